/* tools/kahn_levels.c -- diagnostic: the colour DAG of the sequential fill.
 *
 * For one hole mask (H x W bytes, 1 = hole) runs cv2's two marches as the
 * oracle does (oracle/inpaint_oracle.c, included for its march helpers),
 * records each hole's push stamp, and gives every hole its Kahn level over the
 * positions its colour reads (need3: the radius-3 disk and its 4-neighbours;
 * a hole depends on the holes of smaller stamp there).  Prints the level
 * profile: how many holes each level holds, and how much of the work sits in
 * narrow levels -- what bounds a colour pass on one CU (issue) against k CUs
 * (the dependent chain).
 *
 *   gcc -O2 -o /tmp/kahn_levels tools/kahn_levels.c -lm
 *   /tmp/kahn_levels H W mask.u8 [levels.out]
 */
#include <stdio.h>

#include "../oracle/inpaint_oracle.c"

static int need3(int a, int b) {
#define D3(x, y) ((x) * (x) + (y) * (y) <= 9)
    return D3(a, b) || D3(a + 1, b) || D3(a - 1, b) || D3(a, b + 1) || D3(a, b - 1);
#undef D3
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: kahn_levels H W mask.u8 [levels.out]\n");
        return 2;
    }
    const long H = atol(argv[1]), W = atol(argv[2]);
    const long eh = H + 2, ew = W + 2, en = eh * ew;
    uint8_t *hole = (uint8_t *)malloc((size_t)(H * W));
    FILE *f = fopen(argv[3], "rb");
    if (!f || fread(hole, 1, (size_t)(H * W), f) != (size_t)(H * W)) return 3;
    fclose(f);
    const int range = 3;
    uint8_t *mask = (uint8_t *)calloc((size_t)en, 1), *band = (uint8_t *)calloc((size_t)en, 1);
    uint8_t *out = (uint8_t *)calloc((size_t)en, 1);
    float *t = (float *)malloc(sizeof(float) * (size_t)en);
    uint32_t *stamp = (uint32_t *)calloc((size_t)en, 4);
    int32_t *lev = (int32_t *)calloc((size_t)en, 4);
    for (long k = 0; k < en; ++k) t[k] = T_FAR;
    for (long y = 0; y < H; ++y)
        for (long x = 0; x < W; ++x)
            if (hole[y * W + x]) mask[(y + 1) * ew + x + 1] = INSIDE;
    for (long i = 1; i < eh - 1; ++i)
        for (long j = 1; j < ew - 1; ++j) {
            const long p = i * ew + j;
            if (!mask[p] && (mask[p - 1] || mask[p + 1] || mask[p - ew] || mask[p + ew])) band[p] = 1;
        }
    for (long i = 1; i < eh - 1; ++i)
        for (long j = 1; j < ew - 1; ++j) {
            const long p = i * ew + j;
            if (mask[p] || band[p]) continue;
            int near = 0;
            for (long y = i - range; y <= i + range && !near; ++y)
                for (long x = j - range; x <= j + range; ++x)
                    if (y > 0 && x > 0 && y < eh - 1 && x < ew - 1 && mask[y * ew + x]) { near = 1; break; }
            if (near) out[p] = INSIDE;
        }
    Heap heap = {0}, outq = {0};
    for (long i = 0; i < eh; ++i)
        for (long j = 0; j < ew; ++j)
            if (band[i * ew + j]) {
                heap_push(&heap, i, j, 0.f);
                heap_push(&outq, i, j, 0.f);
                t[i * ew + j] = 0.f;
            }
    long ii, jj;
    while (heap_pop(&outq, &ii, &jj)) {
        out[ii * ew + jj] = CHANGE;
        for (int q = 0; q < 4; ++q) {
            const long i = ii + (q == 0 ? -1 : q == 2 ? 1 : 0), j = jj + (q == 1 ? -1 : q == 3 ? 1 : 0);
            if (i <= 0 || j <= 0 || i > eh || j > ew) continue;
            if (out[i * ew + j] == INSIDE) {
                const float d = fm_dist(i, j, out, t, ew);
                t[i * ew + j] = d;
                out[i * ew + j] = BAND;
                heap_push(&outq, i, j, d);
            }
        }
    }
    for (long k = 0; k < en; ++k)
        if (out[k] == CHANGE) t[k] = -t[k];
    uint32_t seq = 0;
    long nholes = 0;
    int32_t maxl = 0;
    while (heap_pop(&heap, &ii, &jj)) {
        mask[ii * ew + jj] = KNOWN;
        for (int q = 0; q < 4; ++q) {
            const long i = ii + (q == 0 ? -1 : q == 2 ? 1 : 0), j = jj + (q == 1 ? -1 : q == 3 ? 1 : 0);
            if (i <= 0 || j <= 0 || i > eh - 1 || j > ew - 1) continue;
            if (mask[i * ew + j] == INSIDE) {
                const float d = fm_dist(i, j, mask, t, ew);
                t[i * ew + j] = d;
                stamp[i * ew + j] = ++seq;  /* pushed = coloured, in this order */
                int32_t l = 0;
                for (int a = -4; a <= 4; ++a)
                    for (int b = -4; b <= 4; ++b) {
                        if (!need3(a, b) || (a == 0 && b == 0)) continue;
                        const long y = i + a, x = j + b;
                        if (y <= 0 || x <= 0 || y >= eh - 1 || x >= ew - 1) continue;
                        const long pq = y * ew + x;
                        if (stamp[pq] && stamp[pq] < seq && lev[pq] + 1 > l) l = lev[pq] + 1;
                    }
                lev[i * ew + j] = l;
                if (l > maxl) maxl = l;
                ++nholes;
                mask[i * ew + j] = BAND;
                heap_push(&heap, i, j, d);
            }
        }
    }
    long *width = (long *)calloc((size_t)maxl + 1, sizeof(long));
    for (long k = 0; k < en; ++k)
        if (stamp[k]) width[lev[k]]++;
    /* holes in levels of width < w, for a few w; and the level count of each class */
    const long cuts[] = {8, 16, 32, 64, 128, 256, 512, 1024, 1L << 40};
    printf("holes %ld levels %d mean width %.1f\n", nholes, maxl + 1, (double)nholes / (maxl + 1));
    long prev = 0;
    for (int c = 0; c < 9; ++c) {
        long nl = 0, nh = 0;
        for (int32_t l = 0; l <= maxl; ++l)
            if (width[l] >= prev && width[l] < cuts[c]) { ++nl; nh += width[l]; }
        printf("  width [%ld, %ld): %6ld levels, %8ld holes (%.1f%%)\n", prev, cuts[c] > (1L << 39) ? -1 : cuts[c], nl,
               nh, 100.0 * nh / (nholes ? nholes : 1));
        prev = cuts[c];
    }
    /* batches of up to 8 holes per wave: a lower bound on one CU's batch count
     * per level and what the level chain costs at k CUs of 16 waves each */
    for (int k = 1; k <= 8; k *= 2) {
        long batches = 0, rounds = 0;
        for (int32_t l = 0; l <= maxl; ++l) {
            const long b = (width[l] + 7) / 8;
            batches += b;
            rounds += (b + 16 * k - 1) / (16 * k);
        }
        printf("  k=%d: batches %ld, serial wave-rounds %ld\n", k, batches, rounds);
    }
    if (argc > 4) {
        FILE *o = fopen(argv[4], "w");
        for (int32_t l = 0; l <= maxl; ++l) fprintf(o, "%ld\n", width[l]);
        fclose(o);
    }
    return 0;
}
