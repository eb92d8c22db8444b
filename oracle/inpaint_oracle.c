/*
 * oracle/inpaint_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatements of the reference's hole-fill, utils.inpaint
 * (utils.py:136-151).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, as the checker / CPU baseline; the
 * product path (opticalflowfromdepth_amd) never links or calls it.
 *
 * utils.inpaint does two things:
 *   1. mask algebra (utils.py:137-142, restated exactly):
 *        M  = 1 - (valid == collision)            (uint8)
 *        M' = cv2.dilate(M, ones(3,3))            (in-image 3x3 max)
 *        P  = (M' == M)
 *        H' = uint8(valid * P)
 *        inpaint mask = 1 - H'                    (uint8; nonzero = fill)
 *      and the image cast img.permute(1,2,0).numpy().astype(np.uint8)
 *      (utils.py:148; x86 numpy: truncate through int32, keep the low byte).
 *   2. cv2.inpaint(img_u8, mask, 3, cv2.INPAINT_TELEA) (utils.py:149) and the
 *      cast back to float32.  OpenCV is a third-party dependency that is absent
 *      here (nearest pin in the reference: opencv-python==4.5.3.56,
 *      adjusted_gmflow/environment.yml:133).  Sequential mode restates its
 *      published algorithm (modules/photo/src/inpaint.cpp: Telea 2004 fast
 *      marching -- cvInpaint, icvCalcFMM, icvTeleaInpaintFMM): the sorted-list
 *      priority queue (FIFO among equal T), the outer band of negative
 *      distances `range` wide, the padded one-pixel KNOWN border with t = 1e6,
 *      the 2x factor on central colour differences and the km/kp/lm/lp index
 *      shifts at the image border.  PARITY UNPINNED: no OpenCV in this image
 *      and no fixture in the reference pins the fill values.
 *
 * Layered mode restates the product's GPU algorithm (DESIGN.md "Hole-fill"):
 * the same Telea weights and FMM update, but holes are finalised in
 * level-synchronous layers -- layer(p) = L1 distance from p to the nearest
 * known pixel; the outer band likewise by L1 distance to the band -- instead
 * of one pixel at a time in heap order.  Inside a layer every pixel sees
 * exactly the pixels of earlier layers as known, and a hole not yet finalised
 * reads as its input value, so the result does not depend on the order of a
 * layer's pixels; the GPU kernel must match it bit for bit.
 * tests/test_inpaint.py reports its distance from sequential mode.
 *
 * In both modes an INSIDE pixel's distance reads as 1e6 (cv2 never writes t
 * of an INSIDE pixel, so this is exactly its behaviour, and it keeps a
 * layer's concurrent writes invisible).  Images smaller than 2x2 are rejected
 * (-1): cv2's border index shifts read outside them.  Arithmetic follows the
 * C types of the OpenCV source: float image maths, double in
 * FastMarching_solve and in the weight / saturation divisions; built with
 * -ffp-contract=off.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { KNOWN = 0, BAND = 1, INSIDE = 2, CHANGE = 3 };
#define T_FAR 1.0e6f
#define LAY_INF 0x7FFFFFFF

/* ------------------------------------------------------------ mask algebra */
/* numpy float32 -> uint8 on x86: cvttss2si to int32, keep the low byte */
static inline uint8_t to_u8(float v) {
    if (!(v > -2147483648.0f && v < 2147483648.0f)) return 0;
    return (uint8_t)(int32_t)v;
}

/* utils.py:137-142 -> hole[p] = 1 where the inpaint mask is nonzero */
static void hole_mask(const float *valid, const float *coll, long H, long W, uint8_t *hole) {
    uint8_t *M = (uint8_t *)malloc((size_t)(H * W));
    for (long p = 0; p < H * W; ++p) M[p] = (uint8_t)(1 - (valid[p] == coll[p]));
    for (long y = 0; y < H; ++y)
        for (long x = 0; x < W; ++x) {
            uint8_t mp = 0; /* cv2.dilate 3x3: the image border never contributes */
            for (long dy = -1; dy <= 1; ++dy)
                for (long dx = -1; dx <= 1; ++dx) {
                    const long yy = y + dy, xx = x + dx;
                    if (yy >= 0 && yy < H && xx >= 0 && xx < W && M[yy * W + xx] > mp) mp = M[yy * W + xx];
                }
            const long p = y * W + x;
            const uint8_t P = (uint8_t)(mp == M[p]);
            const uint8_t hp = to_u8(valid[p] * (float)P); /* (H * P).astype(uint8) */
            hole[p] = (uint8_t)(1 - hp) != 0;
        }
    free(M);
}

/* cv::saturate_cast<uchar>(float): round half to even, clamp */
static inline uint8_t sat_u8(float v) {
    const long i = lrintf(v);
    return (uint8_t)(i < 0 ? 0 : (i > 255 ? 255 : i));
}

/* ------------------------------------------------------------ FMM update */
/* FastMarching_solve on padded (H+2) x (W+2) flags f / distances t */
static inline float fm_solve(long i1, long j1, long i2, long j2, const uint8_t *f, const float *t, long ew) {
    const int in1 = f[i1 * ew + j1] == INSIDE, in2 = f[i2 * ew + j2] == INSIDE;
    const double a11 = in1 ? T_FAR : t[i1 * ew + j1], a22 = in2 ? T_FAR : t[i2 * ew + j2];
    const double m12 = a11 < a22 ? a11 : a22;
    double sol;
    if (!in1) {
        if (!in2) {
            if (fabs(a11 - a22) >= 1.0)
                sol = 1 + m12;
            else
                sol = (a11 + a22 + sqrt((double)(2 - (a11 - a22) * (a11 - a22)))) * 0.5;
        } else {
            sol = 1 + a11;
        }
    } else if (!in2) {
        sol = 1 + a22;
    } else {
        sol = 1 + m12;
    }
    return (float)sol;
}

static inline float min4f(float a, float b, float c, float d) {
    const float x = a < b ? a : b, y = c < d ? c : d;
    return x < y ? x : y;
}

static inline float fm_dist(long i, long j, const uint8_t *f, const float *t, long ew) {
    return min4f(fm_solve(i - 1, j, i, j - 1, f, t, ew), fm_solve(i + 1, j, i, j - 1, f, t, ew),
                 fm_solve(i - 1, j, i, j + 1, f, t, ew), fm_solve(i + 1, j, i, j + 1, f, t, ew));
}

/* ------------------------------------------------------------ Telea colour */
/* Colour of padded pixel (i, j): the weighted sum over the known pixels
 * (k, l) within `range` (icvTeleaInpaintFMM).  smp(ctx, y, x) reads the
 * channel's value at unpadded (y, x). */
typedef uint8_t (*sample_fn)(const void *ctx, long y, long x);

static uint8_t telea_colour(long i, long j, const uint8_t *f, const float *t, long eh, long ew, int range,
                            sample_fn smp, const void *ctx) {
#define IN(a, b) (f[(a) * ew + (b)] == INSIDE)
#define TT(a, b) t[(a) * ew + (b)]
    float gtx, gty;
    const float tij = TT(i, j);
    if (!IN(i, j + 1))
        gtx = !IN(i, j - 1) ? (TT(i, j + 1) - TT(i, j - 1)) * 0.5f : (TT(i, j + 1) - tij);
    else
        gtx = !IN(i, j - 1) ? (tij - TT(i, j - 1)) : 0.f;
    if (!IN(i + 1, j))
        gty = !IN(i - 1, j) ? (TT(i + 1, j) - TT(i - 1, j)) * 0.5f : (TT(i + 1, j) - tij);
    else
        gty = !IN(i - 1, j) ? (tij - TT(i - 1, j)) : 0.f;
    float Ia = 0, Jx = 0, Jy = 0, s = 1.0e-20f;
    for (long k = i - range; k <= i + range; ++k) {
        const long km = k - 1 + (k == 1), kp = k - 1 - (k == eh - 2);
        for (long l = j - range; l <= j + range; ++l) {
            const long lm = l - 1 + (l == 1), lp = l - 1 - (l == ew - 2);
            if (!(k > 0 && l > 0 && k < eh - 1 && l < ew - 1)) continue;
            if (IN(k, l) || (l - j) * (l - j) + (k - i) * (k - i) > (long)range * range) continue;
            const float ry = (float)(i - k), rx = (float)(j - l);
            const float len2 = rx * rx + ry * ry;
            const float dst = (float)(1. / (len2 * sqrt((double)len2)));
            const float lev = (float)(1. / (1 + fabs((double)(TT(k, l) - tij))));
            float dir = rx * gtx + ry * gty;
            if (fabs((double)dir) <= 0.01) dir = 0.000001f;
            const float w = (float)fabs((double)(dst * lev * dir));
            float gix, giy;
            if (!IN(k, l + 1))
                gix = !IN(k, l - 1) ? (float)((int)smp(ctx, km, lp + 1) - (int)smp(ctx, km, lm - 1)) * 2.0f
                                    : (float)((int)smp(ctx, km, lp + 1) - (int)smp(ctx, km, lm));
            else
                gix = !IN(k, l - 1) ? (float)((int)smp(ctx, km, lp) - (int)smp(ctx, km, lm - 1)) : 0.f;
            if (!IN(k + 1, l))
                giy = !IN(k - 1, l) ? (float)((int)smp(ctx, kp + 1, lm) - (int)smp(ctx, km - 1, lm)) * 2.0f
                                    : (float)((int)smp(ctx, kp + 1, lm) - (int)smp(ctx, km, lm));
            else
                giy = !IN(k - 1, l) ? (float)((int)smp(ctx, kp, lm) - (int)smp(ctx, km - 1, lm)) : 0.f;
            Ia += w * (float)smp(ctx, km, lm);
            Jx -= w * (gix * rx);
            Jy -= w * (giy * ry);
            s += w;
        }
    }
#undef IN
#undef TT
    const float sat = (float)(Ia / s + (Jx + Jy) / (sqrt((double)(Jx * Jx + Jy * Jy)) + 1.0e-20f) + 0.5f);
    return sat_u8(sat);
}

/* ------------------------------------------------------------ sequential (cv2) */
/* Stable min-priority queue on (T, push order): OpenCV's sorted doubly linked
 * list inserts a new element after every element with T <= its own, so equal
 * T pop in push order. */
typedef struct { float T; uint64_t seq; int32_t i, j; } HeapEl;
typedef struct { HeapEl *a; long n, cap; uint64_t seq; } Heap;

static int el_less(const HeapEl *x, const HeapEl *y) { return x->T < y->T || (x->T == y->T && x->seq < y->seq); }

static void heap_push(Heap *h, long i, long j, float T) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 1024;
        h->a = (HeapEl *)realloc(h->a, sizeof(HeapEl) * (size_t)h->cap);
    }
    long c = h->n++;
    const HeapEl e = {T, h->seq++, (int32_t)i, (int32_t)j};
    while (c > 0) {
        const long p = (c - 1) / 2;
        if (!el_less(&e, &h->a[p])) break;
        h->a[c] = h->a[p];
        c = p;
    }
    h->a[c] = e;
}

static int heap_pop(Heap *h, long *i, long *j) {
    if (h->n == 0) return 0;
    *i = h->a[0].i;
    *j = h->a[0].j;
    const HeapEl e = h->a[--h->n];
    long c = 0;
    for (;;) {
        long m = 2 * c + 1;
        if (m >= h->n) break;
        if (m + 1 < h->n && el_less(&h->a[m + 1], &h->a[m])) ++m;
        if (!el_less(&h->a[m], &e)) break;
        h->a[c] = h->a[m];
        c = m;
    }
    if (h->n) h->a[c] = e;
    return 1;
}

typedef struct { const uint8_t *img; long W; } SeqCtx;
static uint8_t seq_sample(const void *ctx, long y, long x) {
    const SeqCtx *c = (const SeqCtx *)ctx;
    return c->img[y * c->W + x];
}

static void telea_seq_image(uint8_t *planes, long C, long H, long W, const uint8_t *hole, int range) {
    const long eh = H + 2, ew = W + 2, en = eh * ew;
    uint8_t *mask = (uint8_t *)calloc((size_t)en, 1), *band = (uint8_t *)calloc((size_t)en, 1);
    uint8_t *out = (uint8_t *)calloc((size_t)en, 1);
    float *t = (float *)malloc(sizeof(float) * (size_t)en);
    for (long k = 0; k < en; ++k) t[k] = T_FAR;
    for (long y = 0; y < H; ++y)
        for (long x = 0; x < W; ++x)
            if (hole[y * W + x]) mask[(y + 1) * ew + x + 1] = INSIDE;
    /* band = cross dilation of the mask minus the mask (border cleared) */
    for (long i = 1; i < eh - 1; ++i)
        for (long j = 1; j < ew - 1; ++j) {
            const long p = i * ew + j;
            if (!mask[p] && (mask[p - 1] || mask[p + 1] || mask[p - ew] || mask[p + ew])) band[p] = 1;
        }
    /* outer ring: square dilation by `range`, minus mask, minus band */
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
    /* icvCalcFMM(out, t, Out, negate = true) */
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
    /* icvTeleaInpaintFMM(mask, t, img, range, Heap) */
    while (heap_pop(&heap, &ii, &jj)) {
        mask[ii * ew + jj] = KNOWN;
        for (int q = 0; q < 4; ++q) {
            const long i = ii + (q == 0 ? -1 : q == 2 ? 1 : 0), j = jj + (q == 1 ? -1 : q == 3 ? 1 : 0);
            if (i <= 0 || j <= 0 || i > eh - 1 || j > ew - 1) continue;
            if (mask[i * ew + j] == INSIDE) {
                const float d = fm_dist(i, j, mask, t, ew);
                t[i * ew + j] = d;
                for (long c = 0; c < C; ++c) {
                    const SeqCtx cx = {planes + c * H * W, W};
                    planes[c * H * W + (i - 1) * W + (j - 1)] = telea_colour(i, j, mask, t, eh, ew, range, seq_sample, &cx);
                }
                mask[i * ew + j] = BAND;
                heap_push(&heap, i, j, d);
            }
        }
    }
    free(heap.a);
    free(outq.a);
    free(mask);
    free(band);
    free(out);
    free(t);
}

/* ------------------------------------------------------------ layered (GPU algorithm) */
typedef struct { const uint8_t *cur, *orig, *hole; const int32_t *lay; long W; int32_t L; } LayCtx;
/* a hole of this layer or a later one still reads as its input value */
static uint8_t lay_sample(const void *ctx, long y, long x) {
    const LayCtx *c = (const LayCtx *)ctx;
    const long q = y * c->W + x;
    return (c->hole[q] && c->lay[q] >= c->L) ? c->orig[q] : c->cur[q];
}

/* L1 distance transform: d[p] = min over q with src[q] != 0 of |dy| + |dx| */
static void l1_dt(const uint8_t *src, long H, long W, int32_t *d) {
    for (long p = 0; p < H * W; ++p) d[p] = src[p] ? 0 : LAY_INF;
    for (long y = 0; y < H; ++y)
        for (long x = 0; x < W; ++x) {
            int32_t v = d[y * W + x];
            if (x > 0 && d[y * W + x - 1] != LAY_INF && d[y * W + x - 1] + 1 < v) v = d[y * W + x - 1] + 1;
            if (y > 0 && d[(y - 1) * W + x] != LAY_INF && d[(y - 1) * W + x] + 1 < v) v = d[(y - 1) * W + x] + 1;
            d[y * W + x] = v;
        }
    for (long y = H - 1; y >= 0; --y)
        for (long x = W - 1; x >= 0; --x) {
            int32_t v = d[y * W + x];
            if (x < W - 1 && d[y * W + x + 1] != LAY_INF && d[y * W + x + 1] + 1 < v) v = d[y * W + x + 1] + 1;
            if (y < H - 1 && d[(y + 1) * W + x] != LAY_INF && d[(y + 1) * W + x] + 1 < v) v = d[(y + 1) * W + x] + 1;
            d[y * W + x] = v;
        }
}

static void telea_layered_image(uint8_t *planes, long C, long H, long W, const uint8_t *hole, int range) {
    const long HW = H * W, eh = H + 2, ew = W + 2, en = eh * ew;
    uint8_t *known = (uint8_t *)malloc((size_t)HW);
    int32_t *din = (int32_t *)malloc(sizeof(int32_t) * (size_t)HW), *dh = (int32_t *)malloc(sizeof(int32_t) * (size_t)HW);
    int32_t *olay = (int32_t *)calloc((size_t)HW, sizeof(int32_t));
    for (long p = 0; p < HW; ++p) known[p] = !hole[p];
    l1_dt(known, H, W, din); /* holes: layer = L1 distance to the nearest known pixel */
    l1_dt(hole, H, W, dh);   /* known: L1 distance to the nearest hole (1 = band) */
    int32_t maxo = 0, maxi = 0;
    for (long y = 0; y < H; ++y)
        for (long x = 0; x < W; ++x) {
            const long p = y * W + x;
            if (hole[p]) {
                if (din[p] != LAY_INF && din[p] > maxi) maxi = din[p];
                continue;
            }
            if (dh[p] <= 1 || dh[p] == LAY_INF) continue;
            /* outer ring: a hole within Chebyshev distance `range`; layer = L1 distance to the band */
            int near = 0;
            for (long yy = y - range; yy <= y + range && !near; ++yy)
                for (long xx = x - range; xx <= x + range; ++xx)
                    if (yy >= 0 && xx >= 0 && yy < H && xx < W && hole[yy * W + xx]) { near = 1; break; }
            if (near) {
                olay[p] = dh[p] - 1;
                if (olay[p] > maxo) maxo = olay[p];
            }
        }
    /* bucket the ring pixels and the holes by layer (raster order inside a layer) */
    long *obeg = (long *)calloc((size_t)maxo + 2, sizeof(long)), *ibeg = (long *)calloc((size_t)maxi + 2, sizeof(long));
    for (long p = 0; p < HW; ++p) {
        if (olay[p] > 0) ++obeg[olay[p] + 1];
        if (hole[p] && din[p] != LAY_INF) ++ibeg[din[p] + 1];
    }
    for (int32_t L = 1; L <= maxo; ++L) obeg[L + 1] += obeg[L];
    for (int32_t L = 1; L <= maxi; ++L) ibeg[L + 1] += ibeg[L];
    long *olist = (long *)malloc(sizeof(long) * (size_t)(obeg[maxo + 1] + 1));
    long *ilist = (long *)malloc(sizeof(long) * (size_t)(ibeg[maxi + 1] + 1));
    {
        long *oc = (long *)malloc(sizeof(long) * ((size_t)maxo + 2)), *ic = (long *)malloc(sizeof(long) * ((size_t)maxi + 2));
        memcpy(oc, obeg, sizeof(long) * ((size_t)maxo + 2));
        memcpy(ic, ibeg, sizeof(long) * ((size_t)maxi + 2));
        for (long p = 0; p < HW; ++p) {
            if (olay[p] > 0) olist[oc[olay[p]]++] = p;
            if (hole[p] && din[p] != LAY_INF) ilist[ic[din[p]]++] = p;
        }
        free(oc);
        free(ic);
    }
    uint8_t *f = (uint8_t *)calloc((size_t)en, 1);
    float *t = (float *)malloc(sizeof(float) * (size_t)en);
    for (long k = 0; k < en; ++k) t[k] = T_FAR;
    for (long p = 0; p < HW; ++p)
        if (!hole[p] && dh[p] == 1) t[(p / W + 1) * ew + p % W + 1] = 0.f;
    /* outer pass: ring pixels of layer >= L are INSIDE */
    for (long p = 0; p < HW; ++p) f[(p / W + 1) * ew + p % W + 1] = olay[p] > 0 ? INSIDE : KNOWN;
    for (int32_t L = 1; L <= maxo; ++L) {
        for (long n = obeg[L]; n < obeg[L + 1]; ++n) {
            const long p = olist[n];
            t[(p / W + 1) * ew + p % W + 1] = fm_dist(p / W + 1, p % W + 1, f, t, ew);
        }
        for (long n = obeg[L]; n < obeg[L + 1]; ++n) f[(olist[n] / W + 1) * ew + olist[n] % W + 1] = KNOWN;
    }
    for (long p = 0; p < HW; ++p)
        if (!hole[p] && (dh[p] == 1 || olay[p] > 0)) t[(p / W + 1) * ew + p % W + 1] *= -1.f;
    uint8_t *orig = (uint8_t *)malloc((size_t)(C * HW));
    memcpy(orig, planes, (size_t)(C * HW));
    /* inner pass: holes of layer >= L are INSIDE */
    for (long p = 0; p < HW; ++p) f[(p / W + 1) * ew + p % W + 1] = hole[p] ? INSIDE : KNOWN;
    for (int32_t L = 1; L <= maxi; ++L) {
        for (long n = ibeg[L]; n < ibeg[L + 1]; ++n) {
            const long p = ilist[n], y = p / W + 1, x = p % W + 1;
            t[y * ew + x] = fm_dist(y, x, f, t, ew);
            for (long c = 0; c < C; ++c) {
                const LayCtx cx = {planes + c * HW, orig + c * HW, hole, din, W, L};
                planes[c * HW + p] = telea_colour(y, x, f, t, eh, ew, range, lay_sample, &cx);
            }
        }
        for (long n = ibeg[L]; n < ibeg[L + 1]; ++n) f[(ilist[n] / W + 1) * ew + ilist[n] % W + 1] = KNOWN;
    }
    free(olist);
    free(ilist);
    free(obeg);
    free(ibeg);
    free(orig);
    free(f);
    free(t);
    free(olay);
    free(known);
    free(din);
    free(dh);
}

/* ------------------------------------------------------------ entry points */
/* utils.inpaint over a batch: img [B,C,H,W] f32, valid / collision [B,1,H,W]
 * f32 -> out [B,C,H,W] f32 (float of uint8).  layered = 0: cv2 sequential
 * restatement; 1: the GPU's layered algorithm.  range = cv2 inpaintRange
 * (cvRound'ed and clamped to [1, 100] as cvInpaint does). */
int oracle_inpaint_f32(const float *img, const float *valid, const float *coll, float *outp, long B, long C, long H,
                       long W, int range, int layered, int nthreads) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return -1;
    if (B * C * H * W == 0) return 0;
    if (H < 2 || W < 2) return -1;
    range = range < 1 ? 1 : (range > 100 ? 100 : range);
    const long HW = H * W;
    long b;
    (void)nthreads;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())
    for (b = 0; b < B; ++b) {
        uint8_t *hole = (uint8_t *)malloc((size_t)HW);
        uint8_t *planes = (uint8_t *)malloc((size_t)(C * HW));
        hole_mask(valid + b * HW, coll + b * HW, H, W, hole);
        for (long k = 0; k < C * HW; ++k) planes[k] = to_u8(img[b * C * HW + k]);
        if (layered)
            telea_layered_image(planes, C, H, W, hole, range);
        else
            telea_seq_image(planes, C, H, W, hole, range);
        for (long k = 0; k < C * HW; ++k) outp[b * C * HW + k] = (float)planes[k];
        free(planes);
        free(hole);
    }
    return 0;
}

/* the mask algebra alone (utils.py:137-142): hole [B,H,W] uint8, 1 = fill */
int oracle_inpaint_mask(const float *valid, const float *coll, uint8_t *hole, long B, long H, long W) {
    if (B < 0 || H < 0 || W < 0) return -1;
    for (long b = 0; b < B; ++b) hole_mask(valid + b * H * W, coll + b * H * W, H, W, hole + b * H * W);
    return 0;
}
