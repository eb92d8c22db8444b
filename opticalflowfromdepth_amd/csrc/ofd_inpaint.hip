// ofd_inpaint.hip -- MI355X (gfx950) hole-fill: layered Telea inpainting.
//
// Replaces utils.inpaint (utils.py:136-151), which the reference runs on the
// CPU after every warp: D2H copy, the keep-mask algebra (:137-142), a uint8
// cast (:148), cv2.inpaint(..., 3, cv2.INPAINT_TELEA) (:149), H2D copy.
//
// cv2's Telea fill is a sequential fast march: a heap pops the hole pixel of
// smallest distance T, which fixes its neighbours' T and colours one at a
// time.  Here holes are finalised in level-synchronous layers instead --
// layer(p) = L1 distance from p to the nearest known pixel -- and every pixel
// of a layer is computed in parallel from exactly the pixels of earlier
// layers, with cv2's own weights (distance, level-set and direction terms,
// the gradient-corrected sample, the 2x central differences and border index
// shifts) and its FastMarching_solve update.  The outer band of negative
// distances around the holes is built the same way, by L1 distance to the
// band.  A hole not yet finalised reads as its input value and its distance
// as 1e6, which is what cv2 does for a pixel still INSIDE, so a layer's
// results do not depend on the order of its pixels.  The CPU restatement is
// oracle/inpaint_oracle.c (layered mode); cv2 parity is unpinned (no OpenCV).
//
// Four launches per chunk of images:
//   PREP   one thread per pixel: keep mask (3x3 dilation of valid != coll),
//          hole bits, out = float(uint8(img)) for every pixel.
//   COLS   one thread per column: vertical distances to the nearest known /
//          hole pixel (two sweeps).
//   ROWS   one thread per row: the row pass of both L1 distance transforms,
//          the Chebyshev-radius test of the outer band; writes the per-pixel
//          code (hole layer / band / ring layer / far) and initial T.
//   TELEA  one 1024-thread workgroup per image: counting sort of the pixels by
//          layer (LDS histogram + block scan), then the outer-band layers and
//          the hole layers, one workgroup barrier per layer.
//
// Plain HIP for gfx950; FP contraction off so the float / double sequence is
// the oracle's.

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "ofd_fw.h"
#include "ofd_inpaint.h"

#pragma clang fp contract(off)

namespace {

constexpr float T_FAR = 1.0e6f;
// per-pixel code: bit 15 hole, bit 14 outer ring, bit 13 far known, low 13
// bits the layer (holes: L1 distance to the known region, LAY_INF = none;
// ring: L1 distance to the band); 0 = band (known, 4-adjacent to a hole)
constexpr unsigned C_HOLE = 0x8000u, C_RING = 0x4000u, C_FAR = 0x2000u, LAY = 0x1FFFu, LAY_INF = 0x1FFFu;
constexpr int DINF = 0x3FFF;  // distance "infinity" in the transforms (> H + W)
constexpr int kMaxHW = 8192;  // H + W limit: layers fit 13 bits, bins fit LDS
constexpr int kMaxRange = 100;
constexpr int kMaxBins = kMaxHW + 2 * kMaxRange;
constexpr int kTeleaThreads = 1024;
constexpr int kChanGroup = 4;  // channels accumulated together per window pass

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

size_t per_image(int64_t H, int64_t W) {
    const size_t HW = size_t(H) * size_t(W);
    return align256(HW * 2) + align256(HW * 4) * 3;  // code, T, list (= ROWS temp), gcol
}

struct IpWs {
    uint16_t *code;
    float *T;
    uint32_t *list;
    uint32_t *gcol;
};

IpWs carve(void *ws, int64_t G, int64_t HW) {
    char *p = static_cast<char *>(ws);
    IpWs w;
    w.code = reinterpret_cast<uint16_t *>(p);
    p += align256(size_t(G) * size_t(HW) * 2);
    w.T = reinterpret_cast<float *>(p);
    p += align256(size_t(G) * size_t(HW) * 4);
    w.list = reinterpret_cast<uint32_t *>(p);
    p += align256(size_t(G) * size_t(HW) * 4);
    w.gcol = reinterpret_cast<uint32_t *>(p);
    return w;
}

// numpy float32 -> uint8 on x86 (utils.py:148): truncate through int32, keep the low byte
__device__ __forceinline__ unsigned to_u8(float v) {
    if (!(v > -2147483648.0f && v < 2147483648.0f)) return 0u;
    return unsigned(int(v)) & 0xFFu;
}

// cv::saturate_cast<uchar>(float): round half to even, clamp
__device__ __forceinline__ unsigned sat_u8(float v) {
    const float r = __builtin_rintf(v);
    return r < 0.f ? 0u : (r > 255.f ? 255u : unsigned(r));
}

// ---------------------------------------------------------------- PREP
// utils.py:137-142: M = valid != coll; M' = 3x3 max (border excluded);
// P = M' == M; H' = uint8(valid * P); fill where 1 - H' != 0.
__global__ __launch_bounds__(256) void ip_prep_kernel(const float *__restrict__ img, const float *__restrict__ valid,
                                                      const float *__restrict__ coll, float *__restrict__ out,
                                                      uint16_t *__restrict__ code, int C, int H, int W, int64_t b0) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.z, b = b0 + bl;
    const float *v = valid + b * HW, *cl = coll + b * HW;
    const int64_t p = int64_t(y) * W + x;
    unsigned mp = 0;
    for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
            const int yy = y + dy, xx = x + dx;
            if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
                const int64_t q = int64_t(yy) * W + xx;
                mp |= v[q] != cl[q] ? 1u : 0u;
            }
        }
    const unsigned M = v[p] != cl[p] ? 1u : 0u;
    const unsigned P = mp == M ? 1u : 0u;
    const unsigned hp = to_u8(v[p] * float(P));
    code[bl * HW + p] = hp != 1u ? uint16_t(C_HOLE) : uint16_t(0);
    const float *ib = img + b * int64_t(C) * HW;
    float *ob = out + b * int64_t(C) * HW;
    for (int c = 0; c < C; ++c) ob[c * HW + p] = float(to_u8(ib[c * HW + p]));
}

// ---------------------------------------------------------------- COLS
// gcol = (vertical distance to the nearest known pixel) | (to the nearest hole) << 16
__global__ __launch_bounds__(256) void ip_cols_kernel(const uint16_t *__restrict__ code, uint32_t *__restrict__ gcol,
                                                      int H, int W) {
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= W) return;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.y;
    const uint16_t *cb = code + bl * HW;
    uint32_t *gb = gcol + bl * HW;
    int lk = -DINF, lh = -DINF;
    for (int y = 0; y < H; ++y) {
        const bool hole = cb[int64_t(y) * W + x] & C_HOLE;
        if (hole) lh = y; else lk = y;
        const int gk = min(y - lk, DINF), gh = min(y - lh, DINF);
        gb[int64_t(y) * W + x] = uint32_t(gk) | (uint32_t(gh) << 16);
    }
    int nk = 2 * DINF, nh = 2 * DINF;
    for (int y = H - 1; y >= 0; --y) {
        const int64_t p = int64_t(y) * W + x;
        const bool hole = cb[p] & C_HOLE;
        if (hole) nh = y; else nk = y;
        const uint32_t g = gb[p];
        const int gk = min(int(g & 0xFFFFu), min(nk - y, DINF)), gh = min(int(g >> 16), min(nh - y, DINF));
        gb[p] = uint32_t(gk) | (uint32_t(gh) << 16);
    }
}

// ---------------------------------------------------------------- ROWS
// Row pass of the L1 distance transforms, d(x) = min_x' g(x') + |x - x'|,
// and the outer-band test "a hole within Chebyshev distance r" = some x' in
// [x - r, x + r] with vertical hole distance <= r.  tmp = forward results.
__global__ __launch_bounds__(64) void ip_rows_kernel(uint16_t *__restrict__ code, float *__restrict__ T,
                                                     const uint32_t *__restrict__ gcol, uint32_t *__restrict__ tmp,
                                                     int H, int W, int r) {
    const int y = blockIdx.x * 64 + threadIdx.x;
    if (y >= H) return;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.y;
    const int64_t row = bl * HW + int64_t(y) * W;
    int fk = DINF, fh = DINF, lastok = -2 * DINF;
    for (int x = 0; x < W; ++x) {
        const uint32_t g = gcol[row + x];
        const int gk = int(g & 0xFFFFu), gh = int(g >> 16);
        fk = min(gk, fk + 1);
        fh = min(gh, fh + 1);
        if (gh <= r) lastok = x;
        tmp[row + x] = uint32_t(fk) | (uint32_t(fh) << 16) | (x - lastok <= r ? 0x80000000u : 0u);
    }
    int bk = DINF, bh = DINF, nextok = 2 * DINF;
    for (int x = W - 1; x >= 0; --x) {
        const uint32_t f = tmp[row + x];
        const uint32_t g = gcol[row + x];
        bk = min(int(f & 0x7FFFu), bk + 1);
        bh = min(int((f >> 16) & 0x7FFFu), bh + 1);
        if (int(g >> 16) <= r) nextok = x;
        const bool near = (f >> 31) || nextok - x <= r;
        const bool hole = code[row + x] & C_HOLE;
        unsigned cd;
        float t = T_FAR;
        if (hole) {
            cd = C_HOLE | unsigned(bk >= int(LAY_INF) ? LAY_INF : bk);
        } else if (bh == 1) {
            cd = 0u;  // band
            t = 0.f;
        } else if (near && bh < DINF) {
            cd = C_RING | unsigned(bh - 1);
        } else {
            cd = C_FAR;
        }
        code[row + x] = uint16_t(cd);
        T[row + x] = t;
    }
}

// ---------------------------------------------------------------- TELEA
struct Img {  // one image's state inside the TELEA workgroup
    const uint16_t *code;
    float *T;
    const float *img;  // input planes (uint8 values of not-yet-final holes)
    float *out;        // output planes (final values of earlier layers)
    int H, W, C;
    int64_t HW;
};

// inner pass: a hole of layer >= L is INSIDE; outer pass: a ring pixel of layer >= L
template <bool kOuter>
__device__ __forceinline__ bool inside(const Img &m, int y, int x, unsigned L) {
    if (y < 0 || x < 0 || y >= m.H || x >= m.W) return false;  // cv2's padded border is KNOWN
    const unsigned c = m.code[int64_t(y) * m.W + x];
    return (c & (kOuter ? C_RING : C_HOLE)) && (c & LAY) >= L;
}

template <bool kOuter>
__device__ __forceinline__ float tval(const Img &m, int y, int x, unsigned L, bool &in) {
    in = inside<kOuter>(m, y, x, L);
    if (in || y < 0 || x < 0 || y >= m.H || x >= m.W) return T_FAR;
    return m.T[int64_t(y) * m.W + x];
}

// FastMarching_solve (double), with cv2's flag cases
__device__ __forceinline__ float fm_solve(float t1, bool in1, float t2, bool in2) {
    const double a11 = t1, a22 = t2;
    const double m12 = a11 < a22 ? a11 : a22;
    double sol;
    if (!in1) {
        if (!in2) {
            if (fabs(a11 - a22) >= 1.0)
                sol = 1 + m12;
            else
                sol = (a11 + a22 + sqrt(double(2 - (a11 - a22) * (a11 - a22)))) * 0.5;
        } else {
            sol = 1 + a11;
        }
    } else if (!in2) {
        sol = 1 + a22;
    } else {
        sol = 1 + m12;
    }
    return float(sol);
}

__device__ __forceinline__ float min4f(float a, float b, float c, float d) {
    const float x = a < b ? a : b, y = c < d ? c : d;
    return x < y ? x : y;
}

template <bool kOuter>
__device__ __forceinline__ float fm_dist(const Img &m, int y, int x, unsigned L) {
    bool iu, id, il, ir;
    const float tu = tval<kOuter>(m, y - 1, x, L, iu), td = tval<kOuter>(m, y + 1, x, L, id);
    const float tl = tval<kOuter>(m, y, x - 1, L, il), tr = tval<kOuter>(m, y, x + 1, L, ir);
    return min4f(fm_solve(tu, iu, tl, il), fm_solve(td, id, tl, il), fm_solve(tu, iu, tr, ir),
                 fm_solve(td, id, tr, ir));
}

// channel value at (y, x): a hole of this layer or later reads as its input
__device__ __forceinline__ int sample(const Img &m, int y, int x, int c, unsigned L) {
    const int64_t q = int64_t(y) * m.W + x;
    const unsigned cd = m.code[q];
    if ((cd & C_HOLE) && (cd & LAY) >= L) return int(to_u8(m.img[c * m.HW + q]));
    return int(m.out[c * m.HW + q]);
}

// Telea colour of hole (y, x) at layer L, channels [c0, c0 + n): the
// weighted sum over the finalised pixels within `range` (icvTeleaInpaintFMM).
__device__ void telea_colour(const Img &m, int y, int x, unsigned L, float tij, int range, int c0, int n,
                             unsigned res[kChanGroup]) {
    bool in_r, in_l, in_d, in_u;
    const float t_r = tval<false>(m, y, x + 1, L, in_r), t_l = tval<false>(m, y, x - 1, L, in_l);
    const float t_d = tval<false>(m, y + 1, x, L, in_d), t_u = tval<false>(m, y - 1, x, L, in_u);
    float gtx, gty;
    if (!in_r)
        gtx = !in_l ? (t_r - t_l) * 0.5f : (t_r - tij);
    else
        gtx = !in_l ? (tij - t_l) : 0.f;
    if (!in_d)
        gty = !in_u ? (t_d - t_u) * 0.5f : (t_d - tij);
    else
        gty = !in_u ? (tij - t_u) : 0.f;
    float Ia[kChanGroup], Jx[kChanGroup], Jy[kChanGroup];
#pragma unroll
    for (int c = 0; c < kChanGroup; ++c) Ia[c] = Jx[c] = Jy[c] = 0.f;
    float s = 1.0e-20f;
    const int H = m.H, W = m.W;
    for (int k = y - range; k <= y + range; ++k) {
        if (k < 0 || k >= H) continue;
        // cv2's border shifts (padded k == 1 <-> image row 0, k == rows-2 <-> H-1)
        const int km = k + (k == 0), kp = k - (k == H - 1);
        for (int l = x - range; l <= x + range; ++l) {
            if (l < 0 || l >= W) continue;
            if ((l - x) * (l - x) + (k - y) * (k - y) > range * range) continue;
            if (inside<false>(m, k, l, L)) continue;
            const int lm = l + (l == 0), lp = l - (l == W - 1);
            const float ry = float(y - k), rx = float(x - l);
            const float len2 = rx * rx + ry * ry;
            const float dst = float(1. / (double(len2) * sqrt(double(len2))));
            const float tkl = m.T[int64_t(k) * W + l];
            const float lev = float(1. / (1 + fabs(double(tkl - tij))));
            float dir = rx * gtx + ry * gty;
            if (fabs(double(dir)) <= 0.01) dir = 0.000001f;
            const float w = float(fabs(double(dst * lev * dir)));
            const bool nr = !inside<false>(m, k, l + 1, L), nl = !inside<false>(m, k, l - 1, L);
            const bool nd = !inside<false>(m, k + 1, l, L), nu = !inside<false>(m, k - 1, l, L);
            for (int c = 0; c < n; ++c) {
                const int cc = c0 + c;
                float gix, giy;
                if (nr)
                    gix = nl ? float(sample(m, km, lp + 1, cc, L) - sample(m, km, lm - 1, cc, L)) * 2.0f
                             : float(sample(m, km, lp + 1, cc, L) - sample(m, km, lm, cc, L));
                else
                    gix = nl ? float(sample(m, km, lp, cc, L) - sample(m, km, lm - 1, cc, L)) : 0.f;
                if (nd)
                    giy = nu ? float(sample(m, kp + 1, lm, cc, L) - sample(m, km - 1, lm, cc, L)) * 2.0f
                             : float(sample(m, kp + 1, lm, cc, L) - sample(m, km, lm, cc, L));
                else
                    giy = nu ? float(sample(m, kp, lm, cc, L) - sample(m, km - 1, lm, cc, L)) : 0.f;
                Ia[c] += w * float(sample(m, km, lm, cc, L));
                Jx[c] -= w * (gix * rx);
                Jy[c] -= w * (giy * ry);
            }
            s += w;
        }
    }
#pragma unroll
    for (int c = 0; c < kChanGroup; ++c) {
        const float sat = float(double(Ia[c] / s) +
                                double(Jx[c] + Jy[c]) / (sqrt(double(Jx[c] * Jx[c] + Jy[c] * Jy[c])) + double(1.0e-20f)) +
                                double(0.5f));
        res[c] = sat_u8(sat);
    }
}

// exclusive block scan of bins[0, n) in place (1024 threads)
__device__ void block_exclusive_scan(unsigned *bins, int n, unsigned *wsum) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n + kTeleaThreads - 1) / kTeleaThreads;
    const int beg = min(tid * per, n), end = min(beg + per, n);
    unsigned sum = 0;
    for (int i = beg; i < end; ++i) sum += bins[i];
    unsigned incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    if (tid == 0) {
        unsigned acc = 0;
        for (int k = 0; k < kTeleaThreads / 64; ++k) {
            const unsigned v = wsum[k];
            wsum[k] = acc;
            acc += v;
        }
    }
    __syncthreads();
    unsigned excl = incl - sum + wsum[wave];
    for (int i = beg; i < end; ++i) {
        const unsigned v = bins[i];
        bins[i] = excl;
        excl += v;
    }
    __syncthreads();
}

__global__ __launch_bounds__(kTeleaThreads) void ip_telea_kernel(const float *__restrict__ img, float *__restrict__ out,
                                                                 IpWs ws, int C, int H, int W, int range, int64_t b0) {
    __shared__ unsigned bins[kMaxBins];
    __shared__ unsigned wsum[kTeleaThreads / 64];
    __shared__ unsigned maxin;
    const int tid = threadIdx.x;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.x, b = b0 + bl;
    Img m;
    m.code = ws.code + bl * HW;
    m.T = ws.T + bl * HW;
    m.img = img + b * int64_t(C) * HW;
    m.out = out + b * int64_t(C) * HW;
    m.H = H;
    m.W = W;
    m.C = C;
    m.HW = HW;
    uint32_t *list = ws.list + bl * HW;
    const int nring = 2 * range;  // ring layers are 1 .. 2r - 1
    // ---- counting sort of ring pixels (bins 0 .. nring-1) and holes (bins nring ..) by layer
    for (int k = tid; k < kMaxBins; k += kTeleaThreads) bins[k] = 0;
    if (tid == 0) maxin = 0;
    __syncthreads();
    for (int64_t p = tid; p < HW; p += kTeleaThreads) {
        const unsigned cd = m.code[p], l = cd & LAY;
        if (cd & C_HOLE) {
            if (l != LAY_INF) {
                atomicAdd(&bins[nring + int(l) - 1], 1u);
                atomicMax(&maxin, l);
            }
        } else if (cd & C_RING) {
            atomicAdd(&bins[int(l) - 1], 1u);
        }
    }
    __syncthreads();
    const int nbins = nring + int(maxin);
    block_exclusive_scan(bins, nbins, wsum);
    for (int64_t p = tid; p < HW; p += kTeleaThreads) {
        const unsigned cd = m.code[p], l = cd & LAY;
        int bin = -1;
        if (cd & C_HOLE) {
            if (l != LAY_INF) bin = nring + int(l) - 1;
        } else if (cd & C_RING) {
            bin = int(l) - 1;
        }
        if (bin >= 0) list[atomicAdd(&bins[bin], 1u)] = uint32_t(p);
    }
    __syncthreads();
    // bin k now spans [k ? bins[k-1] : 0, bins[k])
    // ---- outer band: icvCalcFMM over the ring, layer by layer, then negated
    for (int L = 1; L < nring; ++L) {
        const unsigned beg = L > 1 ? bins[L - 2] : 0u, end = bins[L - 1];
        for (unsigned i = beg + tid; i < end; i += kTeleaThreads) {
            const uint32_t p = list[i];
            const int y = int(p / unsigned(W)), x = int(p - unsigned(y) * unsigned(W));
            m.T[p] = fm_dist<true>(m, y, x, unsigned(L));
        }
        __syncthreads();
    }
    {
        const unsigned end = bins[nring - 1];
        for (unsigned i = tid; i < end; i += kTeleaThreads) {
            const uint32_t p = list[i];
            m.T[p] = -m.T[p];
        }
    }
    __syncthreads();
    // ---- holes, layer by layer
    for (int L = 1; L <= int(maxin); ++L) {
        const int k = nring + L - 1;
        const unsigned beg = bins[k - 1], end = bins[k];
        for (unsigned i = beg + tid; i < end; i += kTeleaThreads) {
            const uint32_t p = list[i];
            const int y = int(p / unsigned(W)), x = int(p - unsigned(y) * unsigned(W));
            const float t = fm_dist<false>(m, y, x, unsigned(L));
            m.T[p] = t;
            for (int c0 = 0; c0 < C; c0 += kChanGroup) {
                const int n = min(kChanGroup, C - c0);
                unsigned res[kChanGroup];
                telea_colour(m, y, x, unsigned(L), t, range, c0, n, res);
                for (int c = 0; c < n; ++c) m.out[(c0 + c) * HW + p] = float(res[c]);
            }
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" {

size_t ofd_inpaint_workspace_bytes(int64_t B, int64_t H, int64_t W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return size_t(B) * per_image(H, W) + 256;
}

int ofd_inpaint_telea_f32(const float *img, const float *valid, const float *collision, float *out, int64_t B,
                          int64_t C, int64_t H, int64_t W, int radius, void *workspace, size_t workspace_bytes,
                          void *stream) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return OFD_FW_EINVAL;
    if (B * C * H * W == 0) return OFD_FW_OK;
    if (!img || !valid || !collision || !out) return OFD_FW_EINVAL;
    if (H < 2 || W < 2) return OFD_FW_EINVAL;
    if (H + W > kMaxHW || H * W >= (int64_t(1) << 31)) return OFD_FW_ETOOBIG;
    const int r = radius < 1 ? 1 : (radius > kMaxRange ? kMaxRange : radius);
    const int64_t HW = H * W;
    const size_t pi = per_image(H, W);
    if (!workspace || (reinterpret_cast<uintptr_t>(workspace) & 255u)) return OFD_FW_EWORKSPACE;
    int64_t G = int64_t(workspace_bytes / pi);
    if (G < 1) return OFD_FW_EWORKSPACE;
    if (G > B) G = B;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const IpWs w = carve(workspace, G, HW);
    for (int64_t b0 = 0; b0 < B; b0 += G) {
        const int64_t nb = B - b0 < G ? B - b0 : G;
        hipLaunchKernelGGL(ip_prep_kernel, dim3(unsigned((W + 63) / 64), unsigned((H + 3) / 4), unsigned(nb)),
                           dim3(256), 0, st, img, valid, collision, out, w.code, int(C), int(H), int(W), b0);
        hipLaunchKernelGGL(ip_cols_kernel, dim3(unsigned((W + 255) / 256), unsigned(nb)), dim3(256), 0, st, w.code,
                           w.gcol, int(H), int(W));
        hipLaunchKernelGGL(ip_rows_kernel, dim3(unsigned((H + 63) / 64), unsigned(nb)), dim3(64), 0, st, w.code, w.T,
                           w.gcol, w.list, int(H), int(W), r);
        hipLaunchKernelGGL(ip_telea_kernel, dim3(unsigned(nb)), dim3(kTeleaThreads), 0, st, img, out, w, int(C),
                           int(H), int(W), r, b0);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

}  // extern "C"
