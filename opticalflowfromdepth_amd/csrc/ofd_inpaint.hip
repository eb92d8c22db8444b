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
// Launches per chunk of images:
//   PREP   one thread per pixel: keep mask (3x3 dilation of valid != coll),
//          hole bits, out = float(uint8(img)) for every pixel.
//   COLS   64 columns x 8 row segments per workgroup: vertical distances to
//          the nearest known / hole pixel (two sweeps).
//   ROWS   one wave per row (prefix / suffix scans): the row pass of both L1 distance transforms,
//          the Chebyshev-radius test of the outer band; writes the per-pixel
//          code (hole layer / band / ring layer / far) and initial T.
//   SORT   chip-wide counting sort of ring pixels and holes by layer (LDS
//          histograms, one scan, one scatter); the counts stay on the device.
//   LAYERS one launch per outer-band layer and per hole layer over every
//          image of the chunk, each reading its layer's size and offset from
//          the device; a persistent deep-tail kernel runs any layer deeper
//          than the launches (no inter-workgroup waits anywhere).  Grids and the number of
//          launches come from recent calls' counts read back asynchronously
//          (LaggedStats): the host never waits.
//
// Plain HIP for gfx950; FP contraction off so the float / double sequence is
// the oracle's.

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "ofd_fw.h"
#include "ofd_inpaint.h"

#pragma clang fp contract(off)

// Fault word of the layered fill (ofd_inpaint_faults): bit 8 = the deep
// tail's wait for a previous layer passed its bound (unreachable: every part
// it waits for is held by a running workgroup; the wait gives up rather than
// hang, and the output is then incomplete).  Bits 1-2 are the sequential
// fill's.
__device__ unsigned g_ip_fault;
// layers run by the deep-tail kernel (ofd_inpaint_tail_layers)
__device__ unsigned g_ip_tail_layers;

unsigned ofd_sq_fault_read(int reset);  // ofd_inpaint_seq.hip

namespace {

#include "ip_common.h"

// Diagnostic build only (tools/probe_ip.hip defines OFD_IP_STAMPS): thread 0
// of the first block of each path of a hole-layer launch records shader-clock
// stamps along the per-hole chain; the product build compiles them out.
#ifdef OFD_IP_STAMPS
__device__ unsigned long long *g_ip_stamps;
__device__ __forceinline__ void ip_stamp(unsigned slot, unsigned k) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    if (g_ip_stamps) g_ip_stamps[slot * 8 + k] = __builtin_amdgcn_s_memtime();
}
#define IP_STAMP(slot, k, cond) do { if (cond) ip_stamp(slot, k); } while (0)
#else
#define IP_STAMP(slot, k, cond) do { } while (0)
#endif

// per-pixel code: bit 15 hole, bit 14 outer ring, bit 13 far known, low 13
// bits the layer (holes: L1 distance to the known region, LAY_INF = none;
// ring: L1 distance to the band); 0 = band (known, 4-adjacent to a hole)
constexpr unsigned C_HOLE = 0x8000u, C_RING = 0x4000u, C_FAR = 0x2000u, LAY = 0x1FFFu, LAY_INF = 0x1FFFu;
constexpr int DINF = 0x3FFF;  // distance "infinity" in the transforms (> H + W)
constexpr int kMaxHW = 4096;  // H + W limit: layers fit 13 bits, 2 bins per layer fit LDS
constexpr int kMaxRange = 100;
constexpr int kMaxBins = 2 * kMaxHW + 2 * kMaxRange;
constexpr int kChanGroup = 4;
constexpr unsigned kCsSplitMax = 262144;  // interior holes of a layer above which one thread takes a whole hole  // channels accumulated together per window pass

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

// Four consecutive pixels per thread (W % 4 == 0, 16-byte aligned planes):
// the 3x3 neighbourhood of the quad is 3 rows x 6 columns of valid /
// collision, loaded as one float4 plus two edge values per row (18 loads per
// 4 pixels instead of 18 per pixel), and the C channel planes move as float4.
__global__ __launch_bounds__(256) void ip_prep4_kernel(const float *__restrict__ img, const float *__restrict__ valid,
                                                       const float *__restrict__ coll, float *__restrict__ out,
                                                       uint16_t *__restrict__ code, int C, int H, int W, int64_t b0) {
    const int x = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4, y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= W || y >= H) return;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.z, b = b0 + bl;
    const float *v = valid + b * HW, *cl = coll + b * HW;
    const int64_t p = int64_t(y) * W + x;
    unsigned mrow[3] = {0u, 0u, 0u};  // bit k: M at column x - 1 + k (0 outside the image)
    float vc[4];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int yy = y - 1 + r;
        if (yy < 0 || yy >= H) continue;
        const int64_t q = int64_t(yy) * W + x;
        const float4 a = *reinterpret_cast<const float4 *>(v + q), c = *reinterpret_cast<const float4 *>(cl + q);
        unsigned m = ((a.x != c.x) ? 2u : 0u) | ((a.y != c.y) ? 4u : 0u) | ((a.z != c.z) ? 8u : 0u) |
                     ((a.w != c.w) ? 16u : 0u);
        if (x > 0) m |= (v[q - 1] != cl[q - 1]) ? 1u : 0u;
        if (x + 4 < W) m |= (v[q + 4] != cl[q + 4]) ? 32u : 0u;
        mrow[r] = m;
        if (r == 1) { vc[0] = a.x; vc[1] = a.y; vc[2] = a.z; vc[3] = a.w; }
    }
    const unsigned mo = mrow[0] | mrow[1] | mrow[2];
    ushort4 cd;
    unsigned short *cde = reinterpret_cast<unsigned short *>(&cd);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const unsigned mp = (mo >> e) & 7u ? 1u : 0u;
        const unsigned M = (mrow[1] >> (e + 1)) & 1u;
        const unsigned P = mp == M ? 1u : 0u;
        const unsigned hp = to_u8(vc[e] * float(P));
        cde[e] = hp != 1u ? uint16_t(C_HOLE) : uint16_t(0);
    }
    *reinterpret_cast<ushort4 *>(code + bl * HW + p) = cd;
    const float *ib = img + b * int64_t(C) * HW;
    float *ob = out + b * int64_t(C) * HW;
    for (int c = 0; c < C; ++c) {
        const float4 a = *reinterpret_cast<const float4 *>(ib + c * HW + p);
        *reinterpret_cast<float4 *>(ob + c * HW + p) =
            make_float4(float(to_u8(a.x)), float(to_u8(a.y)), float(to_u8(a.z)), float(to_u8(a.w)));
    }
}

// ---------------------------------------------------------------- COLS
// gcol = (vertical distance to the nearest known pixel) | (to the nearest hole) << 16
// Workgroup = 64 columns x kColSegs row segments; thread (segment, column).
// Pass 1 sweeps the segment downwards with segment-local state (DINF where
// the segment has no known pixel / hole above), and records the segment's
// first and last known / hole rows in LDS; pass 2 sweeps upwards with the
// state entering from the segments below, patches the DINF entries with the
// state entering from above, and takes the min of both directions.  Same
// values as one sequential sweep per column (thread per column before:
// 620 us per 64 images at one wave per SIMD).
constexpr int kColSegs = 8;
__global__ __launch_bounds__(64 * kColSegs) void ip_cols_kernel(const uint16_t *__restrict__ code,
                                                                 uint32_t *__restrict__ gcol, int H, int W) {
    __shared__ int lastk[kColSegs][64], lasth[kColSegs][64], firstk[kColSegs][64], firsth[kColSegs][64];
    const int cx = threadIdx.x & 63, sg = threadIdx.x >> 6;
    const int x = blockIdx.x * 64 + cx;
    const int SL = (H + kColSegs - 1) / kColSegs, y0 = min(sg * SL, H), y1 = min(y0 + SL, H);
    const int64_t HW = int64_t(H) * W, bl = blockIdx.y;
    const uint16_t *cb = code + bl * HW;
    uint32_t *gb = gcol + bl * HW;
    int lk = -DINF, lh = -DINF, fk = 2 * DINF, fh = 2 * DINF;
    if (x < W)
        for (int y = y0; y < y1; ++y) {
            const bool hole = cb[int64_t(y) * W + x] & C_HOLE;
            if (hole) {
                lh = y;
                fh = min(fh, y);
            } else {
                lk = y;
                fk = min(fk, y);
            }
            const int gk = min(y - lk, DINF), gh = min(y - lh, DINF);
            gb[int64_t(y) * W + x] = uint32_t(gk) | (uint32_t(gh) << 16);
        }
    lastk[sg][cx] = lk;
    lasth[sg][cx] = lh;
    firstk[sg][cx] = fk;
    firsth[sg][cx] = fh;
    __syncthreads();
    int lk_in = -DINF, lh_in = -DINF, nk = 2 * DINF, nh = 2 * DINF;
    for (int t = 0; t < sg; ++t) {
        lk_in = max(lk_in, lastk[t][cx]);
        lh_in = max(lh_in, lasth[t][cx]);
    }
    for (int t = kColSegs - 1; t > sg; --t) {
        nk = min(nk, firstk[t][cx]);
        nh = min(nh, firsth[t][cx]);
    }
    if (x >= W) return;
    for (int y = y1 - 1; y >= y0; --y) {
        const int64_t p = int64_t(y) * W + x;
        const bool hole = cb[p] & C_HOLE;
        if (hole) nh = y; else nk = y;
        const uint32_t g = gb[p];
        int fwk = int(g & 0xFFFFu), fwh = int(g >> 16);
        if (fwk == DINF) fwk = min(y - lk_in, DINF);
        if (fwh == DINF) fwh = min(y - lh_in, DINF);
        const int gk = min(fwk, min(nk - y, DINF)), gh = min(fwh, min(nh - y, DINF));
        gb[p] = uint32_t(gk) | (uint32_t(gh) << 16);
    }
}

// ---------------------------------------------------------------- ROWS
// Row pass of the L1 distance transforms, d(x) = min_x' g(x') + |x - x'|,
// and the outer-band test "a hole within Chebyshev distance r" = some x' in
// [x - r, x + r] with vertical hole distance <= r.  One wave per row, 64
// columns per step (coalesced), using the closed forms of the two sweeps:
//   forward  f(x) = x + min_{x' <= x} (g(x') - x')     (prefix min)
//   backward d(x) = -x + min_{x' >= x} (f(x') + x')    (suffix min)
// and, for the band test, the last / next column x' with g_hole(x') <= r
// (prefix max / suffix min).  tmp holds the forward results.
constexpr int kBig = 1 << 28;

__device__ __forceinline__ int wave_prefix_min(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(v, d);
        if (lane >= d) v = min(v, o);
    }
    return v;
}
__device__ __forceinline__ int wave_prefix_max(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(v, d);
        if (lane >= d) v = max(v, o);
    }
    return v;
}
__device__ __forceinline__ int wave_suffix_min(int v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_down(v, d);
        if (lane + d < 64) v = min(v, o);
    }
    return v;
}

__global__ __launch_bounds__(256) void ip_rows_kernel(uint16_t *__restrict__ code, float *__restrict__ T,
                                                      const uint32_t *__restrict__ gcol, uint32_t *__restrict__ tmp,
                                                      int H, int W, int r) {
    const int y = blockIdx.x * 4 + int(threadIdx.x >> 6);
    if (y >= H) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.y;
    const int64_t row = bl * HW + int64_t(y) * W;
    int ck = kBig, ch = kBig, cl = -kBig;
    for (int x0 = 0; x0 < W; x0 += 64) {
        const int x = x0 + lane;
        int vk = kBig, vh = kBig, lo = -kBig;
        if (x < W) {
            const uint32_t g = gcol[row + x];
            const int gk = int(g & 0xFFFFu), gh = int(g >> 16);
            vk = gk - x;
            vh = gh - x;
            lo = gh <= r ? x : -kBig;
        }
        vk = min(wave_prefix_min(vk), ck);
        vh = min(wave_prefix_min(vh), ch);
        lo = max(wave_prefix_max(lo), cl);
        ck = __shfl(vk, 63);
        ch = __shfl(vh, 63);
        cl = __shfl(lo, 63);
        if (x < W)
            tmp[row + x] = uint32_t(x + vk) | (uint32_t(x + vh) << 16) | (x - lo <= r ? 0x80000000u : 0u);
    }
    int sk = kBig, sh = kBig, sn = kBig;
    for (int x0 = ((W - 1) / 64) * 64; x0 >= 0; x0 -= 64) {
        const int x = x0 + lane;
        int uk = kBig, uh = kBig, nx = kBig;
        uint32_t f = 0;
        if (x < W) {
            f = tmp[row + x];
            const uint32_t g = gcol[row + x];
            uk = int(f & 0x7FFFu) + x;
            uh = int((f >> 16) & 0x7FFFu) + x;
            nx = int(g >> 16) <= r ? x : kBig;
        }
        uk = min(wave_suffix_min(uk), sk);
        uh = min(wave_suffix_min(uh), sh);
        nx = min(wave_suffix_min(nx), sn);
        sk = __shfl(uk, 0);
        sh = __shfl(uh, 0);
        sn = __shfl(nx, 0);
        if (x < W) {
            const int bk = uk - x, bh = uh - x;
            const bool near = (f >> 31) || nx - x <= r;
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
}

// ROWS for W <= 64 * kRowRegs: the whole row lives in registers (kRowRegs
// values per lane), so every gcol / code load of the row issues up front and
// the forward results never round-trip through tmp.  Same arithmetic as
// ip_rows_kernel (which ran one dependent load per 64-column step).
constexpr int kRowRegs = 16;
__global__ __launch_bounds__(256) void ip_rows_reg_kernel(uint16_t *__restrict__ code, float *__restrict__ T,
                                                          const uint32_t *__restrict__ gcol, int H, int W, int r) {
    const int y = blockIdx.x * 4 + int(threadIdx.x >> 6);
    if (y >= H) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.y;
    const int64_t row = bl * HW + int64_t(y) * W;
    const int nst = (W + 63) / 64;
    uint32_t g[kRowRegs], f[kRowRegs];
    bool hole[kRowRegs];
#pragma unroll
    for (int s = 0; s < kRowRegs; ++s) {
        const int x = s * 64 + lane;
        g[s] = 0u;
        hole[s] = false;
        if (s < nst && x < W) {
            g[s] = gcol[row + x];
            hole[s] = code[row + x] & C_HOLE;
        }
    }
    int ck = kBig, ch = kBig, cl = -kBig;
#pragma unroll
    for (int s = 0; s < kRowRegs; ++s) {
        const int x = s * 64 + lane;
        int vk = kBig, vh = kBig, lo = -kBig;
        if (s < nst && x < W) {  // steps past the row hold the scan identities
            const int gk = int(g[s] & 0xFFFFu), gh = int(g[s] >> 16);
            vk = gk - x;
            vh = gh - x;
            lo = gh <= r ? x : -kBig;
        }
        vk = min(wave_prefix_min(vk), ck);
        vh = min(wave_prefix_min(vh), ch);
        lo = max(wave_prefix_max(lo), cl);
        ck = __shfl(vk, 63);
        ch = __shfl(vh, 63);
        cl = __shfl(lo, 63);
        f[s] = uint32_t(x + vk) | (uint32_t(x + vh) << 16) | (x - lo <= r ? 0x80000000u : 0u);
    }
    int sk = kBig, sh = kBig, sn = kBig;
#pragma unroll
    for (int s = kRowRegs - 1; s >= 0; --s) {
        const int x = s * 64 + lane;
        int uk = kBig, uh = kBig, nx = kBig;
        if (s < nst && x < W) {
            uk = int(f[s] & 0x7FFFu) + x;
            uh = int((f[s] >> 16) & 0x7FFFu) + x;
            nx = int(g[s] >> 16) <= r ? x : kBig;
        }
        uk = min(wave_suffix_min(uk), sk);
        uh = min(wave_suffix_min(uh), sh);
        nx = min(wave_suffix_min(nx), sn);
        sk = __shfl(uk, 0);
        sh = __shfl(uh, 0);
        sn = __shfl(nx, 0);
        if (s < nst && x < W) {
            const int bk = uk - x, bh = uh - x;
            const bool near = (f[s] >> 31) || nx - x <= r;
            unsigned cd;
            float t = T_FAR;
            if (hole[s]) {
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

// The Telea colour for range 3 (the reference's inpaintRange) with register
// patches: the 9x9 patches of INSIDE flags, distances and channel values
// around the hole are loaded once (every load independent of the others),
// then weights and sums are formed in cv2's exact (k, l) order (hole_wave), so
// the result is bit-identical.
//   kBorder = false: window plus one-pixel halo inside the image, no border
//     index shifts; every sampled position is then a finalised pixel, so
//     values come straight from `out`.
//   kBorder = true: any position; out-of-image patch entries read as KNOWN
//     with t = 1e6 (cv2's padded border), cv2's km / kp / lm / lp shifts at
//     the image border become selects between neighbouring patch entries, and
//     a sampled pixel still INSIDE reads as its input value (sample()).
constexpr bool in_disk3(int a, int b) { return a * a + b * b <= 9; }
constexpr bool need3(int a, int b) {  // in the disk, or a 4-neighbour of a disk position
    return in_disk3(a, b) || in_disk3(a - 1, b) || in_disk3(a + 1, b) || in_disk3(a, b - 1) || in_disk3(a, b + 1);
}
constexpr int pidx(int a, int b) { return (a + 4) * 9 + (b + 4); }

template <bool kBorder>
__device__ __forceinline__ void telea_pixel_r3(const Img &m, int y, int x, unsigned L, int64_t p, int c_lo, int c_hi) {
    const int W = m.W, H = m.H;
    // patch position (a, b) -> in-image flag and (clamped) pixel index; every
    // load below is unconditional, so they all issue before the first use
    auto inimg = [&](int a, int b) -> bool {
        return !kBorder || (y + a >= 0 && y + a < H && x + b >= 0 && x + b < W);
    };
    auto at = [&](int a, int b) -> int64_t {
        if (!kBorder) return p + int64_t(a) * W + b;
        const int yy = min(max(y + a, 0), H - 1), xx = min(max(x + b, 0), W - 1);
        return int64_t(yy) * W + xx;
    };
    unsigned cds[81];
#pragma unroll
    for (int a = -4; a <= 4; ++a)
#pragma unroll
        for (int b = -4; b <= 4; ++b)
            if (need3(a, b)) cds[pidx(a, b)] = m.code[at(a, b)];
    float tk[81];
#pragma unroll
    for (int a = -3; a <= 3; ++a)
#pragma unroll
        for (int b = -3; b <= 3; ++b)
            if (in_disk3(a, b) && (a || b)) tk[pidx(a, b)] = m.T[at(a, b)];
    uint32_t ib[3] = {0u, 0u, 0u};  // INSIDE bit per patch position (0 outside the image)
#pragma unroll
    for (int a = -4; a <= 4; ++a)
#pragma unroll
        for (int b = -4; b <= 4; ++b) {
            if (!need3(a, b)) continue;
            const unsigned cd = cds[pidx(a, b)];
            const unsigned in = (inimg(a, b) && (cd & C_HOLE) && (cd & LAY) >= L) ? 1u : 0u;
            ib[pidx(a, b) >> 5] |= in << (pidx(a, b) & 31);
        }
    auto IN = [&](int a, int b) -> bool { return (ib[pidx(a, b) >> 5] >> (pidx(a, b) & 31)) & 1u; };
    // distances as tval() reads them: INSIDE or outside the image -> 1e6
#pragma unroll
    for (int a = -3; a <= 3; ++a)
#pragma unroll
        for (int b = -3; b <= 3; ++b)
            if (in_disk3(a, b) && (a || b)) tk[pidx(a, b)] = (IN(a, b) || !inimg(a, b)) ? T_FAR : tk[pidx(a, b)];
    IP_STAMP(2 * L, 2, threadIdx.x == 0 && blockIdx.x == 0);
    // fm_dist<false>
    const float tij = min4f(fm_solve(tk[pidx(-1, 0)], IN(-1, 0), tk[pidx(0, -1)], IN(0, -1)),
                            fm_solve(tk[pidx(1, 0)], IN(1, 0), tk[pidx(0, -1)], IN(0, -1)),
                            fm_solve(tk[pidx(-1, 0)], IN(-1, 0), tk[pidx(0, 1)], IN(0, 1)),
                            fm_solve(tk[pidx(1, 0)], IN(1, 0), tk[pidx(0, 1)], IN(0, 1)));
    if (c_lo == 0) m.T[p] = tij;
    float gtx, gty;
    if (!IN(0, 1))
        gtx = !IN(0, -1) ? (tk[pidx(0, 1)] - tk[pidx(0, -1)]) * 0.5f : (tk[pidx(0, 1)] - tij);
    else
        gtx = !IN(0, -1) ? (tij - tk[pidx(0, -1)]) : 0.f;
    if (!IN(1, 0))
        gty = !IN(-1, 0) ? (tk[pidx(1, 0)] - tk[pidx(-1, 0)]) * 0.5f : (tk[pidx(1, 0)] - tij);
    else
        gty = !IN(-1, 0) ? (tij - tk[pidx(-1, 0)]) : 0.f;
    auto used = [&](int a, int b) -> bool { return in_disk3(a, b) && (a || b) && inimg(a, b) && !IN(a, b); };
    float wt[81];
    float s = 1.0e-20f;
#pragma unroll
    for (int a = -3; a <= 3; ++a)
#pragma unroll
        for (int b = -3; b <= 3; ++b) {
            if (!in_disk3(a, b) || !(a || b)) continue;
            const float ry = float(-a), rx = float(-b);
            const float len2 = rx * rx + ry * ry;
            const float dst = float(1. / (double(len2) * sqrt(double(len2))));
            const float lev = float(1. / (1 + fabs(double(tk[pidx(a, b)] - tij))));
            float dir = rx * gtx + ry * gty;
            if (fabs(double(dir)) <= 0.01) dir = 0.000001f;
            const float w = float(fabs(double(dst * lev * dir)));
            wt[pidx(a, b)] = used(a, b) ? w : 0.f;
            s = used(a, b) ? s + w : s;
        }
    for (int c = c_lo; c < c_hi; ++c) {
        const float *ob = m.out + int64_t(c) * m.HW;
        const float *ib0 = m.img + int64_t(c) * m.HW;
        float V[81];
#pragma unroll
        for (int a = -4; a <= 4; ++a)
#pragma unroll
            for (int b = -4; b <= 4; ++b) {
                if (kBorder) {
                    const float vo = ob[at(a, b)], vi = float(to_u8(ib0[at(a, b)]));
                    V[pidx(a, b)] = IN(a, b) ? vi : vo;  // outside the image: never sampled
                } else if (need3(a, b) && (a || b)) {
                    V[pidx(a, b)] = ob[at(a, b)];
                }
            }
        float Ia = 0.f, Jx = 0.f, Jy = 0.f;
#pragma unroll
        for (int a = -3; a <= 3; ++a)
#pragma unroll
            for (int b = -3; b <= 3; ++b) {
                if (!in_disk3(a, b) || !(a || b)) continue;
                const float ry = float(-a), rx = float(-b), w = wt[pidx(a, b)];
                const bool nr = !IN(a, b + 1), nl = !IN(a, b - 1), nd = !IN(a + 1, b), nu = !IN(a - 1, b);
                float sc, gix, giy;
                if (!kBorder) {
                    sc = V[pidx(a, b)];
                    gix = nr ? (nl ? (V[pidx(a, b + 1)] - V[pidx(a, b - 1)]) * 2.0f : (V[pidx(a, b + 1)] - sc))
                             : (nl ? (sc - V[pidx(a, b - 1)]) : 0.f);
                    giy = nd ? (nu ? (V[pidx(a + 1, b)] - V[pidx(a - 1, b)]) * 2.0f : (V[pidx(a + 1, b)] - sc))
                             : (nu ? (sc - V[pidx(a - 1, b)]) : 0.f);
                } else {
                    // cv2's shifted rows / columns: km = k + (k == 0), kp = k - (k == H-1),
                    // lm = l + (l == 0), lp = l - (l == W-1) (hole_wave)
                    const bool t0 = y + a == 0, tH = y + a == H - 1, l0 = x + b == 0, lW = x + b == W - 1;
                    auto Vs = [&](int r0, bool rs, int c0, bool cs) -> float {  // V(r0 + rs, c0 + cs)
                        const float v00 = V[pidx(r0, c0)], v01 = V[pidx(r0, c0 + 1)];
                        const float v10 = V[pidx(r0 + 1, c0)], v11 = V[pidx(r0 + 1, c0 + 1)];
                        return rs ? (cs ? v11 : v10) : (cs ? v01 : v00);
                    };
                    // rows: km in {a, a+1}, km-1 in {a-1, a}, kp in {a-1, a}, kp+1 in {a, a+1}
                    // cols: lm in {b, b+1}, lm-1 in {b-1, b}, lp in {b-1, b}, lp+1 in {b, b+1}
                    sc = Vs(a, t0, b, l0);                     // (km, lm)
                    const float v_km_lp1 = Vs(a, t0, b, !lW);  // (km, lp+1)
                    const float v_km_lmm = Vs(a, t0, b - 1, l0);
                    const float v_km_lp = Vs(a, t0, b - 1, !lW);
                    const float v_kp1_lm = Vs(a, !tH, b, l0);
                    const float v_kmm_lm = Vs(a - 1, t0, b, l0);
                    const float v_kp_lm = Vs(a - 1, !tH, b, l0);
                    gix = nr ? (nl ? (v_km_lp1 - v_km_lmm) * 2.0f : (v_km_lp1 - sc)) : (nl ? (v_km_lp - v_km_lmm) : 0.f);
                    giy = nd ? (nu ? (v_kp1_lm - v_kmm_lm) * 2.0f : (v_kp1_lm - sc)) : (nu ? (v_kp_lm - v_kmm_lm) : 0.f);
                }
                // unused positions have w == 0: adding +-0 never changes a sum of finite terms
                // except the sign of an exact zero, which the final expression cannot see
                if (used(a, b)) {
                    Ia += w * sc;
                    Jx -= w * (gix * rx);
                    Jy -= w * (giy * ry);
                }
            }
        const float sat =
            float(double(Ia / s) + double(Jx + Jy) / (sqrt(double(Jx * Jx + Jy * Jy)) + double(1.0e-20f)) + double(0.5f));
        IP_STAMP(2 * L, 3, threadIdx.x == 0 && blockIdx.x == 0);
        m.out[int64_t(c) * m.HW + p] = float(sat_u8(sat));
    }
}

// ---------------------------------------------------------------- SORT
// After SCATTER, cursor[k] holds the END of bin k (its start + hist[k]); the
// layer launches read both.
// Counting sort of the chunk's ring pixels and holes by layer, chip-wide:
// bins 0 .. nring-1 = ring layers 1 .., bins nring .. = hole layers 1 ..; an
// entry is bl * HW + p (chunk-local image bl, pixel p).  HIST and SCATTER
// aggregate per workgroup in LDS, so the global atomics are one per
// (workgroup, nonempty bin).  Order inside a bin is irrelevant.
constexpr int kSortThreads = 256;
constexpr int kSortSpan = 16384;  // pixels per sort workgroup

// bins: ring layer l -> l-1; hole layer l -> nring + 2(l-1) for holes the
// register-patch kernel takes (radius 3, window and halo inside the image),
// nring + 2(l-1) + 1 for the others (one wave per hole)
__device__ __forceinline__ bool patch_interior(int64_t e, int64_t HW, int H, int W, bool r3) {
    // entries fit 31 bits (gcap in ofd_inpaint_telea_f32): 32-bit division
    const unsigned p = unsigned(e) % unsigned(HW);
    const int y = int(p / unsigned(W)), x = int(p - unsigned(y) * unsigned(W));
    return r3 && y >= 4 && y < H - 4 && x >= 4 && x < W - 4;
}
__device__ __forceinline__ int bin_of(unsigned cd, int nring, int64_t e, int64_t HW, int H, int W, bool r3) {
    const unsigned l = cd & LAY;
    if (cd & C_HOLE)
        return l != LAY_INF ? nring + 2 * (int(l) - 1) + (patch_interior(e, HW, H, W, r3) ? 0 : 1) : -1;
    if (cd & C_RING) return int(l) - 1;
    return -1;
}

__global__ __launch_bounds__(kSortThreads) void ip_hist_kernel(const uint16_t *__restrict__ code,
                                                               unsigned *__restrict__ hist, int64_t total, int nring,
                                                               int H, int W, bool r3) {
    const int64_t HW = int64_t(H) * W;
    __shared__ unsigned h[kMaxBins];
    for (int k = threadIdx.x; k < kMaxBins; k += kSortThreads) h[k] = 0;
    __syncthreads();
    const int64_t beg = int64_t(blockIdx.x) * kSortSpan, end = min(beg + kSortSpan, total);
    for (int64_t e = beg + threadIdx.x; e < end; e += kSortThreads) {
        const int bin = bin_of(code[e], nring, e, HW, H, W, r3);
        if (bin >= 0) atomicAdd(&h[bin], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kMaxBins; k += kSortThreads)
        if (h[k]) atomicAdd(&hist[k], h[k]);
}

// cursor[k] = exclusive prefix sum of hist (one workgroup); meta[0] = the
// deepest non-empty hole layer (0: no holes), which bounds the device-side
// layer loop of the deep tail kernel.
__global__ __launch_bounds__(1024) void ip_scan_kernel(const unsigned *__restrict__ hist, unsigned *__restrict__ cursor,
                                                       int n, int nring, unsigned *__restrict__ meta) {
    __shared__ unsigned wsum[16];
    __shared__ unsigned lmax;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int per = (n + 1023) / 1024;
    const int beg = min(tid * per, n), end = min(beg + per, n);
    if (tid == 0) lmax = 0;
    unsigned sum = 0, lm = 0;
    for (int i = beg; i < end; ++i) {
        sum += hist[i];
        if (i >= nring && hist[i]) lm = unsigned((i - nring) / 2 + 1);
    }
    unsigned incl = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    if (lm) atomicMax(&lmax, lm);
    if (tid == 0) {
        unsigned acc = 0;
        for (int k = 0; k < 16; ++k) {
            const unsigned v = wsum[k];
            wsum[k] = acc;
            acc += v;
        }
    }
    __syncthreads();
    unsigned excl = incl - sum + wsum[wave];
    for (int i = beg; i < end; ++i) {
        cursor[i] = excl;
        excl += hist[i];
    }
    if (tid == 0) {
        meta[0] = lmax;
        meta[1] = 0u;  // the deep tail's ticket counter
        meta[2] = 0u;  // ... and its count of finished parts
    }
}

__global__ __launch_bounds__(kSortThreads) void ip_scatter_kernel(const uint16_t *__restrict__ code,
                                                                  unsigned *__restrict__ cursor,
                                                                  uint32_t *__restrict__ list, int64_t total,
                                                                  int nring, int H, int W, bool r3) {
    const int64_t HW = int64_t(H) * W;
    __shared__ unsigned h[kMaxBins];
    for (int k = threadIdx.x; k < kMaxBins; k += kSortThreads) h[k] = 0;
    __syncthreads();
    const int64_t beg = int64_t(blockIdx.x) * kSortSpan, end = min(beg + kSortSpan, total);
    for (int64_t e = beg + threadIdx.x; e < end; e += kSortThreads) {
        const int bin = bin_of(code[e], nring, e, HW, H, W, r3);
        if (bin >= 0) atomicAdd(&h[bin], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kMaxBins; k += kSortThreads)
        if (h[k]) h[k] = atomicAdd(&cursor[k], h[k]);  // this workgroup's range of bin k
    __syncthreads();
    for (int64_t e = beg + threadIdx.x; e < end; e += kSortThreads) {
        const int bin = bin_of(code[e], nring, e, HW, H, W, r3);
        if (bin >= 0) list[atomicAdd(&h[bin], 1u)] = uint32_t(e);
    }
}

// ---------------------------------------------------------------- LAYERS
// One launch per layer over every image of the chunk, one thread per pixel.
__device__ __forceinline__ unsigned blocks_for_dev(unsigned n, unsigned per) { return (n + per - 1u) / per; }
struct Chunk {
    const uint16_t *code;
    float *T;
    const float *img;
    float *out;
    int C, H, W;
    int64_t HW, b0;
};

__device__ __forceinline__ Img image_of(const Chunk &ch, uint32_t e, int &y, int &x, int64_t &p) {
    // entries fit 31 bits (gcap in ofd_inpaint_telea_f32): 32-bit divisions
    const unsigned ble = e / unsigned(ch.HW), pe = e - ble * unsigned(ch.HW);
    const int64_t bl = int64_t(ble), b = ch.b0 + bl;
    p = int64_t(pe);
    y = int(pe / unsigned(ch.W));
    x = int(pe - unsigned(y) * unsigned(ch.W));
    Img m;
    m.code = ch.code + bl * ch.HW;
    m.T = ch.T + bl * ch.HW;
    m.img = ch.img + b * int64_t(ch.C) * ch.HW;
    m.out = ch.out + b * int64_t(ch.C) * ch.HW;
    m.H = ch.H;
    m.W = ch.W;
    m.C = ch.C;
    m.HW = ch.HW;
    return m;
}

// Layer launches read their sizes and list offsets from the device (the
// sort's hist / cursor), so the host never waits for them: a fixed grid walks
// each list grid-stride.

// outer band (icvCalcFMM over the ring): ring layer L = bin L - 1
__global__ __launch_bounds__(256) void ip_ring_layer_kernel(Chunk ch, const uint32_t *__restrict__ list,
                                                            const unsigned *__restrict__ hist,
                                                            const unsigned *__restrict__ cursor, unsigned L) {
    const unsigned n = hist[L - 1];
    const uint32_t *lst = list + (cursor[L - 1] - n);  // SCATTER advanced cursor[] to each bin's end
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        int y, x;
        int64_t p;
        const Img m = image_of(ch, lst[i], y, x, p);
        m.T[p] = fm_dist<true>(m, y, x, L);
    }
}

// the outer band's distances are negative (icvCalcFMM negate = true): every
// ring entry, bins 0 .. nring - 1 (list[0, end of bin nring - 1))
__global__ __launch_bounds__(256) void ip_negate_kernel(float *__restrict__ T, const uint32_t *__restrict__ list,
                                                        const unsigned *__restrict__ cursor, int nring) {
    const unsigned n = cursor[nring - 1];
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) T[list[i]] = -T[list[i]];
}

// hole layer L: distance, then every channel's Telea colour
// Patch-interior holes, kCS threads per hole: thread i takes hole i / kCS and
// the channels c = i % kCS, c + kCS, ... of it.  Every thread of a hole
// recomputes the same weights (the code / distance patch loads of one hole
// coalesce into the same lines); only the channel-0 thread writes T.  More,
// shorter threads: a mid-size layer of ~48 k holes otherwise leaves under one
// wave per SIMD, each running the whole serial chain of one hole.
template <int kCS>
__device__ __forceinline__ void hole_patch(const Chunk &ch, const uint32_t *__restrict__ list, unsigned n, unsigned i,
                                           unsigned L) {
    const unsigned h = i / unsigned(kCS), c0 = i - h * unsigned(kCS);
    if (h >= n) return;
    int y, x;
    int64_t p;
    const Img m = image_of(ch, list[h], y, x, p);
    IP_STAMP(2 * L, 1, i == 0);
    if (kCS == 1) {
        telea_pixel_r3<false>(m, y, x, L, p, 0, m.C);  // the sort put only radius-3 interior holes here
    } else {
        for (int c = int(c0); c < m.C; c += kCS) telea_pixel_r3<false>(m, y, x, L, p, c, c + 1);  // C >= 1
    }
    IP_STAMP(2 * L, 4, i == 0);
}

__device__ __forceinline__ float rl(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}

__device__ __forceinline__ void hole_wave(const Chunk &ch, const uint32_t *__restrict__ list, unsigned n, unsigned i,
                                          unsigned L, int range) {
    if (i >= n) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    int y, x;
    int64_t p;
    const Img m = image_of(ch, list[i], y, x, p);
    const int H = m.H, W = m.W, R = range, D = 2 * range + 1, npos = D * D;
    const float tij = fm_dist<false>(m, y, x, L);
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
    for (int c0 = 0; c0 < m.C; c0 += kChanGroup) {
        const int nc = min(kChanGroup, m.C - c0);
        float Ia[kChanGroup], Jx[kChanGroup], Jy[kChanGroup];
#pragma unroll
        for (int c = 0; c < kChanGroup; ++c) Ia[c] = Jx[c] = Jy[c] = 0.f;
        float s = 1.0e-20f;
        for (int base = 0; base < npos; base += 64) {
            const int idx = base + lane;
            const int k = y - R + idx / D, l = x - R + idx % D;
            bool valid = idx < npos && k >= 0 && k < H && l >= 0 && l < W && (l - x) * (l - x) + (k - y) * (k - y) <= R * R;
            valid = valid && !inside<false>(m, k, l, L);
            float w = 0.f, ti[kChanGroup], tx[kChanGroup], ty[kChanGroup];
#pragma unroll
            for (int c = 0; c < kChanGroup; ++c) ti[c] = tx[c] = ty[c] = 0.f;
            if (valid) {
                const int km = k + (k == 0), kp = k - (k == H - 1), lm = l + (l == 0), lp = l - (l == W - 1);
                const float ry = float(y - k), rx = float(x - l);
                const float len2 = rx * rx + ry * ry;
                const float dst = float(1. / (double(len2) * sqrt(double(len2))));
                const float lev = float(1. / (1 + fabs(double(m.T[int64_t(k) * W + l] - tij))));
                float dir = rx * gtx + ry * gty;
                if (fabs(double(dir)) <= 0.01) dir = 0.000001f;
                w = float(fabs(double(dst * lev * dir)));
                const bool nr = !inside<false>(m, k, l + 1, L), nl = !inside<false>(m, k, l - 1, L);
                const bool nd = !inside<false>(m, k + 1, l, L), nu = !inside<false>(m, k - 1, l, L);
                for (int c = 0; c < nc; ++c) {
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
                    ti[c] = w * float(sample(m, km, lm, cc, L));
                    tx[c] = w * (gix * rx);
                    ty[c] = w * (giy * ry);
                }
            }
            const uint64_t vm = __ballot(valid);
            for (int j = 0; j < 64; ++j) {
                if (!((vm >> j) & 1ull)) continue;  // uniform
                for (int c = 0; c < nc; ++c) {
                    Ia[c] += rl(ti[c], j);
                    Jx[c] -= rl(tx[c], j);
                    Jy[c] -= rl(ty[c], j);
                }
                s += rl(w, j);
            }
        }
        if (lane == 0) {
            for (int c = 0; c < nc; ++c) {
                const float sat = float(double(Ia[c] / s) +
                                        double(Jx[c] + Jy[c]) / (sqrt(double(Jx[c] * Jx[c] + Jy[c] * Jy[c])) + double(1.0e-20f)) +
                                        double(0.5f));
                m.out[(c0 + c) * m.HW + p] = float(sat_u8(sat));
            }
        }
    }
    if (lane == 0) m.T[p] = tij;
}

// Wave per hole, radius <= 3: the same arithmetic as hole_wave, but the 9x9
// patch around the hole (INSIDE flags, distances, and per channel group the
// sample() values) is loaded into LDS in ONE round of unconditional, clamped
// loads (entry e = lane, lane + 64).  hole_wave's chain of dependent rounds
// (list -> code -> T -> code -> sample code -> value) becomes list -> patch.
constexpr int kPatch = 9, kPatchN = kPatch * kPatch;
struct WavePatch {
    int fl[kPatchN];                // bit 0: inside the image, bit 1: INSIDE (hole of layer >= L)
    float t[kPatchN];               // T (raw)
    int sv[kChanGroup][kPatchN];    // sample() of the current channel group
    float4 q[64][kChanGroup];       // per window position, per channel: (w*sc, w*gix*rx, w*giy*ry, w)
};

// cv2's distance weight dst = 1 / (|r|^2 * sqrt(|r|^2)) (double, rounded to
// float) for the integer |r|^2 of a radius-3 window: the values the
// double expression gives, bit for bit (host IEEE double = device double).
__device__ __forceinline__ float dst_r3(int len2) {
    switch (len2) {
        case 1: return 0x1p+0f;
        case 2: return 0x1.6a09e6p-2f;
        case 4: return 0x1p-3f;
        case 5: return 0x1.6e5b7ep-4f;
        case 8: return 0x1.6a09e6p-5f;
        default: return 0x1.2f684cp-5f;  // 9
    }
}

// The 28 positions of the radius-3 disk (centre excluded) in raster order of
// the 7 x 7 window, as window indices (dy + 3) * 7 + (dx + 3).
__device__ constexpr int kDisk3[28] = {3,  8,  9,  10, 11, 12, 15, 16, 17, 18, 19, 21, 22, 23,
                                       25, 26, 27, 29, 30, 31, 32, 33, 36, 37, 38, 39, 40, 45};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void hole_wave_lds(const Chunk &ch, const uint32_t *__restrict__ list, unsigned n,
                                              unsigned i, unsigned L, int range, WavePatch &P) {
    if (i >= n) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    int y, x;
    int64_t p;
    const Img m = image_of(ch, list[i], y, x, p);
    IP_STAMP(2 * L + 1, 1, i == 0 && lane == 0);
    const int H = m.H, W = m.W, R = range, D = 2 * range + 1, npos = D * D;
    int64_t qe[2];
    unsigned hge[2];  // sample()'s test: hole of layer >= L
    float vo0[2][kChanGroup], vi0[2][kChanGroup];  // first channel group, loaded with the flags
    const int nc0 = min(kChanGroup, m.C);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int e = lane + 64 * u;
        const int k = y - 4 + e / kPatch, l = x - 4 + e % kPatch;
        const bool inimg = k >= 0 && k < H && l >= 0 && l < W;
        const int kc = min(max(k, 0), H - 1), lc = min(max(l, 0), W - 1);
        qe[u] = int64_t(kc) * W + lc;
#pragma unroll
        for (int c = 0; c < kChanGroup; ++c) {
            vo0[u][c] = vi0[u][c] = 0.f;
            if (c < nc0 && e < kPatchN) {
                vo0[u][c] = m.out[int64_t(c) * m.HW + qe[u]];
                vi0[u][c] = m.img[int64_t(c) * m.HW + qe[u]];
            }
        }
        if (e < kPatchN) {
            const unsigned cd = m.code[qe[u]];
            const float tq = m.T[qe[u]];
            hge[u] = ((cd & C_HOLE) && (cd & LAY) >= L) ? 1u : 0u;
            P.fl[e] = (inimg ? 1 : 0) | ((inimg && hge[u]) ? 2 : 0);
            P.t[e] = tq;
        }
    }
    wave_lds_sync();
    IP_STAMP(2 * L + 1, 2, i == 0 && lane == 0);
    auto IN = [&](int e) -> bool { return (P.fl[e] & 2) != 0; };
    auto TV = [&](int e, bool &in) -> float {
        const int f = P.fl[e];
        in = (f & 2) != 0;
        return (in || !(f & 1)) ? T_FAR : P.t[e];
    };
    constexpr int ctr = 4 * kPatch + 4;
    bool iu, id, il, ir;
    const float tu = TV(ctr - kPatch, iu), td = TV(ctr + kPatch, id);
    const float tl = TV(ctr - 1, il), tr = TV(ctr + 1, ir);
    const float tij = min4f(fm_solve(tu, iu, tl, il), fm_solve(td, id, tl, il), fm_solve(tu, iu, tr, ir),
                            fm_solve(td, id, tr, ir));
    float gtx, gty;
    if (!ir)
        gtx = !il ? (tr - tl) * 0.5f : (tr - tij);
    else
        gtx = !il ? (tij - tl) : 0.f;
    if (!id)
        gty = !iu ? (td - tu) * 0.5f : (td - tij);
    else
        gty = !iu ? (tij - tu) : 0.f;
    for (int c0 = 0; c0 < m.C; c0 += kChanGroup) {
        const int nc = min(kChanGroup, m.C - c0);
        if (c0 > 0) wave_lds_sync();  // the previous group's reads are done
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = lane + 64 * u;
            if (e < kPatchN) {
                if (c0 == 0) {
#pragma unroll
                    for (int c = 0; c < kChanGroup; ++c)
                        if (c < nc) P.sv[c][e] = hge[u] ? int(to_u8(vi0[u][c])) : int(vo0[u][c]);
                } else {
                    for (int c = 0; c < nc; ++c) {
                        const int cc = c0 + c;
                        const float vo = m.out[int64_t(cc) * m.HW + qe[u]], vi = m.img[int64_t(cc) * m.HW + qe[u]];
                        P.sv[c][e] = hge[u] ? int(to_u8(vi)) : int(vo);
                    }
                }
            }
        }
        wave_lds_sync();
        // npos <= 49: one pass
        const int idx = lane;
        const int k = y - R + idx / D, l = x - R + idx % D;
        const int pk = 4 - R + idx / D, pl = 4 - R + idx % D, e = pk * kPatch + pl;
        bool valid = idx < npos && k >= 0 && k < H && l >= 0 && l < W && (l - x) * (l - x) + (k - y) * (k - y) <= R * R;
        valid = valid && !IN(e);
        float w = 0.f, ti[kChanGroup], tx[kChanGroup], ty[kChanGroup];
#pragma unroll
        for (int c = 0; c < kChanGroup; ++c) ti[c] = tx[c] = ty[c] = 0.f;
        if (valid) {
            const int km = pk + (k == 0), kp = pk - (k == H - 1), lm = pl + (l == 0), lp = pl - (l == W - 1);
            const float ry = float(y - k), rx = float(x - l);
            const float len2 = rx * rx + ry * ry;
            const float dst = R <= 3 ? dst_r3(int(len2)) : float(1. / (double(len2) * sqrt(double(len2))));
            const float lev = float(1. / (1 + fabs(double(P.t[e] - tij))));
            float dir = rx * gtx + ry * gty;
            if (fabsf(dir) <= 0.01f) dir = 0.000001f;  // |dir| <= 0.01 (double) <=> |dir| <= 0.01f: no float lies between
            w = fabsf(dst * lev * dir);                // float(fabs(double(f))) == fabsf(f)
            const bool nr = !IN(e + 1), nl = !IN(e - 1), nd = !IN(e + kPatch), nu = !IN(e - kPatch);
            auto S = [&](int c, int a, int b) -> int { return P.sv[c][a * kPatch + b]; };
            for (int c = 0; c < nc; ++c) {
                float gix, giy;
                if (nr)
                    gix = nl ? float(S(c, km, lp + 1) - S(c, km, lm - 1)) * 2.0f : float(S(c, km, lp + 1) - S(c, km, lm));
                else
                    gix = nl ? float(S(c, km, lp) - S(c, km, lm - 1)) : 0.f;
                if (nd)
                    giy = nu ? float(S(c, kp + 1, lm) - S(c, km - 1, lm)) * 2.0f : float(S(c, kp + 1, lm) - S(c, km, lm));
                else
                    giy = nu ? float(S(c, kp, lm) - S(c, km - 1, lm)) : 0.f;
                ti[c] = w * float(S(c, km, lm));
                tx[c] = w * (gix * rx);
                ty[c] = w * (giy * ry);
            }
        }
        // The sums run over the window in raster order (cv2's k, l loops).
        // Transposed through LDS: lane idx leaves its position's terms, then
        // lane c < nc walks the positions in order and accumulates channel c
        // (and s, the same sequence in every channel lane) -- four independent
        // chains per lane instead of a wave-wide fold of 4 x nc + 1 readlanes
        // per position.
        const uint64_t vm = __ballot(valid);
#pragma unroll
        for (int c = 0; c < kChanGroup; ++c)
            if (c < nc) P.q[lane][c] = make_float4(ti[c], tx[c], ty[c], w);
        wave_lds_sync();
        if (lane < nc) {
            float a = 0.f, jx = 0.f, jy = 0.f, sw = 1.0e-20f;
            if (R == 3) {
                // the disk's 28 positions, unconditionally: a position that is
                // not used carries +0 terms, and adding / subtracting +0 leaves
                // every running sum unchanged (a and sw never hold -0: their
                // terms are >= 0), so the sums equal cv2's skipping ones
#pragma unroll
                for (int b0 = 0; b0 < 28; b0 += 7) {
                    float4 v[7];
#pragma unroll
                    for (int t = 0; t < 7; ++t) v[t] = P.q[kDisk3[b0 + t]][lane];
#pragma unroll
                    for (int t = 0; t < 7; ++t) {
                        a += v[t].x;
                        jx -= v[t].y;
                        jy -= v[t].z;
                        sw += v[t].w;
                    }
                }
            } else {
                for (int j = 0; j < npos; ++j) {
                    if (!((vm >> j) & 1ull)) continue;  // uniform
                    const float4 v = P.q[j][lane];
                    a += v.x;
                    jx -= v.y;
                    jy -= v.z;
                    sw += v.w;
                }
            }
            IP_STAMP(2 * L + 1, 3, i == 0 && lane == 0 && c0 == 0);
            const float sat = float(double(a / sw) + double(jx + jy) / (sqrt(double(jx * jx + jy * jy)) + double(1.0e-20f)) +
                                    double(0.5f));
            m.out[(c0 + lane) * m.HW + p] = float(sat_u8(sat));
        }
    }
    if (lane == 0) m.T[p] = tij;
    IP_STAMP(2 * L + 1, 4, i == 0 && lane == 0);
}

// One hole layer over the grid.  The layer's two bins (patch-interior holes,
// the others) are read from the device.  A thin layer (at most thin_cap
// holes, radius <= 3) runs every hole on the wave path, whose per-hole chain
// is the shorter one; otherwise blocks [0, gb) take the patch-interior holes
// (thread per hole, or kCS threads per hole up to kCsSplitMax holes) and the
// rest of the grid the others (wave per hole), each part grid-stride.  The
// two sets of a layer are independent; every block runs one path.
// Block `bx` of a G-block partition of hole layer L (a launch's blockIdx.x /
// gridDim.x, or one of the tail kernel's kTailParts parts).
__device__ __forceinline__ void hole_layer_body(const Chunk &ch, const uint32_t *__restrict__ list,
                                                const unsigned *__restrict__ hist, const unsigned *__restrict__ cursor,
                                                int nring, unsigned L, int range, unsigned thin_cap, WavePatch *patch,
                                                unsigned bx, unsigned G) {
    const int bi = nring + 2 * (int(L) - 1);
    const unsigned ni = hist[bi], nw = hist[bi + 1];
    if (ni + nw == 0u) return;
    // SCATTER advanced cursor[] to each bin's end: a bin starts at cursor - count
    const uint32_t *lp = list + (cursor[bi] - ni), *lw = list + (cursor[bi + 1] - nw);
    const unsigned wave = threadIdx.x >> 6;
    IP_STAMP(2 * L, 0, bx == 0 && threadIdx.x == 0);
    IP_STAMP(2 * L + 1, 0, bx == G - 1 && threadIdx.x == 0);
    if (range <= 3 && ni + nw <= thin_cap) {
        for (unsigned h = bx * 4u + wave; h < ni + nw; h += G * 4u) {
            if (h < ni)
                hole_wave_lds(ch, lp, ni, h, L, range, patch[wave]);
            else
                hole_wave_lds(ch, lw, nw, h - ni, L, range, patch[wave]);
        }
        return;
    }
    const unsigned cs = ni > kCsSplitMax ? 1u : 3u;
    const unsigned bt = blocks_for_dev(ni * cs, 256u), bw = blocks_for_dev(nw, 4u);
    // split the grid in proportion to the two parts' blocks (each part at least one block)
    unsigned gb = bt + bw <= G ? bt : (bw == 0u ? G : (bt == 0u ? 0u : max(1u, unsigned(uint64_t(G) * bt / (bt + bw)))));
    if (bw && gb >= G) gb = G - 1u;
    if (bx < gb) {
        for (unsigned i = bx * 256u + threadIdx.x; i < ni * cs; i += gb * 256u) {
            if (cs == 1u)
                hole_patch<1>(ch, lp, ni, i, L);
            else
                hole_patch<3>(ch, lp, ni, i, L);
        }
    } else {
        const unsigned gw = G - gb;
        for (unsigned h = (bx - gb) * 4u + wave; h < nw; h += gw * 4u) {
            if (range <= 3)
                hole_wave_lds(ch, lw, nw, h, L, range, patch[wave]);
            else
                hole_wave(ch, lw, nw, h, L, range);
        }
    }
}

// One launch per hole layer L (the host launches layers 1 .. K).
__global__ __launch_bounds__(256) void ip_hole_layer_kernel(Chunk ch, const uint32_t *__restrict__ list,
                                                            const unsigned *__restrict__ hist,
                                                            const unsigned *__restrict__ cursor, int nring, unsigned L,
                                                            int range, unsigned thin_cap) {
    __shared__ WavePatch patch[4];
    hole_layer_body(ch, list, hist, cursor, nring, L, range, thin_cap, patch, blockIdx.x, gridDim.x);
}

// The layers beyond the ones the host launched (L0 .. meta[0], the deepest
// layer the sort found), on a grid of kTailGrid workgroups: every layer is
// cut into kTailParts parts (the partition of a kTailParts-block layer
// launch), and the parts of all tail layers are tickets taken in order from
// one counter (meta[1]).  A workgroup holding a part of layer L waits until
// every part of layer L - 1 has finished (meta[2], the count of finished
// parts: parts of layer L + 1 only finish after layer L has, so the first
// (L - L0 + 1) * kTailParts finishes are exactly layers L0 .. L).
// Deadlock-free without co-residency: tickets are taken in increasing order,
// so every part a workgroup waits for was taken earlier -- by a running
// workgroup, which finishes it (its own wait is on an earlier layer still;
// layer L0 waits for nothing).  A workgroup that never starts holds no
// ticket.  Results cross workgroups (and XCDs) through agent-scope
// release / acquire fences around the counters.  The previous tail was one
// workgroup doing the 16 parts of each layer one after another: a deep call
// after a history of shallow ones at the same shape spent 600 ms there
// (308 layers at 16 x 768x1024, tools/tail_cliff.py).
// Exits at once when meta[0] < L0: the host launches every layer of the
// recent calls at this shape (and every possible one when it has no
// statistics yet), so the tail only runs for a call deeper than those.
constexpr unsigned kTailParts = 64, kTailGrid = 64;
constexpr unsigned kTailSpinBound = 1u << 20;  // polls before the wait gives up (~seconds; never reached)

__global__ __launch_bounds__(256) void ip_hole_tail_kernel(Chunk ch, const uint32_t *__restrict__ list,
                                                           const unsigned *__restrict__ hist,
                                                           const unsigned *__restrict__ cursor, unsigned *meta,
                                                           int nring, unsigned L0, int range, unsigned thin_cap) {
    __shared__ WavePatch patch[4];
    __shared__ unsigned tk[2];  // [ticket, gave up]
    const unsigned lmax = meta[0];
    if (lmax < L0) return;  // uniform: no layer beyond the launched ones
    if (threadIdx.x == 0 && blockIdx.x == 0) atomicAdd(&g_ip_tail_layers, lmax - L0 + 1u);
    const unsigned total = (lmax - L0 + 1u) * kTailParts;
    const unsigned lane = threadIdx.x & 63u;
    // Every branch below is uniform across the workgroup or across wave 0
    // (values broadcast with shuffles / readfirstlane), so the loop's barriers
    // are met the same number of times by every wave.
    for (;;) {
        if (threadIdx.x < 64u) {  // wave 0 takes the next ticket and waits for the layer before it
            unsigned t = 0u;
            if (lane == 0u) t = atomicAdd(&meta[1], 1u);
            t = __builtin_amdgcn_readfirstlane(t);
            unsigned gave_up = 0u;
            if (t < total && t >= kTailParts) {
                const unsigned need = (t / kTailParts) * kTailParts;
                for (unsigned spins = 0;; ++spins) {
                    unsigned done = 0u;
                    // the polling lane's agent-scope acquire load pairs with
                    // the publishing thread's release add below
                    if (lane == 0u) done = __hip_atomic_load(&meta[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                    done = __builtin_amdgcn_readfirstlane(done);
                    if (done >= need) break;
                    if (spins >= kTailSpinBound) {
                        if (lane == 0u) atomicOr(&g_ip_fault, 8u);
                        gave_up = 1u;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            }
            if (lane == 0u) {
                tk[0] = t;
                tk[1] = gave_up;
            }
        }
        __syncthreads();
        const unsigned t = __builtin_amdgcn_readfirstlane(tk[0]);
        const unsigned give_up = __builtin_amdgcn_readfirstlane(tk[1]);
        __syncthreads();  // every thread has read tk before wave 0 rewrites it
        if (t >= total || give_up) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the previous layers' T and colours
        hole_layer_body(ch, list, hist, cursor, nring, L0 + t / kTailParts, range, thin_cap, patch, t % kTailParts,
                        kTailParts);
        // every wave completes its own stores (vmcnt is per wave), the barrier
        // orders them before thread 0, whose agent-scope release add publishes
        // the part (HIP / HSA memory model: release after the barrier, on the
        // publishing thread)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(&meta[2], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

inline unsigned blocks_for(unsigned n, unsigned per) { return (n + per - 1) / per; }

// Layers of at most this many holes run every hole on the wave path
// (OFD_IP_THIN or ofd_inpaint_set_schedule override; probes and tests).
int g_thin_cap = -1, g_launch_layers = -1;
unsigned thin_layer_cap() {
    if (g_thin_cap >= 0) return unsigned(g_thin_cap);
    static const unsigned v = [] {
        const char *e = getenv("OFD_IP_THIN");
        return e ? unsigned(atoi(e)) : 4096u;
    }();
    return v;
}

// Grid of a layer launch when its size is unknown, and the cap otherwise:
// 8 workgroups per CU.
unsigned default_layer_grid() {
    static const unsigned v = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                    hipSuccess || cus <= 0)
            cus = 256;
        return unsigned(cus) * 8u;
    }();
    return v;
}

// Per-shape layer statistics of recent calls, read back without ever
// blocking the host: every call enqueues an asynchronous copy of its layer
// histogram and depth into pinned memory behind an event; a later call uses
// them (to size its grids and the number of layer launches) only once that
// event has completed.  They steer launch sizes only, never results.  The
// view is the elementwise maximum over the last kHistory completed copies: a
// caller that alternates shallow and deep fills at one shape (the pipeline's
// flip / rotation / shear augmentations) then launches the deep calls' layers
// -- an unneeded layer launch costs ~1.6 us, a layer left to the one-
// workgroup tail kernel runs on a single CU.
struct LaggedStats {
    static constexpr size_t kHistory = 8;
    std::mutex mu;
    unsigned *pinned = nullptr;  // [kMaxBins + 1]: hist, then the depth (meta[0])
    hipEvent_t ev = nullptr;
    bool pending = false;
    std::vector<std::vector<unsigned>> recent;  // completed copies, oldest first; [nbins] hist + depth
    std::vector<unsigned> hist;                 // elementwise max over `recent`
    unsigned lmax = 0, ring = 0;
    bool valid = false;
    struct View {
        bool valid = false;
        std::vector<unsigned> hist;
        unsigned lmax = 0, ring = 0;
    };
    View snapshot(int nbins, int nring) {
        std::lock_guard<std::mutex> lk(mu);
        if (pending && hipEventQuery(ev) == hipSuccess) {
            std::vector<unsigned> h(pinned, pinned + nbins);
            h.push_back(pinned[kMaxBins]);
            if (!recent.empty() && recent.back().size() != h.size()) recent.clear();
            recent.push_back(std::move(h));
            if (recent.size() > kHistory) recent.erase(recent.begin());
            hist.assign(size_t(nbins), 0u);
            lmax = 0;
            for (const auto &r : recent) {
                for (int k = 0; k < nbins; ++k) hist[size_t(k)] = std::max(hist[size_t(k)], r[size_t(k)]);
                lmax = std::max(lmax, r.back());
            }
            ring = 0;
            for (int k = 0; k < nring && k < nbins; ++k) ring += hist[size_t(k)];
            valid = true;
            pending = false;
        }
        View v;
        v.valid = valid && int(hist.size()) == nbins;
        if (v.valid) {
            v.hist = hist;
            v.lmax = lmax;
            v.ring = ring;
        }
        return v;
    }
    void record(const unsigned *dhist, const unsigned *dmeta, int nbins, hipStream_t st) {
        std::lock_guard<std::mutex> lk(mu);
        if (pending) return;  // the previous copy is still in flight: keep it
        if (!pinned) {
            if (hipHostMalloc(reinterpret_cast<void **>(&pinned), (kMaxBins + 1) * sizeof(unsigned),
                              hipHostMallocDefault) != hipSuccess) {
                pinned = nullptr;
                return;
            }
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;
        }
        if (hipMemcpyAsync(pinned, dhist, size_t(nbins) * 4, hipMemcpyDeviceToHost, st) != hipSuccess) return;
        if (hipMemcpyAsync(pinned + kMaxBins, dmeta, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return;
        if (hipEventRecord(ev, st) == hipSuccess) pending = true;
    }
};

LaggedStats &lagged_stats(int64_t nb, int64_t H, int64_t W, int r) {
    static std::mutex mu;
    static std::map<std::tuple<int64_t, int64_t, int64_t, int>, std::unique_ptr<LaggedStats>> m;
    std::lock_guard<std::mutex> lk(mu);
    auto &p = m[std::make_tuple(nb, H, W, r)];
    if (!p) p.reset(new LaggedStats());
    return *p;
}

}  // namespace

extern "C" {

int ofd_inpaint_tail_layers(int reset) {
    unsigned v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ip_tail_layers), sizeof(v)) != hipSuccess) return -1;
    if (reset) {
        const unsigned z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ip_tail_layers), &z, sizeof(z)) != hipSuccess) return -1;
    }
    return int(v);
}

int ofd_inpaint_faults(int reset) {
    unsigned v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_ip_fault), sizeof(v)) != hipSuccess) return -1;
    if (reset) {
        const unsigned z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ip_fault), &z, sizeof(z)) != hipSuccess) return -1;
    }
    const unsigned q = ofd_sq_fault_read(reset);
    if (q == ~0u) return -1;
    return int(v | (q & (2u | 4u | 32u)));
}

int ofd_inpaint_set_schedule(int launch_layers, int thin_cap) {
    g_launch_layers = launch_layers < 0 ? -1 : launch_layers;
    g_thin_cap = thin_cap < 0 ? -1 : thin_cap;
    return OFD_FW_OK;
}

size_t ofd_inpaint_workspace_bytes(int64_t B, int64_t H, int64_t W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return size_t(B) * per_image(H, W) + 2 * align256(size_t(kMaxBins) * 4) + 256;
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
    const int nring = 2 * r;  // ring layers 1 .. 2r-1 (a Chebyshev-r neighbour is <= 2r away in L1)
    const int64_t HW = H * W;
    const size_t pi = per_image(H, W);
    const size_t fixed = 2 * align256(size_t(kMaxBins) * 4) + 256;
    if (!workspace || (reinterpret_cast<uintptr_t>(workspace) & 255u)) return OFD_FW_EWORKSPACE;
    if (workspace_bytes < fixed + pi) return OFD_FW_EWORKSPACE;
    int64_t G = int64_t((workspace_bytes - fixed) / pi);
    const int64_t gcap = ((int64_t(1) << 31) - 1) / HW;  // list entries bl * HW + p fit 31 bits
    if (G > gcap) G = gcap;
    if (G > B) G = B;
    hipStream_t st = static_cast<hipStream_t>(stream);
    char *wsb = static_cast<char *>(workspace);
    unsigned *hist = reinterpret_cast<unsigned *>(wsb);
    unsigned *cursor = reinterpret_cast<unsigned *>(wsb + align256(size_t(kMaxBins) * 4));
    unsigned *meta = reinterpret_cast<unsigned *>(wsb + 2 * align256(size_t(kMaxBins) * 4));
    const IpWs w = carve(wsb + fixed, G, HW);
    const int nbins = nring + 2 * int(H + W);
    const unsigned thin_cap = thin_layer_cap();
    const unsigned gdef = default_layer_grid();
    for (int64_t b0 = 0; b0 < B; b0 += G) {
        const int64_t nb = B - b0 < G ? B - b0 : G;
        const int64_t total = nb * HW;
        const bool vec4 = W % 4 == 0 && ((reinterpret_cast<uintptr_t>(img) | reinterpret_cast<uintptr_t>(valid) |
                                          reinterpret_cast<uintptr_t>(collision) | reinterpret_cast<uintptr_t>(out)) &
                                         15u) == 0;
        if (vec4)
            hipLaunchKernelGGL(ip_prep4_kernel, dim3(unsigned((W / 4 + 63) / 64), unsigned((H + 3) / 4), unsigned(nb)),
                               dim3(256), 0, st, img, valid, collision, out, w.code, int(C), int(H), int(W), b0);
        else
            hipLaunchKernelGGL(ip_prep_kernel, dim3(unsigned((W + 63) / 64), unsigned((H + 3) / 4), unsigned(nb)),
                               dim3(256), 0, st, img, valid, collision, out, w.code, int(C), int(H), int(W), b0);
        hipLaunchKernelGGL(ip_cols_kernel, dim3(unsigned((W + 63) / 64), unsigned(nb)), dim3(64 * kColSegs), 0, st, w.code,
                           w.gcol, int(H), int(W));
        if (W <= 64 * kRowRegs)
            hipLaunchKernelGGL(ip_rows_reg_kernel, dim3(unsigned((H + 3) / 4), unsigned(nb)), dim3(256), 0, st, w.code,
                               w.T, w.gcol, int(H), int(W), r);
        else
            hipLaunchKernelGGL(ip_rows_kernel, dim3(unsigned((H + 3) / 4), unsigned(nb)), dim3(256), 0, st, w.code, w.T,
                           w.gcol, w.list, int(H), int(W), r);
        hipError_t e = hipMemsetAsync(hist, 0, size_t(kMaxBins) * 4, st);
        if (e != hipSuccess) return int(e);
        const unsigned sblocks = unsigned((total + kSortSpan - 1) / kSortSpan);
        hipLaunchKernelGGL(ip_hist_kernel, dim3(sblocks), dim3(kSortThreads), 0, st, w.code, hist, total, nring,
                           int(H), int(W), r == 3);
        hipLaunchKernelGGL(ip_scan_kernel, dim3(1), dim3(1024), 0, st, hist, cursor, nbins, nring, meta);
        hipLaunchKernelGGL(ip_scatter_kernel, dim3(sblocks), dim3(kSortThreads), 0, st, w.code, cursor, w.list, total,
                           nring, int(H), int(W), r == 3);
        // Launch sizes: the layer counts stay on the device (each launch reads
        // its own); the host only picks grid sizes and how many layers to
        // launch, from the previous call's counts at this shape when those have
        // arrived (LaggedStats) -- the deep tail kernel covers whatever layers
        // lie beyond, so the result never depends on them.
        LaggedStats::View lag = lagged_stats(nb, H, W, r).snapshot(nbins, nring);
        auto grid_for_bin = [&](int bin, unsigned per_block, unsigned per_item) -> unsigned {
            if (!lag.valid) return gdef;
            const uint64_t n = uint64_t(lag.hist[size_t(bin)]) * per_item;
            const uint64_t g = (n + per_block - 1) / per_block;
            return unsigned(g < 16 ? 16 : (g > gdef ? gdef : g + g / 8 + 4));
        };
        const Chunk ch{w.code, w.T, img, out, int(C), int(H), int(W), HW, b0};
        for (int L = 1; L < nring; ++L)  // outer band, then negated
            hipLaunchKernelGGL(ip_ring_layer_kernel, dim3(grid_for_bin(L - 1, 256, 1)), dim3(256), 0, st, ch, w.list,
                               hist, cursor, unsigned(L));
        hipLaunchKernelGGL(ip_negate_kernel, dim3(lag.valid ? std::max(16u, std::min(gdef, lag.ring / 256u + 4u)) : gdef),
                           dim3(256), 0, st, w.T, w.list, cursor, nring);
        // no statistics yet at this shape: every possible layer (an empty
        // launch costs ~1.6 us), so the deep tail is left idle
        const int lmax_launch = g_launch_layers >= 0 ? std::min(g_launch_layers, int(H + W))
                                : int(lag.valid ? std::min<unsigned>(lag.lmax + 2u, unsigned(H + W)) : unsigned(H + W));
        for (int L = 1; L <= lmax_launch; ++L) {
            const int bi = nring + 2 * (L - 1);
            unsigned g = gdef;
            if (lag.valid) {
                const unsigned ni = lag.hist[size_t(bi)], nwv = lag.hist[size_t(bi) + 1];
                const unsigned cs = ni > kCsSplitMax ? 1u : 3u;
                const unsigned need = (ni + nwv <= thin_cap) ? blocks_for(ni + nwv, 4)
                                                              : blocks_for(ni * cs, 256) + blocks_for(nwv, 4);
                g = std::max(16u, std::min(gdef, need + need / 8 + 4));
            }
            hipLaunchKernelGGL(ip_hole_layer_kernel, dim3(g), dim3(256), 0, st, ch, w.list, hist, cursor, nring,
                               unsigned(L), r, thin_cap);
        }
        hipLaunchKernelGGL(ip_hole_tail_kernel, dim3(kTailGrid), dim3(256), 0, st, ch, w.list, hist, cursor, meta,
                           nring, unsigned(lmax_launch + 1), r, thin_cap);
        lagged_stats(nb, H, W, r).record(hist, meta, nbins, st);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

}  // extern "C"
