// ofd_fw.hip -- MI355X (gfx950) forward-warp engine: z-buffered splat + resolve.
//
// Replaces the reference's single-workgroup serial kernel
// (alt_cuda/fw_cuda_kernel.cu:9-49: grid <<<B, C>>>, one thread walks all H*W
// sources of one (image, channel)) with data-parallel kernels.  The z-test is
// restated as a lexicographic minimum: every source s landing on target t
// with depth < 1000 offers the 64-bit key
//       key(s) = orderable(depth[s]) << 32 | s          (s = raster index j*W+i)
// and the winner of t is the source with the smallest key -- exactly the
// source the reference's raster loop keeps with its strict `<` (ties keep the
// earliest source).  Sources with depth >= 1000 or NaN
// offer KEY_NOWIN, which marks the target valid without a winner (the
// reference's collision = 1 case, fw_cuda_kernel.cu:38-45).  The min is
// commutative, so the result is bit-identical however the work is scheduled.
//
// Two engines share the key algebra:
//
//  TILE (default).  Targets are cut into TW x TH tiles whose z-buffer lives in
//  LDS (ds_min_u64 is ~25x the chip rate of a global 64-bit atomic min,
//  tools/microbench.hip).  Sources are cut into 16 x 4 blocks, 8 blocks to a
//  128 x 4 segment.  Three kernels per chunk of images:
//    BIN     : one wave per segment loads its coordinates (16-byte loads),
//              and writes the tile-space bounding box of every block and of
//              the segment (8-byte records, no atomics).
//    SPLAT   : one workgroup per target tile scans the segment boxes, then
//              the block boxes of the selected segments, re-reads the selected
//              blocks' coordinates and depths, folds their keys into the LDS
//              z-buffer and publishes the tile: winner index (u32), valid,
//              collision.
//    RESOLVE : one target per thread: reads the winner index, gathers the
//              winner's C channels and writes them (streaming, HBM-bound).
//    Blocks whose box spans more than MAX_TILES_PER_BLOCK tiles (non-smooth
//    flow) go through global atomics on a per-image key slab instead
//    (pre-reduced over runs of equal targets inside the wave); SPLAT merges
//    the slab for the tiles BIN flagged.
//
//  ATOMIC (OFD_FW_MODE=atomic; and the float64 op).  One global 64-bit atomic
//  min per source into a per-image key slab, then a resolve pass.
//
// Workspace invariant: every call leaves the key slabs and tile flags all-ones
// (keys = KEY_UNTOUCHED, flags ~0), so the workspace is initialised once
// (ofd_fw_workspace_init) and never cleared; the per-block target boxes are
// scratch rewritten by every call.
//
// Plain HIP for gfx950; no CUDA compatibility layer, no dual paths.

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <type_traits>
#include <unordered_map>

#include "ofd_fw.h"

namespace {

constexpr int kBlock = 256;
constexpr unsigned long long KEY_UNTOUCHED = ~0ull;                 // no source landed
constexpr unsigned long long KEY_NOWIN = 0xFFFFFFFF00000000ull;     // landed, none < 1000
constexpr unsigned long long ZKEY_UNTOUCHED = ~0ull;                // f64 op depth keys
constexpr unsigned long long ZKEY_NOWIN = ~0ull - 1ull;
constexpr unsigned int IDX_NONE = ~0u;

// tile engine geometry
#ifndef OFD_PROBE_TW  // tile shape: overridable only by the diagnostic probe build (tools/probe_tile.py)
#define OFD_PROBE_TW 128
#define OFD_PROBE_TH 32
#endif
constexpr int TW = OFD_PROBE_TW, TH = OFD_PROBE_TH;  // target tile (LDS z-buffer 32 KiB)
// Tile-shape invariants are asserted where they are used: the packed target's
// 12-bit offset (pack_target) and the fused publish's rounds (splat_tile: every
// thread takes kGT targets per round, so TW * TH must be a multiple of
// threads x kGT).  Round 5's 128 x 16 probe build broke the latter -- 2048
// targets, 512 threads x 8 in flight -- and its publish read past the LDS
// z-buffer into the block list, gathering obj at garbage winner indices
// (the illegal address it faulted on).
constexpr int SBW = 16, SBH = 4;          // source block = one wave (64 px)
constexpr int SEGB = 8;                   // source blocks per segment (128 x 4 px)
constexpr int MAX_TILES_PER_BLOCK = 12;   // wider boxes go through the global path
constexpr int kSplatU = 2;                // 4-block slots in flight per wave (SPLAT, f32 coords; 3 spills)
#ifndef OFD_BIN_MINW  // BIN waves per SIMD the register budget must allow (probe builds override)
#define OFD_BIN_MINW 8
#endif
constexpr int kBinSPW = 1;                // segments per BIN wave (bin_kernel; 2 measured slower, also for depth-only sources)


// Default chunk: 64M source pixels (85 images of 768x1024, a ~830 MB slab).
// Every kernel of a chunk then has a grid many times the resident slots
// (measured per 64-image step: 16 / 32 / 64-image chunks = 1.15 / 1.05 / 1.02
// ms of summed launches).
constexpr size_t kDefaultChunkPixels = size_t(64) << 20;

// ---------------------------------------------------------------- key helpers
// Monotone map float -> uint32 (total order of non-NaN floats), -0 == +0.
__device__ __forceinline__ unsigned int orderable32(float d) {
    unsigned int u = __float_as_uint(d);
    if (u == 0x80000000u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long orderable64(double d) {
    unsigned long long u = (unsigned long long)__double_as_longlong(d);
    if (u == 0x8000000000000000ull) u = 0ull;
    return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}

// fw_cuda_kernel.cu:34 compares `depth < dlut` with dlut initialised to 1000
// (:58): only depth < 1000 can ever win; NaN never compares true.
__device__ __forceinline__ unsigned long long make_key(float d, unsigned int src) {
    return (d < 1000.0f) ? ((unsigned long long)orderable32(d) << 32) | src : KEY_NOWIN;
}

// The float32 depth a winning key carries: the inverse of orderable32 for
// keys below KEY_NOWIN.  -0 was folded onto +0, so a decoded 0 is ambiguous
// and the caller re-reads the depth plane for it.
__device__ __forceinline__ float depth_from_key(unsigned long long key) {
    const unsigned o = unsigned(key >> 32);
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}

// ---------------------------------------------------------------- target maps
// Op level: coordinates as given to fw_cuda.forward_warping.  The reference
// indexes its accessor with them, i.e. converts float -> int32 by truncation
// (fw_cuda_kernel.cu:31-35); an out-of-range index is UB there and a dropped
// source (tx = -1) here.
template <typename T>
__device__ __forceinline__ void target_safe(T x, T y, int H, int W, int &tx, int &ty) {
    if (!(x > T(-1)) || !(x < T(W)) || !(y > T(-1)) || !(y < T(H))) { tx = ty = -1; return; }
    tx = int(x);
    ty = int(y);
}

// FW level: fw.py:27-42.  p1 = p0 + flow in the flow's dtype (p0 is the
// float32 meshgrid, exact for any pixel index < 2^24), clamp to [0, W-1] x
// [0, H-1], truncate through int64.  NaN survives torch.clamp and is dropped.
template <typename F>
__device__ __forceinline__ void target_flow(int i, int j, F fx, F fy, int H, int W, int &tx, int &ty) {
    F px = F(i) + fx;
    F py = F(j) + fy;
    if (px != px || py != py) { tx = ty = -1; return; }
    px = px < F(0) ? F(0) : (px > F(W - 1) ? F(W - 1) : px);
    py = py < F(0) ? F(0) : (py > F(H - 1) ? F(H - 1) : py);
    tx = int(px);
    ty = int(py);
}

// Four consecutive pixels p..p+3 (n of them inside the row).  kVec: one
// 16-byte load per plane (float4, or two double2) -- the caller guarantees
// 16-byte alignment of every row start (W % 4 == 0, aligned base pointers).
template <bool kVec, typename T>
__device__ __forceinline__ void load4(const T *__restrict__ q, T v[4], int n) {
    if constexpr (kVec && sizeof(T) == 4) {
        const float4 f = *reinterpret_cast<const float4 *>(q);
        v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    } else if constexpr (kVec) {
        const double2 f0 = reinterpret_cast<const double2 *>(q)[0], f1 = reinterpret_cast<const double2 *>(q)[1];
        v[0] = f0.x; v[1] = f0.y; v[2] = f1.x; v[3] = f1.y;
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = e < n ? q[e] : T(0);
    }
}

// BIN's target range of one source: the exact target (lo == hi) for every
// coordinate source except the ego-motion one (EgoCoords::target_range).
#define TARGET_RANGE_EXACT                                                                              \
    __device__ __forceinline__ void target_range(int64_t b, int i, int j, V x, V y, int H_, int W_, int &tx0, \
                                                 int &tx1, int &ty0, int &ty1) const {                 \
        target(b, i, j, x, y, H_, W_, tx0, ty0);                                                      \
        tx1 = tx0;                                                                                    \
        ty1 = ty0;                                                                                    \
    }

// Coordinate sources whose z-test depth is the separate float32 depth plane
// and that generate no obj channels.
#define KEY_DEPTH_FROM_PLANE                                                                            \
    static constexpr int kGen = 0, kGenGT = 0;                                                        \
    static constexpr bool kPackable = true;                                                           \
    template <bool kVec>                                                                              \
    __device__ __forceinline__ void load4k(int64_t b, int64_t p, float dk[4], int n,                  \
                                           const float *depth) const {                                \
        ::load4<kVec>(depth + b * HW + p, dk, n);                                                     \
    }                                                                                                 \
    template <bool kVec>                                                                              \
    __device__ __forceinline__ void load4d(int64_t b, int64_t p, V x[4], V y[4], float dk[4], int n,  \
                                           const float *depth) const {                                \
        load4<kVec>(b, p, x, y, n);                                                                   \
        ::load4<kVec>(depth + b * HW + p, dk, n);                                                     \
    }                                                                                                 \
    __device__ __forceinline__ float key_depth(int64_t b, int64_t p, const float *depth) const {     \
        return depth[b * HW + p];                                                                     \
    }                                                                                                 \
    __device__ __forceinline__ void gen_key(int64_t, unsigned, unsigned long long, float *) const {}      \
    TARGET_RANGE_EXACT

// Coordinate sources: the target of the source at pixel p = j*W + i of image b.

struct SafeF32 {  // fw_cuda.forward_warping inputs: safe_y, safe_x [B,1,H,W]
    using V = float;
    const float *sy, *sx;
    int64_t HW;
    __device__ __forceinline__ void load(int64_t b, int64_t p, V &x, V &y) const {
        x = sx[b * HW + p];
        y = sy[b * HW + p];
    }
    template <bool kVec>
    __device__ __forceinline__ void load4(int64_t b, int64_t p, V x[4], V y[4], int n) const {
        ::load4<kVec>(sx + b * HW + p, x, n);
        ::load4<kVec>(sy + b * HW + p, y, n);
    }
    __host__ bool vec_ok() const { return (uintptr_t(sx) | uintptr_t(sy)) % 16 == 0; }
    __device__ __forceinline__ void target(int64_t, int, int, V x, V y, int H, int W, int &tx, int &ty) const {
        target_safe<float>(x, y, H, W, tx, ty);
    }
    KEY_DEPTH_FROM_PLANE
};

template <typename F>
struct FlowCoords {  // FW.forward input: flow [B,2,H,W], ch0 = x, ch1 = y
    using V = F;
    const F *flow;
    int64_t HW;
    __device__ __forceinline__ void load(int64_t b, int64_t p, V &x, V &y) const {
        const F *f = flow + b * 2 * HW + p;
        x = f[0];
        y = f[HW];
    }
    template <bool kVec>
    __device__ __forceinline__ void load4(int64_t b, int64_t p, V x[4], V y[4], int n) const {
        const F *f = flow + b * 2 * HW + p;
        ::load4<kVec>(f, x, n);
        ::load4<kVec>(f + HW, y, n);
    }
    __host__ bool vec_ok() const { return uintptr_t(flow) % 16 == 0; }
    __device__ __forceinline__ void target(int64_t, int i, int j, V x, V y, int H, int W, int &tx, int &ty) const {
        target_flow<F>(i, j, x, y, H, W, tx, ty);
    }
    KEY_DEPTH_FROM_PLANE
};

// Fused depth -> disparity -> flow (preprocess.py:239-254 / :356-359):
// disparity = s * B * f / depth with s * 50 * 1 in float32 and the division in
// the depth's dtype; flow = cat(disparity, 0) * -1.0, so the x flow is
// -disparity and the y flow -0.0; obj = cat(rgb, depth, flow * -1.0).  The
// flow is never stored: BIN and SPLAT derive it from the depth they load, and
// SPLAT generates obj's three middle channels (depth, disparity, +0) from the
// winner's depth.  The z-test key is the float32 depth (fw.py:43).
template <typename D>
struct DisparityCoords {
    using V = D;
    static constexpr int kGen = 3, kGenGT = 8;
    static constexpr bool kPackable = false;  // SPLAT reads only the depth already
    const D *depth;
    const float *s;  // [B] per-image scale
    int64_t HW;
    __device__ __forceinline__ D disp(int64_t b, D d) const { return D(s[b] * 50.0f * 1.0f) / d; }
    __device__ __forceinline__ void load(int64_t b, int64_t p, V &x, V &y) const {
        x = -disp(b, depth[b * HW + p]);
        y = -D(0);
    }
    template <bool kVec>
    __device__ __forceinline__ void load4(int64_t b, int64_t p, V x[4], V y[4], int n) const {
        D d[4];
        ::load4<kVec>(depth + b * HW + p, d, n);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            x[e] = -disp(b, d[e]);
            y[e] = -D(0);
        }
    }
    template <bool kVec>
    __device__ __forceinline__ void load4d(int64_t b, int64_t p, V x[4], V y[4], float dk[4], int n,
                                           const float *) const {
        D d[4];
        ::load4<kVec>(depth + b * HW + p, d, n);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            x[e] = -disp(b, d[e]);
            y[e] = -D(0);
            dk[e] = float(d[e]);
        }
    }
    __device__ __forceinline__ float key_depth(int64_t b, int64_t p, const float *) const {
        return float(depth[b * HW + p]);
    }
    // The winner's depth: a float32 depth is the key's high half (no gather);
    // a float64 depth is re-read (the key holds only its float32 rounding).
    __device__ __forceinline__ D winner_depth(int64_t b, unsigned w, unsigned long long key) const {
        if constexpr (std::is_same<D, float>::value) {
            const float d = depth_from_key(key);
            return d != 0.0f ? d : depth[b * HW + w];
        } else {
            return depth[b * HW + w];
        }
    }
    // generated obj channels of winner w: depth, flow_x * -1.0 = disparity, flow_y * -1.0 = +0
    __device__ __forceinline__ void gen_key(int64_t b, unsigned w, unsigned long long key, float g[3]) const {
        const D d = winner_depth(b, w, key);
        g[0] = float(d);
        g[1] = float(disp(b, d));
        g[2] = 0.0f;
    }
    __host__ bool vec_ok() const { return uintptr_t(depth) % 16 == 0; }
    __device__ __forceinline__ void target(int64_t, int i, int j, V x, V y, int H, int W, int &tx, int &ty) const {
        target_flow<D>(i, j, x, y, H, W, tx, ty);
    }
    TARGET_RANGE_EXACT
};

// Ego-motion flow (Convert.depth_to_random_flow, preprocess.py:265-298, with
// geometry.BackprojectDepth / Project3D, geometry.py:17-67) of the source at
// pixel (i, j) with depth d, in the reference's operation order:
//   cam   = inv_K[:3,:3] @ [i, j, 1]                      (geometry.py:38)
//   cam   = float32(d * cam)  (in d's dtype)              (:39-40)
//   cp    = P @ [cam, 1],  P = (K @ T)[:3]                (:57-59)
//   pix   = cp[:2] / (cp[2] + 1e-7)                       (:61)
//   pix   = (pix / (size - 1) - 0.5) * 2                  (:64-66)
//   p1    = (pix + 1) / 2 * (size - 1);  flow = p1 - p0   (preprocess.py:284-291)
// The two small matrix products accumulate k = 0, 1, ... with fused
// multiply-adds, as a GEMM inner loop does; torch's own GEMM order is not
// specified, so the flow matches the reference to float32 rounding (not
// bit-exact; tests/test_ego.py).  Every use of this function -- the flow
// plane kernel, BIN, SPLAT and the generated channels -- runs the same code,
// so the fused warp is bit-identical to FW on ofd_fw_ego_flow's plane.
struct EgoCam {
    float ik[9];  // inv_K[:3,:3], row-major (the same for every image)
};

// kApprox: the four divisions become multiplications by v_rcp_f32 (1 ulp);
// every other operation is the exact sequence's.  Only BIN's conservative
// target-tile boxes use it (ego_box_range), never a published value.
template <typename D, bool kApprox = false>
__device__ __forceinline__ void ego_flow_at(const EgoCam &cam, const float *__restrict__ Pb, int i, int j, D d,
                                            int H, int W, float &fx, float &fy) {
    auto dv = [](float a, float b) -> float { return kApprox ? a * __builtin_amdgcn_rcpf(b) : a / b; };
    const float x = float(i), y = float(j);
    float c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) c[k] = fmaf(cam.ik[3 * k + 2], 1.0f, fmaf(cam.ik[3 * k + 1], y, cam.ik[3 * k] * x));
    float X[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) X[k] = float(d * D(c[k]));
    float cp[3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        cp[k] = fmaf(Pb[4 * k + 3], 1.0f, fmaf(Pb[4 * k + 2], X[2], fmaf(Pb[4 * k + 1], X[1], Pb[4 * k] * X[0])));
    const float den = cp[2] + 1e-7f;
    float u = dv(cp[0], den), v = dv(cp[1], den);
    u = dv(u, float(W - 1));
    v = dv(v, float(H - 1));
    u = (u - 0.5f) * 2.0f;
    v = (v - 0.5f) * 2.0f;
    u = (u + 1.0f) / 2.0f;
    v = (v + 1.0f) / 2.0f;
    u = u * float(W - 1);
    v = v * float(H - 1);
    fx = u - x;
    fy = v - y;
}

// [lo, hi] bounds on trunc(clamp(p_exact, 0, n - 1)) from the approximate
// coordinate p (= i + fx of ego_flow_at<D, true>).  Replacing the four
// divisions by v_rcp_f32 products moves p by at most
// 2^-24 * (~20 |p| + ~3.2 n) (rcp 1 ulp, each later rounding 1/2 ulp, the
// normalise / denormalise steps scaling the error by n - 1); the margin
// 32 * 2^-24 * (|p| + n + 1) covers it.  false: p is not finite (NaN depth,
// a zero denominator) -- the caller takes the exact target.
__device__ __forceinline__ bool approx_trunc_range(float p, int n, int &lo, int &hi) {
    if (!(fabsf(p) < 1.0e30f)) return false;
    const float m = 1.9073486328125e-06f * (fabsf(p) + float(n) + 1.0f);
    const float a = fminf(fmaxf(p - m, 0.0f), float(n - 1)), b = fminf(fmaxf(p + m, 0.0f), float(n - 1));
    lo = int(a);
    hi = int(b);
    return true;
}

// Fused depth -> ego-motion flow -> splat: the flow is derived from the depth
// (and the image's P) in BIN and SPLAT, and SPLAT generates obj's channels
// depth, flow * -1.0 (x, y) from the winner (preprocess.py:371-373, :385-386).
template <typename D>
struct EgoCoords {
    // The coordinate registers carry the source's depth (x; y is unused):
    // the flow is computed in target(), after every load of a batch of
    // sources has been issued, which keeps SPLAT's loads in flight together.
    using V = D;
    static constexpr int kGen = 3, kGenGT = 4;
    static constexpr bool kPackable = false;  // BIN bounds targets approximately; SPLAT reads only the depth
    const D *depth;
    const float *P;  // [B][3][4] float32 (K @ T)[:3]
    EgoCam cam;
    int64_t HW;
    int H, W;
    // b is wave-uniform at every call site (BIN: one segment per wave; SPLAT:
    // one image per tile): the image's P is read through the scalar cache
    __device__ __forceinline__ const float *Pof(int64_t b) const {
        return P + 12 * int64_t(__builtin_amdgcn_readfirstlane(int(b)));
    }
    template <bool kVec>
    __device__ __forceinline__ void load4d(int64_t b, int64_t p, V x[4], V y[4], float dk[4], int n,
                                           const float *) const {
        ::load4<kVec>(depth + b * HW + p, x, n);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            y[e] = D(0);
            dk[e] = float(x[e]);
        }
    }
    template <bool kVec>
    __device__ __forceinline__ void load4(int64_t b, int64_t p, V x[4], V y[4], int n) const {
        ::load4<kVec>(depth + b * HW + p, x, n);
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = D(0);
    }
    __device__ __forceinline__ void load(int64_t b, int64_t p, V &x, V &y) const {
        x = depth[b * HW + p];
        y = D(0);
    }
    __device__ __forceinline__ float key_depth(int64_t b, int64_t p, const float *) const {
        return float(depth[b * HW + p]);
    }
    __device__ __forceinline__ D winner_depth(int64_t b, unsigned w, unsigned long long key) const {
        if constexpr (std::is_same<D, float>::value) {
            const float d = depth_from_key(key);
            return d != 0.0f ? d : depth[b * HW + w];
        } else {
            return depth[b * HW + w];
        }
    }
    // generated obj channels of winner w: depth, flow_x * -1.0, flow_y * -1.0
    __device__ __forceinline__ void gen_key(int64_t b, unsigned w, unsigned long long key, float g[3]) const {
        const D d = winner_depth(b, w, key);
        const unsigned j = w / unsigned(W), i = w - j * unsigned(W);
        float fx, fy;
        ego_flow_at<D>(cam, Pof(b), int(i), int(j), d, H, W, fx, fy);
        g[0] = float(d);
        g[1] = fx * -1.0f;
        g[2] = fy * -1.0f;
    }
    __host__ bool vec_ok() const { return uintptr_t(depth) % 16 == 0; }
    __device__ __forceinline__ void target(int64_t b, int i, int j, V d, V, int H_, int W_, int &tx,
                                           int &ty) const {
        float fx, fy;
        ego_flow_at<D>(cam, Pof(b), i, j, d, H, W, fx, fy);
        target_flow<float>(i, j, fx, fy, H_, W_, tx, ty);
    }
    // BIN's boxes only need a superset of the target tiles: the approximate
    // flow widened by its error bound (approx_trunc_range), exact only where
    // the approximation is not finite.
    __device__ __forceinline__ void target_range(int64_t b, int i, int j, V d, V y, int H_, int W_, int &tx0,
                                                 int &tx1, int &ty0, int &ty1) const {
        float fx, fy;
        ego_flow_at<D, true>(cam, Pof(b), i, j, d, H, W, fx, fy);
        if (!approx_trunc_range(float(i) + fx, W_, tx0, tx1) || !approx_trunc_range(float(j) + fy, H_, ty0, ty1)) {
            target(b, i, j, d, y, H_, W_, tx0, ty0);
            tx1 = tx0;
            ty1 = ty0;
        }
    }
};

// FW on a flow plane the caller already holds, with obj's depth and flow
// channels generated instead of concatenated (preprocess.py:371-373, :385-387,
// :400-402, :414-417 all call FW(cat(img, depth, flow * -1.0[, mask]), flow,
// depth)): the flow plane is read for the targets, the winner's depth is the
// key's high half, its flow * -1.0 is gathered from the same plane, and the
// concatenation is never stored.  F: the flow's dtype (float64 flows add in
// float64, fw.py:31); D: the depth's.  The torch.cat promotes the obj to the
// widest dtype, then fw.py:40 casts it to float32: generated channel values
// are float32(depth) and float32(flow * -1.0), exactly those casts.
template <typename F, typename D>
struct FlowCatCoords {
    using V = F;
    // targets in flight per publish thread: every target's two flow gathers
    // stay live until the stores, so float64 flows keep 4 (8 spilled)
    static constexpr int kGen = 3, kGenGT = sizeof(F) == 8 ? 4 : 8;
    static constexpr bool kPackable = true;
    const F *flow;   // [B,2,H,W]
    const D *depth;  // [B,1,H,W]
    int64_t HW;
    template <bool kVec>
    __device__ __forceinline__ void load4k(int64_t b, int64_t p, float dk[4], int n, const float *) const {
        D d[4];
        ::load4<kVec>(depth + b * HW + p, d, n);
#pragma unroll
        for (int e = 0; e < 4; ++e) dk[e] = float(d[e]);
    }
    __device__ __forceinline__ void load(int64_t b, int64_t p, V &x, V &y) const {
        const F *f = flow + b * 2 * HW + p;
        x = f[0];
        y = f[HW];
    }
    template <bool kVec>
    __device__ __forceinline__ void load4(int64_t b, int64_t p, V x[4], V y[4], int n) const {
        const F *f = flow + b * 2 * HW + p;
        ::load4<kVec>(f, x, n);
        ::load4<kVec>(f + HW, y, n);
    }
    template <bool kVec>
    __device__ __forceinline__ void load4d(int64_t b, int64_t p, V x[4], V y[4], float dk[4], int n,
                                           const float *) const {
        load4<kVec>(b, p, x, y, n);
        D d[4];
        ::load4<kVec>(depth + b * HW + p, d, n);
#pragma unroll
        for (int e = 0; e < 4; ++e) dk[e] = float(d[e]);
    }
    __device__ __forceinline__ float key_depth(int64_t b, int64_t p, const float *) const {
        return float(depth[b * HW + p]);
    }
    // the winner's float32 depth: the key's high half (a decoded 0 may have
    // been -0: re-read)
    __device__ __forceinline__ float winner_depth32(int64_t b, unsigned w, unsigned long long key) const {
        const float d = depth_from_key(key);
        return d != 0.0f ? d : float(depth[b * HW + w]);
    }
    __device__ __forceinline__ void gen_key(int64_t b, unsigned w, unsigned long long key, float g[3]) const {
        const F *f = flow + b * 2 * HW + w;
        g[0] = winner_depth32(b, w, key);
        g[1] = float(f[0] * F(-1.0));
        g[2] = float(f[HW] * F(-1.0));
    }
    // The publish's split form (kGenSplit): gen_vals has no branch and no
    // store, so a thread issues every target's flow gathers before its first
    // output store (gen_key's per-target loads, each behind the previous
    // target's stores, serialised the publish: 683 vs ~640 us per 64 images
    // of the plain FW on the same flows); the depth channel comes from the
    // key, and gen_fix rewrites the rare winner whose key decodes to 0 (the
    // depth plane holds the sign the key folded).
    static constexpr bool kGenSplit = true;
    __device__ __forceinline__ void gen_vals(int64_t b, unsigned w, unsigned long long key, float g[3]) const {
        const F *f = flow + b * 2 * HW + w;
        g[0] = depth_from_key(key);
        g[1] = float(f[0] * F(-1.0));
        g[2] = float(f[HW] * F(-1.0));
    }
    __device__ __forceinline__ void gen_fix(int64_t b, unsigned w, unsigned long long key, float *dst) const {
        if (depth_from_key(key) == 0.0f) __builtin_nontemporal_store(float(depth[b * HW + w]), dst);
    }
    __host__ bool vec_ok() const { return (uintptr_t(flow) | uintptr_t(depth)) % 16 == 0; }
    __device__ __forceinline__ void target(int64_t, int i, int j, V x, V y, int H, int W, int &tx, int &ty) const {
        target_flow<F>(i, j, x, y, H, W, tx, ty);
    }
    TARGET_RANGE_EXACT
};

// The ego-motion flow plane itself ([B,2,H,W] float32), four pixels of a row
// per thread.
template <typename D>
__global__ __launch_bounds__(256) void ego_flow_kernel(EgoCoords<D> co, float *__restrict__ flow, int64_t B) {
    const int64_t q = int64_t(blockIdx.x) * 256 + threadIdx.x;  // quad index over [B][H][ceil(W/4)]
    const int64_t qpr = (co.W + 3) / 4;
    const int64_t row = q / qpr;
    if (row >= B * co.H) return;
    const int64_t b = row / co.H;
    const int j = int(row - b * co.H), i0 = int(q - row * qpr) * 4;
    const float *Pb = co.P + 12 * b;
    float *fxp = flow + b * 2 * co.HW + int64_t(j) * co.W, *fyp = fxp + co.HW;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int i = i0 + e;
        if (i >= co.W) break;
        float fx, fy;
        ego_flow_at<D>(co.cam, Pb, i, j, co.depth[b * co.HW + int64_t(j) * co.W + i], co.H, co.W, fx, fy);
        fxp[i] = fx;
        fyp[i] = fy;
    }
}

template <typename C, typename = void>
struct GenSplit : std::false_type {};
template <typename C>
struct GenSplit<C, std::void_t<decltype(C::kGenSplit)>> : std::integral_constant<bool, C::kGenSplit> {};

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations (lgkmcnt), not for its outstanding global loads and stores --
// __syncthreads() would also drain every store, e.g. a tile's published
// output before the next tile of a persistent loop may start.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Packed min of two unsigned 16-bit halves (one v_pk_min_u16).
__device__ __forceinline__ unsigned pk_min_u16(unsigned a, unsigned b) {
    unsigned r;
    asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Global atomic min of `key` into base[t] for every lane with t >= 0, issuing
// one atomic per run of consecutive lanes with the same t (border clamping
// sends long runs to one pixel).  Segmented inclusive min-scan over the runs;
// every lane of the wave must call it.
__device__ __forceinline__ void wave_run_atomic_min(unsigned long long *base, int t, unsigned long long key) {
    const int lane = lane_id();
    const int tprev = __shfl_up(t, 1);
    const bool head = lane == 0 || tprev != t;
    const unsigned long long heads = __ballot(head);
    const unsigned long long le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1ull);
    const int seg_start = 63 - __clzll(heads & le);
    unsigned int lo = (unsigned int)key, hi = (unsigned int)(key >> 32);
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned int olo = __shfl_up(lo, d), ohi = __shfl_up(hi, d);
        if (lane - d >= seg_start) {
            const unsigned long long o = ((unsigned long long)ohi << 32) | olo;
            const unsigned long long k = ((unsigned long long)hi << 32) | lo;
            if (o < k) { lo = olo; hi = ohi; }
        }
    }
    const int tnext = __shfl_down(t, 1);
    const bool tail = lane == 63 || tnext != t;
    if (tail && t >= 0) atomicMin(base + t, ((unsigned long long)hi << 32) | lo);
}

// ---------------------------------------------------------------- workspace layout
struct TileGeom {
    int tilesX, tilesY, ntiles;  // target tiles per image
    int nsbx, nsby, nsb;         // source blocks per image
    int nsegx, nseg;             // segments (SEGB blocks of one block row) per image
};

// th: the tile height (TH, or kShortTH for short calls: run_f32)
inline TileGeom make_geom(int64_t H, int64_t W, int th = TH) {
    TileGeom g;
    g.tilesX = int((W + TW - 1) / TW);
    g.tilesY = int((H + th - 1) / th);
    g.ntiles = g.tilesX * g.tilesY;
    g.nsbx = int((W + SBW - 1) / SBW);
    g.nsby = int((H + SBH - 1) / SBH);
    g.nsb = g.nsbx * g.nsby;
    g.nsegx = (g.nsbx + SEGB - 1) / SEGB;
    g.nseg = g.nsegx * g.nsby;
    return g;
}

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// Per-image workspace: key slab (HW u64, only touched by spills), winner map
// (HW u32), per-tile spill flags, and the target-tile boxes of every source
// segment and block; plus, once per chunk slab, the persistent SPLAT's tile
// queue words (inside the per-image slack).
// Sized (and carved) for the shorter tiles, which have the most tiles: one
// layout serves both tile heights, so a call may pick either.
constexpr int kShortTH = 16;  // tile height of short calls (run_f32)
static_assert(kShortTH <= TH && TH % kShortTH == 0, "short tiles");
inline size_t per_image_bytes(int64_t H, int64_t W) {
    const TileGeom g = make_geom(H, W, kShortTH);
    return size_t(H) * size_t(W) * 12 + size_t(g.ntiles) * 4 + size_t(g.nseg) * 8 + size_t(g.nsb) * 8 + 256;
}

struct Ws {  // views of one chunk's workspace (G images)
    unsigned long long *keys;  // [G][HW]      KEY_UNTOUCHED between calls
    unsigned int *winner;      // [G][HW]      scratch: winning source index, ~0 = none (split engine)
    unsigned short *code;      // [G][HW]      scratch, aliases winner's first half: packed targets (fused engine)
    unsigned int *flag;        // [G][ntiles]  0 = merge key slab, ~0 = clean
    ushort4 *segrec;           // [G][nseg]    scratch: target tile box (t0x,t1x,t0y,t1y) of a segment
    ushort4 *blkrec;           // [G][nsb]     scratch: same per source block
    unsigned int *queue;       // [16]         persistent SPLAT: 8 per-XCD tile queues + exit count, ~0 between calls
};

inline Ws carve(void *ws, int64_t G, int64_t HW, const TileGeom &g) {
    Ws w;
    char *p = static_cast<char *>(ws);
    w.keys = reinterpret_cast<unsigned long long *>(p);
    p += align16(size_t(G) * size_t(HW) * 8);
    w.winner = reinterpret_cast<unsigned int *>(p);
    w.code = reinterpret_cast<unsigned short *>(p);  // never used by the same call as winner
    p += align16(size_t(G) * size_t(HW) * 4);
    w.flag = reinterpret_cast<unsigned int *>(p);
    p += align16(size_t(G) * g.ntiles * 4);
    w.segrec = reinterpret_cast<ushort4 *>(p);
    p += align16(size_t(G) * g.nseg * 8);
    w.blkrec = reinterpret_cast<ushort4 *>(p);
    p += align16(size_t(G) * g.nsb * 8);
    w.queue = reinterpret_cast<unsigned int *>(p);
    return w;
}

// empty box: no t0x <= x holds
__device__ __forceinline__ ushort4 empty_box() { return make_ushort4(0xFFFF, 0, 0xFFFF, 0); }
__device__ __forceinline__ bool box_has(const ushort4 &r, int tx, int ty) {
    return int(r.x) <= tx && tx <= int(r.y) && int(r.z) <= ty && ty <= int(r.w);
}

// ---------------------------------------------------------------- TILE engine
// Three kernels per chunk of images, each with a grid far larger than the
// resident slots:
//
// BIN     : one wave per source segment (SEGB blocks of 16x4 px).  Streams the
//           flow, writes each block's target-tile box and the segment's union
//           box.  No atomics, no lists.  A block whose box spans more than
//           MAX_TILES_PER_BLOCK tiles (non-smooth flow) is not boxed: its
//           sources go to the key slab by global atomic min (pre-reduced over
//           runs of equal targets) and flag their target tiles.
// SPLAT   : one workgroup per 128x32 target tile.  Finds its source blocks by
//           scanning the segment boxes of the image, then the block boxes of
//           the selected segments (both L2-resident), folds the selected
//           blocks' keys into an LDS z-buffer (ds_min_u64), merges the key
//           slab if flagged, and publishes the tile: winner index (u32),
//           valid, collision.
// RESOLVE : one target per thread, lane-consecutive: reads the winner index
//           and gathers / writes the C channels.  A pure streaming kernel
//           (tools/microbench.hip resolve_sim: 5.9 TB/s on this access shape,
//           against ~4.4 TB/s when the resolve ran inside the tile workgroup
//           behind its latency-bound scan / splat phases).
constexpr int kWarpThreads = 512;
constexpr int kWaves = kWarpThreads / 64;
constexpr int kSegCap = 768;    // selected segments held in LDS (else: scan all blocks)
constexpr int kListCap = 1024;  // candidate blocks examined per batch
constexpr int kResolveWX = 2, kResolveRows = 8;  // RESOLVE workgroup = 128 x 8 targets
constexpr unsigned int WIN_NONE = 0xFFFFFFFFu;

template <int kTH>
struct TileLdsT {
    unsigned long long zk[TW * kTH];
    unsigned int seg[kSegCap];
    unsigned int blk[kListCap];
    unsigned int nseg, nblk, flag;
    unsigned int next;  // persistent SPLAT: the tile thread 0 dequeued
};

struct ChunkArgs {  // one chunk of images
    Ws ws;
    int64_t b0;     // first image of the chunk
    int nimg;       // images in the chunk
};

// ---- BIN: wave w of workgroup blockIdx.x boxes segment blockIdx.x * kWaves + w.
// A segment is 128 x 4 px (SEGB = 8 blocks of 16 x 4).  Lane l owns the 4
// consecutive pixels 4*(l%32)..+3 of rows 2q + l/32 (q = 0, 1): one 16-byte
// load per plane and row pair (kVec), so the segment's coordinates arrive in
// 4 wave-wide 1 KiB loads instead of 16 of 256 B (dword loads capped BIN at
// ~3.3 TB/s).  Block k = lanes 4k..4k+3 of both halves: a lane folds its 8
// pixels in registers, a quad DPP reduction and one xor-32 swap give every
// lane its block's tile box.
__device__ __forceinline__ unsigned quad_min_pk16(unsigned v) {
    constexpr int ident = -1;
    v = pk_min_u16(v, unsigned(__builtin_amdgcn_update_dpp(ident, int(v), 0xB1, 0xF, 0xF, false)));  // [1,0,3,2]
    v = pk_min_u16(v, unsigned(__builtin_amdgcn_update_dpp(ident, int(v), 0x4E, 0xF, 0xF, false)));  // [2,3,0,1]
    return pk_min_u16(v, unsigned(__shfl_xor(int(v), 32)));
}

// Records: after the quad reduction every lane of quad k holds block k's box,
// so lanes 4k (k < SEGB) store the 8 block records in ONE 64-byte store
// instruction, and the segment box is a 3-step xor reduction over the quads
// (8 readlanes and 9 single-lane stores before: 98 -> 72 us per 64 images,
// and 76 -> 56 VGPRs, i.e. 8 waves per SIMD).
// Packed target (kPack; coordinate sources with exact BIN targets): BIN
// writes every source's target as 16 bits relative to its block's box --
// (tile index within the box, <= 11) << 12 | offset inside that tile (ly * TW
// + lx) -- so SPLAT re-reads 2 bytes per source instead of the coordinate
// planes (8 bytes for a float32 flow) and needs no target arithmetic: a
// source lands in SPLAT's tile iff its code's high nibble is the tile's index
// in the block's box, and the low 12 bits are its z-buffer slot.  0xFFFF:
// dropped source (NaN coordinate; no box holds 15 tiles).
static_assert(TW * TH <= 4096 && MAX_TILES_PER_BLOCK <= 15, "packed target: 12-bit tile offset, 4-bit tile index");
constexpr unsigned short CODE_NONE = 0xFFFF;

template <int TH>
__device__ __forceinline__ unsigned short pack_target(int tx, int ty, int t0x, int t0y, int bw) {
    if (tx < 0) return CODE_NONE;
    const int k = (ty / TH - t0y) * bw + (tx / TW - t0x);
    return (unsigned short)((unsigned(k) << 12) | unsigned((ty % TH) * TW + tx % TW));
}

template <typename Coords, bool kPack = false, bool kVec = false, int kTH = TH>
__device__ __forceinline__ void bin_segment(const Coords &co, const float *__restrict__ depth, const ChunkArgs &a,
                                               int H, int W, int64_t HW, const TileGeom &g, int64_t sgg,
                                               const typename Coords::V (&x)[2][4], const typename Coords::V (&y)[2][4]) {
    constexpr int TH = kTH;  // this call's tile height (shadows the default)
    const Ws &ws = a.ws;
    const int lane = lane_id();
    const int bl = int(sgg / g.nseg);
    const int sg = int(sgg - int64_t(bl) * g.nseg);
    const int sby = sg / g.nsegx, sgx = sg - sby * g.nsegx;
    const int64_t b = a.b0 + bl;
    const int i0 = sgx * (SEGB * SBW) + (lane & 31) * 4;
    const int jh = sby * SBH + (lane >> 5);
    unsigned mn = 0xFFFFFFFFu, mxi = 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int j = jh + 2 * q;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            int tx0 = -1, tx1 = -1, ty0 = -1, ty1 = -1;
            if (i0 + e < W && j < H) co.target_range(b, i0 + e, j, x[q][e], y[q][e], H, W, tx0, tx1, ty0, ty1);
            if (tx0 >= 0) {
                mn = pk_min_u16(mn, unsigned(tx0 / TW) | (unsigned(ty0 / TH) << 16));
                mxi = pk_min_u16(mxi, (0xFFFFu - unsigned(tx1 / TW)) | ((0xFFFFu - unsigned(ty1 / TH)) << 16));
            }
        }
    }
    mn = quad_min_pk16(mn);
    mxi = quad_min_pk16(mxi);
    const int k = (lane & 31) >> 2;  // this lane's block in the segment
    const int sbx = sgx * SEGB + k;
    const bool nonempty = (mn & 0xFFFFu) != 0xFFFFu;
    const int t0x = int(mn & 0xFFFFu), t0y = int(mn >> 16);
    const int t1x = int(0xFFFFu - (mxi & 0xFFFFu)), t1y = int(0xFFFFu - (mxi >> 16));
    const bool is_wide = nonempty && (t1x - t0x + 1) * (t1y - t0y + 1) > MAX_TILES_PER_BLOCK;
    const bool boxed = nonempty && !is_wide;
    // segment union of the boxed blocks (quads hold equal values: xor 4, 8, 16)
    unsigned smn = boxed ? mn : 0xFFFFFFFFu, smx = boxed ? mxi : 0xFFFFFFFFu;
#pragma unroll
    for (int m = 4; m < 32; m <<= 1) {
        smn = pk_min_u16(smn, unsigned(__shfl_xor(int(smn), m)));
        smx = pk_min_u16(smx, unsigned(__shfl_xor(int(smx), m)));
    }
    if (lane < 32 && (lane & 3) == 0 && sbx < g.nsbx)
        ws.blkrec[int64_t(bl) * g.nsb + int64_t(sby) * g.nsbx + sbx] =
            boxed ? make_ushort4((unsigned short)t0x, (unsigned short)t1x, (unsigned short)t0y, (unsigned short)t1y)
                  : empty_box();
    if constexpr (kPack) {
        // this lane's 2 x 4 sources: one 8-byte store per row (kVec); the
        // exact targets are recomputed (keeping 8 of them live through the
        // box reduction would spill at BIN's 64-VGPR budget)
        const int bw = t1x - t0x + 1;
        unsigned short *cb = ws.code + int64_t(bl) * HW;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = jh + 2 * q;
            if (j >= H || i0 >= W) continue;
            unsigned short c[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                int tx = -1, ty = -1;
                if (boxed && i0 + e < W) co.target(b, i0 + e, j, x[q][e], y[q][e], H, W, tx, ty);
                c[e] = pack_target<TH>(tx, ty, t0x, t0y, bw);
            }
            const int64_t p = int64_t(j) * W + i0;
            if constexpr (kVec) {
                *reinterpret_cast<uint2 *>(cb + p) =
                    make_uint2(unsigned(c[0]) | (unsigned(c[1]) << 16), unsigned(c[2]) | (unsigned(c[3]) << 16));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (i0 + e < W) cb[p + e] = c[e];
            }
        }
    }
    if (lane == 0)
        ws.segrec[sgg] = (smn & 0xFFFFu) == 0xFFFFu
                             ? empty_box()
                             : make_ushort4((unsigned short)(smn & 0xFFFFu), (unsigned short)(0xFFFFu - (smx & 0xFFFFu)),
                                            (unsigned short)(smn >> 16), (unsigned short)(0xFFFFu - (smx >> 16)));
    // wide blocks as a bit mask over k (bit 4k of the ballot of lanes < 32)
    const unsigned long long wb = __ballot(is_wide && lane < 32 && (lane & 3) == 0);
    if (wb == 0ull) return;  // wave-uniform
    // non-smooth flow (rare): the wide blocks' sources go to the key slab by
    // global atomic min and flag their target tiles for SPLAT's merge
    const bool mine_lane = (wb >> (4 * k)) & 1ull;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int j = jh + 2 * q;
            int tx = -1, ty = -1;
            if (mine_lane && i0 + e < W && j < H) co.target(b, i0 + e, j, x[q][e], y[q][e], H, W, tx, ty);
            const bool ok = tx >= 0;
            const int64_t p = int64_t(j) * W + i0 + e;
            const unsigned long long key = ok ? make_key(co.key_depth(b, p, depth), unsigned(p)) : 0ull;
            wave_run_atomic_min(ws.keys + int64_t(bl) * HW, ok ? ty * W + tx : -1, key);
            if (ok) ws.flag[int64_t(bl) * g.ntiles + (ty / TH) * g.tilesX + tx / TW] = 0u;
        }
}

// kSPW segments per wave (consecutive in the image's segment order): every
// segment's coordinate loads are issued before the first one is folded
// (2 / 4: 0.754 / 0.763 ms per 64-image step vs 0.737 at 1).
// BIN's register budget: 8 waves per SIMD (<= 64 VGPRs) for the float
// coordinate sources, which fit it without spilling (66 -> 64 VGPRs lifts BIN
// from 3 to 4 workgroups per CU, no measurable change in time: BIN streams at
// ~5.6 TB/s either way); the double and ego-motion sources keep the
// compiler's own choice (they would spill).
template <typename C>
struct BinMinW {
    static constexpr int value = sizeof(typename C::V) == 4 ? OFD_BIN_MINW : 1;
};
template <typename D>
struct BinMinW<EgoCoords<D>> {
    static constexpr int value = 1;
};

template <typename Coords, bool kVec, int kSPW = 1, bool kPack = false, int kTH = TH>
__global__ __launch_bounds__(kWarpThreads, BinMinW<Coords>::value) void bin_kernel(Coords co, const float *__restrict__ depth, ChunkArgs a,
                                                              int H, int W, int64_t HW, TileGeom g) {
    using V = typename Coords::V;
    const int lane = lane_id();
    const int64_t sg0 = (int64_t(blockIdx.x) * kWaves + (threadIdx.x >> 6)) * kSPW;
    const int64_t nsg = int64_t(a.nimg) * g.nseg;
    if (sg0 >= nsg) return;  // wave-uniform
    V x[kSPW][2][4], y[kSPW][2][4];
#pragma unroll
    for (int s = 0; s < kSPW; ++s) {
        const int64_t sgg = sg0 + s < nsg ? sg0 + s : nsg - 1;  // a clamped duplicate is loaded, not binned
        const int bl = int(sgg / g.nseg);
        const int sg = int(sgg - int64_t(bl) * g.nseg);
        const int sby = sg / g.nsegx, sgx = sg - sby * g.nsegx;
        const int i0 = sgx * (SEGB * SBW) + (lane & 31) * 4;
        const int jh = sby * SBH + (lane >> 5);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int j = jh + 2 * q;
            if (i0 < W && j < H) co.template load4<kVec>(a.b0 + bl, int64_t(j) * W + i0, x[s][q], y[s][q], W - i0);
        }
    }
#pragma unroll
    for (int s = 0; s < kSPW; ++s)
        if (sg0 + s < nsg) bin_segment<Coords, kPack, kVec, kTH>(co, depth, a, H, W, HW, g, sg0 + s, x[s], y[s]);  // wave-uniform
}

// ---- SPLAT.  Workgroup id -> XCD-aware tile: dispatch is round-robin over the
// 8 XCDs (workgroups b and b+8 share one), so each XCD gets a contiguous run
// of a band-major tile order -- tile-row band k of every image in turn -- so
// neighbouring tiles share source blocks and box records in one L2, and every
// XCD sees every image (whole images per XCD left the XCDs holding the
// heavier ego-motion images running ~60 us after the rest had drained).
// Placement only affects speed, never results.
//
// Inside a band the heavy tiles of every image come first (longest job
// first): the warp clamps out-of-image targets onto the border
// (fw.py:37-42), so border tiles collect every source that leaves the image
// and take up to 5x a median tile; dequeued last they set the drain tail.
// OFD_TILE_ORDER: 0 = plain band-major, 1 = corner tiles first, 3 = border
// tiles first.
#ifndef OFD_TILE_ORDER
#define OFD_TILE_ORDER 0
#endif
// heavy columns of tile row r: 0 = none, 1 = the two end columns, 2 = all
[[maybe_unused]] __device__ __forceinline__ int heavy_kind(int r, const TileGeom &g) {
    const bool edge_row = r == 0 || r == g.tilesY - 1;
    if constexpr (OFD_TILE_ORDER == 1) return edge_row ? 1 : 0;
    else if constexpr (OFD_TILE_ORDER == 3) return edge_row ? 2 : 1;
    else return 0;
}
[[maybe_unused]] __device__ __forceinline__ int n_heavy(int kind, int tx) { return kind == 0 ? 0 : kind == 2 ? tx : (tx > 1 ? 2 : 1); }

__device__ __forceinline__ void band_major_tile(unsigned lin, int nimg, const TileGeom &g, int &bl, int &tile) {
    unsigned start = 0;
    for (int k = 0; k < 8; ++k) {
        const int r0 = k * g.tilesY / 8, r1 = (k + 1) * g.tilesY / 8;
        const unsigned per_img = unsigned(r1 - r0) * unsigned(g.tilesX);
        const unsigned cnt = per_img * unsigned(nimg);
        if (lin < start + cnt || k == 7) {
            unsigned idx = lin - start;
            if constexpr (OFD_TILE_ORDER == 0) {
                bl = int(idx / per_img);
                tile = r0 * g.tilesX + int(idx - unsigned(bl) * per_img);
            } else {
                unsigned nh = 0;
                for (int r = r0; r < r1; ++r) nh += unsigned(n_heavy(heavy_kind(r, g), g.tilesX));
                const bool heavy = idx < nh * unsigned(nimg);
                const unsigned per = heavy ? nh : per_img - nh;
                if (!heavy) idx -= nh * unsigned(nimg);
                bl = int(idx / per);
                int kk = int(idx - unsigned(bl) * per);
                tile = r0 * g.tilesX;
                for (int r = r0; r < r1; ++r) {
                    const int kind = heavy_kind(r, g), nhr = n_heavy(kind, g.tilesX);
                    const int n = heavy ? nhr : g.tilesX - nhr;
                    if (kk < n) {
                        const int col = heavy ? (kind == 2 ? kk : (kk == 0 ? 0 : g.tilesX - 1)) : (kind == 0 ? kk : 1 + kk);
                        tile = r * g.tilesX + col;
                        break;
                    }
                    kk -= n;
                }
            }
            return;
        }
        start += cnt;
    }
}

// What SPLAT writes.  Split engine: valid, collision and the winner map (the
// workspace's); fused engine (kFuse): valid, collision and the C output
// planes, gathered from obj right out of the LDS z-buffer.
struct SplatIO {
    float *valid, *coll;
    const void *obj;   // kFuse only: [B][Cobj][H][W] of the element type E (float, or bf16 bits)
    void *out;         // kFuse only: [B][C][H][W], E
    int C;             // output channels
    int Cobj, gen_at;  // obj channels; output channel of the first of Coords::kGen generated ones
};

// SPLAT launch shape: threads per workgroup, gather targets in flight per
// thread (fused publish), minimum waves per SIMD (__launch_bounds__), 4-block
// slots in flight per wave, publish store policy, tile order (probe knobs).
template <int kThr_, int kGT_, int kMinW_, int kUF_ = kSplatU, int kNTPub_ = 1, int kMap_ = 0, int kTH_ = TH>
struct SplatCfg {
    static constexpr int kThr = kThr_, kWaves = kThr_ / 64, kGT = kGT_, kMinW = kMinW_, kUF = kUF_, kNTPub = kNTPub_,
                         kMap = kMap_, kTH = kTH_;  // kTH: target tile height
};

// (image, tile) of linear index `lin` of the chunk's tile order
template <typename Cfg>
__device__ __forceinline__ void tile_of(unsigned lin, const ChunkArgs &a, const TileGeom &g, int &bl, int &tile) {
    if constexpr (Cfg::kMap == 0) {
        band_major_tile(lin, a.nimg, g, bl, tile);
    } else if constexpr (Cfg::kMap == 1) {  // whole images, image k, k+8, ... on XCD k
        const unsigned s0 = lin / unsigned(g.ntiles);
        tile = int(lin - s0 * unsigned(g.ntiles));
        const unsigned nq = unsigned(a.nimg) / 8u, nr = unsigned(a.nimg) % 8u;
        // s0-th image of the order sorted by (image % 8, image / 8)
        unsigned k = 0, before = 0;
        while (before + nq + (k < nr ? 1u : 0u) <= s0) { before += nq + (k < nr ? 1u : 0u); ++k; }
        bl = int((s0 - before) * 8u + k);
    } else {  // whole images, contiguous
        bl = int(lin / unsigned(g.ntiles));
        tile = int(lin - unsigned(bl) * unsigned(g.ntiles));
    }
}

// The segments (SEGB source blocks) of image bl whose target-tile box holds
// tile (txi, tyi), appended to L.seg; *cnt counts them (> kSegCap: too many,
// the tile scans every block instead).  All loads of a thread in flight
// together.
template <typename Cfg, typename Lds>
__device__ __forceinline__ void seg_scan(Lds &L, unsigned *cnt, const ushort4 *segrec, const TileGeom &g, int txi,
                                         int tyi) {
    for (int s0 = threadIdx.x; s0 < g.nseg; s0 += Cfg::kThr * 4) {
        ushort4 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int sidx = s0 + u * Cfg::kThr;
            r[u] = sidx < g.nseg ? segrec[sidx] : empty_box();
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (box_has(r[u], txi, tyi)) {
                const unsigned idx = atomicAdd(cnt, 1u);
                if (idx < unsigned(kSegCap)) L.seg[idx] = unsigned(s0 + u * Cfg::kThr);
            }
        }
    }
}

// Persistent SPLAT's tile queue (thread 0): the next tile, ~0u when every
// queue is drained; the last workgroup to find them drained restores the
// queue words for the next launch.
__device__ __forceinline__ unsigned dequeue_tile(unsigned *queue, unsigned home, unsigned per, unsigned total,
                                                 unsigned &drained) {
    unsigned lin = ~0u;
    for (unsigned k = 0; k < 8u && lin == ~0u; ++k) {
        const unsigned qx = (home + k) & 7u;
        if ((drained >> qx) & 1u) continue;
        const unsigned idx = ~atomicSub(queue + qx, 1u);
        const unsigned l = qx * per + idx;
        if (idx < per && l < total) lin = l;
        else drained |= 1u << qx;
    }
    if (lin == ~0u && ~atomicSub(queue + 8, 1u) == gridDim.x - 1u) {
        // every other workgroup has finished dequeuing: restore the queues
        for (int k = 0; k < 9; ++k) atomicExch(queue + k, ~0u);
    }
    return lin;
}

// One target tile (linear index `lin` of the chunk's band-major tile order).
// Every barrier is LDS-only: global loads are consumed by the thread that
// issued them, and the published stores are never waited for.
template <typename Coords, bool kVec, bool kFuse, bool kStamp, typename Cfg, typename E = float, bool kPack = false>
__device__ __forceinline__ void splat_tile(TileLdsT<Cfg::kTH> &L, unsigned lin, int bl, int tile, const Coords &co,
                                           const float *__restrict__ depth, const SplatIO &io, const ChunkArgs &a,
                                           int H, int W, int64_t HW, const TileGeom &g, unsigned long long *stamps) {
    constexpr int TH = Cfg::kTH;  // this call's tile height (shadows the default)
    unsigned long long *ph = kStamp ? stamps + 8 * lin : nullptr;
    if constexpr (kStamp) { if (threadIdx.x == 0) ph[0] = wall_clock64(); }

    const Ws &ws = a.ws;
    const unsigned fid = unsigned(bl) * unsigned(g.ntiles) + unsigned(tile);  // flag slot
    const int tyi = tile / g.tilesX, txi = tile - tyi * g.tilesX;
    const int x0 = txi * TW, y0 = tyi * TH;
    const int64_t b = a.b0 + bl;
    unsigned long long *keys = ws.keys + int64_t(bl) * HW;
    const ushort4 *segrec = ws.segrec + int64_t(bl) * g.nseg;
    const ushort4 *blkrec = ws.blkrec + int64_t(bl) * g.nsb;

    if (threadIdx.x == 0) {
        L.flag = ws.flag[fid];
        ws.flag[fid] = 0xFFFFFFFFu;  // restore the workspace invariant for the next call
        L.nseg = 0;
        L.nblk = 0;
    }
    for (int k = threadIdx.x; k < TW * TH; k += Cfg::kThr) L.zk[k] = KEY_UNTOUCHED;
    lds_barrier();

    // ---- 1. segments whose box holds this tile
    seg_scan<Cfg>(L, &L.nseg, segrec, g, txi, tyi);
    lds_barrier();
    if constexpr (kStamp) { if (threadIdx.x == 0) ph[4] = wall_clock64(); }
    const int nsel = int(L.nseg);
    // candidates: the blocks of the selected segments, or every block of the
    // image if too many segments matched
    const bool all_blocks = nsel > kSegCap;
    const int ncand = all_blocks ? g.nsb : nsel * SEGB;
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    [[maybe_unused]] unsigned nblk_tot = 0;  // kStamp: candidate blocks splatted

    for (int c0 = 0; c0 < ncand; c0 += kListCap) {
        // ---- 2. candidate blocks whose box holds this tile -> L.blk
#pragma unroll
        for (int u = 0; u < kListCap / Cfg::kThr; ++u) {
            const int c = c0 + int(threadIdx.x) + u * Cfg::kThr;
            int sb = -1;
            if (c < ncand) {
                if (all_blocks) {
                    sb = c;
                } else {
                    const int sg = int(L.seg[c / SEGB]);
                    const int sby = sg / g.nsegx, sbx = (sg - sby * g.nsegx) * SEGB + c % SEGB;
                    sb = sbx < g.nsbx ? sby * g.nsbx + sbx : -1;
                }
            }
            if (sb >= 0) {
                const ushort4 r = blkrec[sb];
                if (box_has(r, txi, tyi)) {
                    const unsigned idx = atomicAdd(&L.nblk, 1u);
                    // kPack: this tile's index in the block's box rides in the top nibble
                    const unsigned kt = kPack ? unsigned((tyi - int(r.z)) * (int(r.y) - int(r.x) + 1) + (txi - int(r.x))) : 0u;
                    L.blk[idx] = unsigned(sb) | (kt << 28);
                }
            }
        }
        lds_barrier();
        // ---- 3. splat the selected blocks into the LDS z-buffer.  A slot is 4
        // blocks: lane = (block lane/16, row (lane/4)%4, pixels 4*(lane%4)..+3),
        // one 16-byte load per plane (kVec); kU slots in flight per wave.
        using V = typename Coords::V;
        constexpr int kU = sizeof(V) == 4 ? Cfg::kUF : 1;  // 64-VGPR budget
        const int nb = int(L.nblk);
        if constexpr (kStamp) nblk_tot += unsigned(nb);
        const int sub = lane >> 4, rr = (lane >> 2) & 3, c4 = (lane & 3) * 4;
        if constexpr (kPack) {
            // packed targets (BIN): 8 bytes of codes + 16 of depth per lane and
            // slot, no target arithmetic
            constexpr int kUP = Cfg::kUF;
            const unsigned short *cb = ws.code + int64_t(bl) * HW;
            for (int e0 = wave * 4; e0 < nb; e0 += Cfg::kWaves * 4 * kUP) {
                unsigned cw[kUP][2];
                float d[kUP][4];
                int ii[kUP], jj[kUP];
                unsigned kt[kUP];
#pragma unroll
                for (int u = 0; u < kUP; ++u) {
                    const int e = e0 + sub + u * Cfg::kWaves * 4;
                    ii[u] = W;
                    jj[u] = 0;
                    kt[u] = 0;
                    if (e < nb) {
                        const unsigned be = L.blk[e];
                        const int sb = int(be & 0x0FFFFFFFu);
                        kt[u] = be >> 28;
                        const int sby = sb / g.nsbx, sbx = sb - sby * g.nsbx;
                        const int i = sbx * SBW + c4, j = sby * SBH + rr;
                        if (i < W && j < H) {
                            ii[u] = i;
                            jj[u] = j;
                            const int64_t p = int64_t(j) * W + i;
                            if constexpr (kVec) {
                                const uint2 v = *reinterpret_cast<const uint2 *>(cb + p);
                                cw[u][0] = v.x;
                                cw[u][1] = v.y;
                            } else {
                                unsigned short c[4];
#pragma unroll
                                for (int q = 0; q < 4; ++q) c[q] = i + q < W ? cb[p + q] : CODE_NONE;
                                cw[u][0] = unsigned(c[0]) | (unsigned(c[1]) << 16);
                                cw[u][1] = unsigned(c[2]) | (unsigned(c[3]) << 16);
                            }
                            co.template load4k<kVec>(b, p, d[u], W - i, depth);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < kUP; ++u) {
                    if (ii[u] >= W) continue;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int i = ii[u] + q;
                        if (i >= W) break;
                        const unsigned c = (cw[u][q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
                        if ((c >> 12) == kt[u])
                            atomicMin(&L.zk[c & 0xFFFu], make_key(d[u][q], unsigned(jj[u] * W + i)));
                    }
                }
            }
        } else
        for (int e0 = wave * 4; e0 < nb; e0 += Cfg::kWaves * 4 * kU) {
            V cx[kU][4], cy[kU][4];
            float d[kU][4];
            int ii[kU], jj[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const int e = e0 + sub + u * Cfg::kWaves * 4;
                ii[u] = W;
                jj[u] = 0;
                if (e < nb) {
                    const int sb = int(L.blk[e] & 0x0FFFFFFFu);
                    const int sby = sb / g.nsbx, sbx = sb - sby * g.nsbx;
                    const int i = sbx * SBW + c4, j = sby * SBH + rr;
                    if (i < W && j < H) {
                        ii[u] = i;
                        jj[u] = j;
                        const int64_t p = int64_t(j) * W + i;
                        co.template load4d<kVec>(b, p, cx[u], cy[u], d[u], W - i, depth);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                if (ii[u] >= W) continue;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int i = ii[u] + q, j = jj[u];
                    if (i >= W) break;
                    int tx, ty;
                    co.target(b, i, j, cx[u][q], cy[u][q], H, W, tx, ty);
                    const int lx = tx - x0, ly = ty - y0;
                    if (tx >= 0 && unsigned(lx) < unsigned(TW) && unsigned(ly) < unsigned(TH))
                        atomicMin(&L.zk[ly * TW + lx], make_key(d[u][q], unsigned(j * W + i)));
                }
            }
        }
        lds_barrier();
        if (threadIdx.x == 0) L.nblk = 0;
        lds_barrier();
    }
    if constexpr (kStamp) { if (threadIdx.x == 0) ph[5] = wall_clock64(); }
    // ---- 4. merge the key slab where BIN spilled into it
    if (L.flag == 0u) {
        for (int k = threadIdx.x; k < TW * TH; k += Cfg::kThr) {
            const int ly = k / TW, lx = k - ly * TW;
            const int tx = x0 + lx, ty = y0 + ly;
            if (tx < W && ty < H) {
                unsigned long long *gk = keys + int64_t(ty) * W + tx;
                const unsigned long long v = *gk;
                if (v != KEY_UNTOUCHED) {
                    atomicMin(&L.zk[k], v);
                    *gk = KEY_UNTOUCHED;
                }
            }
        }
        lds_barrier();
    }
    if constexpr (kStamp) { if (threadIdx.x == 0) { ph[6] = wall_clock64(); ph[7] = L.nseg; } }
    // ---- 5. publish (lane-consecutive rows of the tile)
    float *vb = io.valid + b * HW;
    float *cb = io.coll + b * HW;
    if constexpr (kFuse && Coords::kGen > 0) {
        // Coordinate sources that generate obj channels (fused first-stage
        // warps): the Cobj obj channels are gathered for kT targets at once,
        // the kGen generated ones (depth, flow * -1.0) are computed once per
        // target from the winner's depth -- the key's high half for a float32
        // depth -- while those gathers are in flight.  Output channel c is
        // obj channel c below gen_at, generated c - gen_at, then obj c - kGen.
        constexpr int kT = Cfg::kGT, kCh = 4, kG = Coords::kGen;
        static_assert((TW * TH) % (Cfg::kThr * kT) == 0, "publish rounds must tile the z-buffer exactly");
        const int C = io.C, Cobj = io.Cobj, ga = io.gen_at;
        const float *ob = static_cast<const float *>(io.obj) + b * int64_t(Cobj) * HW;
        float *oo = static_cast<float *>(io.out) + b * int64_t(C) * HW;
        const unsigned uHW = unsigned(HW);
#pragma unroll
        for (int k = 0; k < TW * TH / Cfg::kThr; k += kT) {
            unsigned t[kT], w[kT];
            unsigned long long kk[kT];
            bool in[kT];
#pragma unroll
            for (int u = 0; u < kT; ++u) {
                const int q = int(threadIdx.x) + (k + u) * Cfg::kThr;
                const int ly = q / TW, lx = q - ly * TW;
                const int ty = y0 + ly, tx = x0 + lx;
                in[u] = ty < H && tx < W;
                kk[u] = L.zk[q];
                const bool touched = kk[u] != KEY_UNTOUCHED;
                const bool nowin = kk[u] == KEY_NOWIN;
                t[u] = unsigned(ty) * unsigned(W) + unsigned(tx);
                w[u] = (in[u] && touched && !nowin) ? unsigned(kk[u] & 0xFFFFFFFFull) : WIN_NONE;
                if (in[u]) {
                    __builtin_nontemporal_store(touched ? 1.f : 0.f, vb + t[u]);
                    __builtin_nontemporal_store(nowin ? 1.f : 0.f, cb + t[u]);
                }
            }
            for (int c0 = 0; c0 < (Cobj > 0 ? Cobj : 1); c0 += kCh) {
                float o[kT][kCh];
#pragma unroll
                for (int u = 0; u < kT; ++u)
#pragma unroll
                    for (int cc = 0; cc < kCh; ++cc)
                        o[u][cc] = (w[u] != WIN_NONE && c0 + cc < Cobj) ? ob[unsigned(c0 + cc) * uHW + w[u]] : 0.f;
                if (c0 == 0) {  // the generated channels, computed while the first gathers fly
                    if constexpr (GenSplit<Coords>::value) {
                        // every target's gathers first, then the stores
                        float g[kT][kG];
#pragma unroll
                        for (int u = 0; u < kT; ++u) co.gen_vals(b, w[u] != WIN_NONE ? w[u] : 0u, kk[u], g[u]);
#pragma unroll
                        for (int u = 0; u < kT; ++u)
                            if (in[u])
#pragma unroll
                                for (int e = 0; e < kG; ++e)
                                    __builtin_nontemporal_store(w[u] != WIN_NONE ? g[u][e] : 0.f,
                                                                oo + unsigned(ga + e) * uHW + t[u]);
                    } else {
#pragma unroll
                        for (int u = 0; u < kT; ++u) {
                            float g[kG];
#pragma unroll
                            for (int e = 0; e < kG; ++e) g[e] = 0.f;
                            if (w[u] != WIN_NONE) co.gen_key(b, w[u], kk[u], g);
                            if (in[u])
#pragma unroll
                                for (int e = 0; e < kG; ++e)
                                    __builtin_nontemporal_store(g[e], oo + unsigned(ga + e) * uHW + t[u]);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < kT; ++u)
#pragma unroll
                    for (int cc = 0; cc < kCh; ++cc) {
                        const int c = c0 + cc;
                        if (in[u] && c < Cobj)
                            __builtin_nontemporal_store(o[u][cc], oo + unsigned(c < ga ? c : c + kG) * uHW + t[u]);
                    }
            }
            if constexpr (GenSplit<Coords>::value) {
                // the rare winner whose key decodes to a zero depth: its sign
                // from the depth plane (after this thread's stores: same address)
#pragma unroll
                for (int u = 0; u < kT; ++u)
                    if (in[u] && w[u] != WIN_NONE) co.gen_fix(b, w[u], kk[u], oo + unsigned(ga) * uHW + t[u]);
            }
        }
    } else if constexpr (kFuse) {
        // valid, collision, and the winners' C channels: kT targets per thread
        // with all their gathers in flight before any store.  The output
        // planes and masks are touched once: non-temporal.
        // E = unsigned short: bf16 planes moved as raw bits (the warp only
        // selects a source value, so no rounding happens anywhere)
        static_assert(Coords::kGen == 0, "generated channels take the branch above");
        constexpr int kT = Cfg::kGT, kCh = 8;
        static_assert((TW * TH) % (Cfg::kThr * kT) == 0, "publish rounds must tile the z-buffer exactly");
        const int C = io.C;
        const E *ob = static_cast<const E *>(io.obj) + b * int64_t(io.Cobj) * HW;
        E *oo = static_cast<E *>(io.out) + b * int64_t(C) * HW;
        const unsigned uHW = unsigned(HW);
        auto source = [&](int c, unsigned wi) -> E { return ob[unsigned(c) * uHW + wi]; };
#pragma unroll
        for (int k = 0; k < TW * TH / Cfg::kThr; k += kT) {
            unsigned t[kT], w[kT];
            bool in[kT];
#pragma unroll
            for (int u = 0; u < kT; ++u) {
                const int q = int(threadIdx.x) + (k + u) * Cfg::kThr;
                const int ly = q / TW, lx = q - ly * TW;
                const int ty = y0 + ly, tx = x0 + lx;
                in[u] = ty < H && tx < W;
                const unsigned long long key = L.zk[q];
                const bool touched = key != KEY_UNTOUCHED;
                const bool nowin = key == KEY_NOWIN;
                t[u] = unsigned(ty) * unsigned(W) + unsigned(tx);
                w[u] = (in[u] && touched && !nowin) ? unsigned(key & 0xFFFFFFFFull) : WIN_NONE;
                if (in[u]) {
                    __builtin_nontemporal_store(touched ? 1.f : 0.f, vb + t[u]);
                    __builtin_nontemporal_store(nowin ? 1.f : 0.f, cb + t[u]);
                }
            }
            // channels generated from the winner (Coords::kGen of them at output
            // channel gen_at; obj supplies the others): one source read per target
            for (int c0 = 0; c0 < C; c0 += kCh) {
                E o[kT][kCh];
#pragma unroll
                for (int u = 0; u < kT; ++u)
#pragma unroll
                    for (int cc = 0; cc < kCh; ++cc)
                        o[u][cc] = (w[u] != WIN_NONE && c0 + cc < C) ? source(c0 + cc, w[u]) : E(0);
#pragma unroll
                for (int u = 0; u < kT; ++u)
#pragma unroll
                    for (int cc = 0; cc < kCh; ++cc)
                        if (in[u] && c0 + cc < C)
                            __builtin_nontemporal_store(o[u][cc], oo + unsigned(c0 + cc) * uHW + t[u]);
            }
        }
    } else {
        unsigned int *win = ws.winner + int64_t(bl) * HW;
        static_assert((TW * TH) % Cfg::kThr == 0, "publish rounds must tile the z-buffer exactly");
#pragma unroll
        for (int k = 0; k < TW * TH / Cfg::kThr; ++k) {
            const int q = int(threadIdx.x) + k * Cfg::kThr;
            const int ly = q / TW, lx = q - ly * TW;
            const int ty = y0 + ly, tx = x0 + lx;
            if (ty >= H || tx >= W) continue;
            const unsigned long long key = L.zk[q];
            const bool touched = key != KEY_UNTOUCHED;
            const bool nowin = key == KEY_NOWIN;
            const unsigned t = unsigned(ty) * unsigned(W) + unsigned(tx);
            const unsigned wv = (touched && !nowin) ? unsigned(key & 0xFFFFFFFFull) : WIN_NONE;
            if constexpr (Cfg::kNTPub >= 2) __builtin_nontemporal_store(wv, win + t);
            else win[t] = wv;
            if constexpr (Cfg::kNTPub >= 1) {
                __builtin_nontemporal_store(touched ? 1.f : 0.f, vb + t);
                __builtin_nontemporal_store(nowin ? 1.f : 0.f, cb + t);
            } else {
                vb[t] = touched ? 1.f : 0.f;
                cb[t] = nowin ? 1.f : 0.f;
            }
        }
    }
    if constexpr (kStamp) {
        lds_barrier();
        if (threadIdx.x == 0) { ph[1] = wall_clock64(); ph[2] = nblk_tot; ph[3] = lin; }
    }
}

using SplitCfg = SplatCfg<512, 2, 8>;  // split engine: 4 workgroups / CU, light publish
// fused engine: 2 workgroups / CU (VGPR-bound), every target's gathers of a
// thread (8 x C) in flight at once.  Measured at 64 x 768x1024, C = 6
// (tools/probe_tile.py): 512 threads / 2 in flight / 4 per CU 702 us;
// 512 / 8 / 2 per CU 675; as a persistent kernel 655; 256 threads 715.
#ifndef OFD_PROBE_THR  // SPLAT workgroup shape: overridable only by the diagnostic probe build
#define OFD_PROBE_THR 512
#define OFD_PROBE_MINW 4
#endif
#ifndef OFD_PROBE_GT  // targets in flight per thread in the publish (probe builds override)
#define OFD_PROBE_GT 8
#endif
#ifndef OFD_PROBE_UF  // 4-block splat slots in flight per wave (probe builds override)
#define OFD_PROBE_UF kSplatU
#endif
// targets in flight per thread, at most the tile's targets per thread (a
// 128 x 16 tile at 512 threads holds 4 per thread)
constexpr int gt_cap(int gt, int thr, int th = TH) { return gt < TW * th / thr ? gt : TW * th / thr; }
using FusedCfg = SplatCfg<OFD_PROBE_THR, gt_cap(OFD_PROBE_GT, OFD_PROBE_THR), OFD_PROBE_MINW, OFD_PROBE_UF>;
// short calls (run_f32): 128 x 16 tiles, one workgroup per tile, 4 targets in
// flight per thread (2048 targets / 512 threads)
using FusedShortCfg = SplatCfg<OFD_PROBE_THR, gt_cap(OFD_PROBE_GT, OFD_PROBE_THR, kShortTH), OFD_PROBE_MINW, OFD_PROBE_UF,
                               1, 0, kShortTH>;
// coordinate sources that generate channels carry the generated values and a
// division per source: 4 targets in flight keeps them inside 128 VGPRs
// (Coords::kGenGT of them: 4 for the disparity source, 2 for the ego-motion
// source, whose per-target projection is the heavier)
template <typename Coords>
using FusedGenCfg = SplatCfg<512, gt_cap(Coords::kGenGT, 512), 4>;
template <typename Coords>
using FusedCfgFor = typename std::conditional<Coords::kGen == 0, FusedCfg, FusedGenCfg<Coords>>::type;

// One workgroup per tile (grid = the chunk's tiles, rounded up to 8): tile
// lin = (blockIdx % 8) * per + blockIdx / 8, so the workgroups of one XCD
// (round-robin placement) take consecutive tiles of the band-major order.
// The fused TILE engine uses it for calls of few tiles per resident slot,
// where the hardware's dispatch of fresh workgroups balances the last tiles
// better than the persistent kernel's queues (see run_f32).
template <typename Coords, bool kVec, bool kFuse = false, bool kStamp = false, typename Cfg = SplitCfg,
          typename E = float, bool kPack = false>
__global__ __launch_bounds__(Cfg::kThr, Cfg::kMinW) void splat_kernel(Coords co, const float *__restrict__ depth,
                                                                SplatIO io, ChunkArgs a, int H, int W, int64_t HW,
                                                                TileGeom g, unsigned long long *stamps = nullptr) {
    __shared__ TileLdsT<Cfg::kTH> L;
    const unsigned total = unsigned(a.nimg) * unsigned(g.ntiles);
    const unsigned per = (total + 7u) / 8u;
    const unsigned lin = (blockIdx.x % 8u) * per + blockIdx.x / 8u;
    if (lin >= total) return;
    int bl, tile;
    tile_of<Cfg>(lin, a, g, bl, tile);
    splat_tile<Coords, kVec, kFuse, kStamp, Cfg, E, kPack>(L, lin, bl, tile, co, depth, io, a, H, W, HW, g, stamps);
}

// Persistent SPLAT: one workgroup per resident slot, looping over tiles.  The
// band-major tile order is cut into 8 contiguous queues, queue k served first
// by the workgroups with blockIdx % 8 == k (one XCD under round-robin
// placement); a workgroup whose queue is drained takes tiles from the next
// queues.  Queue words count down from ~0 (the workspace's initial state);
// the last workgroup out restores them, so the next launch starts clean.
// Placement and order affect speed only: every tile is processed exactly
// once, and no workgroup ever waits for another.
template <typename Coords, bool kVec, bool kFuse = true, bool kStamp = false, typename Cfg = FusedCfg,
          typename E = float, bool kPack = false>
__global__ __launch_bounds__(Cfg::kThr, Cfg::kMinW) void splat_persist_kernel(Coords co, const float *__restrict__ depth,
                                                                        SplatIO io, ChunkArgs a, int H, int W,
                                                                        int64_t HW, TileGeom g,
                                                                        unsigned long long *stamps = nullptr) {
    __shared__ TileLdsT<Cfg::kTH> L;
    unsigned *queue = a.ws.queue;
    const unsigned total = unsigned(a.nimg) * unsigned(g.ntiles);
    const unsigned per = (total + 7u) / 8u;
    const unsigned home = blockIdx.x % 8u;
    unsigned drained = 0;  // thread 0: queues seen empty
    for (;;) {
        if (threadIdx.x == 0) L.next = dequeue_tile(queue, home, per, total, drained);
        lds_barrier();
        const unsigned lin = L.next;
        if (lin == ~0u) return;
        int bl, tile;
        tile_of<Cfg>(lin, a, g, bl, tile);
        splat_tile<Coords, kVec, kFuse, kStamp, Cfg, E, kPack>(L, lin, bl, tile, co, depth, io, a, H, W, HW, g, stamps);
        // splat_tile ends with LDS reads of the z-buffer; the next iteration's
        // barrier orders them before the next tile's initialisation
    }
}

// ---- RESOLVE: one target per thread over 2-D target patches -- workgroup =
// 64*kWX columns x kRows rows (wave = one 64-pixel row segment), grid (x, y,
// image) so no division is needed.  The gathers of neighbouring targets,
// whose sources share cache lines under rotated / sheared flows, run on one
// CU at the same time.  The output planes and the winner map are touched once,
// so they go non-temporal (kNT / kNTW) and leave the caches to the gathered
// source lines.  tools/probe_tile.py sweep at 64 x 768x1024, C=6: 128x8 nt
// 462 us, 64x16 nt 474, 64x16 plain 487, 1024x1 plain 553.  32-bit offsets
// inside an image (C*H*W < 2^30 is checked on the host); the gathers of up to
// kChan channels are in flight before the stores.
template <int kChan, int kRows, int kWX = 1, bool kNT = false, bool kNTW = false>
__global__ __launch_bounds__(64 * kWX * kRows) void resolve2d_kernel(const float *__restrict__ obj,
                                                                     const unsigned int *__restrict__ winner,
                                                                     float *__restrict__ out, int C, int H, int W,
                                                                     int64_t HW, int64_t b0) {
    const unsigned wave = threadIdx.x >> 6;
    const unsigned x = (blockIdx.x * unsigned(kWX) + wave % unsigned(kWX)) * 64u + (threadIdx.x & 63u);
    const unsigned y = blockIdx.y * unsigned(kRows) + wave / unsigned(kWX);
    if (x >= unsigned(W) || y >= unsigned(H)) return;
    const int64_t bl = blockIdx.z, b = b0 + bl;
    const unsigned p = y * unsigned(W) + x;
    const unsigned w = kNTW ? __builtin_nontemporal_load(winner + bl * HW + p) : winner[bl * HW + p];
    const float *ob = obj + b * C * HW;
    float *oo = out + b * C * HW;
    const unsigned uHW = unsigned(HW);
    const bool win = w != WIN_NONE;
    for (int c0 = 0; c0 < C; c0 += kChan) {
        float o[kChan];
#pragma unroll
        for (int cc = 0; cc < kChan; ++cc)
            o[cc] = (win && c0 + cc < C) ? ob[unsigned(c0 + cc) * uHW + w] : 0.f;
#pragma unroll
        for (int cc = 0; cc < kChan; ++cc)
            if (c0 + cc < C) {
                if constexpr (kNT)
                    __builtin_nontemporal_store(o[cc], oo + unsigned(c0 + cc) * uHW + p);
                else
                    oo[unsigned(c0 + cc) * uHW + p] = o[cc];
            }
    }
}

// ---------------------------------------------------------------- ATOMIC engine
// Lane-strided: a wave covers 64*4 consecutive chunk pixels, lane l takes
// pixels l, l+64, l+128, l+192, so every atomic / load / store wave-instruction
// touches one contiguous span (thread-contiguous spans measured 3.5x slower
// for 64-bit atomics, tools/microbench.hip).
template <typename Coords>
__global__ __launch_bounds__(kBlock) void splat_atomic_kernel(Coords co, const float *__restrict__ depth,
                                                              unsigned long long *__restrict__ keys, int H, int W,
                                                              int64_t HW, int64_t b0, int64_t chunk_px) {
    const int64_t base = (int64_t(blockIdx.x) * kBlock + (threadIdx.x & ~63)) * 4 + lane_id();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t q = base + k * 64;
        int t = -1;
        unsigned long long key = 0;
        if (q < chunk_px) {
            const int64_t bl = q / HW, p = q - bl * HW, b = b0 + bl;
            const int j = int(p / W), i = int(p - int64_t(j) * W);
            typename Coords::V x, y;
            co.load(b, p, x, y);
            int tx, ty;
            co.target(b, i, j, x, y, H, W, tx, ty);
            if (tx >= 0) {
                t = int(bl * HW) + ty * W + tx;  // chunk-local slot (chunk_px < 2^31)
                key = make_key(co.key_depth(b, p, depth), unsigned(p));
            }
        }
        wave_run_atomic_min(keys, t, key);
    }
}

__global__ __launch_bounds__(kBlock) void resolve_atomic_kernel(const float *__restrict__ obj,
                                                                unsigned long long *__restrict__ keys,
                                                                float *__restrict__ out, float *__restrict__ valid,
                                                                float *__restrict__ coll, int C, int64_t HW,
                                                                int64_t b0, int64_t chunk_px) {
    const int64_t base = (int64_t(blockIdx.x) * kBlock + (threadIdx.x & ~63)) * 4 + lane_id();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t q = base + k * 64;
        if (q >= chunk_px) break;
        const int64_t bl = q / HW, p = q - bl * HW, b = b0 + bl;
        const unsigned long long key = keys[q];
        keys[q] = KEY_UNTOUCHED;
        const bool touched = key != KEY_UNTOUCHED;
        const bool win = touched && key != KEY_NOWIN;
        const int64_t s = int64_t(key & 0xFFFFFFFFull);
        valid[b * HW + p] = touched ? 1.f : 0.f;
        coll[b * HW + p] = (touched && !win) ? 1.f : 0.f;
        const float *ob = obj + b * C * HW;
        float *oo = out + b * C * HW + p;
        for (int c = 0; c < C; ++c) oo[int64_t(c) * HW] = win ? ob[int64_t(c) * HW + s] : 0.f;
    }
}

// ---------------------------------------------------------------- f64 op (atomic)
// Exact double depths do not fit a 32-bit key half, so the double path keys
// on the full 64-bit orderable depth first, then resolves ties by a 32-bit
// index min among the sources that hold the minimum depth.
__global__ __launch_bounds__(kBlock) void splat_f64_depth_kernel(
        const double *__restrict__ sy, const double *__restrict__ sx, const double *__restrict__ depth,
        unsigned long long *__restrict__ zkeys, int H, int W, int64_t HW, int64_t b0, int64_t chunk_px) {
    const int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (q >= chunk_px) return;
    const int64_t g = b0 * HW + q;
    int tx, ty;
    target_safe<double>(sx[g], sy[g], H, W, tx, ty);
    if (tx < 0) return;
    const double d = depth[g];
    const unsigned long long z = (d < 1000.0) ? orderable64(d) : ZKEY_NOWIN;
    atomicMin(zkeys + (q / HW) * HW + int64_t(ty) * W + tx, z);
}

__global__ __launch_bounds__(kBlock) void splat_f64_index_kernel(
        const double *__restrict__ sy, const double *__restrict__ sx, const double *__restrict__ depth,
        const unsigned long long *__restrict__ zkeys, unsigned int *__restrict__ idx,
        int H, int W, int64_t HW, int64_t b0, int64_t chunk_px) {
    const int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (q >= chunk_px) return;
    const int64_t g = b0 * HW + q;
    const double d = depth[g];
    if (!(d < 1000.0)) return;
    int tx, ty;
    target_safe<double>(sx[g], sy[g], H, W, tx, ty);
    if (tx < 0) return;
    const int64_t slot = (q / HW) * HW + int64_t(ty) * W + tx;
    if (zkeys[slot] == orderable64(d)) atomicMin(idx + slot, (unsigned int)(q % HW));
}

__global__ __launch_bounds__(kBlock) void resolve_f64_kernel(
        const double *__restrict__ obj, unsigned long long *__restrict__ zkeys, unsigned int *__restrict__ idx,
        double *__restrict__ out, double *__restrict__ valid, double *__restrict__ coll,
        int C, int64_t HW, int64_t b0, int64_t chunk_px) {
    const int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (q >= chunk_px) return;
    const int64_t bl = q / HW, p = q - bl * HW, b = b0 + bl;
    const unsigned long long z = zkeys[q];
    const unsigned int s = idx[q];
    zkeys[q] = ZKEY_UNTOUCHED;
    idx[q] = IDX_NONE;
    const bool touched = z != ZKEY_UNTOUCHED;
    const bool win = touched && z != ZKEY_NOWIN;
    valid[b * HW + p] = touched ? 1.0 : 0.0;
    coll[b * HW + p] = (touched && !win) ? 1.0 : 0.0;
    const double *ob = obj + b * C * HW;
    double *oo = out + b * C * HW + p;
    for (int c = 0; c < C; ++c) oo[int64_t(c) * HW] = win ? ob[int64_t(c) * HW + s] : 0.0;
}

// ---------------------------------------------------------------- host side
inline unsigned grid_for(int64_t work_items, int per_block = kBlock) {
    return unsigned((work_items + per_block - 1) / per_block);
}

inline bool aligned(const void *p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

int check_dims(int64_t B, int64_t C, int64_t H, int64_t W) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return OFD_FW_EINVAL;
    if (H * W >= (int64_t(1) << 31)) return OFD_FW_ETOOBIG;
    return OFD_FW_OK;
}

enum class Mode { Tile = 0, Atomic = 1, TileSplit = 2 };

// Engine selection: OFD_FW_MODE=atomic|split in the environment, or
// ofd_fw_set_engine() at run time (tests and benchmarks compare them).
int g_engine = -1;

Mode engine_mode() {
    if (g_engine < 0) {
        const char *e = getenv("OFD_FW_MODE");
        g_engine = (e && strcmp(e, "atomic") == 0)  ? int(Mode::Atomic)
                   : (e && strcmp(e, "split") == 0) ? int(Mode::TileSplit)
                                                    : int(Mode::Tile);
    }
    return Mode(g_engine);
}

// images per chunk for a workspace of `bytes`; chunk pixels stay < 2^31
int64_t chunk_images(int64_t B, int64_t HW, size_t per_image, size_t bytes) {
    int64_t g = int64_t(bytes / per_image);
    const int64_t cap = ((int64_t(1) << 31) - 1) / HW;
    if (g > cap) g = cap;
    return g < B ? g : B;
}

// C == 0: the reference launches no channel-0 thread, so valid and collision
// stay as allocated, all zero (fw_cuda_kernel.cu:59-60, :38).
int zero_masks(void *valid, void *coll, size_t bytes, hipStream_t st) {
    hipError_t e = hipMemsetAsync(valid, 0, bytes, st);
    if (e == hipSuccess) e = hipMemsetAsync(coll, 0, bytes, st);
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

// Which slab layout last left each workspace's key slabs and flags
// all-ones.  A workspace initialised by ofd_fw_workspace_init is clean for
// every layout; a call with a different layout (other H, W or chunking) than
// the last one re-initialises the slabs it uses before launching, because the
// previous layout's scratch boxes may sit where this layout keeps keys/flags.
struct LayoutSig {
    int64_t H, W, G;
    int nslab;
    bool operator==(const LayoutSig &o) const { return H == o.H && W == o.W && G == o.G && nslab == o.nslab; }
};
constexpr LayoutSig kCleanSig{-1, -1, -1, -1};
std::mutex g_layout_mu;
std::unordered_map<const void *, LayoutSig> g_layout;

void mark_clean(const void *ws) {
    std::lock_guard<std::mutex> lk(g_layout_mu);
    g_layout[ws] = kCleanSig;
}

// true if the caller must re-initialise the slabs before using layout `sig`
bool claim_layout(const void *ws, const LayoutSig &sig) {
    std::lock_guard<std::mutex> lk(g_layout_mu);
    auto it = g_layout.find(ws);
    const bool ok = it != g_layout.end() && (it->second == sig || it->second == kCleanSig);
    g_layout[ws] = sig;
    return !ok;
}

// Resident workgroup slots of a kernel on the current device (the persistent
// SPLAT's grid); queried once per kernel instantiation.
template <typename K>
unsigned resident_slots(K kernel, int threads) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void *>(kernel), threads, 0) !=
            hipSuccess ||
        cus <= 0 || per <= 0)
        return 1024u;
    if (const char *e = getenv("OFD_SPLAT_WG_PER_CU")) {  // probe knob: workgroups per CU of the grid
        const int v = atoi(e);
        if (v > 0) per = v;
    }
    return unsigned(cus) * unsigned(per);
}

template <typename Coords, bool kVec, typename Cfg = FusedCfgFor<Coords>, typename E = float, bool kPack = false>
unsigned persist_slots() {
    static const unsigned slots =
        resident_slots(splat_persist_kernel<Coords, kVec, true, false, Cfg, E, kPack>, Cfg::kThr);
    return slots;
}

template <typename Coords, bool kVec, typename Cfg = FusedCfgFor<Coords>, typename E = float, bool kPack = false>
unsigned persist_grid(unsigned tiles) {
    const unsigned slots = persist_slots<Coords, kVec, Cfg, E, kPack>();
    return tiles < slots ? tiles : slots;
}

// Packed targets in the fused TILE engine (coordinate sources with exact BIN
// targets): on by default; OFD_FW_PACK=0 or ofd_fw_set_pack(0) turns them off
// (A/B and cross-check; results never depend on it).
int g_pack = -1;
bool pack_enabled() {
    if (g_pack < 0) {
        const char *e = getenv("OFD_FW_PACK");
        g_pack = e ? (atoi(e) != 0) : 1;
    }
    return g_pack != 0;
}

// Calls with fewer than persist_min() tiles per resident SPLAT slot launch
// one workgroup per tile instead of the persistent kernel (OFD_PERSIST_MIN
// overrides; 0 = always persistent).  Whole calls (tools/ab_env.sh, ms):
// config 2 (32 x 480x640, 4.7 tiles per slot) 0.156 one-per-tile vs 0.184
// persistent; config 5 (64 x 368x560, 7.5) 0.218 vs 0.234; 32 x 768x1024 (12)
// 0.383 vs 0.387; 16 x 768x1024 (6) 0.218 vs 0.216; the headline (24) 0.741
// vs 0.721 -- the persistent queues pay off only on long calls.
int g_persist_min = -1;  // ofd_fw_set_persist_min; -1 = not set (OFD_PERSIST_MIN, else 16)
unsigned persist_min() {
    if (g_persist_min < 0) {
        const char *e = getenv("OFD_PERSIST_MIN");
        g_persist_min = e ? atoi(e) : 16;
        if (g_persist_min < 0) g_persist_min = 16;
    }
    return unsigned(g_persist_min);
}

// Short calls on 128 x kShortTH tiles (ofd_fw_set_short_tiles; OFD_FW_SHORT_TILES,
// default on).  Results never depend on it.
int g_short_tiles = -1;
bool short_tiles_enabled() {
    if (g_short_tiles < 0) {
        const char *e = getenv("OFD_FW_SHORT_TILES");
        g_short_tiles = (e && e[0] == '0') ? 0 : 1;
    }
    return g_short_tiles != 0;
}

// Optional timing hook (ofd_fw_set_profile_events): events recorded on the
// launch stream right before the first and right after the last RESOLVE
// launch of a call -- the dominant kernel -- so a benchmark can time it with
// HIP events on the stream it runs on.
hipEvent_t g_prof_start = nullptr, g_prof_stop = nullptr;
hipEvent_t g_prof_bin = nullptr;  // ofd_fw_set_profile_bin_event: before the first BIN

// E: the obj / output element type -- float, or unsigned short for bf16
// planes (fused TILE engine only, like coordinate sources that generate
// channels).
template <typename Coords, typename E = float>
int run_f32(Coords co, const E *obj, const float *depth, E *out, float *valid, float *coll,
            int64_t B, int64_t C, int64_t H, int64_t W, void *ws, size_t ws_bytes, hipStream_t st,
            int gen_at = -1) {
    constexpr bool kTileOnly = Coords::kGen > 0 || !std::is_same<E, float>::value;
    const int64_t HW = H * W;
    if (gen_at < 0) gen_at = int(C);
    if (B == 0 || HW == 0) return OFD_FW_OK;
    if (C == 0) return zero_masks(valid, coll, size_t(B * HW) * sizeof(float), st);
    if (!ws || !aligned(ws, 16)) return OFD_FW_EWORKSPACE;
    const size_t per_image = per_image_bytes(H, W);
    const TileGeom g = make_geom(H, W);
    // the tile engine's gathers use 32-bit offsets inside one image
    // Coordinate sources that generate obj channels run on the fused TILE
    // engine only (the gather is where the channels are generated).
    if (kTileOnly && C * HW >= (int64_t(1) << 30)) return OFD_FW_ETOOBIG;
    const Mode mode = kTileOnly ? Mode::Tile : (C * HW < (int64_t(1) << 30)) ? engine_mode() : Mode::Atomic;

    // One slab of G images, shared by both engines (so the all-ones key /
    // flag regions are the same bytes whichever engine ran last).  Chunks are
    // large: every kernel's grid is then many times the resident slots, which
    // measured best (a two-stream pipeline of small, cache-resident chunks
    // lost: ~10 us per cross-stream event hop, and the latency-bound BIN ran
    // 3-4x slower beside a streaming RESOLVE).
    const int64_t G = chunk_images(B, HW, per_image, ws_bytes);
    if (G < 1) return OFD_FW_EWORKSPACE;
    const int64_t nch = (B + G - 1) / G;
    if (claim_layout(ws, LayoutSig{H, W, G, 1})) {
        const hipError_t e = hipMemsetAsync(ws, 0xFF, size_t(G) * per_image, st);
        if (e != hipSuccess) return int(e);
    }
    const Ws slab = carve(ws, G, HW, make_geom(H, W, kShortTH));  // the layout of both tile heights
    // 16-byte coordinate / depth loads in BIN and SPLAT
    const bool vec = W % 4 == 0 && co.vec_ok() && uintptr_t(depth) % 16 == 0;
    for (int64_t c = 0; c < nch; ++c) {
        const int64_t b0 = c * G;
        const int64_t nb = (B - b0) < G ? (B - b0) : G;
        const int64_t px = nb * HW;
        if constexpr (!kTileOnly) {
            if (mode == Mode::Atomic) {
                hipLaunchKernelGGL((splat_atomic_kernel<Coords>), dim3(grid_for(px, kBlock * 4)), dim3(kBlock), 0,
                                   st, co, depth, slab.keys, int(H), int(W), HW, b0, px);
                if (c == 0 && g_prof_start) (void)hipEventRecord(g_prof_start, st);
                hipLaunchKernelGGL(resolve_atomic_kernel, dim3(grid_for(px, kBlock * 4)), dim3(kBlock), 0, st,
                                   obj, slab.keys, out, valid, coll, int(C), HW, b0, px);
                if (c == nch - 1 && g_prof_stop) (void)hipEventRecord(g_prof_stop, st);
                continue;
            }
        }
        {
            const ChunkArgs a{slab, b0, int(nb)};
            const SplatIO io{valid, coll, obj, out, int(C), int(C) - Coords::kGen, gen_at};
            const dim3 bgrid(grid_for(nb * g.nseg, kWaves * kBinSPW));
            const dim3 sgrid((unsigned(nb * g.ntiles) + 7u) / 8u * 8u);
            if (mode == Mode::Tile) {
                // fused: BIN, then a persistent SPLAT gathers the output planes
                // itself (dominant kernel); one SPLAT workgroup per tile on
                // short calls
                const unsigned tiles = unsigned(nb * g.ntiles);
                using Cfg = FusedCfgFor<Coords>;
                auto fused = [&](auto vec_c, auto pack_c) {
                    constexpr bool kV = decltype(vec_c)::value, kP = decltype(pack_c)::value;
                    const bool short_call = tiles < persist_min() * persist_slots<Coords, kV, Cfg, E, kP>();
                    if (c == 0 && g_prof_bin) (void)hipEventRecord(g_prof_bin, st);
                    if constexpr (Coords::kGen == 0) {
                        // short calls of plain coordinate sources: 128 x 16
                        // tiles, twice the workgroups of the one-per-tile grid,
                        // so the last tiles drain sooner (config 2: 0.154 ->
                        // 0.150 ms, profiles/r06_t16_probe.txt)
                        if (short_call && short_tiles_enabled()) {
                            const TileGeom gs = make_geom(H, W, kShortTH);
                            hipLaunchKernelGGL((bin_kernel<Coords, kV, kBinSPW, kP, kShortTH>), bgrid, dim3(kWarpThreads),
                                               0, st, co, depth, a, int(H), int(W), HW, gs);
                            if (c == 0 && g_prof_start) (void)hipEventRecord(g_prof_start, st);
                            hipLaunchKernelGGL((splat_kernel<Coords, kV, true, false, FusedShortCfg, E, kP>),
                                               dim3((unsigned(nb * gs.ntiles) + 7u) / 8u * 8u), dim3(FusedShortCfg::kThr),
                                               0, st, co, depth, io, a, int(H), int(W), HW, gs, nullptr);
                            return;
                        }
                    }
                    hipLaunchKernelGGL((bin_kernel<Coords, kV, kBinSPW, kP>), bgrid, dim3(kWarpThreads), 0, st, co,
                                       depth, a, int(H), int(W), HW, g);
                    if (c == 0 && g_prof_start) (void)hipEventRecord(g_prof_start, st);
                    if (short_call)
                        hipLaunchKernelGGL((splat_kernel<Coords, kV, true, false, Cfg, E, kP>), sgrid, dim3(Cfg::kThr),
                                           0, st, co, depth, io, a, int(H), int(W), HW, g, nullptr);
                    else
                        hipLaunchKernelGGL((splat_persist_kernel<Coords, kV, true, false, Cfg, E, kP>),
                                           dim3(persist_grid<Coords, kV, Cfg, E, kP>(tiles)), dim3(Cfg::kThr), 0, st,
                                           co, depth, io, a, int(H), int(W), HW, g, nullptr);
                };
                using T_ = std::true_type;
                using F_ = std::false_type;
                bool packed = false;
                if constexpr (Coords::kPackable) {
                    if (pack_enabled()) {
                        packed = true;
                        if (vec) fused(T_{}, T_{});
                        else fused(F_{}, T_{});
                    }
                }
                if (!packed) {
                    if (vec) fused(T_{}, F_{});
                    else fused(F_{}, F_{});
                }
                if (c == nch - 1 && g_prof_stop) (void)hipEventRecord(g_prof_stop, st);
                continue;
            }
            if (vec)
                hipLaunchKernelGGL((bin_kernel<Coords, true, kBinSPW>), bgrid, dim3(kWarpThreads), 0, st, co, depth, a,
                                   int(H), int(W), HW, g);
            else
                hipLaunchKernelGGL((bin_kernel<Coords, false, kBinSPW>), bgrid, dim3(kWarpThreads), 0, st, co, depth,
                                   a, int(H), int(W), HW, g);
            if constexpr (!kTileOnly) {
            if (vec)
                hipLaunchKernelGGL((splat_kernel<Coords, true>), sgrid, dim3(kWarpThreads), 0, st, co, depth, io, a,
                                   int(H), int(W), HW, g, nullptr);
            else
                hipLaunchKernelGGL((splat_kernel<Coords, false>), sgrid, dim3(kWarpThreads), 0, st, co, depth, io, a,
                                   int(H), int(W), HW, g, nullptr);
            const dim3 rgrid(unsigned((W + 64 * kResolveWX - 1) / (64 * kResolveWX)),
                             unsigned((H + kResolveRows - 1) / kResolveRows), unsigned(nb));
            const dim3 rblock(64 * kResolveWX * kResolveRows);
            if (c == 0 && g_prof_start) (void)hipEventRecord(g_prof_start, st);
            if (C <= 8)
                hipLaunchKernelGGL((resolve2d_kernel<8, kResolveRows, kResolveWX, true, true>), rgrid, rblock, 0, st,
                                   obj, slab.winner, out, int(C), int(H), int(W), HW, b0);
            else
                hipLaunchKernelGGL((resolve2d_kernel<4, kResolveRows, kResolveWX, true, true>), rgrid, rblock, 0, st,
                                   obj, slab.winner, out, int(C), int(H), int(W), HW, b0);
            if (c == nch - 1 && g_prof_stop) (void)hipEventRecord(g_prof_stop, st);
            }
        }
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

}  // namespace

namespace {
// Disparity warps (preprocess.py:356-359) move every source along its own
// row: the flow is (-s*50/d, -0), and fw.py's clamp keeps y + -0 = y.  So the
// fused disparity warp needs no BIN and no tile lists: one workgroup per
// image row folds the row's keys into an LDS z-buffer (ds_min_u64 on the
// same lexmin key as every engine) and publishes the row -- the winners' obj
// channels (same row: L1 / L2 hits), the generated depth / disparity / +0
// channels, valid and collision.  Bit-identical to the tile engine on the
// same call (tests/test_fused.py); 48 B/px of HBM traffic at C = 6.
constexpr int kRowThr = 256;
typedef float RowF4 __attribute__((ext_vector_type(4)));
constexpr int kRowMaxW = 8192;  // 64 KB of keys per workgroup

template <typename D, bool kVec>
__global__ __launch_bounds__(kRowThr) void disp_row_kernel(DisparityCoords<D> co, const float *__restrict__ obj,
                                                         float *__restrict__ out, float *__restrict__ valid,
                                                         float *__restrict__ coll, int Cobj, int gen_at, int H, int W) {
    extern __shared__ unsigned long long zrow[];
    const int64_t row = blockIdx.x;
    const int64_t b = row / H;
    const int j = int(row - b * H);
    const int64_t HW = int64_t(H) * W;
    for (int x = threadIdx.x; x < W; x += kRowThr) zrow[x] = KEY_UNTOUCHED;
    __syncthreads();
    const D *dr = co.depth + b * HW + int64_t(j) * W;
    // kVec (W % 4 == 0, 16-byte aligned planes): four consecutive pixels per
    // thread, 16-byte loads and stores
    constexpr int kP = kVec ? 4 : 1;
    for (int x0 = kP * threadIdx.x; x0 < W; x0 += kP * kRowThr) {
        D d[kP];
        if constexpr (kVec)
            ::load4<true>(dr + x0, d, 4);
        else
            d[0] = dr[x0];
#pragma unroll
        for (int e = 0; e < kP; ++e) {
            int tx, ty;
            target_flow<D>(x0 + e, j, -co.disp(b, d[e]), -D(0), H, W, tx, ty);
            if (tx >= 0) atomicMin(&zrow[tx], make_key(float(d[e]), unsigned(j * W + x0 + e)));
        }
    }
    __syncthreads();
    const int C = Cobj + 3;
    const float *ob = obj + b * int64_t(Cobj) * HW;
    float *oo = out + b * int64_t(C) * HW;
    const unsigned uHW = unsigned(HW);
    auto put = [&](float *dst, const float v[kP]) {
        if constexpr (kVec)
            __builtin_nontemporal_store(RowF4{v[0], v[1], v[2], v[3]}, reinterpret_cast<RowF4 *>(dst));
        else
            __builtin_nontemporal_store(v[0], dst);
    };
    for (int x0 = kP * threadIdx.x; x0 < W; x0 += kP * kRowThr) {
        unsigned long long key[kP];
        unsigned w[kP];
        float vv[kP], cv[kP];
#pragma unroll
        for (int e = 0; e < kP; ++e) {
            key[e] = zrow[x0 + e];
            const bool touched = key[e] != KEY_UNTOUCHED, nowin = key[e] == KEY_NOWIN;
            w[e] = (touched && !nowin) ? unsigned(key[e] & 0xFFFFFFFFull) : WIN_NONE;
            vv[e] = touched ? 1.f : 0.f;
            cv[e] = nowin ? 1.f : 0.f;
        }
        const unsigned t = unsigned(j) * unsigned(W) + unsigned(x0);
        put(valid + b * HW + t, vv);
        put(coll + b * HW + t, cv);
        for (int c = 0; c < Cobj; ++c) {
            float v[kP];
#pragma unroll
            for (int e = 0; e < kP; ++e) v[e] = w[e] != WIN_NONE ? ob[unsigned(c) * uHW + w[e]] : 0.f;
            put(oo + unsigned(c < gen_at ? c : c + 3) * uHW + t, v);
        }
        float g[3][kP];
#pragma unroll
        for (int e = 0; e < kP; ++e) {
            float ge[3] = {0.f, 0.f, 0.f};
            if (w[e] != WIN_NONE) co.gen_key(b, w[e], key[e], ge);
#pragma unroll
            for (int q = 0; q < 3; ++q) g[q][e] = ge[q];
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) put(oo + unsigned(gen_at + q) * uHW + t, g[q]);
    }
}

int g_disp_rows = -1;  // ofd_fw_set_disparity_rows; -1: OFD_DISP_ROW (default on)

bool disp_row_enabled() {
    static const bool env_on = [] {
        const char *e = getenv("OFD_DISP_ROW");
        return !(e && e[0] == '0');
    }();
    return g_disp_rows < 0 ? env_on : g_disp_rows != 0;
}

template <typename D>
int warp_disparity_rows(DisparityCoords<D> co, const float *obj, int64_t Cobj, float *output, float *valid,
                        float *collision, int64_t B, int64_t H, int64_t W, hipStream_t st) {
    const int gen_at = int(Cobj < 3 ? Cobj : 3);
    const bool vec = W % 4 == 0 && aligned(co.depth, 16) && aligned(output, 16) && aligned(valid, 16) &&
                     aligned(collision, 16);
    if (vec)
        hipLaunchKernelGGL((disp_row_kernel<D, true>), dim3(unsigned(B * H)), dim3(kRowThr), size_t(W) * 8, st, co, obj,
                           output, valid, collision, int(Cobj), gen_at, int(H), int(W));
    else
        hipLaunchKernelGGL((disp_row_kernel<D, false>), dim3(unsigned(B * H)), dim3(kRowThr), size_t(W) * 8, st, co,
                           obj, output, valid, collision, int(Cobj), gen_at, int(H), int(W));
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

bool rows_ok(int64_t B, int64_t C, int64_t H, int64_t W) {
    return disp_row_enabled() && W <= kRowMaxW && C * H * W < (int64_t(1) << 31) && B * H < (int64_t(1) << 31);
}
}  // namespace

extern "C" {

int ofd_fw_abi_version(void) { return OFD_FW_ABI_VERSION; }

#ifndef OFD_BUILD_ID
#define OFD_BUILD_ID "unknown"
#endif
const char *ofd_fw_build_id(void) { return OFD_BUILD_ID; }

int ofd_fw_set_profile_events(void *start_event, void *stop_event) {
    g_prof_start = static_cast<hipEvent_t>(start_event);
    g_prof_stop = static_cast<hipEvent_t>(stop_event);
    return OFD_FW_OK;
}

int ofd_fw_set_profile_bin_event(void *bin_start_event) {
    g_prof_bin = static_cast<hipEvent_t>(bin_start_event);
    return OFD_FW_OK;
}

int ofd_fw_set_disparity_rows(int on) {
    const int prev = disp_row_enabled() ? 1 : 0;
    if (on == 0 || on == 1) g_disp_rows = on;
    return prev;
}

int ofd_fw_set_persist_min(int tiles_per_slot) {
    const int prev = int(persist_min());
    if (tiles_per_slot >= 0) g_persist_min = tiles_per_slot;
    return prev;
}

int ofd_fw_set_short_tiles(int on) {
    const int prev = short_tiles_enabled() ? 1 : 0;
    if (on == 0 || on == 1) g_short_tiles = on;
    return prev;
}

int ofd_fw_set_pack(int on) {
    const int prev = pack_enabled() ? 1 : 0;
    if (on == 0 || on == 1) g_pack = on;
    return prev;
}

int ofd_fw_set_engine(int engine) {
    const int prev = int(engine_mode());
    if (engine == OFD_FW_ENGINE_TILE || engine == OFD_FW_ENGINE_ATOMIC || engine == OFD_FW_ENGINE_TILE_SPLIT)
        g_engine = engine;
    return prev;
}

const char *ofd_fw_strerror(int code) {
    switch (code) {
        case OFD_FW_OK: return "success";
        case OFD_FW_EINVAL: return "invalid argument (null pointer or negative dimension)";
        case OFD_FW_ETOOBIG: return "H*W must be < 2^31";
        case OFD_FW_EWORKSPACE: return "workspace missing, misaligned or smaller than one image's slab";
        case OFD_FW_EALIGN: return "pointer misaligned for its dtype";
        default: return code > 0 ? hipGetErrorString(hipError_t(code)) : "unknown error";
    }
}

size_t ofd_fw_workspace_bytes(int64_t B, int64_t H, int64_t W, int f64) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    if (f64) return size_t(B < 8 ? B : 8) * size_t(H) * size_t(W) * (sizeof(unsigned long long) + sizeof(unsigned int));
    const size_t per_image = per_image_bytes(H, W);
    // chunk = the images whose slabs and re-read planes stay cache-resident
    // between a chunk's BIN and TILE roles; OFD_FW_CHUNK_IMAGES overrides.
    size_t g = kDefaultChunkPixels / (size_t(H) * size_t(W));
    if (const char *e = getenv("OFD_FW_CHUNK_IMAGES")) g = size_t(atoi(e));
    if (g < 1) g = 1;
    if (g > size_t(B)) g = size_t(B);
    return g * per_image;
}

int ofd_fw_workspace_init(void *workspace, size_t bytes, void *stream) {
    if (!workspace && bytes) return OFD_FW_EINVAL;
    if (!bytes) return OFD_FW_OK;
    const hipError_t e = hipMemsetAsync(workspace, 0xFF, bytes, static_cast<hipStream_t>(stream));
    if (e == hipSuccess) mark_clean(workspace);
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

int ofd_fw_forward_warping_f32(const float *obj, const float *safe_y, const float *safe_x,
                               const float *depth, float *output, float *valid, float *collision,
                               int64_t B, int64_t C, int64_t H, int64_t W, void *workspace,
                               size_t workspace_bytes, void *stream) {
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!safe_y || !safe_x || !depth || !valid || !collision || (C > 0 && (!obj || !output))))
        return OFD_FW_EINVAL;
    SafeF32 co{safe_y, safe_x, H * W};
    return run_f32(co, obj, depth, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream));
}

int ofd_fw_forward_warp_flow_f32(const float *obj, const float *flow, const float *depth, float *output,
                                 float *valid, float *collision, int64_t B, int64_t C, int64_t H, int64_t W,
                                 void *workspace, size_t workspace_bytes, void *stream) {
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!flow || !depth || !valid || !collision || (C > 0 && (!obj || !output))))
        return OFD_FW_EINVAL;
    FlowCoords<float> co{flow, H * W};
    return run_f32(co, obj, depth, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream));
}

int ofd_fw_forward_warp_flow_f64flow(const float *obj, const double *flow, const float *depth, float *output,
                                     float *valid, float *collision, int64_t B, int64_t C, int64_t H,
                                     int64_t W, void *workspace, size_t workspace_bytes, void *stream) {
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!flow || !depth || !valid || !collision || (C > 0 && (!obj || !output))))
        return OFD_FW_EINVAL;
    if (!aligned(flow, 8)) return OFD_FW_EALIGN;
    FlowCoords<double> co{flow, H * W};
    return run_f32(co, obj, depth, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream));
}

int ofd_fw_forward_warp_flow_bf16(const uint16_t *obj, const float *flow, const float *depth, uint16_t *output,
                                  float *valid, float *collision, int64_t B, int64_t C, int64_t H, int64_t W,
                                  void *workspace, size_t workspace_bytes, void *stream) {
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!flow || !depth || !valid || !collision || (C > 0 && (!obj || !output))))
        return OFD_FW_EINVAL;
    if ((C > 0 && (!aligned(obj, 2) || !aligned(output, 2)))) return OFD_FW_EALIGN;
    FlowCoords<float> co{flow, H * W};
    return run_f32<FlowCoords<float>, unsigned short>(
        co, reinterpret_cast<const unsigned short *>(obj), depth, reinterpret_cast<unsigned short *>(output), valid,
        collision, B, C, H, W, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
}

int ofd_fw_warp_disparity_f32(const float *obj, int64_t Cobj, const float *depth, const float *s, float *output,
                              float *valid, float *collision, int64_t B, int64_t H, int64_t W, void *workspace,
                              size_t workspace_bytes, void *stream) {
    if (Cobj < 0) return OFD_FW_EINVAL;
    const int64_t C = Cobj + 3;
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!depth || !s || !valid || !collision || !output || (Cobj > 0 && !obj)))
        return OFD_FW_EINVAL;
    DisparityCoords<float> co{depth, s, H * W};
    if (B * H * W > 0 && rows_ok(B, C, H, W))
        return warp_disparity_rows(co, obj, Cobj, output, valid, collision, B, H, W, static_cast<hipStream_t>(stream));
    return run_f32(co, obj, nullptr, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream), int(Cobj < 3 ? Cobj : 3));
}

int ofd_fw_warp_disparity_f64depth(const float *obj, int64_t Cobj, const double *depth, const float *s,
                                   float *output, float *valid, float *collision, int64_t B, int64_t H, int64_t W,
                                   void *workspace, size_t workspace_bytes, void *stream) {
    if (Cobj < 0) return OFD_FW_EINVAL;
    const int64_t C = Cobj + 3;
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!depth || !s || !valid || !collision || !output || (Cobj > 0 && !obj)))
        return OFD_FW_EINVAL;
    if (!aligned(depth, 8)) return OFD_FW_EALIGN;
    DisparityCoords<double> co{depth, s, H * W};
    if (B * H * W > 0 && rows_ok(B, C, H, W))
        return warp_disparity_rows(co, obj, Cobj, output, valid, collision, B, H, W, static_cast<hipStream_t>(stream));
    return run_f32(co, obj, nullptr, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream), int(Cobj < 3 ? Cobj : 3));
}

}  // extern "C"

namespace {
template <typename D>
int ego_flow(const D *depth, const float *P, const float *inv_K, float *flow, int64_t B, int64_t H, int64_t W,
             void *stream) {
    if (int rc = check_dims(B, 1, H, W)) return rc;
    if (B * H * W == 0) return OFD_FW_OK;
    if (!depth || !P || !inv_K || !flow) return OFD_FW_EINVAL;
    if (!aligned(depth, sizeof(D)) || !aligned(P, 4) || !aligned(flow, 4)) return OFD_FW_EALIGN;
    EgoCoords<D> co{depth, P, {}, H * W, int(H), int(W)};
    for (int k = 0; k < 9; ++k) co.cam.ik[k] = inv_K[k];
    const int64_t quads = B * H * ((W + 3) / 4);
    hipLaunchKernelGGL((ego_flow_kernel<D>), dim3(grid_for(quads)), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       co, flow, B);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

// SpecialFlow._rotate's flows (preprocess.py:31-41, :63-77): p1 = (p0 - c0)
// @ R + c0, flow = p1 - p0, for R = rotate and reverse_rotate.  The 2-term
// product is evaluated the way a GEMM accumulates it -- the k = 0 product
// rounded, then a fused multiply-add of the k = 1 term -- which is the rounding
// of the reference's matmul (checked bit for bit against its CPU run,
// tests/golden/ppa_fill_large.npz); the library is built with contraction off,
// so every other operation rounds on its own.  params [B][10] float32:
// c0x, c0y, R (r00, r01, r10, r11), reverse R (q00, q01, q10, q11).
__global__ __launch_bounds__(kBlock) void rotation_flow_kernel(const float *__restrict__ params, float *__restrict__ flow,
                                                              float *__restrict__ back, int H, int W, int64_t n) {
    const int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (q >= n) return;
    const int64_t HW = int64_t(H) * W;
    const int64_t b = q / HW;
    const int p = int(q - b * HW);
    const int j = p / W, i = p - j * W;
    const float *pr = params + b * 10;
    const float x = float(i), y = float(j);
    const float dx = x - pr[0], dy = y - pr[1];
    float *fo = flow + b * 2 * HW + p, *bo = back + b * 2 * HW + p;
    {
        const float px = fmaf(dy, pr[4], dx * pr[2]), py = fmaf(dy, pr[5], dx * pr[3]);
        fo[0] = (px + pr[0]) - x;
        fo[HW] = (py + pr[1]) - y;
    }
    {
        const float px = fmaf(dy, pr[8], dx * pr[6]), py = fmaf(dy, pr[9], dx * pr[7]);
        bo[0] = (px + pr[0]) - x;
        bo[HW] = (py + pr[1]) - y;
    }
}

int rotation_flow(const float *params, float *flow, float *back, int64_t B, int64_t H, int64_t W, void *stream) {
    if (int rc = check_dims(B, 2, H, W)) return rc;
    if (B * H * W == 0) return OFD_FW_OK;
    if (!params || !flow || !back) return OFD_FW_EINVAL;
    if (!aligned(params, 4) || !aligned(flow, 4) || !aligned(back, 4)) return OFD_FW_EALIGN;
    const int64_t n = B * H * W;
    hipLaunchKernelGGL(rotation_flow_kernel, dim3(grid_for(n)), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       params, flow, back, int(H), int(W), n);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

template <typename D>
int warp_ego(const float *obj, int64_t Cobj, const D *depth, const float *P, const float *inv_K, float *output,
             float *valid, float *collision, int64_t B, int64_t H, int64_t W, void *workspace, size_t workspace_bytes,
             void *stream) {
    if (Cobj < 0) return OFD_FW_EINVAL;
    const int64_t C = Cobj + 3;
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!depth || !P || !inv_K || !valid || !collision || !output || (Cobj > 0 && !obj)))
        return OFD_FW_EINVAL;
    if (!aligned(depth, sizeof(D))) return OFD_FW_EALIGN;
    EgoCoords<D> co{depth, P, {}, H * W, int(H), int(W)};
    if (inv_K)
        for (int k = 0; k < 9; ++k) co.cam.ik[k] = inv_K[k];
    return run_f32(co, obj, nullptr, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream), int(Cobj < 3 ? Cobj : 3));
}
}  // namespace

extern "C" {

int ofd_fw_warp_flow_cat(const float *obj, int64_t Cobj, const void *flow, int flow_f64, const void *depth,
                         int depth_f64, float *output, float *valid, float *collision, int64_t B, int64_t H,
                         int64_t W, void *workspace, size_t workspace_bytes, void *stream) {
    if (Cobj < 0) return OFD_FW_EINVAL;
    const int64_t C = Cobj + 3;
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!flow || !depth || !valid || !collision || !output || (Cobj > 0 && !obj)))
        return OFD_FW_EINVAL;
    if (!aligned(flow, flow_f64 ? 8 : 4) || !aligned(depth, depth_f64 ? 8 : 4)) return OFD_FW_EALIGN;
    const int gen_at = int(Cobj < 3 ? Cobj : 3);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t HW = H * W;
#define OFD_FLOW_CAT(F, D)                                                                                   \
    run_f32(FlowCatCoords<F, D>{static_cast<const F *>(flow), static_cast<const D *>(depth), HW}, obj, nullptr, \
            output, valid, collision, B, C, H, W, workspace, workspace_bytes, st, gen_at)
    if (flow_f64) return depth_f64 ? OFD_FLOW_CAT(double, double) : OFD_FLOW_CAT(double, float);
    return depth_f64 ? OFD_FLOW_CAT(float, double) : OFD_FLOW_CAT(float, float);
#undef OFD_FLOW_CAT
}

int ofd_fw_ego_flow_f32(const float *depth, const float *P, const float *inv_K, float *flow, int64_t B, int64_t H,
                        int64_t W, void *stream) {
    return ego_flow(depth, P, inv_K, flow, B, H, W, stream);
}

int ofd_fw_ego_flow_f64depth(const double *depth, const float *P, const float *inv_K, float *flow, int64_t B,
                             int64_t H, int64_t W, void *stream) {
    return ego_flow(depth, P, inv_K, flow, B, H, W, stream);
}

int ofd_fw_rotation_flow_f32(const float *params, float *flow, float *back_flow, int64_t B, int64_t H, int64_t W,
                             void *stream) {
    return rotation_flow(params, flow, back_flow, B, H, W, stream);
}

int ofd_fw_warp_ego_f32(const float *obj, int64_t Cobj, const float *depth, const float *P, const float *inv_K,
                        float *output, float *valid, float *collision, int64_t B, int64_t H, int64_t W,
                        void *workspace, size_t workspace_bytes, void *stream) {
    return warp_ego(obj, Cobj, depth, P, inv_K, output, valid, collision, B, H, W, workspace, workspace_bytes, stream);
}

int ofd_fw_warp_ego_f64depth(const float *obj, int64_t Cobj, const double *depth, const float *P,
                             const float *inv_K, float *output, float *valid, float *collision, int64_t B, int64_t H,
                             int64_t W, void *workspace, size_t workspace_bytes, void *stream) {
    return warp_ego(obj, Cobj, depth, P, inv_K, output, valid, collision, B, H, W, workspace, workspace_bytes, stream);
}

int ofd_fw_forward_warping_f64(const double *obj, const double *safe_y, const double *safe_x,
                               const double *depth, double *output, double *valid, double *collision,
                               int64_t B, int64_t C, int64_t H, int64_t W, void *workspace,
                               size_t workspace_bytes, void *stream) {
    if (int rc = check_dims(B, C, H, W)) return rc;
    const int64_t HW = H * W;
    if (B == 0 || HW == 0) return OFD_FW_OK;
    if (!safe_y || !safe_x || !depth || !valid || !collision || (C > 0 && (!obj || !output)))
        return OFD_FW_EINVAL;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (C == 0) return zero_masks(valid, collision, size_t(B * HW) * sizeof(double), st);
    if (!workspace || !aligned(workspace, 16)) return OFD_FW_EWORKSPACE;
    const size_t per_image = size_t(HW) * (sizeof(unsigned long long) + sizeof(unsigned int));
    const int64_t G = chunk_images(B, HW, per_image, workspace_bytes);
    if (G < 1) return OFD_FW_EWORKSPACE;
    auto *zkeys = static_cast<unsigned long long *>(workspace);
    auto *idx = reinterpret_cast<unsigned int *>(zkeys + G * HW);
    // The f32 engines keep scratch records in parts of the shared workspace,
    // so the float64 op (a rare path) initialises the region it uses.
    {
        const hipError_t e = hipMemsetAsync(workspace, 0xFF, size_t(G) * per_image, st);
        if (e != hipSuccess) return int(e);
    }
    for (int64_t b0 = 0; b0 < B; b0 += G) {
        const int64_t nb = (B - b0) < G ? (B - b0) : G;
        const int64_t px = nb * HW;
        hipLaunchKernelGGL(splat_f64_depth_kernel, dim3(grid_for(px)), dim3(kBlock), 0, st,
                           safe_y, safe_x, depth, zkeys, int(H), int(W), HW, b0, px);
        hipLaunchKernelGGL(splat_f64_index_kernel, dim3(grid_for(px)), dim3(kBlock), 0, st,
                           safe_y, safe_x, depth, zkeys, idx, int(H), int(W), HW, b0, px);
        hipLaunchKernelGGL(resolve_f64_kernel, dim3(grid_for(px)), dim3(kBlock), 0, st,
                           obj, zkeys, idx, output, valid, collision, int(C), HW, b0, px);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

}  // extern "C"
