// ofd_fw.hip -- MI355X (gfx950) forward-warp engine: z-buffered splat + resolve.
//
// Replaces the reference's single-workgroup serial kernel
// (alt_cuda/fw_cuda_kernel.cu:9-49, grid <<<B, C>>>, one thread walks all H*W
// sources of one (image, channel)) with a data-parallel two-phase design:
//
//   splat   : one lane per source pixel.  Computes the target pixel (from the
//             flow, fw.py:27-42 fused in, or from given safe coordinates) and
//             folds a 64-bit key  (orderable(depth) << 32) | raster_index  into
//             the target's slot with one native 64-bit atomic min
//             (global_atomic_umin_x2).  Sources with depth >= 1000 / NaN mark
//             the slot "touched, no winner" (KEY_NOWIN) so valid/collision are
//             reproduced.  The lexicographic (depth, raster index) minimum is
//             exactly the winner of the reference's raster loop with its strict
//             `<` (ties keep the earliest source): SURVEY.md 0.1 item 1.
//   resolve : one lane per target pixel.  Reads the key, gathers the winner's C
//             channel values, writes output / valid / collision exactly once
//             (16-byte stores), and resets the key slot to KEY_UNTOUCHED so the
//             workspace needs no clearing pass before the next call.
//
// Images are processed in chunks whose key slab fits the workspace the caller
// passes (ofd_fw_workspace_bytes suggests a slab that stays resident in the
// 256 MiB Infinity Cache, so the key traffic does not reach HBM).
//
// Everything here is plain HIP for gfx950; no CUDA compatibility layer.

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "ofd_fw.h"

namespace {

constexpr int kBlock = 256;
constexpr unsigned long long KEY_UNTOUCHED = ~0ull;                 // no source landed
constexpr unsigned long long KEY_NOWIN = 0xFFFFFFFF00000000ull;     // landed, none < 1000
// f64 op: depth keys are full 64-bit orderable doubles, index kept aside
constexpr unsigned long long ZKEY_UNTOUCHED = ~0ull;
constexpr unsigned long long ZKEY_NOWIN = ~0ull - 1ull;
constexpr unsigned int IDX_NONE = ~0u;

// Default key slab: 8 images of 768x1024 (48 MiB) -- resident in the MALL
// together with the chunk's streamed planes.
constexpr size_t kDefaultSlabBytes = size_t(48) << 20;

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

// ---------------------------------------------------------------- target maps
// Op level: coordinates as given to fw_cuda.forward_warping.  The reference
// indexes its accessor with them, i.e. converts float -> int32 by truncation
// (fw_cuda_kernel.cu:31-35); an out-of-range index is UB there and a dropped
// source here.
template <typename T>
__device__ __forceinline__ int target_safe(T x, T y, int H, int W) {
    if (!(x > T(-1)) || !(x < T(W)) || !(y > T(-1)) || !(y < T(H))) return -1;
    return int(y) * W + int(x);
}

// FW level: fw.py:27-42.  p1 = p0 + flow in the flow's dtype (p0 is the
// float32 meshgrid, exact for any pixel index < 2^24), clamp to [0, W-1] x
// [0, H-1], truncate through int64.  NaN survives torch.clamp and is dropped.
template <typename F>
__device__ __forceinline__ int target_flow(int i, int j, F fx, F fy, int H, int W) {
    F px = F(i) + fx;
    F py = F(j) + fy;
    if (px != px || py != py) return -1;
    px = px < F(0) ? F(0) : (px > F(W - 1) ? F(W - 1) : px);
    py = py < F(0) ? F(0) : (py > F(H - 1) ? F(H - 1) : py);
    return int(py) * W + int(px);
}

// Coordinate sources.  load<VEC>() fetches the raw per-source values of VEC
// consecutive sources (vectorised when VEC == 4), target() maps one of them.
struct SafeF32 {  // fw_cuda.forward_warping inputs: safe_y, safe_x [B,1,H,W]
    using V = float;
    const float *sy, *sx;
    int64_t HW;
    template <int VEC>
    __device__ __forceinline__ void load(int64_t g, int64_t, V (&x)[VEC], V (&y)[VEC]) const {
        if constexpr (VEC == 4) {
            const float4 a = *reinterpret_cast<const float4 *>(sx + g);
            const float4 c = *reinterpret_cast<const float4 *>(sy + g);
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
            y[0] = c.x; y[1] = c.y; y[2] = c.z; y[3] = c.w;
        } else {
#pragma unroll
            for (int k = 0; k < VEC; ++k) { x[k] = sx[g + k]; y[k] = sy[g + k]; }
        }
    }
    __device__ __forceinline__ int target(int, int, V x, V y, int H, int W) const {
        return target_safe<float>(x, y, H, W);
    }
};

template <typename F>
struct FlowCoords {  // FW.forward input: flow [B,2,H,W], ch0 = x, ch1 = y
    using V = F;
    const F *flow;
    int64_t HW;
    template <int VEC>
    __device__ __forceinline__ void load(int64_t, int64_t bp, V (&x)[VEC], V (&y)[VEC]) const {
        // bp = b*2*HW + p: the x plane sample; the y plane is HW further on
        const F *fx = flow + bp;
        const F *fy = fx + HW;
        if constexpr (VEC == 4 && sizeof(F) == 4) {
            const float4 a = *reinterpret_cast<const float4 *>(fx);
            const float4 c = *reinterpret_cast<const float4 *>(fy);
            x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
            y[0] = c.x; y[1] = c.y; y[2] = c.z; y[3] = c.w;
        } else if constexpr (VEC == 4 && sizeof(F) == 8) {
            const double2 a0 = *reinterpret_cast<const double2 *>(fx);
            const double2 a1 = *reinterpret_cast<const double2 *>(fx + 2);
            const double2 c0 = *reinterpret_cast<const double2 *>(fy);
            const double2 c1 = *reinterpret_cast<const double2 *>(fy + 2);
            x[0] = a0.x; x[1] = a0.y; x[2] = a1.x; x[3] = a1.y;
            y[0] = c0.x; y[1] = c0.y; y[2] = c1.x; y[3] = c1.y;
        } else {
#pragma unroll
            for (int k = 0; k < VEC; ++k) { x[k] = fx[k]; y[k] = fy[k]; }
        }
    }
    __device__ __forceinline__ int target(int i, int j, V x, V y, int H, int W) const {
        return target_flow<F>(i, j, x, y, H, W);
    }
};

// ---------------------------------------------------------------- splat (f32 depth)
// One thread handles VEC consecutive sources of one image (HW % VEC == 0).
// Runs of equal targets inside the thread (border clamping, flat regions)
// are merged before touching memory.
template <int VEC, typename Coords>
__global__ __launch_bounds__(kBlock) void splat_f32_kernel(
        Coords co, const float *__restrict__ depth, unsigned long long *__restrict__ keys,
        int H, int W, int64_t HW, int64_t b0, int64_t chunk_px) {
    const int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) * VEC;  // chunk-local
    if (q >= chunk_px) return;
    const int64_t bl = q / HW;
    const int64_t p = q - bl * HW;  // pixel in image
    const int64_t b = b0 + bl;
    const int64_t g = b * HW + p;   // global plane index

    float d[VEC];
    if constexpr (VEC == 4) {
        const float4 v = *reinterpret_cast<const float4 *>(depth + g);
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) d[k] = depth[g + k];
    }
    typename Coords::V cx[VEC], cy[VEC];
    co.template load<VEC>(g, b * 2 * HW + p, cx, cy);
    int j = int(p / W);
    int i = int(p - int64_t(j) * W);
    unsigned long long *kb = keys + bl * HW;

    int run_t = -1;
    unsigned long long run_key = KEY_UNTOUCHED;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const int t = co.target(i, j, cx[k], cy[k], H, W);
        const unsigned long long key = make_key(d[k], (unsigned int)(p + k));
        if (t != run_t) {
            if (run_t >= 0) atomicMin(kb + run_t, run_key);
            run_t = t;
            run_key = key;
        } else if (key < run_key) {
            run_key = key;
        }
        if (++i == W) { i = 0; ++j; }
    }
    if (run_t >= 0) atomicMin(kb + run_t, run_key);
}

// ---------------------------------------------------------------- resolve (f32)
template <int VEC>
__global__ __launch_bounds__(kBlock) void resolve_f32_kernel(
        const float *__restrict__ obj, unsigned long long *__restrict__ keys,
        float *__restrict__ out, float *__restrict__ valid, float *__restrict__ coll,
        int C, int64_t HW, int64_t b0, int64_t chunk_px) {
    const int64_t q = (int64_t(blockIdx.x) * kBlock + threadIdx.x) * VEC;
    if (q >= chunk_px) return;
    const int64_t bl = q / HW;
    const int64_t p = q - bl * HW;
    const int64_t b = b0 + bl;

    unsigned long long key[VEC];
    if constexpr (VEC == 4) {
        const ulonglong2 k01 = *reinterpret_cast<const ulonglong2 *>(keys + q);
        const ulonglong2 k23 = *reinterpret_cast<const ulonglong2 *>(keys + q + 2);
        key[0] = k01.x; key[1] = k01.y; key[2] = k23.x; key[3] = k23.y;
        const ulonglong2 ones = {KEY_UNTOUCHED, KEY_UNTOUCHED};
        *reinterpret_cast<ulonglong2 *>(keys + q) = ones;
        *reinterpret_cast<ulonglong2 *>(keys + q + 2) = ones;
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) { key[k] = keys[q + k]; keys[q + k] = KEY_UNTOUCHED; }
    }

    int src[VEC];
    float vv[VEC], cc[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        const bool touched = key[k] != KEY_UNTOUCHED;
        const bool nowin = key[k] == KEY_NOWIN;
        vv[k] = touched ? 1.f : 0.f;
        cc[k] = nowin ? 1.f : 0.f;
        src[k] = (touched && !nowin) ? int(key[k] & 0xFFFFFFFFull) : -1;
    }

    const float *ob = obj + b * C * HW;
    float *oo = out + b * C * HW + p;
    for (int c = 0; c < C; ++c) {
        const float *plane = ob + int64_t(c) * HW;
        float o[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) o[k] = src[k] >= 0 ? plane[src[k]] : 0.f;
        if constexpr (VEC == 4) {
            *reinterpret_cast<float4 *>(oo + int64_t(c) * HW) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int k = 0; k < VEC; ++k) oo[int64_t(c) * HW + k] = o[k];
        }
    }
    if constexpr (VEC == 4) {
        *reinterpret_cast<float4 *>(valid + b * HW + p) = make_float4(vv[0], vv[1], vv[2], vv[3]);
        *reinterpret_cast<float4 *>(coll + b * HW + p) = make_float4(cc[0], cc[1], cc[2], cc[3]);
    } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) { valid[b * HW + p + k] = vv[k]; coll[b * HW + p + k] = cc[k]; }
    }
}

// ---------------------------------------------------------------- f64 op
// Exact double depths do not fit a 32-bit key half, so the double path keys
// on the full 64-bit orderable depth first, then resolves ties by a 32-bit
// index min among the sources that hold the minimum depth.
__global__ __launch_bounds__(kBlock) void splat_f64_depth_kernel(
        const double *__restrict__ sy, const double *__restrict__ sx, const double *__restrict__ depth,
        unsigned long long *__restrict__ zkeys, int H, int W, int64_t HW, int64_t b0, int64_t chunk_px) {
    const int64_t q = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (q >= chunk_px) return;
    const int64_t g = b0 * HW + q;
    const int t = target_safe<double>(sx[g], sy[g], H, W);
    if (t < 0) return;
    const double d = depth[g];
    const unsigned long long z = (d < 1000.0) ? orderable64(d) : ZKEY_NOWIN;
    atomicMin(zkeys + (q / HW) * HW + t, z);
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
    const int t = target_safe<double>(sx[g], sy[g], H, W);
    if (t < 0) return;
    const int64_t slot = (q / HW) * HW + t;
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
inline unsigned grid_for(int64_t work_items) {
    return unsigned((work_items + kBlock - 1) / kBlock);
}

inline bool aligned(const void *p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

int check_dims(int64_t B, int64_t C, int64_t H, int64_t W) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return OFD_FW_EINVAL;
    if (H * W >= (int64_t(1) << 31)) return OFD_FW_ETOOBIG;
    return OFD_FW_OK;
}

// images per chunk for a workspace of `bytes` (per-image slab `per_image`)
int64_t chunk_images(int64_t B, int64_t per_image, size_t bytes) {
    int64_t g = int64_t(bytes / size_t(per_image));
    return g < B ? g : B;
}

template <typename Coords>
int run_f32(Coords co, bool coords_vec_ok, const float *obj, const float *depth, float *out, float *valid,
            float *coll, int64_t B, int64_t C, int64_t H, int64_t W, void *ws, size_t ws_bytes,
            hipStream_t st) {
    const int64_t HW = H * W;
    if (B == 0 || HW == 0) return OFD_FW_OK;
    const int64_t per_image = HW * int64_t(sizeof(unsigned long long));
    if (!ws || !aligned(ws, 16)) return OFD_FW_EWORKSPACE;
    const int64_t G = chunk_images(B, per_image, ws_bytes);
    if (G < 1) return OFD_FW_EWORKSPACE;
    auto *keys = static_cast<unsigned long long *>(ws);
    const bool vec = (HW % 4 == 0) && coords_vec_ok && aligned(depth, 16) && aligned(obj, 4) &&
                     aligned(out, 16) && aligned(valid, 16) && aligned(coll, 16);
    for (int64_t b0 = 0; b0 < B; b0 += G) {
        const int64_t nb = (B - b0) < G ? (B - b0) : G;
        const int64_t px = nb * HW;
        if (vec) {
            hipLaunchKernelGGL((splat_f32_kernel<4, Coords>), dim3(grid_for(px / 4)), dim3(kBlock), 0, st,
                               co, depth, keys, int(H), int(W), HW, b0, px);
            hipLaunchKernelGGL((resolve_f32_kernel<4>), dim3(grid_for(px / 4)), dim3(kBlock), 0, st,
                               obj, keys, out, valid, coll, int(C), HW, b0, px);
        } else {
            hipLaunchKernelGGL((splat_f32_kernel<1, Coords>), dim3(grid_for(px)), dim3(kBlock), 0, st,
                               co, depth, keys, int(H), int(W), HW, b0, px);
            hipLaunchKernelGGL((resolve_f32_kernel<1>), dim3(grid_for(px)), dim3(kBlock), 0, st,
                               obj, keys, out, valid, coll, int(C), HW, b0, px);
        }
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

}  // namespace

extern "C" {

int ofd_fw_abi_version(void) { return OFD_FW_ABI_VERSION; }

const char *ofd_fw_strerror(int code) {
    switch (code) {
        case OFD_FW_OK: return "success";
        case OFD_FW_EINVAL: return "invalid argument (null pointer or negative dimension)";
        case OFD_FW_ETOOBIG: return "H*W must be < 2^31";
        case OFD_FW_EWORKSPACE: return "workspace missing, misaligned or smaller than one image's key slab";
        case OFD_FW_EALIGN: return "pointer misaligned for its dtype";
        default: return code > 0 ? hipGetErrorString(hipError_t(code)) : "unknown error";
    }
}

size_t ofd_fw_workspace_bytes(int64_t B, int64_t H, int64_t W, int f64) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    const size_t per_image = size_t(H) * size_t(W) * (f64 ? (sizeof(unsigned long long) + sizeof(unsigned int))
                                                           : sizeof(unsigned long long));
    size_t g = kDefaultSlabBytes / per_image;
    if (g < 1) g = 1;
    if (g > size_t(B)) g = size_t(B);
    return g * per_image;
}

int ofd_fw_workspace_init(void *workspace, size_t bytes, void *stream) {
    if (!workspace && bytes) return OFD_FW_EINVAL;
    if (!bytes) return OFD_FW_OK;
    const hipError_t e = hipMemsetAsync(workspace, 0xFF, bytes, static_cast<hipStream_t>(stream));
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
    const bool vec_ok = aligned(safe_y, 16) && aligned(safe_x, 16);
    return run_f32(co, vec_ok, obj, depth, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream));
}

int ofd_fw_forward_warp_flow_f32(const float *obj, const float *flow, const float *depth, float *output,
                                 float *valid, float *collision, int64_t B, int64_t C, int64_t H, int64_t W,
                                 void *workspace, size_t workspace_bytes, void *stream) {
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!flow || !depth || !valid || !collision || (C > 0 && (!obj || !output))))
        return OFD_FW_EINVAL;
    FlowCoords<float> co{flow, H * W};
    return run_f32(co, aligned(flow, 16), obj, depth, output, valid, collision, B, C, H, W, workspace,
                   workspace_bytes, static_cast<hipStream_t>(stream));
}

int ofd_fw_forward_warp_flow_f64flow(const float *obj, const double *flow, const float *depth, float *output,
                                     float *valid, float *collision, int64_t B, int64_t C, int64_t H,
                                     int64_t W, void *workspace, size_t workspace_bytes, void *stream) {
    if (int rc = check_dims(B, C, H, W)) return rc;
    if (B * H * W > 0 && (!flow || !depth || !valid || !collision || (C > 0 && (!obj || !output))))
        return OFD_FW_EINVAL;
    if (!aligned(flow, 8)) return OFD_FW_EALIGN;
    FlowCoords<double> co{flow, H * W};
    return run_f32(co, aligned(flow, 16), obj, depth, output, valid, collision, B, C, H, W, workspace, workspace_bytes,
                   static_cast<hipStream_t>(stream));
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
    if (!workspace || !aligned(workspace, 16)) return OFD_FW_EWORKSPACE;
    const int64_t per_image = HW * int64_t(sizeof(unsigned long long) + sizeof(unsigned int));
    const int64_t G = chunk_images(B, per_image, workspace_bytes);
    if (G < 1) return OFD_FW_EWORKSPACE;
    auto *zkeys = static_cast<unsigned long long *>(workspace);
    auto *idx = reinterpret_cast<unsigned int *>(zkeys + G * HW);
    hipStream_t st = static_cast<hipStream_t>(stream);
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
