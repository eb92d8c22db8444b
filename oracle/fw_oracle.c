/*
 * oracle/fw_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference forward-warp (z-buffered splat).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the CPU baseline.  The product path
 * (opticalflowfromdepth_amd) never links or calls it.
 *
 * What it restates (paths relative to the reference checkout):
 *   - oracle_forward_warping_*   : alt_cuda/fw_cuda_kernel.cu:52-83 (host: zeros
 *     output, dlut = 1000, zero valid/collision) and :28-47 (the serial raster
 *     loop that one CUDA thread runs per (b, c)).  Written as that literal loop:
 *     strict `<` against the per-channel dlut, channel 0 writes valid/collision.
 *   - oracle_fw_flow_*           : alt_cuda/fw.py:27-43 (p0 meshgrid + flow in the
 *     flow's dtype, clamp to [0,W-1]/[0,H-1], truncate through int64, back to
 *     float32) followed by the loop above.
 *
 * Behaviour the reference leaves undefined, defined here identically to the
 * HIP product path (documented in DESIGN.md "Defined behaviour"):
 *   - a coordinate that is NaN, or whose truncation falls outside the image,
 *     drops the source: it is never written and does not mark valid
 *     (reference: out-of-bounds accessor write, fw_cuda_kernel.cu:31-45).
 *
 * Parallelism: OpenMP over (b, c) planes, exactly the reference's
 * grid <<<B, C>>> decomposition (fw_cuda_kernel.cu:67-68); each plane is a
 * serial loop.  `nthreads` <= 0 means "OpenMP default".
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* float -> int index the way the reference's PackedTensorAccessor32 indexing
 * converts it (implicit conversion to int32 = truncation toward zero).
 * Returns -1 when the reference would index out of bounds (UB there). */
static inline long idx_f(double v, long n) {
    if (!(v > -1.0) || !(v < (double)n)) return -1; /* NaN fails both */
    return (long)v;                                 /* trunc toward zero */
}

#define DEFINE_LOOP(NAME, T)                                                         \
static void NAME(const T *obj, const T *sy, const T *sx, const T *depth, T *out,   \
                 T *valid, T *coll, long B, long C, long H, long W, int nthreads) { \
    const long HW = H * W;                                                          \
    memset(out, 0, sizeof(T) * (size_t)(B * C * HW));       /* zeros_like(obj)  */  \
    memset(valid, 0, sizeof(T) * (size_t)(B * HW));         /* zeros_like(depth)*/  \
    memset(coll, 0, sizeof(T) * (size_t)(B * HW));                                  \
    long plane;                                                                     \
    (void)nthreads;                                                                 \
    _Pragma("omp parallel for schedule(dynamic,1) num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())") \
    for (plane = 0; plane < B * C; ++plane) {                                       \
        const long b = plane / C, c = plane % C;                                    \
        T *dlut = (T *)malloc(sizeof(T) * (size_t)HW);      /* ones_like*1000   */  \
        for (long k = 0; k < HW; ++k) dlut[k] = (T)1000.;                           \
        const T *o = obj + (b * C + c) * HW;                                        \
        T *oo = out + (b * C + c) * HW;                                             \
        const T *py = sy + b * HW, *px = sx + b * HW, *pd = depth + b * HW;         \
        T *pv = valid + b * HW, *pc = coll + b * HW;                                \
        for (long j = 0; j < H; ++j) {                                              \
            for (long i = 0; i < W; ++i) {                                          \
                const long s = j * W + i;                                           \
                const long x = idx_f((double)px[s], W);                             \
                const long y = idx_f((double)py[s], H);                             \
                if (x < 0 || y < 0) continue;                                       \
                const long t = y * W + x;                                           \
                if (pd[s] < dlut[t]) {                                              \
                    oo[t] = o[s];                                                   \
                    dlut[t] = pd[s];                                                \
                }                                                                   \
                if (c == 0) {                                                       \
                    pv[t] = 1;                                                      \
                    if (dlut[t] != (T)1000.) pc[t] = 0; else pc[t] = 1;             \
                }                                                                   \
            }                                                                       \
        }                                                                           \
        free(dlut);                                                                 \
    }                                                                               \
}

#ifndef _OPENMP
static int omp_get_max_threads(void) { return 1; }
#endif

DEFINE_LOOP(loop_f32, float)
DEFINE_LOOP(loop_f64, double)

int oracle_forward_warping_f32(const float *obj, const float *safe_y, const float *safe_x,
                               const float *depth, float *output, float *valid,
                               float *collision, long B, long C, long H, long W,
                               int nthreads) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return -1;
    loop_f32(obj, safe_y, safe_x, depth, output, valid, collision, B, C, H, W, nthreads);
    return 0;
}

int oracle_forward_warping_f64(const double *obj, const double *safe_y, const double *safe_x,
                               const double *depth, double *output, double *valid,
                               double *collision, long B, long C, long H, long W,
                               int nthreads) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return -1;
    loop_f64(obj, safe_y, safe_x, depth, output, valid, collision, B, C, H, W, nthreads);
    return 0;
}

/* fw.py:27-43 -- safe coordinates from a flow.  p0 is float32 (fw.py:28); the
 * add happens in the flow's dtype (fw.py:31: float32 + float64 -> float64);
 * clamp (fw.py:37-38); .type(int64).type(float32) truncates (fw.py:41-42).
 * NaN stays NaN through torch.clamp and is dropped by the loop above. */
static void safe_from_flow_f32(const float *flow, float *sy, float *sx, long B, long H, long W) {
    const long HW = H * W;
    for (long b = 0; b < B; ++b)
        for (long j = 0; j < H; ++j)
            for (long i = 0; i < W; ++i) {
                const long s = j * W + i;
                float p1x = (float)i + flow[(b * 2 + 0) * HW + s];
                float p1y = (float)j + flow[(b * 2 + 1) * HW + s];
                if (!isnan(p1x)) { p1x = p1x < 0.f ? 0.f : p1x; p1x = p1x > (float)(W - 1) ? (float)(W - 1) : p1x; p1x = (float)(int64_t)p1x; }
                if (!isnan(p1y)) { p1y = p1y < 0.f ? 0.f : p1y; p1y = p1y > (float)(H - 1) ? (float)(H - 1) : p1y; p1y = (float)(int64_t)p1y; }
                sx[b * HW + s] = p1x;
                sy[b * HW + s] = p1y;
            }
}

static void safe_from_flow_f64(const double *flow, float *sy, float *sx, long B, long H, long W) {
    const long HW = H * W;
    for (long b = 0; b < B; ++b)
        for (long j = 0; j < H; ++j)
            for (long i = 0; i < W; ++i) {
                const long s = j * W + i;
                double p1x = (double)(float)i + flow[(b * 2 + 0) * HW + s];
                double p1y = (double)(float)j + flow[(b * 2 + 1) * HW + s];
                float ox = NAN, oy = NAN;
                if (!isnan(p1x)) { p1x = p1x < 0. ? 0. : p1x; p1x = p1x > (double)(W - 1) ? (double)(W - 1) : p1x; ox = (float)(int64_t)p1x; }
                if (!isnan(p1y)) { p1y = p1y < 0. ? 0. : p1y; p1y = p1y > (double)(H - 1) ? (double)(H - 1) : p1y; oy = (float)(int64_t)p1y; }
                sx[b * HW + s] = ox;
                sy[b * HW + s] = oy;
            }
}

/* Whole FW.forward (fw.py:19-59), batched: obj/depth already float32. */
int oracle_fw_flow_f32(const float *obj, const float *flow, const float *depth, float *output,
                       float *valid, float *collision, long B, long C, long H, long W,
                       int nthreads) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return -1;
    float *sy = (float *)malloc(sizeof(float) * (size_t)(B * H * W + 1));
    float *sx = (float *)malloc(sizeof(float) * (size_t)(B * H * W + 1));
    if (!sy || !sx) { free(sy); free(sx); return -2; }
    safe_from_flow_f32(flow, sy, sx, B, H, W);
    loop_f32(obj, sy, sx, depth, output, valid, collision, B, C, H, W, nthreads);
    free(sy); free(sx);
    return 0;
}

int oracle_fw_flow_f64flow(const float *obj, const double *flow, const float *depth, float *output,
                           float *valid, float *collision, long B, long C, long H, long W,
                           int nthreads) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return -1;
    float *sy = (float *)malloc(sizeof(float) * (size_t)(B * H * W + 1));
    float *sx = (float *)malloc(sizeof(float) * (size_t)(B * H * W + 1));
    if (!sy || !sx) { free(sy); free(sx); return -2; }
    safe_from_flow_f64(flow, sy, sx, B, H, W);
    loop_f32(obj, sy, sx, depth, output, valid, collision, B, C, H, W, nthreads);
    free(sy); free(sx);
    return 0;
}
