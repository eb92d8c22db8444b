// tools/microbench.hip -- design probes for the forward-warp engine (gfx950).
// Measures: HBM stream-copy ceiling; global 64-bit atomicMin throughput by
// access shape and footprint; 32-bit atomicMin; LDS 64-bit atomicMin.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int U>
__global__ __launch_bounds__(256) void copyU(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    size_t base = (blockIdx.x * (size_t)256 * U) + threadIdx.x;
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (base + u * 256 < n) v[u] = a[base + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) if (base + u * 256 < n) b[base + u * 256] = v[u];
}

__global__ __launch_bounds__(256) void read4(const float4* __restrict__ a, float* out, size_t n) {
    size_t base = (blockIdx.x * (size_t)256 * 4) + threadIdx.x;
    float acc = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) { float4 v = a[base + u * 256]; acc += v.x + v.y + v.z + v.w; }
    if (acc == 12345.f) out[0] = acc;
}

__global__ __launch_bounds__(256) void copy1(const float* __restrict__ a, float* __restrict__ b, size_t n) {
    size_t i = blockIdx.x * (size_t)256 + threadIdx.x;
    if (i < n) b[i] = a[i];
}

// resolve-like: per target read a u32 source index, gather C planes, write C + 2 planes
template <int C, int PER>
__global__ __launch_bounds__(256) void resolve_sim(const unsigned* __restrict__ idx, const float* __restrict__ obj,
                                                    float* __restrict__ out, size_t hw, size_t n) {
    size_t t0 = blockIdx.x * (size_t)256 * PER + threadIdx.x;
#pragma unroll
    for (int p = 0; p < PER; ++p) {
        size_t t = t0 + p * 256;
        if (t >= n) return;
        size_t img = t / hw, pix = t - img * hw;
        unsigned s = idx[t];
        const float* ob = obj + img * C * hw;
        float* oo = out + img * (C + 2) * hw + pix;
        float v[C];
#pragma unroll
        for (int c = 0; c < C; ++c) v[c] = ob[c * hw + s];
#pragma unroll
        for (int c = 0; c < C; ++c) oo[c * hw] = v[c];
        oo[C * hw] = 1.f;
        oo[(C + 1) * hw] = 0.f;
    }
}

__global__ void init_idx(unsigned* idx, size_t hw, size_t n) {
    size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
    if (t >= n) return;
    size_t pix = t % hw;
    long s = (long)pix + 17 - (long)((pix / 1024) % 7);   // coherent, shifted sources
    if (s < 0) s = 0;
    if (s >= (long)hw) s = hw - 1;
    idx[t] = (unsigned)s;
}

__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    size_t st = (size_t)gridDim.x * blockDim.x;
    for (; i < n; i += st) b[i] = a[i];
}

// each thread: VEC atomics; shape 0 = lane-contiguous per instruction (addr = base + k*64 + lane)
// shape 1 = thread-contiguous (addr = base + lane*VEC + k)  (v1 kernel's shape)
template <int SHAPE, typename T>
__global__ void atom(T* __restrict__ buf, size_t n_atomics, size_t mask, unsigned salt) {
    const int VEC = 4;
    size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    size_t wave = t / 64, lane = t % 64;
    size_t base = wave * 64 * VEC;
    if (base >= n_atomics) return;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
        size_t idx = SHAPE == 0 ? base + k * 64 + lane : base + lane * VEC + k;
        atomicMin(buf + (idx & mask), (T)(idx ^ salt));
    }
}

__global__ void lds_atom(unsigned long long* out, int iters) {
    __shared__ unsigned long long z[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) z[i] = ~0ull;
    __syncthreads();
    unsigned long long v = blockIdx.x * 7919ull + threadIdx.x;
    for (int it = 0; it < iters; ++it) {
        int a = (threadIdx.x * 13 + it * 64) & 4095;
        atomicMin(&z[a], v ^ (unsigned long long)it);
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = z[blockIdx.x & 4095];
}

template <typename F>
float timeit(F f, int reps = 10) {
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    f(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const size_t n4 = (size_t)1 << 28;  // 4 GiB as float4? no: 2^28 float4 = 4 GiB; use 2^26 = 1 GiB
    size_t n = (size_t)1 << 26;
    float4 *a, *b; CK(hipMalloc(&a, n * 16)); CK(hipMalloc(&b, n * 16));
    CK(hipMemset(a, 0, n * 16));
    float ms = timeit([&] { copy4<<<2048 * 4, 256>>>(a, b, n); });
    printf("copy float4 1GiB->1GiB: %.3f ms  %.1f GB/s (read+write)\n", ms, 2.0 * n * 16 / ms / 1e6);
    ms = timeit([&] { copyU<1><<<n / 256, 256>>>(a, b, n); });
    printf("copyU<1> : %.3f ms  %.1f GB/s\n", ms, 2.0 * n * 16 / ms / 1e6);
    ms = timeit([&] { copyU<4><<<n / 1024, 256>>>(a, b, n); });
    printf("copyU<4> : %.3f ms  %.1f GB/s\n", ms, 2.0 * n * 16 / ms / 1e6);
    ms = timeit([&] { copyU<8><<<n / 2048, 256>>>(a, b, n); });
    printf("copyU<8> : %.3f ms  %.1f GB/s\n", ms, 2.0 * n * 16 / ms / 1e6);
    ms = timeit([&] { copy1<<<n * 4 / 256, 256>>>((const float*)a, (float*)b, n * 4); });
    printf("copy1 (dword/lane): %.3f ms  %.1f GB/s\n", ms, 2.0 * n * 16 / ms / 1e6);
    {
        const size_t hw = 768 * 1024, nimg = 32, npx = hw * nimg;
        unsigned* idx; float* obj; float* out;
        CK(hipMalloc(&idx, npx * 4)); CK(hipMalloc(&obj, npx * 6 * 4)); CK(hipMalloc(&out, npx * 8 * 4));
        init_idx<<<npx / 256, 256>>>(idx, hw, npx);
        float m1 = timeit([&] { resolve_sim<6, 1><<<npx / 256, 256>>>(idx, obj, out, hw, npx); });
        float m4 = timeit([&] { resolve_sim<6, 4><<<npx / 1024, 256>>>(idx, obj, out, hw, npx); });
        const double bytes = npx * (4.0 + 24 + 32);
        printf("resolve_sim C=6 (60 B/px): PER=1 %.3f ms %.1f GB/s | PER=4 %.3f ms %.1f GB/s\n", m1, bytes / m1 / 1e6, m4, bytes / m4 / 1e6);
    }
    float* o1; CK(hipMalloc(&o1, 64));
    ms = timeit([&] { read4<<<n / 1024, 256>>>(a, o1, n); });
    printf("read-only: %.3f ms  %.1f GB/s\n", ms, 1.0 * n * 16 / ms / 1e6);
    (void)n4;

    const size_t NA = 50331648;  // one headline step of sources
    unsigned long long* keys; CK(hipMalloc(&keys, ((size_t)1 << 26) * 8));
    unsigned* k32; CK(hipMalloc(&k32, ((size_t)1 << 26) * 4));
    const size_t blocks = (NA / 4 + 255) / 256;
    for (size_t lg : {26, 23, 19}) {
        size_t mask = ((size_t)1 << lg) - 1;
        CK(hipMemset(keys, 0xFF, ((size_t)1 << 26) * 8));
        float m0 = timeit([&] { atom<0, unsigned long long><<<blocks, 256>>>(keys, NA, mask, 12345u); });
        float m1 = timeit([&] { atom<1, unsigned long long><<<blocks, 256>>>(keys, NA, mask, 12345u); });
        float m2 = timeit([&] { atom<0, unsigned><<<blocks, 256>>>(k32, NA, mask, 12345u); });
        printf("footprint %zu slots: u64 lane-contig %.3f ms (%.1f Gatom/s)  u64 thread-contig %.3f ms (%.1f)  u32 lane-contig %.3f ms (%.1f)\n",
               mask + 1, m0, NA / m0 / 1e6, m1, NA / m1 / 1e6, m2, NA / m2 / 1e6);
    }
    unsigned long long* o; CK(hipMalloc(&o, 1 << 20));
    int iters = 4096;
    float ml = timeit([&] { lds_atom<<<2048, 256>>>(o, iters); });
    printf("LDS u64 atomicMin: %.3f ms  %.1f Gatom/s chip\n", ml, 2048.0 * 256 * iters / ml / 1e6);
    return 0;
}
