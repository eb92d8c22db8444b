// tools/sync_bench.hip -- what a cross-workgroup barrier costs on MI355X, for
// the chip-wide fast-march design: a march's large
// bucket split over several workgroups needs a barrier between its phases.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sync_bench tools/sync_bench.hip && /tmp/sync_bench
// 1. cooperative grid barrier (cooperative_groups grid.sync) over one
//    1024-thread workgroup per CU;
// 2. a barrier of workgroup pairs (counter + agent-scope release / acquire
//    fences, what two workgroups of one image's march would use), with and
//    without 64 KB of fresh global stores per workgroup between barriers.
// Every wait is bounded (a broken barrier ends the kernel; the result line
// says so).  Prints one line per case: microseconds per barrier.
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <stdio.h>

namespace cg = cooperative_groups;

__global__ __launch_bounds__(1024) void grid_sync_kernel(int iters, unsigned *sink) {
    cg::grid_group g = cg::this_grid();
    unsigned acc = 0;
    for (int i = 0; i < iters; ++i) {
        acc += threadIdx.x ^ unsigned(i);
        g.sync();
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

// pairs of workgroups (2p, 2p+1): generation barrier on ctr[p]
__global__ __launch_bounds__(1024) void pair_kernel(int iters, unsigned *ctr, float *scratch, int store_words,
                                                    unsigned *fault) {
    const unsigned pair = blockIdx.x / 2u;
    unsigned *c = ctr + pair * 32u;  // one 128-byte line per pair
    float *mine = scratch + size_t(blockIdx.x) * size_t(store_words);
    __shared__ unsigned bad;
    if (threadIdx.x == 0) bad = 0u;
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        for (int k = threadIdx.x; k < store_words; k += 1024) mine[k] = float(i + k);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (threadIdx.x == 0) {
            atomicAdd(c, 1u);
            const unsigned target = 2u * unsigned(i + 1);
            unsigned spins = 0;
            while (atomicAdd(c, 0u) < target) {
                if (++spins > (1u << 22)) {
                    bad = 1u;
                    atomicOr(fault, 1u);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (bad) return;
    }
}

int main() {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    unsigned *sink = nullptr, *ctr = nullptr, *fault = nullptr;
    float *scratch = nullptr;
    hipMalloc(&sink, 64);
    hipMalloc(&ctr, size_t(cus) * 128);
    hipMalloc(&fault, 4);
    hipMalloc(&scratch, size_t(cus) * 16384 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // 1. cooperative grid barrier
    for (int wpc : {1}) {
        int iters = 2000;
        void *args[] = {&iters, &sink};
        const unsigned grid = unsigned(cus * wpc);
        hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<void *>(grid_sync_kernel), dim3(grid), dim3(1024),
                                                  args, 0, nullptr);
        hipDeviceSynchronize();
        hipEventRecord(a);
        e = hipLaunchCooperativeKernel(reinterpret_cast<void *>(grid_sync_kernel), dim3(grid), dim3(1024), args, 0,
                                       nullptr);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        printf("cooperative grid.sync, %u workgroups x 1024 threads: %s %.3f us per barrier\n", grid,
               e == hipSuccess ? "ok" : hipGetErrorString(e), ms * 1e3f / iters);
    }
    // 2. pair barriers (one workgroup per CU, cus / 2 pairs)
    for (int words : {0, 16384}) {
        const int iters = 2000;
        hipMemset(ctr, 0, size_t(cus) * 128);
        hipMemset(fault, 0, 4);
        const unsigned grid = unsigned(cus) & ~1u;
        hipLaunchKernelGGL(pair_kernel, dim3(grid), dim3(1024), 0, nullptr, 10, ctr, scratch, words, fault);
        hipDeviceSynchronize();
        hipMemset(ctr, 0, size_t(cus) * 128);
        hipEventRecord(a);
        hipLaunchKernelGGL(pair_kernel, dim3(grid), dim3(1024), 0, nullptr, iters, ctr, scratch, words, fault);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        unsigned f = 0;
        hipMemcpy(&f, fault, 4, hipMemcpyDeviceToHost);
        printf("pair barrier (agent fences), %u workgroups, %d KB stored per workgroup per step: %.3f us per barrier%s\n",
               grid, words * 4 / 1024, ms * 1e3f / iters, f ? " (FAULT: a wait gave up)" : "");
    }
    hipFree(sink);
    hipFree(ctr);
    hipFree(fault);
    hipFree(scratch);
    return 0;
}
