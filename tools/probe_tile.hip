// tools/probe_tile.hip -- diagnostic build of the TILE engine (not shipped).
// Same translation unit as the product (#include), with per-workgroup wall
// clock stamps in the SPLAT kernel (splat_kernel<..., kStamp = true>) so a
// Python driver can time BIN / SPLAT / RESOLVE separately and see the SPLAT
// workgroups' phase split.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude \
//         -o tools/_build/libprobe_tile.so tools/probe_tile.hip
#include "../opticalflowfromdepth_amd/csrc/ofd_fw.hip"

// which: 0 = BIN, 1 = SPLAT (stamped), 2 = RESOLVE
extern "C" int probe_launch(int which, const float *obj, const float *flow, const float *depth, float *out,
                            float *valid, float *coll, int64_t C, int64_t H, int64_t W, void *slab, int64_t b0,
                            int nimg, unsigned long long *stamps, void *stream) {
    const int64_t HW = H * W;
    const TileGeom g = make_geom(H, W);
    FlowCoords<float> co{flow, HW};
    const ChunkArgs a{carve(slab, nimg, HW, g), b0, nimg};
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (which == 0) {
        hipLaunchKernelGGL((bin_kernel<FlowCoords<float>, true>), dim3(grid_for(int64_t(nimg) * g.nseg, kWaves)),
                           dim3(kWarpThreads), 0, st, co, depth, a, int(H), int(W), HW, g);
    } else if (which == 7 || which == 8) {
        // SPLAT tile orders: 7 = whole images strided over XCDs, 8 = whole images contiguous
        const unsigned tiles = unsigned(nimg * g.ntiles);
        const dim3 grid((tiles + 7u) / 8u * 8u);
        if (which == 7)
            hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true, true, 2, kSplatU, 1>), grid, dim3(kWarpThreads), 0,
                               st, co, depth, valid, coll, a, int(H), int(W), HW, g, stamps);
        else
            hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true, true, 2, kSplatU, 2>), grid, dim3(kWarpThreads), 0,
                               st, co, depth, valid, coll, a, int(H), int(W), HW, g, stamps);
    } else if (which == 5 || which == 6) {
        // SPLAT with 3 / 4 slots of 4 blocks in flight per wave
        const unsigned tiles = unsigned(nimg * g.ntiles);
        const dim3 grid((tiles + 7u) / 8u * 8u);
        if (which == 5)
            hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true, true, 2, 3>), grid, dim3(kWarpThreads), 0, st, co,
                               depth, valid, coll, a, int(H), int(W), HW, g, stamps);
        else
            hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true, true, 2, 4>), grid, dim3(kWarpThreads), 0, st, co,
                               depth, valid, coll, a, int(H), int(W), HW, g, stamps);
    } else if (which == 1 || which == 3 || which == 4) {
        // 1: product SPLAT (stamped; valid / collision non-temporal); 3 / 4: all plain / all non-temporal
        const unsigned tiles = unsigned(nimg * g.ntiles);
        const dim3 grid((tiles + 7u) / 8u * 8u);
        if (which == 1)
            hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true, true>), grid, dim3(kWarpThreads), 0, st, co, depth,
                               valid, coll, a, int(H), int(W), HW, g, stamps);
        else if (which == 3)
            hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true, true, 0>), grid, dim3(kWarpThreads), 0, st, co, depth,
                               valid, coll, a, int(H), int(W), HW, g, stamps);
        else
            hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true, true, 2>), grid, dim3(kWarpThreads), 0, st, co, depth,
                               valid, coll, a, int(H), int(W), HW, g, stamps);
    } else {
        // which 2: product RESOLVE; 10+v: RESOLVE shape / store variants
        const int v = which == 2 ? 0 : which - 10;
#define RV(WX, R, NT, ...)                                                                                         \
    hipLaunchKernelGGL((resolve2d_kernel<8, R, WX, NT __VA_OPT__(,) __VA_ARGS__>),                                                       \
                       dim3(unsigned((W + 64 * WX - 1) / (64 * WX)), unsigned((H + R - 1) / R), unsigned(nimg)), \
                       dim3(64 * WX * R), 0, st, obj, a.ws.winner, out, int(C), int(H), int(W), HW, b0)
        switch (v) {
        case 0: RV(kResolveWX, kResolveRows, true, true); break;
        case 1: RV(1, 16, true, true); break;
        case 2: RV(4, 4, false); break;
        case 3: RV(1, 8, false); break;
        case 4: RV(2, 4, false); break;
        case 5: RV(1, 4, false); break;
        case 6: RV(1, 16, true); break;
        case 7: RV(2, 8, true); break;
        case 8: RV(4, 4, true); break;
        case 9: RV(8, 2, true); break;
        case 10: RV(2, 4, true); break;
        case 11: RV(2, 8, true, true); break;
        case 12: RV(4, 4, true, true); break;
        case 13: RV(16, 1, true); break;
        default: return -1;
        }
#undef RV
    }
    return int(hipGetLastError());
}

extern "C" size_t probe_slab_bytes(int64_t G, int64_t H, int64_t W) { return size_t(G) * per_image_bytes(H, W); }
