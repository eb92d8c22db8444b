// tools/probe_tile.hip -- diagnostic build of the TILE engine (not shipped).
// Same translation unit as the product (#include), with per-workgroup wall
// clock stamps in the SPLAT kernel (splat_kernel<..., kStamp = true>) so a
// Python driver can time BIN / SPLAT / RESOLVE separately, compare kernel
// variants, and see the SPLAT workgroups' phase split.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude \
//         -o tools/_build/libprobe_tile.so tools/probe_tile.hip
#include "../opticalflowfromdepth_amd/csrc/ofd_fw.hip"

// which:  0 / 3 / 4 = BIN with 1 / 2 / 4 segments per wave
//         1 = SPLAT, split engine (stamped)       5 = SPLAT, split engine
//         6 = SPLAT, fused engine (stamped)       7 = SPLAT, fused engine (product FusedCfg)
//         8 = persistent fused SPLAT (stamped)    9 = persistent fused SPLAT
//        10..14 = fused SPLAT launch-shape variants (see the cases)
//         2 = RESOLVE (product shape)
//        15 = BIN writing packed targets, 16 / 17 = packed persistent fused SPLAT (stamped / not)
using C256 = SplatCfg<256, 8, 4>;
using C512u3 = SplatCfg<512, 8, 4, 3>;
using C256u3 = SplatCfg<256, 8, 4, 3>;

extern "C" int probe_launch(int which, const float *obj, const float *flow, const float *depth, float *out,
                            float *valid, float *coll, int64_t C, int64_t H, int64_t W, void *slab, int64_t b0,
                            int nimg, unsigned long long *stamps, void *stream) {
    const int64_t HW = H * W;
    const TileGeom g = make_geom(H, W);
    using Co = FlowCoords<float>;
    Co co{flow, HW};
    const ChunkArgs a{carve(slab, nimg, HW, g), b0, nimg};
    const SplatIO io{valid, coll, obj, out, int(C), int(C), int(C)};  // Cobj = C, no generated channels
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 sgrid((unsigned(nimg * g.ntiles) + 7u) / 8u * 8u), blk(kWarpThreads);
    const int64_t nsg = int64_t(nimg) * g.nseg;
    switch (which) {
    case 0: hipLaunchKernelGGL((bin_kernel<Co, true, 1>), dim3(grid_for(nsg, kWaves)), blk, 0, st, co, depth, a,
                               int(H), int(W), HW, g); break;
    case 3: hipLaunchKernelGGL((bin_kernel<Co, true, 2>), dim3(grid_for(nsg, kWaves * 2)), blk, 0, st, co, depth, a,
                               int(H), int(W), HW, g); break;
    case 4: hipLaunchKernelGGL((bin_kernel<Co, true, 4>), dim3(grid_for(nsg, kWaves * 4)), blk, 0, st, co, depth, a,
                               int(H), int(W), HW, g); break;
    case 1: hipLaunchKernelGGL((splat_kernel<Co, true, false, true>), sgrid, blk, 0, st, co, depth, io, a, int(H),
                               int(W), HW, g, stamps); break;
    case 5: hipLaunchKernelGGL((splat_kernel<Co, true, false, false>), sgrid, blk, 0, st, co, depth, io, a, int(H),
                               int(W), HW, g, nullptr); break;
    case 6: hipLaunchKernelGGL((splat_kernel<Co, true, true, true, FusedCfg>), sgrid, blk, 0, st, co, depth, io, a,
                               int(H), int(W), HW, g, stamps); break;
    case 7: hipLaunchKernelGGL((splat_kernel<Co, true, true, false, FusedCfg>), sgrid, blk, 0, st, co, depth, io, a,
                               int(H), int(W), HW, g, nullptr); break;
    case 8: hipLaunchKernelGGL((splat_persist_kernel<Co, true, true, true>), dim3(persist_grid<Co, true>(sgrid.x)),
                               dim3(FusedCfg::kThr), 0, st, co, depth, io, a, int(H), int(W), HW, g, stamps); break;
    case 9: hipLaunchKernelGGL((splat_persist_kernel<Co, true, true, false>), dim3(persist_grid<Co, true>(sgrid.x)),
                               dim3(FusedCfg::kThr), 0, st, co, depth, io, a, int(H), int(W), HW, g, nullptr); break;
#define FV(CFG) hipLaunchKernelGGL((splat_kernel<Co, true, true, false, CFG>), sgrid, dim3(CFG::kThr), 0, st, co, depth, \
                                   io, a, int(H), int(W), HW, g, nullptr)
    case 10: FV(SplitCfg); break;                      // 512 threads, 2 targets in flight, 4 WG / CU
    case 11: FV(C256); break;    // 256 threads, 8 in flight, LDS-bound 4 WG / CU
    case 13: FV(C512u3); break;  // + 3 splat slots per wave
    case 14: FV(C256u3); break;
#undef FV
    case 12: {
        using P = SplatCfg<256, 8, 4>;
        hipLaunchKernelGGL((splat_persist_kernel<Co, true, true, false, P>), dim3(persist_grid<Co, true, P>(sgrid.x)),
                           dim3(P::kThr), 0, st, co, depth, io, a, int(H), int(W), HW, g, nullptr);
        break;
    }
    case 15: hipLaunchKernelGGL((bin_kernel<Co, true, 1, true>), dim3(grid_for(nsg, kWaves)), blk, 0, st, co, depth, a,
                                int(H), int(W), HW, g); break;  // BIN writing packed targets
    case 16: hipLaunchKernelGGL((splat_persist_kernel<Co, true, true, true, FusedCfg, float, true>),
                                dim3(persist_grid<Co, true, FusedCfg, float, true>(sgrid.x)), dim3(FusedCfg::kThr), 0, st,
                                co, depth, io, a, int(H), int(W), HW, g, stamps); break;  // packed, stamped
    case 17: hipLaunchKernelGGL((splat_persist_kernel<Co, true, true, false, FusedCfg, float, true>),
                                dim3(persist_grid<Co, true, FusedCfg, float, true>(sgrid.x)), dim3(FusedCfg::kThr), 0, st,
                                co, depth, io, a, int(H), int(W), HW, g, nullptr); break;  // packed
    case 2:
        hipLaunchKernelGGL((resolve2d_kernel<8, kResolveRows, kResolveWX, true, true>),
                           dim3(unsigned((W + 64 * kResolveWX - 1) / (64 * kResolveWX)),
                                unsigned((H + kResolveRows - 1) / kResolveRows), unsigned(nimg)),
                           dim3(64 * kResolveWX * kResolveRows), 0, st, obj, a.ws.winner, out, int(C), int(H), int(W),
                           HW, b0);
        break;
    default: return -1;
    }
    return int(hipGetLastError());
}

extern "C" size_t probe_slab_bytes(int64_t G, int64_t H, int64_t W) { return size_t(G) * per_image_bytes(H, W); }
