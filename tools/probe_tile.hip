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
        hipLaunchKernelGGL((bin_kernel<FlowCoords<float>>), dim3(grid_for(int64_t(nimg) * g.nseg, kWaves)),
                           dim3(kWarpThreads), 0, st, co, depth, a, int(H), int(W), HW, g);
    } else if (which == 1) {
        const unsigned tiles = unsigned(nimg * g.ntiles);
        hipLaunchKernelGGL((splat_kernel<FlowCoords<float>, true>), dim3((tiles + 7u) / 8u * 8u),
                           dim3(kWarpThreads), 0, st, co, depth, valid, coll, a, int(H), int(W), HW, g, stamps);
    } else {
        hipLaunchKernelGGL((resolve2d_kernel<8, kResolveRows>),
                           dim3(unsigned((W + 63) / 64), unsigned((H + kResolveRows - 1) / kResolveRows), unsigned(nimg)),
                           dim3(64 * kResolveRows), 0, st, obj, a.ws.winner, out, int(C), int(H), int(W), HW, b0);
    }
    return int(hipGetLastError());
}

extern "C" size_t probe_slab_bytes(int64_t G, int64_t H, int64_t W) { return size_t(G) * per_image_bytes(H, W); }
