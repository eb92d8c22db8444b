// tools/probe_tile.hip -- diagnostic build of the TILE engine (not shipped).
// Same translation unit as the product (#include), with per-workgroup wall
// clock stamps (warp_kernel<..., kStamp = true>) so a Python driver can see
// each role's workgroup latency distribution and the launch spans.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude \
//         -o tools/_build/libprobe_tile.so tools/probe_tile.hip
#include "../opticalflowfromdepth_amd/csrc/ofd_fw.hip"

extern "C" int probe_launch(const float *obj, const float *flow, const float *depth, float *out, float *valid,
                            float *coll, int64_t C, int64_t H, int64_t W, void *slab, int64_t tile_b0,
                            int tile_nimg, int64_t bin_b0, int bin_nimg, int G, unsigned long long *stamps,
                            void *stream) {
    const int64_t HW = H * W;
    const TileGeom g = make_geom(H, W);
    FlowCoords<float> co{flow, HW};
    ChunkArgs t{}, b{};
    Ws w = carve(slab, G, HW, g);
    if (tile_nimg > 0) { t.ws = w; t.b0 = tile_b0; t.nimg = tile_nimg; t.nwg = tile_nimg * g.ntiles; }
    if (bin_nimg > 0) {
        b.ws = w; b.b0 = bin_b0; b.nimg = bin_nimg;
        b.nwg = int((int64_t(bin_nimg) * g.nseg + kWaves - 1) / kWaves);
    }
    const unsigned N = unsigned(t.nwg + b.nwg);
    hipLaunchKernelGGL((warp_kernel<FlowCoords<float>, true>), dim3((N + 7u) / 8u * 8u), dim3(kWarpThreads), 0,
                       static_cast<hipStream_t>(stream), co, obj, depth, out, valid, coll, t, b, int(C), int(H),
                       int(W), HW, g, stamps);
    return int(hipGetLastError());
}

extern "C" size_t probe_slab_bytes(int64_t G, int64_t H, int64_t W) { return size_t(G) * per_image_bytes(H, W); }
