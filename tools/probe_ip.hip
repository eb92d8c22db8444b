// tools/probe_ip.hip -- diagnostic build of the hole-fill (not shipped): the
// product TU with OFD_IP_STAMPS, so thread 0 of the first block of each path
// of every hole-layer launch stamps the per-hole chain (entry, list read,
// patch loaded, colour computed, stores done) in shader clocks.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Iinclude \
//         -o tools/_build/libprobe_ip.so tools/probe_ip.hip
#define OFD_IP_STAMPS 1
#include "../opticalflowfromdepth_amd/csrc/ofd_inpaint.hip"

extern "C" int probe_ip_set_stamps(unsigned long long *p) {
    return int(hipMemcpyToSymbol(HIP_SYMBOL(g_ip_stamps), &p, sizeof(p)));
}
