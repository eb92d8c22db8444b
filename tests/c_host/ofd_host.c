/* ofd_host.c -- the drop-in C ABI driven from plain C (no Python, no torch):
 * what a C / cgo / JNI host of the reference's path would do.  Reads a batch
 * from a file, runs the forward warp (ofd_fw_forward_warp_flow_f32, replacing
 * fw_cuda.forward_warping, alt_cuda/fw_cuda.cpp:15-30) and the cv2-order
 * hole-fill of the warped RGB (ofd_inpaint_telea_seq_f32, replacing
 * utils.inpaint, utils.py:136-151) on the GPU, and writes the results.
 * tests/test_c_host.py checks them against the CPU oracle.
 *
 *   ofd_host IN OUT
 *   IN : int64 B, C, H, W; float32 obj[B][C][H][W], flow[B][2][H][W], depth[B][1][H][W]
 *   OUT: float32 output[B][C][H][W], valid[B][H][W], collision[B][H][W], filled[B][3][H][W]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "ofd_fw.h"
#include "ofd_inpaint.h"

#define HIP_OK(x)                                                               \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 2;                                                           \
        }                                                                       \
    } while (0)

static void *dev_copy(const float *h, size_t n) {
    void *d = NULL;
    if (hipMalloc(&d, n * sizeof(float)) != hipSuccess) return NULL;
    if (h && hipMemcpy(d, h, n * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return NULL;
    return d;
}

int main(int argc, char **argv) {
    if (argc != 3) {
        fprintf(stderr, "usage: %s IN OUT\n", argv[0]);
        return 1;
    }
    FILE *f = fopen(argv[1], "rb");
    if (!f) return 1;
    int64_t dims[4];
    if (fread(dims, sizeof(int64_t), 4, f) != 4) return 1;
    const int64_t B = dims[0], C = dims[1], H = dims[2], W = dims[3], HW = H * W;
    const size_t nobj = (size_t)(B * C * HW), nflow = (size_t)(B * 2 * HW), nd = (size_t)(B * HW);
    float *h = (float *)malloc((nobj + nflow + nd) * sizeof(float));
    if (!h || fread(h, sizeof(float), nobj + nflow + nd, f) != nobj + nflow + nd) return 1;
    fclose(f);
    if (C < 3) return 1;

    hipStream_t st;
    HIP_OK(hipStreamCreate(&st));
    float *obj = dev_copy(h, nobj), *flow = dev_copy(h + nobj, nflow), *depth = dev_copy(h + nobj + nflow, nd);
    float *out = dev_copy(NULL, nobj), *valid = dev_copy(NULL, nd), *coll = dev_copy(NULL, nd);
    float *rgb = dev_copy(NULL, (size_t)(B * 3 * HW)), *filled = dev_copy(NULL, (size_t)(B * 3 * HW));
    if (!obj || !flow || !depth || !out || !valid || !coll || !rgb || !filled) return 2;

    /* the warp: caller-owned workspace, initialised once */
    const size_t nws = ofd_fw_workspace_bytes(B, H, W, 0);
    void *ws = NULL;
    HIP_OK(hipMalloc(&ws, nws));
    int rc = ofd_fw_workspace_init(ws, nws, st);
    if (!rc) rc = ofd_fw_forward_warp_flow_f32(obj, flow, depth, out, valid, coll, B, C, H, W, ws, nws, st);
    if (rc) {
        fprintf(stderr, "forward_warp_flow: %s\n", ofd_fw_strerror(rc));
        return 3;
    }
    /* the caller's masking of the warped RGB (preprocess.py:362: rgb * valid), on the host */
    HIP_OK(hipStreamSynchronize(st));
    float *ho = (float *)malloc(nobj * sizeof(float)), *hv = (float *)malloc(nd * sizeof(float));
    float *hc = (float *)malloc(nd * sizeof(float)), *hr = (float *)malloc((size_t)(B * 3 * HW) * sizeof(float));
    HIP_OK(hipMemcpy(ho, out, nobj * sizeof(float), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(hv, valid, nd * sizeof(float), hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(hc, coll, nd * sizeof(float), hipMemcpyDeviceToHost));
    for (int64_t b = 0; b < B; ++b)
        for (int64_t c = 0; c < 3; ++c)
            for (int64_t p = 0; p < HW; ++p) hr[(b * 3 + c) * HW + p] = ho[(b * C + c) * HW + p] * hv[b * HW + p];
    HIP_OK(hipMemcpy(rgb, hr, (size_t)(B * 3 * HW) * sizeof(float), hipMemcpyHostToDevice));

    /* the hole-fill in cv2's order */
    const size_t nws2 = ofd_inpaint_seq_workspace_bytes(B, H, W);
    void *ws2 = NULL;
    HIP_OK(hipMalloc(&ws2, nws2));
    rc = ofd_inpaint_telea_seq_f32(rgb, valid, coll, filled, B, 3, H, W, 3, ws2, nws2, st);
    if (rc) {
        fprintf(stderr, "inpaint: %s\n", ofd_fw_strerror(rc));
        return 3;
    }
    HIP_OK(hipStreamSynchronize(st));
    HIP_OK(hipMemcpy(hr, filled, (size_t)(B * 3 * HW) * sizeof(float), hipMemcpyDeviceToHost));

    FILE *g = fopen(argv[2], "wb");
    if (!g) return 1;
    fwrite(ho, sizeof(float), nobj, g);
    fwrite(hv, sizeof(float), nd, g);
    fwrite(hc, sizeof(float), nd, g);
    fwrite(hr, sizeof(float), (size_t)(B * 3 * HW), g);
    fclose(g);
    hipFree(ws);
    hipFree(ws2);
    hipStreamDestroy(st);
    printf("ofd_host OK: B=%lld C=%lld H=%lld W=%lld\n", (long long)B, (long long)C, (long long)H, (long long)W);
    return 0;
}
