/*
 * ofd_fw.h -- C ABI of the MI355X forward-warp (z-buffered splat) engine.
 *
 * Plain pointers and sizes only; every device pointer is a gfx950 device
 * allocation, every entry point is asynchronous on the given HIP stream
 * (`stream` is a hipStream_t passed as void*, NULL = the legacy default
 * stream).  All tensors are dense, contiguous, NCHW.
 *
 * Entry point -> reference interface it replaces (paths in the reference
 * checkout AegeanKI/OpticalFlowFromDepth @ 2024_08_07):
 *
 *   ofd_fw_forward_warping_f32 / _f64
 *       fw_cuda.forward_warping(obj, safe_y, safe_x, depth)
 *       -- alt_cuda/fw_cuda.cpp:15-26 (binding), alt_cuda/fw_cuda_kernel.cu:52-83
 *          (host: allocate + launch) and :9-49 (kernel).  Same semantics, any B.
 *   ofd_fw_forward_warp_flow_f32 / _f64flow
 *       alt_cuda.fw.FW.forward(obj, flow, depth)  -- alt_cuda/fw.py:19-59,
 *       batched: the meshgrid add / clamp / int64 truncation of fw.py:27-42 is
 *       done inside the kernel, the add in the flow's dtype (fw.py:31).
 *   ofd_fw_forward_warp_flow_bf16
 *       no reference counterpart (FW is float32-only, fw.py:40-43, and
 *       AT_DISPATCH_FLOATING_TYPES excludes bf16): the on-the-fly training-loop
 *       warp of SURVEY.md 8(d) config 5 / 8(f) rank 4, bf16 obj and output.
 *   ofd_fw_warp_disparity_f32 / _f64depth
 *       preprocess.py:356-359 (Convert.depth_to_disparity, disparity_to_flow,
 *       the obj concatenation and the FW call) fused into one warp: the flow
 *       and obj's depth / flow channels are derived from the depth in-kernel.
 *   ofd_fw_ego_flow_f32 / _f64depth
 *       Convert.depth_to_random_flow (preprocess.py:265-298) with
 *       geometry.BackprojectDepth / Project3D (geometry.py:17-67): the
 *       ego-motion flow plane from depth, inv_K and P = (K @ T)[:3].
 *   ofd_fw_rotation_flow_f32
 *       SpecialFlow._rotate's special / back special flows
 *       (preprocess.py:31-41, :63-77), one kernel for a batch.
 *   ofd_fw_warp_ego_f32 / _f64depth
 *       preprocess.py:371-373 / :385-387 (ego-motion flow, the obj
 *       concatenation and the FW call) fused into one warp.
 *   ofd_fw_workspace_bytes / ofd_fw_workspace_init
 *       no reference counterpart: the reference allocates its z-buffer `dlut`
 *       per call (fw_cuda_kernel.cu:58); here the caller owns a reusable
 *       key workspace that every call leaves in its initial state.
 *
 * Semantics (identical to the serial loop fw_cuda_kernel.cu:28-47):
 *   per target pixel t of image b:
 *     winner(t)    = the source s with the smallest float depth among sources
 *                    landing on t with depth < 1000; ties -> smallest raster
 *                    index s = j*W + i.  (-0.0 == +0.0; NaN never wins.)
 *     output[b,c,t]= obj[b,c,winner] or 0 if no winner
 *     valid[b,0,t] = 1 if any source landed on t, else 0
 *     collision[b,0,t] = 1 if valid and no winner, else 0
 *   Defined where the reference is undefined: a source whose coordinate is
 *   NaN or truncates outside [0,W)x[0,H) is dropped.
 *
 * Return codes: 0 = success; <0 = OFD_FW_E* below; >0 = a hipError_t from the
 * launch.  ofd_fw_strerror() names any of them.
 */
#ifndef OFD_FW_H
#define OFD_FW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OFD_FW_ABI_VERSION 1

enum {
    OFD_FW_OK = 0,
    OFD_FW_EINVAL = -1,      /* null pointer or negative/zero-sized dimension mismatch */
    OFD_FW_ETOOBIG = -2,     /* H*W >= 2^31 (source index must fit 31 bits) */
    OFD_FW_EWORKSPACE = -3,  /* workspace null or smaller than ofd_fw_workspace_bytes() */
    OFD_FW_EALIGN = -4       /* a pointer is not 4-byte (f32) / 8-byte (f64, workspace) aligned */
};

/* ABI version of the loaded library (OFD_FW_ABI_VERSION at build time). */
int ofd_fw_abi_version(void);

/* Build id of the loaded library: the first 16 hex digits of the SHA-256 of
 * the sources it was compiled from (the .hip files and ip_common.h under csrc,
 * the headers under include;
 * opticalflowfromdepth_amd/build.py:source_hash), or "unknown" for a build
 * made without it.  Ties a binary to the commit whose sources it came from. */
const char *ofd_fw_build_id(void);

/* Engines (see csrc/ofd_fw.hip): TILE = LDS z-buffer per target tile whose
 * workgroup also gathers the output (default); TILE_SPLIT = the same z-buffer
 * publishing a winner map, then a separate RESOLVE gather pass; ATOMIC = one
 * global 64-bit atomic min per source.  Results are identical.
 * Selects the engine for subsequent calls in this process (also settable with
 * OFD_FW_MODE=atomic|split); an unknown value only queries.  Returns the
 * previous engine.  Not thread-safe against concurrent calls. */
#define OFD_FW_ENGINE_TILE 0
#define OFD_FW_ENGINE_ATOMIC 1
#define OFD_FW_ENGINE_TILE_SPLIT 2
int ofd_fw_set_engine(int engine);

/* The fused disparity warps (ofd_fw_warp_disparity_*) move every source
 * along its own row, and by default run on a row kernel (one workgroup per
 * image row, LDS z-buffer; rows up to 8192 wide) instead of the TILE engine;
 * results are identical.  on = 1 / 0 selects the row kernel / the TILE
 * engine for subsequent calls (also OFD_DISP_ROW=0); any other value only
 * queries.  Returns the previous setting.  Process-wide, not thread-safe. */
int ofd_fw_set_disparity_rows(int on);

/* Short TILE-engine calls -- fewer than `tiles_per_slot` target tiles per
 * resident SPLAT workgroup -- run one SPLAT workgroup per tile instead of the
 * persistent SPLAT (default 16, also OFD_PERSIST_MIN); 0 = always persistent
 * (tests drive the persistent kernel's queues on small images with it).
 * Results are identical.  A negative value only queries.  Returns the
 * previous setting.  Process-wide, not thread-safe against concurrent calls. */
int ofd_fw_set_persist_min(int tiles_per_slot);

/* Packed targets in the default TILE engine: BIN writes each source's target
 * as 16 bits relative to its source block's tile box and SPLAT re-reads those
 * 2 bytes instead of the coordinate planes (for FW on a flow / safe
 * coordinates and ofd_fw_warp_flow_cat; the fused disparity / ego-motion
 * warps read only the depth anyway).  on = 1 (default) / 0 for subsequent
 * calls (also OFD_FW_PACK=0); any other value only queries.  Results are
 * identical.  Returns the previous setting.  Process-wide, not thread-safe
 * against concurrent calls. */
int ofd_fw_set_pack(int on);

/* Short calls of the fused TILE engine (fewer tiles than persist_min() per
 * resident SPLAT slot: one SPLAT workgroup per tile) on plain coordinate
 * sources (FW on a flow or on safe coordinates, the bf16 warp) use 128 x 16
 * target tiles instead of 128 x 32: twice the workgroups, a shorter drain.
 * on = 1 (default) / 0 for subsequent calls (also OFD_FW_SHORT_TILES=0); any
 * other value only queries.  Results are identical.  Returns the previous
 * setting.  Process-wide, not thread-safe against concurrent calls. */
int ofd_fw_set_short_tiles(int on);

/* Benchmark hook: when non-NULL, the given hipEvent_t's are recorded on the
 * launch stream right before the first and right after the last launch of
 * each subsequent f32 call's dominant kernel: SPLAT (TILE engine), RESOLVE
 * (TILE_SPLIT), the resolve pass (ATOMIC).  Pass NULLs to disable.  Process-
 * wide, not thread-safe; for timing only. */
int ofd_fw_set_profile_events(void *start_event, void *stop_event);

/* Benchmark hook beside ofd_fw_set_profile_events: when non-NULL, the given
 * hipEvent_t is recorded right before the first chunk's BIN launch (TILE
 * engines), so BIN's duration is this event to the start event above.  NULL
 * disables it.  Process-wide, not thread-safe; for timing only. */
int ofd_fw_set_profile_bin_event(void *bin_start_event);

/* Human-readable name of a return code (static storage). */
const char *ofd_fw_strerror(int code);

/* Bytes of workspace recommended for a call with these sizes (f64 != 0 for
 * the float64 op); any size of at least one image's share works, larger
 * workspaces process more images per chunk.  The workspace is reused across
 * calls: initialise it once with ofd_fw_workspace_init(); every successful
 * call leaves the parts that must start initialised (key slabs, tile flags)
 * in that state again.  Calls sharing a workspace must be stream-ordered. */
size_t ofd_fw_workspace_bytes(int64_t B, int64_t H, int64_t W, int f64);

/* Put `bytes` of workspace into its initial state (async on `stream`).  Call
 * it for every new workspace allocation (the library remembers, per workspace
 * address, which layout last used it, and re-initialises on a layout change). */
int ofd_fw_workspace_init(void *workspace, size_t bytes, void *stream);

/* fw_cuda.forward_warping, float32.  obj/output [B,C,H,W]; safe_y, safe_x,
 * depth, valid, collision [B,1,H,W].  Coordinates are truncated toward zero. */
int ofd_fw_forward_warping_f32(const float *obj, const float *safe_y, const float *safe_x,
                               const float *depth, float *output, float *valid,
                               float *collision, int64_t B, int64_t C, int64_t H, int64_t W,
                               void *workspace, size_t workspace_bytes, void *stream);

/* fw_cuda.forward_warping, float64 (AT_DISPATCH_FLOATING_TYPES double path). */
int ofd_fw_forward_warping_f64(const double *obj, const double *safe_y, const double *safe_x,
                               const double *depth, double *output, double *valid,
                               double *collision, int64_t B, int64_t C, int64_t H, int64_t W,
                               void *workspace, size_t workspace_bytes, void *stream);

/* FW.forward, batched.  obj [B,C,H,W] f32, flow [B,2,H,W] (ch0 = x, ch1 = y)
 * f32, depth [B,1,H,W] f32 -> output [B,C,H,W], valid, collision [B,1,H,W]. */
int ofd_fw_forward_warp_flow_f32(const float *obj, const float *flow, const float *depth,
                                 float *output, float *valid, float *collision,
                                 int64_t B, int64_t C, int64_t H, int64_t W,
                                 void *workspace, size_t workspace_bytes, void *stream);

/* FW.forward with a float64 flow: p0 + flow is evaluated in float64 exactly
 * as fw.py:31 promotes it; everything else float32. */
int ofd_fw_forward_warp_flow_f64flow(const float *obj, const double *flow, const float *depth,
                                     float *output, float *valid, float *collision,
                                     int64_t B, int64_t C, int64_t H, int64_t W,
                                     void *workspace, size_t workspace_bytes, void *stream);

/* FW.forward on bf16 planes (raw bf16 bit patterns as uint16_t): obj and
 * output [B,C,H,W] bf16; flow [B,2,H,W], depth, valid, collision [B,1,H,W]
 * f32, the z-test and the coordinate arithmetic exactly as the f32 entry.
 * The warp only selects source values, so output == the f32 entry's output on
 * the same (bf16-valued) obj, bit for bit.  TILE engine only: requires
 * C*H*W < 2^30 (OFD_FW_ETOOBIG); obj / output 2-byte aligned. */
int ofd_fw_forward_warp_flow_bf16(const uint16_t *obj, const float *flow, const float *depth,
                                  uint16_t *output, float *valid, float *collision,
                                  int64_t B, int64_t C, int64_t H, int64_t W,
                                  void *workspace, size_t workspace_bytes, void *stream);

/* Fused depth -> disparity -> flow -> FW: preprocess.py:356-359,
 *     disp0   = Convert.depth_to_disparity(depth)         (s * 50 * 1 / depth, :239-246)
 *     flow01  = Convert.disparity_to_flow(disp0, random_sign=False)   (:249-254)
 *     obj_all = torch.cat((obj[:3], depth, flow01 * -1.0, obj[3:]))   (:358)
 *     FW(obj_all, flow01, depth)                                      (:359)
 * without the flow plane or the concatenated obj ever being stored: the flow
 * is derived from the depth inside the kernels, and output channels 3, 4, 5
 * (depth, disparity, +0) are generated from the winner's depth.
 * obj [B,Cobj,H,W] f32 holds the caller's other channels (the RGB image, and
 * any channels the caller appends, e.g. a validity mask); depth [B,1,H,W] in
 * float32 or float64 (utils.get_depth returns float64; the disparity and the
 * flow add are computed in the depth's dtype, exactly as torch promotes them);
 * s [B] f32 per-image scale (the get_random draw of :240).  Output
 * [B,Cobj+3,H,W], valid / collision [B,1,H,W].  Bit-identical to
 * ofd_fw_forward_warp_flow_* on the materialised inputs.  TILE engine only:
 * requires (Cobj+3)*H*W < 2^30 (OFD_FW_ETOOBIG). */
int ofd_fw_warp_disparity_f32(const float *obj, int64_t Cobj, const float *depth, const float *s,
                              float *output, float *valid, float *collision, int64_t B, int64_t H,
                              int64_t W, void *workspace, size_t workspace_bytes, void *stream);
int ofd_fw_warp_disparity_f64depth(const float *obj, int64_t Cobj, const double *depth, const float *s,
                                   float *output, float *valid, float *collision, int64_t B, int64_t H,
                                   int64_t W, void *workspace, size_t workspace_bytes, void *stream);

/* Ego-motion flow plane (preprocess.py:265-298, geometry.py:17-67):
 *   cam  = float32(depth * inv_K[:3,:3] @ [x, y, 1])
 *   cp   = P @ [cam, 1]
 *   pix  = cp[:2] / (cp[2] + 1e-7), normalised to [-1, 1] and back to pixels
 *   flow = pix - [x, y]
 * depth [B,1,H,W] f32 or f64 (device); P [B,3,4] f32 (device) = (K @ T)[:, :3]
 * as Project3D computes it; inv_K: HOST pointer to the 9 floats of
 * inv_K[:3,:3] (row-major; one camera for the batch, Plausible.K); flow
 * [B,2,H,W] f32 (device).  The products accumulate with fused multiply-adds
 * in k order, so the flow equals the reference's to float32 rounding, not bit
 * for bit (torch's GEMM order is unspecified). */
int ofd_fw_ego_flow_f32(const float *depth, const float *P, const float *inv_K, float *flow, int64_t B, int64_t H,
                        int64_t W, void *stream);
int ofd_fw_ego_flow_f64depth(const double *depth, const float *P, const float *inv_K, float *flow, int64_t B,
                             int64_t H, int64_t W, void *stream);

/* SpecialFlow._rotate (preprocess.py:31-41, :63-77): the rotation special
 * flow and back special flow [B,2,H,W] float32, p1 = (p0 - c0) @ R + c0 minus
 * p0, for R = rotate / reverse_rotate.  params [B][10] float32 (device):
 * c0x, c0y, then R and reverse R row-major (R = [[cos t, -sin t], [sin t,
 * cos t]] as the reference builds it, t and -t).  The 2-term product rounds
 * as a GEMM accumulates it (k = 0 product, then a fused multiply-add of the
 * k = 1 term): bit-identical to the reference's matmul. */
int ofd_fw_rotation_flow_f32(const float *params, float *flow, float *back_flow, int64_t B, int64_t H, int64_t W,
                             void *stream);

/* Fused depth -> ego-motion flow -> FW (preprocess.py:371-373, :385-387):
 *     flow    = the ofd_fw_ego_flow_* plane
 *     obj_all = torch.cat((obj[:3], depth, flow * -1.0, obj[3:]))
 *     FW(obj_all, flow, depth)
 * with neither the flow nor obj_all stored; arguments as ofd_fw_ego_flow_*
 * and ofd_fw_warp_disparity_*.  Bit-identical to ofd_fw_forward_warp_flow_f32
 * on the materialised ofd_fw_ego_flow_* plane (the same device code computes
 * the flow in both).  TILE engine only: (Cobj+3)*H*W < 2^30. */
int ofd_fw_warp_ego_f32(const float *obj, int64_t Cobj, const float *depth, const float *P, const float *inv_K,
                        float *output, float *valid, float *collision, int64_t B, int64_t H, int64_t W,
                        void *workspace, size_t workspace_bytes, void *stream);
int ofd_fw_warp_ego_f64depth(const float *obj, int64_t Cobj, const double *depth, const float *P,
                             const float *inv_K, float *output, float *valid, float *collision, int64_t B, int64_t H,
                             int64_t W, void *workspace, size_t workspace_bytes, void *stream);

/* FW on a flow plane the caller holds, obj's depth and flow channels
 * generated instead of concatenated: preprocess.py:371-373 / :385-387 (the
 * ego-motion warps, whose flow planes are group outputs) and :400-402 /
 * :414-417 (the composed-flow warps) all compute
 *     obj_all = torch.cat((obj[:3], depth, flow * -1.0, obj[3:]))
 *     FW(obj_all, flow, depth)
 * This entry never stores obj_all: the winner's depth and flow * -1.0 are
 * taken from the depth key and the flow plane.  obj [B,Cobj,H,W] f32 (the
 * image and any appended channels, e.g. a validity mask); flow [B,2,H,W] f32
 * (flow_f64 = 0) or f64 (flow_f64 = 1, added in float64 as fw.py:31); depth
 * [B,1,H,W] f32 (depth_f64 = 0) or f64.  Output [B,Cobj+3,H,W], valid /
 * collision [B,1,H,W] f32, bit-identical to ofd_fw_forward_warp_flow_* on the
 * materialised obj_all (cast to float32, fw.py:40).  TILE engine only:
 * (Cobj+3)*H*W < 2^30 (OFD_FW_ETOOBIG). */
int ofd_fw_warp_flow_cat(const float *obj, int64_t Cobj, const void *flow, int flow_f64, const void *depth,
                         int depth_f64, float *output, float *valid, float *collision, int64_t B, int64_t H,
                         int64_t W, void *workspace, size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* OFD_FW_H */
