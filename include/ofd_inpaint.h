/*
 * ofd_inpaint.h -- C ABI of the MI355X hole-fill (Telea inpainting: cv2's sequential
 * order, the default, and the faster layered order).
 *
 * Same conventions as ofd_fw.h: plain pointers and sizes, gfx950 device
 * pointers, dense contiguous NCHW float32, asynchronous on `stream` (a
 * hipStream_t passed as void*, NULL = the legacy default stream); return 0 or
 * an OFD_FW_E* code (< 0) or a hipError_t (> 0), named by ofd_fw_strerror().
 *
 * Entry point -> reference interface it replaces (AegeanKI/OpticalFlowFromDepth
 * @ 2024_08_07):
 *
 *   ofd_inpaint_telea_f32
 *       utils.inpaint(img, valid, collision)  -- utils.py:136-151, batched:
 *       the keep-mask algebra of :137-142 (exact), the uint8 cast of :148, and
 *       cv2.inpaint(img_u8, 1 - H', 3, cv2.INPAINT_TELEA) of :149 replaced by a
 *       level-synchronous Telea fill (DESIGN.md "Hole-fill"): the same Telea
 *       weights and fast-marching update, with holes finalised in layers of
 *       equal L1 distance to the known region instead of one at a time.  The
 *       fill values are therefore not cv2's (parity with cv2 is unpinned: no
 *       OpenCV in the build image); the kernel is bit-exact against its CPU
 *       restatement oracle/inpaint_oracle.c (layered mode).  Specified
 *       divergence from cv2's sequential order: on
 *       warped random-RGB images 85 % of hole values differ, mean 5.7 grey
 *       levels, p99 40; within 1-2 levels on smooth images.
 *   ofd_inpaint_telea_seq_f32
 *       utils.inpaint, as above, with the fill in cv2's sequential order
 *       (bit-exact against oracle/inpaint_oracle.c sequential mode, OpenCV's
 *       icvCalcFMM / icvTeleaInpaintFMM restated): bucketed parallel fast
 *       march + colours in dependency levels.
 *   ofd_inpaint_workspace_bytes, ofd_inpaint_seq_workspace_bytes
 *       no reference counterpart (cv2 allocates its fast-marching state per
 *       call); caller-owned scratch, no initialisation needed.
 *   ofd_inpaint_seq_helper_device, ofd_inpaint_seq_set_pipeline,
 *   ofd_inpaint_seq_set_colour, ofd_inpaint_seq_set_multi
 *       no reference counterpart: the device whose helper stream a call
 *       would use, the record / colour rounds pipelined beside the fast
 *       marches, and the colour pass's form and workgroups per image
 *       (results never depend on any of them).
 *   ofd_inpaint_set_schedule
 *       no reference counterpart: diagnostics / tests only (how many hole
 *       layers are launched one by one before the deep-tail
 *       kernel takes over, and the layer size below which every hole takes the
 *       wave-per-hole path).  Results never depend on it.
 *
 * The call never blocks the host: every launch reads its layer's size from
 * the device.  The host sizes grids and the number of per-layer launches from
 * the layer histograms of recent calls at the same shape (the elementwise
 * maximum over the last 8), read back asynchronously (pinned memory + event,
 * used once it has arrived); layers beyond those launches run in one
 * persistent kernel with grid barriers.
 */
#ifndef OFD_INPAINT_H
#define OFD_INPAINT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bytes of workspace for a call over B images of H x W (any size of at least
 * one image's share works; larger workspaces process more images per launch). */
size_t ofd_inpaint_workspace_bytes(int64_t B, int64_t H, int64_t W);

/* utils.inpaint, batched.  img / out [B,C,H,W] f32 (out holds uint8 values),
 * valid / collision [B,1,H,W] f32.  radius = cv2 inpaintRange (3 in the
 * reference), clamped to [1, 100].  Requires H >= 2, W >= 2 (OFD_FW_EINVAL)
 * and H + W <= 4096 (OFD_FW_ETOOBIG).  out must not alias img. */
int ofd_inpaint_telea_f32(const float *img, const float *valid, const float *collision, float *out,
                          int64_t B, int64_t C, int64_t H, int64_t W, int radius, void *workspace,
                          size_t workspace_bytes, void *stream);

/* Bytes of workspace for ofd_inpaint_telea_seq_f32 over B images of H x W
 * (about 212 bytes per padded pixel: stamps, distances, push log and sort
 * buffers, 160-byte per-hole colour records and the packed colour image of
 * the radius-3 path; any size of at least one image's share works, larger
 * ones process more images per launch -- the fill is latency-bound per
 * image, so a whole batch per launch is the fast choice on 288 GB). */
size_t ofd_inpaint_seq_workspace_bytes(int64_t B, int64_t H, int64_t W);

/* utils.inpaint, batched, in cv2's exact order: the same arguments and
 * conventions as ofd_inpaint_telea_f32, but the fill follows the sequential
 * fast march of cv2.inpaint(..., INPAINT_TELEA) (utils.py:149) -- heap pops in
 * (distance, push order), each pushed hole coloured from the pixels reached
 * before it -- and is bit-exact against its CPU restatement
 * oracle/inpaint_oracle.c (sequential mode).  cv2 itself is absent from the
 * build image, so parity with OpenCV's binary is pinned only through that
 * restatement of OpenCV's published source.  Requires H >= 2, W >= 2 and
 * (H+2)(W+2) < 2^30 (OFD_FW_ETOOBIG).  Asynchronous on `stream`; never blocks
 * the host. */
int ofd_inpaint_telea_seq_f32(const float *img, const float *valid, const float *collision, float *out,
                              int64_t B, int64_t C, int64_t H, int64_t W, int radius, void *workspace,
                              size_t workspace_bytes, void *stream);

/* The pipelined sequential fill (radius 3, C <= 3 -- utils.inpaint's call --
 * on images of at least 2^18 pixels): `rounds` record / colour rounds run on
 * a helper stream beside the fast marches, `round_us` apart, over the holes
 * the inner march has finished (once the image's outer march is done); each
 * colour round stops at the next round's start and carries its frontier
 * over, and the final round after the marches takes the rest.  rounds = 0
 * runs the record and colour passes after the marches only.  force = 1
 * pipelines smaller images too (tests).  Results never depend on any of it.
 * Negative values leave a setting as it is, round_us = 0 restores its
 * default; defaults OFD_SEQ_PIPE (else 12) and OFD_SEQ_PIPE_US (else 2000).
 * Process-wide; returns the previous number of rounds. */
int ofd_inpaint_seq_set_pipeline(int rounds, int round_us, int force);

/* The sequential fill's colour pass: mode 1 = levels-free (a hole is
 * coloured as soon as every earlier hole it reads is; no level barrier),
 * 0 = level-synchronous (one workgroup barrier per Kahn level).  Results
 * never depend on it.  Negative: leave it; default OFD_SEQ_DF (else 1).
 * Process-wide; returns the previous mode. */
int ofd_inpaint_seq_set_colour(int mode);

/* Workgroups per image of the sequential fill's levels-free colour pass
 * (images of at least 2^18 pixels): 1 = one 1024-thread workgroup per image
 * (one CU); k > 1 = k workgroups of 512 threads sharing the image's ready
 * queue (k CUs: the colour pass is VALU-issue-bound on one).  Results are
 * identical for every k (default 4: 37.6 -> 35.5 ms per 64 warped 768x1024
 * images).  force != 0 applies k to smaller images too (tests;
 * k is lowered where an image has fewer than 4608 padded pixels per
 * workgroup).  workgroups < 1 only queries; default OFD_SEQ_MW.  Returns the
 * previous setting.  Process-wide. */
int ofd_inpaint_seq_set_multi(int workgroups, int force);

/* The device whose helper streams a grouped sequential fill on `stream`
 * would use: the stream's own device (helpers are kept per device and
 * created there on first use), or -1 if it cannot be told. */
int ofd_inpaint_seq_helper_device(void *stream);

/* Diagnostics: launch_layers >= 0 launches exactly that many hole layers one
 * by one (the deep-tail kernel does the rest); thin_cap >= 0 sets the layer
 * size up to which every hole takes the wave path.  -1 restores the
 * defaults (launches sized from an earlier call's depth; thin_cap 4096).
 * Process-wide; returns 0. */
int ofd_inpaint_set_schedule(int launch_layers, int thin_cap);

/* Test / debug hook: the OR of the invariant-violation bits any hole-fill
 * kernel raised since the last reset -- 2: a sequential-march bucket index
 * passed its bound; 4: a sequential distance sweep passed its iteration bound;
 * 8: the layered fill's deep tail gave up waiting for a previous layer;
 * 32: a bounded wait of the sequential fill's levels-free colour pass gave
 * up (a neighbour's colour or the ready queue).  Each is unreachable while the
 * algorithm's invariants hold, and each means that call's output is
 * incomplete.  Blocking (a device-to-host copy of the fault words); reset != 0
 * clears them.  Returns the bits (>= 0) or -1 on a HIP error. */
int ofd_inpaint_faults(int reset);

/* Diagnostic: how many hole layers the layered fill's deep-tail kernel has
 * run since the last reset (layers deeper than the launches the host sized
 * from recent calls at the shape -- a call much deeper than the last 8 at its
 * shape).  The tail runs them on a small persistent grid, layer after layer
 * (a wait per layer instead of a launch): results are unchanged.  Blocking;
 * reset != 0 clears the count.  Returns the count (>= 0) or -1 on a HIP
 * error. */
int ofd_inpaint_tail_layers(int reset);

#ifdef __cplusplus
}
#endif

#endif /* OFD_INPAINT_H */
