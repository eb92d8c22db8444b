// ofd_inpaint_seq.hip -- MI355X (gfx950) hole-fill in cv2's exact order.
//
// Replaces utils.inpaint (utils.py:136-151) with results equal to cv2's
// sequential Telea fast march (cv2.inpaint(..., 3, cv2.INPAINT_TELEA), :149)
// as restated by oracle/inpaint_oracle.c (sequential mode): the same pop
// order, distances, and colours, bit for bit.
//
// cv2 pops the band pixel of least (T, push order) from a heap; each pop
// gives its INSIDE 4-neighbours a distance (FastMarching_solve over the
// neighbours reached so far), a colour (Telea's weighted window over the
// pixels reached so far) and pushes them.  Two facts make that order
// reproducible in parallel:
//
//  1. A pushed pixel's distance is at least the popped one's + 1/sqrt(2)
//     (every reached neighbour of an INSIDE pixel is a heap member with
//     T >= the current minimum, and FastMarching_solve adds >= 0.7071 to the
//     smaller argument).  So the pops with T in [k/2, (k+1)/2) are exactly
//     the heap's contents in that range when the range becomes the minimum:
//     none of them pushes anything into its own range.  FMM runs one such
//     bucket at a time: sort the bucket by (T, push order), let every pop
//     claim its INSIDE neighbours (atomicMin over (pop rank, direction): the
//     first claimant is the pusher, as in the serial loop), number the pushes
//     in (rank, direction) order -- cv2's push order -- and solve their
//     distances.  A push may read a neighbour pushed earlier in the same
//     bucket, so the distances are iterated to a fixed point (the system is
//     acyclic in push order, so a sweep with no change is the exact answer).
//  2. Colours do not steer the march: T and the push order depend on the
//     mask only.  With every pixel's push stamp known, a hole's colour reads
//     exactly the holes of smaller stamp in its window (cv2's INSIDE test is
//     "not pushed yet"), so COLOUR evaluates the holes in dependency levels
//     (Kahn's algorithm: a hole runs once every earlier-stamped hole in its
//     window has), all holes of a level in parallel.
//
// Launches per chunk of images (one workgroup per image for the two
// sequential phases):
//   PREP   per pixel: keep mask (utils.py:137-142), out = float(uint8(img)),
//          inner stamps (INF = hole).
//   INIT   one wave per padded row: frame, band (4-adjacent to a hole),
//          outer ring (a hole within Chebyshev `range`), t, owner keys; band
//          count per row.
//   BAND   row offsets, then the band pixels in raster order (cv2 pushes them
//          in that order with T = 0).
//   FMM    per image: the outer march over the ring (icvCalcFMM with negate),
//          its distances negated, then the inner march over the holes.
//   COUNT  per pixel: earlier-stamped holes in the window; level-0 holes.
//   COLOUR per image: Kahn levels, cv2's Telea colour per hole.
//
// Plain HIP for gfx950; FP contraction off so the float / double sequence is
// the oracle's (and OpenCV's source's).

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include <mutex>

#include "ofd_fw.h"
#include "ofd_inpaint.h"

#pragma clang fp contract(off)

// Fault bits of the sequential fill (ofd_inpaint_faults): 2 = a march bucket
// index past its bound, 4 = a distance sweep past its iteration bound (both
// unreachable while the margin argument holds; the kernel stops early and the
// output is incomplete, so a set bit means a wrong result), 32 = a bounded
// wait of the levels-free colour pass gave up (a hole may then be coloured
// from uncoloured neighbours, or left unfilled).
__device__ unsigned g_sq_fault;

namespace {

#include "ip_common.h"

// Probe build only (-DOFD_SQ_PROF, tools/seq_probe.sh): thread 0 of each
// workgroup accumulates shader-clock intervals of its own work into meta[8..].
#ifdef OFD_SQ_PROF
__device__ __forceinline__ uint64_t sq_clock() {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    return __builtin_amdgcn_s_memtime();
}
#define SQ_T(var) uint64_t var = (threadIdx.x == 0) ? sq_clock() : 0
#define SQ_ACC(slot, a, b) do { if (threadIdx.x == 0) prof[slot] += (b) - (a); } while (0)
#else
#define SQ_T(var) do { } while (0)
#define SQ_ACC(slot, a, b) do { } while (0)
#endif

constexpr uint32_t INF = 0xFFFFFFFFu;
constexpr int kThreads = 1024;     // FMM workgroup
constexpr int kColThreads = 256;  // COLOUR workgroup of the any-radius path
constexpr int kCap = 4096;      // bucket keys sorted in LDS; larger buckets merge in global memory
constexpr int kLdsPush = 2048;  // pushes per bucket whose distance sweeps run in LDS
constexpr int kMaxRange = 100;
constexpr int kMeta = 32;  // per image: 0 band count, 1 pushes, 2 frontier count, 3 levels, 4 buckets, 5 error, 6 COLOUR3 rounds, 7 COLOUR3 levels <= 64 holes,
                          // 8..15 FMM / 16..23 COLOUR probe clocks (>> 8)

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// per-image arrays over the padded (H+2) x (W+2) grid (cv2's one-pixel KNOWN frame)
struct SqWs {
    uint32_t *sO;    // outer march stamps: INF = ring pixel not reached yet, else push seq (0 = never in heap)
    uint32_t *sI;    // inner march stamps: INF = hole not reached yet, else push seq (0 = known)
    uint32_t *own;   // FMM: claiming (rank * 4 + direction); COLOUR: pending dependencies
    float *t;        // distances (cv2's t; 1e6 far)
    uint32_t *logp;  // push log: pixel of push seq s (band first, raster order)
    float *logt;     // push log: T of push seq s
    uint64_t *k0;    // large-bucket sort buffers; COLOUR frontiers
    uint64_t *k1;
    uint32_t *rowc;  // band count / offset per padded row
    uint32_t *meta;  // kMeta words per image
    uint32_t *rec;   // radius-3 COLOUR: kRecW words per hole, indexed by padded pixel
    uint32_t *shd;   // radius-3 COLOUR: the image as packed uint8 channels (C <= 3), H x W words
    uint64_t *fr2;   // radius-3 COLOUR: frontier buffers (entries beyond the LDS capacity)
    uint64_t *fr3;
    uint32_t *olog;  // outer march: push log (en), its T (en), sort buffers (2 x 2 en)
    uint32_t *rpx;   // large buckets' pops by rank: inner (en), outer (en)
    uint32_t *kc;    // radius-3 COLOUR: Kahn counters (kK - earlier holes, + 1 per release)
    uint64_t *rq;    // radius-3 COLOUR: holes RECORD found ready (pixel << 32 | pixel)
    uint64_t *cy;    // radius-3 COLOUR: the frontier a time-bounded round carries to the next
    uint32_t *pipe;  // kPipe words per image: pipelined fill control (kP* below)
    int64_t en, eh, ew, hw;
};

// Pipelined fill control words (per image, kPipe words = two 128-byte lines
// apart from meta): the march publishes the first line, the pacing kernel
// owns the second (different writers never share a cache line).
constexpr int kPipe = 64;
constexpr int kPProg = 0;      // inner march: log entries [0, prog) final (release-published)
constexpr int kPOutDone = 1;   // outer march done (its distances negated), release-published
constexpr int kPInDone = 2;    // inner march done
constexpr int kPRecDone = 32;  // holes of stamp < recdone recorded
constexpr int kPLo = 33, kPHi = 34;  // the current RECORD window of stamps [lo, hi)
constexpr int kPRqc = 35;      // ready-queue entries COLOUR3 has consumed
constexpr int kPT0 = 36;       // image 0: the pacing clock origin (2 words)
// timeline (constant-rate clock, 2 words each; tools/seq_time.py): FMM start,
// outer march end, inner march end (march's line); first and last COLOUR3
// round with work, rounds with work (pacing line)
constexpr int kPTFmm = 8, kPTOut = 10, kPTIn = 12, kPTc0 = 40, kPTc1 = 42, kPCRounds = 44;
constexpr int kPCarry = 46;    // frontier entries a COLOUR3 round left in cy for the next
constexpr int kPAllDone = 60;   // image 0: every march of the chunk was done at this round's snapshot (PACE)
constexpr int kPB0Out = 4, kPB0In = 5;  // pushes of bucket 0 (the band) of the outer / inner march (BAND PUSH)
__device__ __forceinline__ void put64(uint32_t *p, uint64_t v) {
    p[0] = uint32_t(v);
    p[1] = uint32_t(v >> 32);
}
constexpr uint32_t kK = 64;    // a hole is ready when its counter reaches kK (> 60 earlier holes)

constexpr int kRecW = 40;  // record words: 32 weights (lane-major), 4 code words, dependants mask (2), weight sum, pad

size_t per_image_bytes(int64_t H, int64_t W) {
    const size_t en = size_t(H + 2) * size_t(W + 2);
    return align256(en * 4) * 6 + align256(en * 8) * 2 + align256(size_t(H + 2) * 4) + kMeta * 4 +
           en * kRecW * 4 + size_t(H) * size_t(W) * 4 + en * 8 + 3 * 256 +
           en * 8 + en * 4 * 6 + en * 4 * 2 + en * 4 + en * 8 + en * 8 + kPipe * 4 + 8 * 256;
}

SqWs carve(void *ws, int64_t G, int64_t H, int64_t W) {
    SqWs w;
    w.eh = H + 2;
    w.ew = W + 2;
    w.en = w.eh * w.ew;
    const size_t n4 = align256(size_t(G) * size_t(w.en) * 4), n8 = align256(size_t(G) * size_t(w.en) * 8);
    char *p = static_cast<char *>(ws);
    w.sO = reinterpret_cast<uint32_t *>(p), p += n4;
    w.sI = reinterpret_cast<uint32_t *>(p), p += n4;
    w.own = reinterpret_cast<uint32_t *>(p), p += n4;
    w.t = reinterpret_cast<float *>(p), p += n4;
    w.logp = reinterpret_cast<uint32_t *>(p), p += n4;
    w.logt = reinterpret_cast<float *>(p), p += n4;
    w.k0 = reinterpret_cast<uint64_t *>(p), p += n8;
    w.k1 = reinterpret_cast<uint64_t *>(p), p += n8;
    w.rowc = reinterpret_cast<uint32_t *>(p), p += align256(size_t(G) * size_t(w.eh) * 4);
    w.meta = reinterpret_cast<uint32_t *>(p), p += align256(size_t(G) * kMeta * 4);
    w.hw = H * W;
    w.rec = reinterpret_cast<uint32_t *>(p), p += align256(size_t(G) * size_t(w.en) * kRecW * 4);
    w.shd = reinterpret_cast<uint32_t *>(p), p += align256(size_t(G) * size_t(w.hw) * 4);
    w.fr2 = reinterpret_cast<uint64_t *>(p), p += align256(size_t(G) * size_t(w.en) * 8);
    w.fr3 = reinterpret_cast<uint64_t *>(p), p += align256(size_t(G) * size_t(w.en) * 8);
    w.olog = reinterpret_cast<uint32_t *>(p), p += align256(size_t(G) * size_t(w.en) * 4 * 6);
    w.rpx = reinterpret_cast<uint32_t *>(p), p += align256(size_t(G) * size_t(w.en) * 4 * 2);
    w.kc = reinterpret_cast<uint32_t *>(p), p += align256(size_t(G) * size_t(w.en) * 4);
    w.rq = reinterpret_cast<uint64_t *>(p), p += align256(size_t(G) * size_t(w.en) * 8);
    w.cy = reinterpret_cast<uint64_t *>(p), p += align256(size_t(G) * size_t(w.en) * 8);
    w.pipe = reinterpret_cast<uint32_t *>(p);
    return w;
}

// One image's view of the workspace
struct Img {
    uint32_t *sO, *sI, *own, *logp, *rowc, *meta, *rec, *shd, *olog, *rpx, *kc, *pipe;
    float *t, *logt;
    uint64_t *k0, *k1, *fr2, *fr3, *rq, *cy;
    int64_t en;
    int eh, ew;
};

__device__ __forceinline__ Img image(const SqWs &w, int64_t bl) {
    Img m;
    m.sO = w.sO + bl * w.en;
    m.sI = w.sI + bl * w.en;
    m.own = w.own + bl * w.en;
    m.t = w.t + bl * w.en;
    m.logp = w.logp + bl * w.en;
    m.logt = w.logt + bl * w.en;
    m.k0 = w.k0 + bl * w.en;
    m.k1 = w.k1 + bl * w.en;
    m.rowc = w.rowc + bl * w.eh;
    m.meta = w.meta + bl * kMeta;
    m.rec = w.rec + bl * w.en * kRecW;
    m.shd = w.shd + bl * w.hw;
    m.fr2 = w.fr2 + bl * w.en;
    m.fr3 = w.fr3 + bl * w.en;
    m.olog = w.olog + bl * w.en * 6;
    m.rpx = w.rpx + bl * w.en * 2;
    m.kc = w.kc + bl * w.en;
    m.rq = w.rq + bl * w.en;
    m.cy = w.cy + bl * w.en;
    m.pipe = w.pipe + bl * kPipe;
    m.en = w.en;
    m.eh = int(w.eh);
    m.ew = int(w.ew);
    return m;
}

// Workgroup barrier after which every thread of the workgroup sees the
// others' global stores and atomics.  Workgroup scope suffices: an image's
// march and colours run inside one workgroup, whose waves share one CU and
// its vector L1 (not in threadgroup-split mode), so no L2 write-back or L1
// invalidation is needed -- agent scope would emit both (buffer_wbl2 /
// buffer_inv) on every level, which measured 4-7 us per load round.
__device__ __forceinline__ void sync_all() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Exclusive scan of one value per thread over the 1024-thread workgroup.
__device__ __forceinline__ uint32_t block_scan(uint32_t v, uint32_t &total, uint32_t *scr /* [40] LDS */) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) scr[wave] = incl;
    __syncthreads();
    if (tid < 64) {
        const uint32_t w = tid < kThreads / 64 ? scr[tid] : 0u;
        uint32_t wi = w;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint32_t o = __shfl_up(wi, d);
            if (lane >= d) wi += o;
        }
        if (tid < kThreads / 64) scr[16 + tid] = wi - w;
        if (tid == kThreads / 64 - 1) scr[32] = wi;
    }
    __syncthreads();
    const uint32_t r = incl - v + scr[16 + wave];
    total = scr[32];
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------- PREP
// utils.py:137-142: M = valid != coll; M' = 3x3 max (border excluded);
// P = M' == M; H' = uint8(valid * P); fill where 1 - H' != 0.  Writes the
// uint8 cast of every channel (utils.py:148) and sI (INF = hole, 0 = known)
// at the padded position.
// On 64 x 16 tiles: M = valid != coll of the tile and a one-pixel halo in
// LDS (read once), so the 3 x 3 maximum costs LDS reads instead of 18 global
// loads per pixel (0.70 ms per 64 images of 768 x 1024 before).  Also zeroes
// the band counts (rowc) the tiled INIT accumulates.
__global__ __launch_bounds__(256) void sq_prep_tile_kernel(const float *__restrict__ img,
                                                           const float *__restrict__ valid,
                                                           const float *__restrict__ coll, float *__restrict__ out,
                                                           SqWs w, int C, int H, int W, int64_t b0, int shadow) {
    constexpr int TW = 64, TH = 16;
    __shared__ uint8_t Mt[TH + 2][TW + 2];
    const int x0 = int(blockIdx.x) * TW, y0 = int(blockIdx.y) * TH;
    const int64_t HW = int64_t(H) * W, bl = blockIdx.z, b = b0 + bl;
    const float *v = valid + b * HW, *cl = coll + b * HW;
    for (int e = threadIdx.x; e < (TH + 2) * (TW + 2); e += 256) {
        const int ry = e / (TW + 2), rx = e - ry * (TW + 2);
        const int y = y0 - 1 + ry, x = x0 - 1 + rx;
        uint8_t mv = 0;
        if (y >= 0 && y < H && x >= 0 && x < W) {
            const int64_t q = int64_t(y) * W + x;
            mv = v[q] != cl[q] ? 1 : 0;
        }
        Mt[ry][rx] = mv;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x = x0 + lane;
    if (x == 0 && blockIdx.x == 0)  // rowc: padded rows y + 1 of this tile, and 0, H + 1
        for (int ly = wave; ly < TH; ly += 4) {
            const int y = y0 + ly;
            if (y < H) {
                uint32_t *rc = w.rowc + bl * w.eh;
                rc[y + 1] = 0u;
                if (y == 0) rc[0] = rc[H + 1] = 0u;
            }
        }
    if (x >= W) return;
    const float *ib = img + b * int64_t(C) * HW;
    float *ob = out + b * int64_t(C) * HW;
    for (int ly = wave; ly < TH; ly += 4) {
        const int y = y0 + ly;
        if (y >= H) break;
        const int64_t p = int64_t(y) * W + x;
        unsigned mp = 0;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) mp |= Mt[ly + dy][lane + dx];
        const unsigned M = Mt[ly + 1][lane + 1];
        const unsigned P = mp == M ? 1u : 0u;
        const unsigned hp = to_u8(v[p] * float(P));
        w.sI[bl * w.en + int64_t(y + 1) * w.ew + (x + 1)] = hp != 1u ? INF : 0u;
        uint32_t pk = 0;
        for (int c = 0; c < C; ++c) {
            const unsigned u = to_u8(ib[c * HW + p]);
            if (shadow)
                pk |= u << (8 * c);  // C <= 3; sq_unpack_kernel writes out
            else
                ob[c * HW + p] = float(u);
        }
        // (byte 3: the coloured flag of the levels-free colour pass -- set on
        // kept pixels, by the colour store on holes; no other reader)
        if (shadow) w.shd[bl * w.hw + p] = pk | (hp == 1u ? 0xFF000000u : 0u);
    }
}

// ---------------------------------------------------------------- INIT
// One wave per padded row.  Holes are read by coordinates (the frame is never
// a hole), so the frame entries this kernel writes are never read here.
__global__ __launch_bounds__(256) void sq_init_kernel(SqWs w, int range) {
    const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const Img m = image(w, blockIdx.y);
    if (i >= m.eh) return;
    const int eh = m.eh, ew = m.ew;
    auto hole = [&](int y, int x) -> bool {
        return y > 0 && x > 0 && y < eh - 1 && x < ew - 1 && m.sI[int64_t(y) * ew + x] == INF;
    };
    uint32_t nband = 0;
    for (int j0 = 0; j0 < ew; j0 += 64) {
        const int j = j0 + lane;
        bool band = false;
        if (j < ew) {
            const int64_t p = int64_t(i) * ew + j;
            const bool frame = i == 0 || j == 0 || i == eh - 1 || j == ew - 1;
            bool ring = false;
            if (!frame && !hole(i, j)) {
                band = hole(i - 1, j) || hole(i + 1, j) || hole(i, j - 1) || hole(i, j + 1);
                if (!band)
                    for (int y = i - range; y <= i + range && !ring; ++y)
                        for (int x = j - range; x <= j + range; ++x)
                            if (hole(y, x)) {
                                ring = true;
                                break;
                            }
            }
            if (frame) m.sI[p] = 0u;
            m.sO[p] = ring ? INF : 0u;
            m.t[p] = band ? 0.f : T_FAR;
            m.own[p] = INF;
            m.kc[p] = 0u;
        }
        nband += __popcll(__ballot(band));
    }
    if (lane == 0) m.rowc[i] = nband;
}

// The same for range <= kInitR, on 64 x 16 tiles of the padded grid: the
// tile's hole flags with a range-wide halo in LDS, the window test as a
// horizontal then a vertical OR (separable), so a pixel costs ~2 (2r + 1)
// LDS reads instead of (2r + 1)^2 global ones (the row kernel above read the
// 7 x 7 window from memory for every pixel far from a hole: 1.6 ms per 64
// images of 768 x 1024).  Band counts per row go to rowc by one atomic per
// wave-row (PREP zeroed rowc).
constexpr int kInitTW = 64, kInitTH = 16, kInitR = 8;
__global__ __launch_bounds__(256) void sq_init_tile_kernel(SqWs w, int range) {
    constexpr int XW = kInitTW + 2 * kInitR, YH = kInitTH + 2 * kInitR;
    __shared__ uint8_t hf[YH][XW];        // hole flags, tile + halo
    __shared__ uint8_t hor[YH][kInitTW];  // OR over [x - r, x + r] of each halo row
    const Img m = image(w, blockIdx.z);
    const int eh = m.eh, ew = m.ew, r = range;
    const int i0 = int(blockIdx.y) * kInitTH, j0 = int(blockIdx.x) * kInitTW;
    const int xw = kInitTW + 2 * r, yh = kInitTH + 2 * r;
    for (int e = threadIdx.x; e < xw * yh; e += 256) {
        const int ry = e / xw, rx = e - ry * xw;
        const int y = i0 - r + ry, x = j0 - r + rx;
        const bool h = y > 0 && x > 0 && y < eh - 1 && x < ew - 1 && m.sI[int64_t(y) * ew + x] == INF;
        hf[ry][rx] = h ? 1 : 0;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < yh * kInitTW; e += 256) {
        const int ry = e / kInitTW, cx = e - ry * kInitTW;
        uint8_t o = 0;
        for (int d = 0; d <= 2 * r; ++d) o |= hf[ry][cx + d];
        hor[ry][cx] = o;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j = j0 + lane;
    for (int li = wave; li < kInitTH; li += 4) {
        const int i = i0 + li;
        if (i >= eh) break;  // wave-uniform
        bool band = false;
        if (j < ew) {
            const int64_t p = int64_t(i) * ew + j;
            const bool frame = i == 0 || j == 0 || i == eh - 1 || j == ew - 1;
            const int hy = li + r, hx = lane + r;  // the pixel in hf
            bool ring = false;
            if (!frame && !hf[hy][hx]) {
                band = hf[hy - 1][hx] || hf[hy + 1][hx] || hf[hy][hx - 1] || hf[hy][hx + 1];
                if (!band)
                    for (int d = 0; d <= 2 * r; ++d) ring = ring || hor[li + d][lane];
            }
            if (frame) m.sI[p] = 0u;
            m.sO[p] = ring ? INF : 0u;
            m.t[p] = band ? 0.f : T_FAR;
            m.own[p] = INF;
            m.kc[p] = 0u;
        }
        const unsigned nb = unsigned(__popcll(__ballot(band)));
        if (lane == 0 && nb) atomicAdd(&m.rowc[i], nb);
    }
}

// Row offsets of the band (exclusive scan over rows), one workgroup per image.
__global__ __launch_bounds__(kThreads) void sq_band_scan_kernel(SqWs w) {
    __shared__ uint32_t scr[40];
    const Img m = image(w, blockIdx.x);
    uint32_t carry = 0;
    for (int i0 = 0; i0 < m.eh; i0 += kThreads) {
        const int i = i0 + threadIdx.x;
        const uint32_t v = i < m.eh ? m.rowc[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_scan(v, tot, scr);
        if (i < m.eh) m.rowc[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        for (int k = 0; k < kMeta; ++k) m.meta[k] = 0u;
        m.meta[0] = carry;
        for (int k = 0; k < kPipe; ++k) m.pipe[k] = 0u;
    }
}

// Band pixels in raster order into the push log (cv2's Heap->Add, T = 0).
__global__ __launch_bounds__(256) void sq_band_write_kernel(SqWs w) {
    const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const Img m = image(w, blockIdx.y);
    if (i >= m.eh) return;
    uint32_t off = m.rowc[i];
    for (int j0 = 0; j0 < m.ew; j0 += 64) {
        const int j = j0 + lane;
        const int64_t p = int64_t(i) * m.ew + j;
        const bool band = j < m.ew && m.t[p] == 0.f;
        const uint64_t bal = __ballot(band);
        if (band) {
            const uint32_t s = off + __popcll(bal & ((uint64_t(1) << lane) - 1));
            m.logp[s] = uint32_t(p);
            m.logt[s] = 0.f;
            m.olog[s] = uint32_t(p);  // the outer march's log (outer_view)
            reinterpret_cast<float *>(m.olog + m.en)[s] = 0.f;
        }
        off += __popcll(bal);
    }
}

// ---------------------------------------------------------------- BAND PUSH
// Bucket 0 of both marches -- its claims, push numbering, stamps and log
// entries -- as raster passes over all images before FMM (one wave per
// padded row), instead of claim atomics and dependent log loads inside the
// one-workgroup marches (~1.6 ms of each march on the deep images).  Bucket 0
// pops the band, whose log is raster order, so a pixel's claimant -- its
// neighbour of least pop rank -- is its first band neighbour in raster order
// (up, left, right, down), and band pixel b pushes its INSIDE neighbour n in
// direction q exactly when no band neighbour of n precedes b:
//   q = 0 (n above b):    none of n's up, left, right neighbours is band;
//   q = 1 (n left of b):  neither n's up nor n's left neighbour is band;
//   q = 2 (n below b):    always (b is n's first neighbour);
//   q = 3 (n right of b): n's up neighbour is not band.
// Pushes are numbered in (rank, direction) order: the pushes of each padded
// row's band pixels (COUNT), an exclusive scan over the rows (SCAN), then
// each band pixel's pushes at its row's offset + the pushes of the row's
// earlier band pixels, in direction order (WRITE).  A pixel is band iff its
// distance is 0 (INIT).  The distances are left to the march's sweeps; the
// claim words (own) are not needed: a pushed pixel is never claimed again.
// blockIdx.z: 0 = the outer march (ring stamps sO, log olog), 1 = the inner
// march (hole stamps sI, log logp).
// Both marches on 64 x 16 tiles of the padded grid (a wave per row of the
// tile: one 64-pixel row chunk): the tile's band flags with a 2-pixel halo
// above and to the left and 1 to the right, and both marches' INSIDE flags
// with a 1-pixel halo, in LDS, so the rule reads LDS.  COUNT stores each row
// chunk's pushes, SCAN turns them into offsets in raster order (per image and
// march), WRITE numbers and stores the pushes in direction order.
constexpr int kBpTW = 64, kBpTH = 16;
struct BandPushLds {
    uint8_t band[kBpTH + 2][kBpTW + 3];  // rows i0 - 2 .., columns j0 - 2 .. j0 + 64
    uint8_t ins[kBpTH + 2][kBpTW + 2];   // rows i0 - 1 .., columns j0 - 1 .. j0 + 64: bit 0 outer INF, bit 1 inner INF
};

__device__ __forceinline__ void band_push_tile(const Img &m, int i0, int j0, BandPushLds &L) {
    const int eh = m.eh, ew = m.ew;
    for (int e = threadIdx.x; e < (kBpTH + 2) * (kBpTW + 3); e += 256) {
        const int r = e / (kBpTW + 3), c = e - r * (kBpTW + 3);
        const int y = i0 - 2 + r, x = j0 - 2 + c;
        L.band[r][c] = (y >= 0 && x >= 0 && y < eh && x < ew && m.t[int64_t(y) * ew + x] == 0.f) ? 1 : 0;
    }
    for (int e = threadIdx.x; e < (kBpTH + 2) * (kBpTW + 2); e += 256) {
        const int r = e / (kBpTW + 2), c = e - r * (kBpTW + 2);
        const int y = i0 - 1 + r, x = j0 - 1 + c;
        uint8_t f = 0;
        if (y >= 0 && x >= 0 && y < eh && x < ew) {
            const int64_t q = int64_t(y) * ew + x;
            f = uint8_t((m.sO[q] == INF ? 1 : 0) | (m.sI[q] == INF ? 2 : 0));
        }
        L.ins[r][c] = f;
    }
}

// push bits of tile pixel (li, lj) for the march whose INSIDE flag is bit mk
__device__ __forceinline__ unsigned band_push_bits(const BandPushLds &L, int li, int lj, unsigned mk) {
    const int br = li + 2, bc = lj + 2, ir = li + 1, ic = lj + 1;  // the pixel in band / ins
    if (!L.band[br][bc]) return 0u;
    const bool bu2 = L.band[br - 2][bc], bul = L.band[br - 1][bc - 1], bur = L.band[br - 1][bc + 1],
               bl2 = L.band[br][bc - 2];
    unsigned v = 0;
    v |= ((L.ins[ir - 1][ic] & mk) && !bu2 && !bul && !bur) ? 1u : 0u;
    v |= ((L.ins[ir][ic - 1] & mk) && !bul && !bl2) ? 2u : 0u;
    v |= (L.ins[ir + 1][ic] & mk) ? 4u : 0u;
    v |= ((L.ins[ir][ic + 1] & mk) && !bur) ? 8u : 0u;
    return v;
}

// wave-wide exclusive prefix and total of a 0..7 count, by bit planes
__device__ __forceinline__ uint32_t wave_scan_small(unsigned v, uint32_t &tot) {
    const uint64_t below = (uint64_t(1) << (threadIdx.x & 63)) - 1;
    uint32_t ex = 0;
    tot = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint64_t bal = __ballot((v >> k) & 1u);
        ex += uint32_t(__popcll(bal & below)) << k;
        tot += uint32_t(__popcll(bal)) << k;
    }
    return ex;
}

// the per-chunk counts / offsets (eh x nch words, a chunk = 64 columns of a
// row): the march's sort buffer, free until FMM
__device__ __forceinline__ uint32_t *band_push_chunks(const Img &m, bool inner) {
    return inner ? reinterpret_cast<uint32_t *>(m.k0) : m.olog + 2 * m.en;
}

// grid: (ceil(ew / 64), ceil(eh / 16), images)
__global__ __launch_bounds__(256) void sq_band_push_count_kernel(SqWs w) {
    __shared__ BandPushLds L;
    const Img m = image(w, blockIdx.z);
    const int i0 = int(blockIdx.y) * kBpTH, j0 = int(blockIdx.x) * kBpTW, c = int(blockIdx.x);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nch = (m.ew + 63) / 64;
    band_push_tile(m, i0, j0, L);
    __syncthreads();
    uint32_t *co = band_push_chunks(m, false), *ci = band_push_chunks(m, true);
    for (int li = wave; li < kBpTH; li += 4) {
        const int i = i0 + li;
        if (i >= m.eh) break;
        const bool in = i >= 1 && i < m.eh - 1 && j0 + lane < m.ew;
        uint32_t to, ti;
        (void)wave_scan_small(in ? unsigned(__popc(band_push_bits(L, li, lane, 1u))) : 0u, to);
        (void)wave_scan_small(in ? unsigned(__popc(band_push_bits(L, li, lane, 2u))) : 0u, ti);
        if (lane == 0) {
            co[int64_t(i) * nch + c] = to;
            ci[int64_t(i) * nch + c] = ti;
        }
    }
}

__global__ __launch_bounds__(kThreads) void sq_band_push_scan_kernel(SqWs w) {
    __shared__ uint32_t scr[40];
    const Img m = image(w, blockIdx.x);
    const bool inner = blockIdx.y != 0;
    uint32_t *cp = band_push_chunks(m, inner);
    const int64_t n = int64_t(m.eh) * ((m.ew + 63) / 64);
    uint32_t carry = 0;
    for (int64_t i0 = 0; i0 < n; i0 += kThreads) {
        const int64_t i = i0 + threadIdx.x;
        const uint32_t v = i < n ? cp[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_scan(v, tot, scr);
        if (i < n) cp[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) m.pipe[inner ? kPB0In : kPB0Out] = carry;
}

__global__ __launch_bounds__(256) void sq_band_push_write_kernel(SqWs w) {
    __shared__ BandPushLds L;
    const Img m = image(w, blockIdx.z);
    const int i0 = int(blockIdx.y) * kBpTH, j0 = int(blockIdx.x) * kBpTW, c = int(blockIdx.x);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, ew = m.ew, nch = (ew + 63) / 64;
    band_push_tile(m, i0, j0, L);
    __syncthreads();  // (every flag the rule reads is in LDS before any stamp store below)
    const int64_t off[4] = {-int64_t(ew), -1, int64_t(ew), 1};
    const uint32_t nb = m.meta[0];
    for (int li = wave; li < kBpTH; li += 4) {
        const int i = i0 + li;
        if (i >= m.eh) break;
        const bool in = i >= 1 && i < m.eh - 1 && j0 + lane < ew;
        const int64_t p = int64_t(i) * ew + j0 + lane;
#pragma unroll
        for (int mk = 0; mk < 2; ++mk) {
            const bool inner = mk != 0;
            const unsigned bits = in ? band_push_bits(L, li, lane, inner ? 2u : 1u) : 0u;
            uint32_t tot;
            uint32_t s = nb + band_push_chunks(m, inner)[int64_t(i) * nch + c] + wave_scan_small(unsigned(__popc(bits)), tot);
            uint32_t *st = inner ? m.sI : m.sO, *logp = inner ? m.logp : m.olog;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (bits & (1u << q)) {
                    st[p + off[q]] = s;
                    logp[s] = uint32_t(p + off[q]);
                    ++s;
                }
        }
    }
}

// INIT fused with bucket 0's push counts (range + 1 <= kInitR): the tile's
// hole flags with a halo of max(3, range + 1), so the band is known on the
// tile with a 2-pixel halo above / left and 1 right, and both marches'
// INSIDE flags (ring, hole) on the tile with a 1-pixel halo -- the BAND PUSH
// rule's inputs.  Besides INIT's outputs it stores, per 64-pixel row chunk,
// the band pixels (the band log's order) and the pushes of each march
// (sq_band3_scan_kernel, sq_band3_write_kernel take it from there; no row
// counts, no BAND / COUNT passes).
static_assert(kInitTW == kBpTW && kInitTH == kBpTH, "INIT and BAND PUSH share their tiles");
__device__ __forceinline__ uint32_t *band_chunks(const Img &m) { return reinterpret_cast<uint32_t *>(m.k1); }

__global__ __launch_bounds__(256) void sq_init_push_kernel(SqWs w, int range) {
    constexpr int XW = kInitTW + 2 * kInitR, YH = kInitTH + 2 * kInitR;
    __shared__ uint8_t hf[YH][XW];               // hole flags, tile + halo h
    __shared__ uint8_t hor[YH][kInitTW + 2];     // OR over the window's columns, for columns j0 - 1 .. j0 + 64
    __shared__ BandPushLds P;                    // band / INSIDE flags of the BAND PUSH rule
    const Img m = image(w, blockIdx.z);
    const int eh = m.eh, ew = m.ew, r = range, h = max(3, range + 1);
    const int i0 = int(blockIdx.y) * kInitTH, j0 = int(blockIdx.x) * kInitTW;
    const int xw = kInitTW + 2 * h, yh = kInitTH + 2 * h;
    for (int e = threadIdx.x; e < xw * yh; e += 256) {
        const int ry = e / xw, rx = e - ry * xw;
        const int y = i0 - h + ry, x = j0 - h + rx;
        hf[ry][rx] = (y > 0 && x > 0 && y < eh - 1 && x < ew - 1 && m.sI[int64_t(y) * ew + x] == INF) ? 1 : 0;
    }
    __syncthreads();
    // hor[ry][k]: a hole in columns (j0 - 1 + k) - r .. + r of halo row ry
    for (int e = threadIdx.x; e < yh * (kInitTW + 2); e += 256) {
        const int ry = e / (kInitTW + 2), k = e - ry * (kInitTW + 2);
        uint8_t o = 0;
        for (int d = 0; d <= 2 * r; ++d) o |= hf[ry][k + h - 1 - r + d];
        hor[ry][k] = o;
    }
    auto hole = [&](int y, int x) -> bool { return hf[y - i0 + h][x - j0 + h] != 0; };  // |y - i0|, |x - j0| in the halo
    auto bandp = [&](int y, int x) -> bool {
        return y > 0 && x > 0 && y < eh - 1 && x < ew - 1 && !hole(y, x) &&
               (hole(y - 1, x) || hole(y + 1, x) || hole(y, x - 1) || hole(y, x + 1));
    };
    for (int e = threadIdx.x; e < (kBpTH + 2) * (kBpTW + 3); e += 256) {
        const int rr = e / (kBpTW + 3), c = e - rr * (kBpTW + 3);
        P.band[rr][c] = bandp(i0 - 2 + rr, j0 - 2 + c) ? 1 : 0;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < (kBpTH + 2) * (kBpTW + 2); e += 256) {
        const int rr = e / (kBpTW + 2), c = e - rr * (kBpTW + 2);
        const int y = i0 - 1 + rr, x = j0 - 1 + c;
        bool ring = false;
        const bool hl = y > 0 && x > 0 && y < eh - 1 && x < ew - 1 && hole(y, x);
        if (y > 0 && x > 0 && y < eh - 1 && x < ew - 1 && !hl && !bandp(y, x))  // (row i0 + 16 is past P.band)
            for (int d = 0; d <= 2 * r && !ring; ++d) ring = hor[rr + h - 1 - r + d][c] != 0;
        P.ins[rr][c] = uint8_t((ring ? 1 : 0) | (hl ? 2 : 0));
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = j0 + lane, c = int(blockIdx.x);
    const int nch = (ew + 63) / 64;
    uint32_t *cb = band_chunks(m), *co = band_push_chunks(m, false), *ci = band_push_chunks(m, true);
    for (int li = wave; li < kInitTH; li += 4) {
        const int i = i0 + li;
        if (i >= eh) break;  // wave-uniform
        bool band = false;
        unsigned po = 0, pi = 0;
        if (j < ew) {
            const int64_t p = int64_t(i) * ew + j;
            const bool frame = i == 0 || j == 0 || i == eh - 1 || j == ew - 1;
            band = P.band[li + 2][lane + 2] != 0;
            if (frame) m.sI[p] = 0u;
            m.sO[p] = (P.ins[li + 1][lane + 1] & 1u) ? INF : 0u;
            m.t[p] = band ? 0.f : T_FAR;
            m.own[p] = INF;
            m.kc[p] = 0u;
            po = band_push_bits(P, li, lane, 1u);
            pi = band_push_bits(P, li, lane, 2u);
        }
        uint32_t tb, to, ti;
        (void)wave_scan_small(band ? 1u : 0u, tb);
        (void)wave_scan_small(unsigned(__popc(po)), to);
        (void)wave_scan_small(unsigned(__popc(pi)), ti);
        if (lane == 0) {
            cb[int64_t(i) * nch + c] = tb;
            co[int64_t(i) * nch + c] = to;
            ci[int64_t(i) * nch + c] = ti;
        }
    }
}

// Offsets of the three per-chunk counts (band, outer pushes, inner pushes) in
// raster order, one workgroup per image; also the per-fill meta / pipe reset
// (sq_band_scan_kernel's) with the band's size in meta[0].
__global__ __launch_bounds__(kThreads) void sq_band3_scan_kernel(SqWs w) {
    __shared__ uint32_t scr[40];
    const Img m = image(w, blockIdx.x);
    const int64_t n = int64_t(m.eh) * ((m.ew + 63) / 64);
    uint32_t tot3[3];
    for (int a = 0; a < 3; ++a) {
        uint32_t *cp = a == 0 ? band_chunks(m) : band_push_chunks(m, a == 2);
        uint32_t carry = 0;
        for (int64_t i0 = 0; i0 < n; i0 += kThreads) {
            const int64_t i = i0 + threadIdx.x;
            const uint32_t v = i < n ? cp[i] : 0u;
            uint32_t tot;
            const uint32_t ex = block_scan(v, tot, scr);
            if (i < n) cp[i] = carry + ex;
            carry += tot;
        }
        tot3[a] = carry;
    }
    if (threadIdx.x == 0) {
        for (int k = 0; k < kMeta; ++k) m.meta[k] = 0u;
        for (int k = 0; k < kPipe; ++k) m.pipe[k] = 0u;
        m.meta[0] = tot3[0];
        m.pipe[kPB0Out] = tot3[1];
        m.pipe[kPB0In] = tot3[2];
    }
}

// The band log (raster order, T = 0, both marches' logs) and bucket 0's
// pushes, on INIT's tiles: the rule's flags come from INIT's outputs (band:
// distance 0; INSIDE: stamp INF), read before any stamp store of this
// workgroup (only a pixel's claimant pushes it: another workgroup's stores
// cannot change a bit this one computes).
__global__ __launch_bounds__(256) void sq_band3_write_kernel(SqWs w) {
    __shared__ BandPushLds L;
    const Img m = image(w, blockIdx.z);
    const int i0 = int(blockIdx.y) * kBpTH, j0 = int(blockIdx.x) * kBpTW, c = int(blockIdx.x);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, ew = m.ew, nch = (ew + 63) / 64;
    band_push_tile(m, i0, j0, L);
    __syncthreads();
    const int64_t off[4] = {-int64_t(ew), -1, int64_t(ew), 1};
    const uint32_t nb = m.meta[0];
    float *ologt = reinterpret_cast<float *>(m.olog + m.en);
    for (int li = wave; li < kBpTH; li += 4) {
        const int i = i0 + li;
        if (i >= m.eh) break;
        const bool in = i >= 1 && i < m.eh - 1 && j0 + lane < ew;
        const int64_t p = int64_t(i) * ew + j0 + lane;
        const int64_t ck = int64_t(i) * nch + c;
        {
            const bool band = in && L.band[li + 2][lane + 2];
            uint32_t tot;
            const uint32_t s = band_chunks(m)[ck] + wave_scan_small(band ? 1u : 0u, tot);
            if (band) {
                m.logp[s] = uint32_t(p);
                m.logt[s] = 0.f;
                m.olog[s] = uint32_t(p);
                ologt[s] = 0.f;
            }
        }
#pragma unroll
        for (int mk = 0; mk < 2; ++mk) {
            const bool inner = mk != 0;
            const unsigned bits = in ? band_push_bits(L, li, lane, inner ? 2u : 1u) : 0u;
            uint32_t tot;
            uint32_t s = nb + band_push_chunks(m, inner)[ck] + wave_scan_small(unsigned(__popc(bits)), tot);
            uint32_t *st = inner ? m.sI : m.sO, *logp = inner ? m.logp : m.olog;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (bits & (1u << q)) {
                    st[p + off[q]] = s;
                    logp[s] = uint32_t(p + off[q]);
                    ++s;
                }
        }
    }
}

// ---------------------------------------------------------------- FMM
constexpr int kHash = 1024;  // distinct-distance sort of large buckets: hash slots
constexpr int kMaxD = 256;   // ... and distinct distances it handles (else the merge sort)

struct FmmLds {
    uint64_t keys[kCap];
    uint64_t keys2[kCap];  // LDS sort ping-pong
    uint32_t scr[40];
    uint32_t tmin, tmax, chg;
    uint32_t chg3[3];  // the LDS distance sweeps' change flags (one barrier per sweep)
    uint32_t hk[kHash], hd[kHash], hc[kHash];  // distinct distance, its rank, its count
    uint32_t wc[kThreads / 64][kMaxD];         // per wave: keys of each rank in the current chunk
    uint32_t base[kMaxD], dv[kMaxD];
    uint32_t nd, ovf;
};

// Bucket k holds T in [k w, (k + 1) w) with w = 1 / bscale.  A push lands at
// least 1/sqrt(2) above the bucket's smallest pop (less float rounding of T:
// half an ulp, under 2^-11 for T < 8192), so any w <= 0.7 keeps every push
// out of its own bucket: w = 0.7 while H + W < 8000 bounds T, else 0.5.
// (Double product: the bucket edges are exact to far below the margin.)
__device__ __forceinline__ uint32_t bucket_of(float T, double bscale) { return uint32_t(double(T) * bscale); }

// distance of padded pixel p pushed with seq s: FastMarching_solve over the
// neighbours reached before it (stamp < s); cv2's fm order (up/left,
// down/left, up/right, down/right)
// The inner march runs beside the outer one (sq_fmm_kernel), whose final
// negation turns the band's distances from +0 to -0 at some point during it;
// the inner march reads a band distance as the -0 it would see after the
// outer march (the only pixels with a zero distance are band pixels).
template <bool kInner>
__device__ __forceinline__ float band_t(float v) {
    return (kInner && v == 0.f) ? -0.f : v;
}

template <bool kInner>
__device__ __forceinline__ float fm_dist_seq(const uint32_t *st, const float *t, int64_t p, int ew, uint32_t s) {
    const int64_t nu = p - ew, nd = p + ew, nl = p - 1, nr = p + 1;
    const bool iu = st[nu] >= s, id = st[nd] >= s, il = st[nl] >= s, ir = st[nr] >= s;
    const float tu = iu ? T_FAR : band_t<kInner>(t[nu]), td = id ? T_FAR : band_t<kInner>(t[nd]),
                tl = il ? T_FAR : band_t<kInner>(t[nl]), tr = ir ? T_FAR : band_t<kInner>(t[nr]);
    return min4f(fm_solve(tu, iu, tl, il), fm_solve(td, id, tl, il), fm_solve(tu, iu, tr, ir),
                 fm_solve(td, id, tr, ir));
}

// bitonic sort of keys[0, m) in LDS, m a power of two
__device__ void lds_bitonic(uint64_t *s, int m) {
    for (int k = 2; k <= m; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < m; i += kThreads) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint64_t a = s[i], b = s[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        s[i] = b;
                        s[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int j) {
    const uint32_t lo = __shfl_xor(uint32_t(v), j), hi = __shfl_xor(uint32_t(v >> 32), j);
    return (uint64_t(hi) << 32) | lo;
}

// bitonic sort of one key per lane over the wave, ascending
__device__ __forceinline__ uint64_t wave_sort64(uint64_t v, int lane) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t o = shfl_xor64(v, j);
            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
            v = keep_min ? (o < v ? o : v) : (o > v ? o : v);
        }
    return v;
}

__device__ __forceinline__ uint32_t lower_bound64(const uint64_t *a, uint32_t n, uint64_t key);

// Sort keys[0, n) (unique), 1 < n <= kCap, in LDS: 64-key runs sorted in
// registers (wave shuffles, no barrier), then merge passes between the two
// LDS buffers (each key's place = its rank in its run + its rank in the
// partner run).  Returns the buffer holding the result.
__device__ uint64_t *lds_sort(FmmLds &L, uint32_t n) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint64_t *src = L.keys, *dst = L.keys2;
    for (uint32_t c = wave; c * 64 < n; c += kThreads / 64) {
        const uint32_t i = c * 64 + lane;
        uint64_t v = i < n ? src[i] : ~uint64_t(0);
        v = wave_sort64(v, lane);
        if (i < n) src[i] = v;
    }
    __syncthreads();
    for (uint32_t wdt = 64; wdt < n; wdt <<= 1) {
        for (uint32_t i = tid; i < n; i += kThreads) {
            const uint32_t lo = i / (2 * wdt) * (2 * wdt), mid = min(lo + wdt, n), hi = min(lo + 2 * wdt, n);
            const uint64_t key = src[i];
            const uint32_t pos = i < mid ? (i - lo) + lower_bound64(src + mid, hi - mid, key)
                                         : (i - mid) + lower_bound64(src + lo, mid - lo, key);
            dst[lo + pos] = key;
        }
        __syncthreads();
        uint64_t *tmp = src;
        src = dst;
        dst = tmp;
    }
    return src;
}

__device__ __forceinline__ uint32_t lower_bound64(const uint64_t *a, uint32_t n, uint64_t key) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t hslot0(uint32_t v) { return (v * 2654435761u) >> 22; }  // kHash = 1024

__device__ __forceinline__ uint32_t hfind(const FmmLds &L, uint32_t v) {
    uint32_t h = hslot0(v);
    while (L.hk[h] != v) h = (h + 1) & (kHash - 1);
    return h;
}

// Stable sort of n keys (distance bits << 32 | log index, in log index order)
// by distance when the bucket holds at most kMaxD distinct distances -- the
// big early buckets hold a handful (0.7071, 1, ...): count the distinct
// values in an LDS hash set, rank them, and scatter the keys in order, one
// 1024-key chunk at a time (rank within a value = earlier lanes of the wave
// with that value + earlier waves + earlier chunks).  Returns false, having
// written nothing, when there are more distinct values.
__device__ bool digit_sort(const uint64_t *g, uint64_t *out, uint32_t n, FmmLds &L, const uint32_t *logp = nullptr,
                           uint32_t *outp = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < kHash; i += kThreads) {
        L.hk[i] = INF;
        L.hc[i] = 0u;
    }
    if (tid == 0) {
        L.nd = 0u;
        L.ovf = 0u;
    }
    __syncthreads();
    for (uint32_t b = 0; b < n; b += kThreads) {
        const uint32_t e = b + tid;
        const bool in = e < n;
        const uint32_t T = in ? uint32_t(g[e] >> 32) : INF;
        uint64_t todo = __ballot(in);
        while (todo) {
            const int ld = __ffsll((unsigned long long)todo) - 1;
            const uint32_t v = __shfl(T, ld);
            const uint64_t mk = __ballot(in && T == v);
            if (lane == ld) {
                uint32_t h = hslot0(v);
                bool ok = false;
                for (int probe = 0; probe < kHash; ++probe) {
                    const uint32_t prev = atomicCAS(&L.hk[h], INF, v);
                    if (prev == INF) {
                        const uint32_t d = atomicAdd(&L.nd, 1u);
                        if (d < uint32_t(kMaxD)) L.dv[d] = v;
                    }
                    if (prev == INF || prev == v) {
                        ok = true;
                        break;
                    }
                    h = (h + 1) & (kHash - 1);
                }
                if (ok)
                    atomicAdd(&L.hc[h], uint32_t(__popcll(mk)));
                else
                    L.ovf = 1u;
            }
            todo &= ~mk;
        }
    }
    __syncthreads();
    const uint32_t nd = L.nd;
    if (L.ovf || nd > uint32_t(kMaxD)) return false;  // uniform
    uint32_t rk = 0, v = 0;
    if (uint32_t(tid) < nd) {
        v = L.dv[tid];
        for (uint32_t j = 0; j < nd; ++j) rk += L.dv[j] < v ? 1u : 0u;  // T >= 0: bits order as values
        L.base[rk] = L.hc[hfind(L, v)];
    }
    __syncthreads();
    uint32_t tot;
    const uint32_t ex = block_scan(uint32_t(tid) < nd ? L.base[tid] : 0u, tot, L.scr);
    if (uint32_t(tid) < nd) {
        L.base[tid] = ex;
        L.hd[hfind(L, v)] = rk;
    }
    __syncthreads();
    const uint64_t below = (uint64_t(1) << lane) - 1;
    for (uint32_t b = 0; b < n; b += kThreads) {
        const uint32_t e = b + tid;
        const bool in = e < n;
        const uint64_t key = in ? g[e] : 0;
        const uint32_t T = uint32_t(key >> 32);
        for (uint32_t k = lane; k < nd; k += 64) L.wc[wave][k] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t d = 0, r = 0;
        uint64_t todo = __ballot(in);
        while (todo) {
            const int ld = __ffsll((unsigned long long)todo) - 1;
            const uint32_t vv = __shfl(T, ld);
            const uint64_t mk = __ballot(in && T == vv);
            const uint32_t dd = L.hd[hfind(L, vv)];
            if (in && T == vv) {
                d = dd;
                r = uint32_t(__popcll(mk & below));
            }
            if (lane == ld) L.wc[wave][dd] = uint32_t(__popcll(mk));
            todo &= ~mk;
        }
        __syncthreads();
        if (in) {
            uint32_t pre = 0;
            for (int w2 = 0; w2 < wave; ++w2) pre += L.wc[w2][d];
            out[L.base[d] + pre + r] = key;
            if (outp) outp[L.base[d] + pre + r] = logp[uint32_t(key)];  // the pop's pixel, by rank
        }
        __syncthreads();
        if (uint32_t(tid) < nd) {
            uint32_t sum = 0;
#pragma unroll
            for (int w2 = 0; w2 < kThreads / 64; ++w2) sum += L.wc[w2][tid];
            L.base[tid] += sum;
        }
        __syncthreads();
    }
    return true;
}

// Sort n > kCap keys held in g[0, n): LDS-sorted runs of kCap, then merge
// passes between g and h (unique keys: each element's place is its rank in
// its own run plus its rank in the partner run).  Returns the buffer that
// holds the result.
__device__ uint64_t *global_sort(uint64_t *g, uint64_t *h, uint32_t n, FmmLds &L) {
    for (uint32_t r0 = 0; r0 < n; r0 += kCap) {
        const uint32_t len = min(uint32_t(kCap), n - r0);
        for (int i = threadIdx.x; i < kCap; i += kThreads) L.keys[i] = uint32_t(i) < len ? g[r0 + i] : ~uint64_t(0);
        __syncthreads();
        lds_bitonic(L.keys, kCap);
        for (int i = threadIdx.x; uint32_t(i) < len; i += kThreads) g[r0 + i] = L.keys[i];
        sync_all();
    }
    uint64_t *src = g, *dst = h;
    for (uint32_t wdt = kCap; wdt < n; wdt <<= 1) {
        for (uint32_t i = threadIdx.x; i < n; i += kThreads) {
            const uint32_t lo = i / (2 * wdt) * (2 * wdt), mid = min(lo + wdt, n), hi = min(lo + 2 * wdt, n);
            const uint64_t key = src[i];
            const uint32_t pos = i < mid ? (i - lo) + lower_bound64(src + mid, hi - mid, key)
                                         : (i - mid) + lower_bound64(src + lo, mid - lo, key);
            dst[lo + pos] = key;
        }
        sync_all();
        uint64_t *tmp = src;
        src = dst;
        dst = tmp;
    }
    return src;
}

// FMM loops handle kFB entries per thread per round (gather, claim, push,
// the global-memory distance sweep)
#ifndef OFD_FMM_B
#define OFD_FMM_B 2
#endif
constexpr int kFB = OFD_FMM_B;

// One fast march (icvCalcFMM / icvTeleaInpaintFMM's heap order) over the
// pixels whose stamp is INF, starting from the band in log[0, nb).  Leaves
// every push's stamp, distance and log entry; returns the number of log
// entries (band + pushes).
// Pipelined fill: the inner march publishes how far its log is final (the
// entries of completed buckets) at most every kPubTicks of the constant-rate
// clock, for the record / colour rounds running beside it.  Called by every
// thread right after a workgroup barrier that followed the bucket's stores:
// thread 0's agent-scope release store then carries every thread's stores
// (each waited for its own before the barrier).
constexpr uint64_t kPubTicks = 10000;  // 100 us at 100 MHz
__device__ __forceinline__ void publish_prog(const Img &m, uint32_t seq, uint64_t &last, bool force) {
    if (threadIdx.x != 0) return;
    const uint64_t now = wall_clock64();
    if (!force && now - last < kPubTicks) return;
    last = now;
    __hip_atomic_store(&m.pipe[kPProg], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool kInner>
__device__ uint32_t fmm_pass(const Img &m, uint32_t *st, uint32_t nb, FmmLds &L, uint32_t &nbuckets, uint64_t *prof,
                         double bscale, bool pub) {
    (void)prof;
    uint64_t last_pub = 0;
    const int tid = threadIdx.x, ew = m.ew;
    const int64_t off[4] = {-int64_t(ew), -1, int64_t(ew), 1};  // cv2's q = 0..3: up, left, down, right
    uint32_t seq = nb;
    uint32_t start[4] = {nb, nb, nb, nb};  // first push of buckets k-3 .. k (ring indexed by k & 3)
    nbuckets = 0;
    for (uint32_t k = 0;; ++k) {
        uint32_t lo, hi = seq;
        if (k == 0) {
            lo = 0;
            hi = nb;
            if (nb == 0) break;
        } else {
            lo = k >= 3 ? start[(k - 3) & 3] : nb;
            if (lo == seq) break;  // nothing pending in buckets >= k
        }
        if (k > 4u * uint32_t(m.en) + 16u) {  // cannot happen: bucket k holds T >= k w >= k / 2 and T < en
            if (tid == 0) { m.meta[5] = 1u; atomicOr(&g_sq_fault, 2u); }
            break;
        }
        start[k & 3] = seq;
        SQ_T(f0);
#ifdef OFD_BUCKET_TRACE
        const uint64_t tb0 = __builtin_amdgcn_s_memtime();
#endif
        // gather bucket k in push order
        if (tid == 0) {
            L.tmin = INF;
            L.tmax = 0u;
        }
        __syncthreads();
        uint32_t n = 0, tmn = INF, tmx = 0u;
        // bucket 0 is the band: every log entry [0, nb), all at T = 0, already
        // in (T, push order) -- its pops are the log itself (no gather, no sort)
        const bool band = k == 0;
        if (band) {
            n = nb;
            tmn = tmx = 0u;
        }
        for (uint32_t b = band ? hi : lo; b < hi; b += kFB * kThreads) {  // kFB consecutive entries per thread
            float T[kFB];
            unsigned sel = 0;
#pragma unroll
            for (int u = 0; u < kFB; ++u) {
                const uint32_t i = b + kFB * tid + u;
                T[u] = i < hi ? m.logt[i] : 0.f;
                if (i < hi && bucket_of(T[u], bscale) == k) sel |= 1u << u;
            }
            uint32_t tot;
            uint32_t pos = block_scan(__popc(sel), tot, L.scr);
#pragma unroll
            for (int u = 0; u < kFB; ++u)
                if (sel & (1u << u)) {
                    const uint32_t i = b + kFB * tid + u;
                    const uint32_t tb = __float_as_uint(T[u] + 0.0f);  // -0 -> +0: the heap compares values
                    const uint64_t key = (uint64_t(tb) << 32) | i;
                    const uint32_t at = n + pos++;
                    if (at < kCap)
                        L.keys[at] = key;
                    else
                        m.k0[at] = key;
                    tmn = min(tmn, tb);
                    tmx = max(tmx, tb);
                }
            n += tot;
        }
        SQ_T(f1);
        SQ_ACC(0, f0, f1);
#ifdef OFD_BUCKET_TRACE
        const uint64_t tb1 = __builtin_amdgcn_s_memtime();
#endif
        if (n == 0) continue;
        ++nbuckets;
#ifdef OFD_SQ_PROF
        const int pb = n > uint32_t(kCap) ? 8 : 0;  // probe: large buckets in prof[8..]
#endif
        if (tmn != INF) atomicMin(&L.tmin, tmn);
        atomicMax(&L.tmax, tmx);
        __syncthreads();
        const bool uniform = L.tmin == L.tmax;  // already in (T, seq) order
        const uint64_t *keys = L.keys;
        const uint32_t *kpx = nullptr;  // pixel of each pop by rank, when the sort provides it
        if (band) {
            keys = nullptr;  // pop rank r is log entry r
        } else if (n > kCap) {
            for (int i = tid; i < kCap; i += kThreads) m.k0[i] = L.keys[i];
            sync_all();
            // the counting sort also lays the pops' pixels out by rank (the
            // claims and pushes of these long buckets then skip one dependent
            // load per pop); the area is free until RECORD
            uint32_t *rank_px = m.rpx + (kInner ? 0 : m.en);
            if (uniform)
                keys = m.k0;
            else if (digit_sort(m.k0, m.k1, n, L, m.logp, rank_px)) {
                keys = m.k1;
                kpx = rank_px;
            } else
                keys = global_sort(m.k0, m.k1, n, L);
        } else if (!uniform && n > 1) {
            keys = lds_sort(L, n);
        }
        SQ_T(f2);
        SQ_ACC(pb + 1, f1, f2);
#ifdef OFD_BUCKET_TRACE
        const uint64_t tb2 = __builtin_amdgcn_s_memtime();
#endif
        // the band's claims and pushes are already made (sq_band_push_*_kernel)
        uint32_t npush = band ? m.pipe[kInner ? kPB0In : kPB0Out] : 0u;
        // pops in order: claim the INSIDE neighbours (first claimant = pusher)
        if (!band)
        for (uint32_t r0 = tid; r0 < n; r0 += kFB * kThreads) {  // 4 pops per thread: one round per load step
            int64_t a[kFB];
            uint32_t sv[kFB][4];
#pragma unroll
            for (int u = 0; u < kFB; ++u) {
                const uint32_t r = r0 + uint32_t(u) * kThreads;
                a[u] = r < n ? int64_t(kpx ? kpx[r] : m.logp[keys ? uint32_t(keys[r]) : r]) : 0;
            }
#pragma unroll
            for (int u = 0; u < kFB; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) sv[u][q] = r0 + uint32_t(u) * kThreads < n ? st[a[u] + off[q]] : 0u;
#pragma unroll
            for (int u = 0; u < kFB; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (sv[u][q] == INF)
                        atomicMin(&m.own[a[u] + off[q]], (r0 + uint32_t(u) * kThreads) * 4u + uint32_t(q));
        }
        sync_all();
        SQ_T(f3);
        SQ_ACC(pb + 2, f2, f3);
#ifdef OFD_BUCKET_TRACE
        const uint64_t tb3 = __builtin_amdgcn_s_memtime();
#endif
        // pushes numbered in (rank, direction) order
        if (!band)
        for (uint32_t b = 0; b < n; b += kFB * kThreads) {  // kFB slices of kThreads ranks, loads first
            int64_t a[kFB];
            uint32_t sv[kFB][4], ov[kFB][4];
#pragma unroll
            for (int u = 0; u < kFB; ++u) {
                const uint32_t r = b + uint32_t(u) * kThreads + tid;
                a[u] = r < n ? int64_t(kpx ? kpx[r] : m.logp[keys ? uint32_t(keys[r]) : r]) : 0;
            }
#pragma unroll
            for (int u = 0; u < kFB; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool in = b + uint32_t(u) * kThreads + tid < n;
                    sv[u][q] = in ? st[a[u] + off[q]] : 0u;
                    ov[u][q] = in ? m.own[a[u] + off[q]] : 0u;
                }
#pragma unroll
            for (int u = 0; u < kFB; ++u) {
                if (b + uint32_t(u) * kThreads >= n) break;  // uniform
                const uint32_t r = b + uint32_t(u) * kThreads + tid;
                unsigned mine = 0;  // a pixel pushed by an earlier bucket keeps a stale key
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (sv[u][q] == INF && ov[u][q] == r * 4u + uint32_t(q)) mine |= 1u << q;
                uint32_t tot;
                uint32_t pos = block_scan(__popc(mine), tot, L.scr);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (mine & (1u << q)) {
                        const uint32_t s = seq + npush + pos++;
                        const int64_t p = a[u] + off[q];
                        st[p] = s;
                        m.logp[s] = uint32_t(p);
                    }
                npush += tot;
            }
        }
        sync_all();
        SQ_T(f4);
        SQ_ACC(pb + 3, f3, f4);
#ifdef OFD_BUCKET_TRACE
        const uint64_t tb4 = __builtin_amdgcn_s_memtime();
        uint32_t nsw = 0;  // probe: sweeps of this bucket
#endif
        // distances: sweep to the fixed point (acyclic in push order: at most
        // npush + 1 sweeps; the cap only guards against a broken invariant).
        // Up to kLdsPush pushes: the bucket's distances live in LDS and each
        // push keeps its neighbours' fixed values in registers -- only a
        // neighbour pushed earlier in this bucket is read per sweep.
        if (npush <= uint32_t(kLdsPush)) {
            float *Tl = reinterpret_cast<float *>(L.keys);
            float fv[2][4];
            int lk[2][4];  // -2: INSIDE, -1: fixed value, >= 0: push index in this bucket
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const uint32_t i = tid + uint32_t(u) * kThreads;
                if (i < npush) {
                    const uint32_t sp = seq + i;
                    const int64_t p = m.logp[sp];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int64_t nq = p + off[q];
                        const uint32_t sn = st[nq];
                        lk[u][q] = sn >= sp ? -2 : (sn >= seq ? int(sn - seq) : -1);
                        fv[u][q] = lk[u][q] == -1 ? band_t<kInner>(m.t[nq]) : T_FAR;
                    }
                    Tl[i] = T_FAR;
                }
            }
            if (tid == 0) L.chg3[0] = 0u;
            __syncthreads();
            // one barrier per sweep: sweep `it` flags changes in chg3[it % 3];
            // chg3[(it + 1) % 3], last read right after barrier it - 2, is
            // zeroed for the next sweep before this sweep's barrier
            for (uint32_t it = 0;; ++it) {
                if (it > npush + 1) {
                    if (tid == 0) { m.meta[5] = 2u; atomicOr(&g_sq_fault, 4u); }
                    break;
                }
                if (tid == 0) L.chg3[(it + 1) % 3] = 0u;
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const uint32_t i = tid + uint32_t(u) * kThreads;
                    if (i < npush) {
                        float tv[4];
                        bool in[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            in[q] = lk[u][q] == -2;
                            tv[q] = lk[u][q] >= 0 ? Tl[lk[u][q]] : fv[u][q];
                        }
                        // cv2's order: (up, left), (down, left), (up, right), (down, right)
                        const float T = min4f(fm_solve(tv[0], in[0], tv[1], in[1]), fm_solve(tv[2], in[2], tv[1], in[1]),
                                              fm_solve(tv[0], in[0], tv[3], in[3]), fm_solve(tv[2], in[2], tv[3], in[3]));
                        if (T != Tl[i]) {
                            Tl[i] = T;
                            L.chg3[it % 3] = 1u;
                        }
                    }
                }
                __syncthreads();
                const uint32_t c = L.chg3[it % 3];
#ifdef OFD_SQ_PROF
                if (tid == 0) prof[pb + 6] += 1;
#endif
#ifdef OFD_BUCKET_TRACE
                nsw = it + 1;
#endif
                if (!c) break;
            }
            for (uint32_t i = tid; i < npush; i += kThreads) {
                const float T = Tl[i];
                m.t[m.logp[seq + i]] = T;
                m.logt[seq + i] = T;
            }
            SQ_T(f5a);
            SQ_ACC(pb + 4, f4, f5a);
            seq += npush;
            sync_all();
            if (kInner && pub) publish_prog(m, seq, last_pub, false);
            SQ_T(f6a);
            SQ_ACC(pb + 5, f5a, f6a);
#ifdef OFD_BUCKET_TRACE
            if (threadIdx.x == 0 && 8 * nbuckets + 8 < 4 * m.en) {  // inner at 8 en, outer at 20 en
                uint32_t *tr = m.rec + (kInner ? 8 : 20) * m.en + 8 * (nbuckets - 1);
                tr[0] = uint32_t((__builtin_amdgcn_s_memtime() - tb0) >> 4);
                tr[4] = uint32_t((tb1 - tb0) >> 4);
                tr[5] = uint32_t((tb2 - tb1) >> 4);
                tr[6] = uint32_t((tb3 - tb2) >> 4);
                tr[7] = uint32_t((tb4 - tb3) >> 4);
                tr[1] = n;
                tr[2] = npush;
                tr[3] = k | (nsw << 16);
                m.rec[(kInner ? 8 : 20) * m.en + 4 * m.en] = nbuckets;
            }
#endif
            continue;
        }
        // More pushes: sweep 0 evaluates every push; each later sweep only the
        // pushes of this bucket next to one whose distance changed in the
        // sweep before (a worklist, deduplicated by a per-sweep tag in own[]:
        // claims are settled, and tags have the top bit, claims not).
        {
            uint32_t *wa = reinterpret_cast<uint32_t *>(m.k0), *wb = reinterpret_cast<uint32_t *>(m.k1);
            uint32_t nw = npush;
            for (uint32_t it = 0;; ++it) {
                if (it > npush + 1) {
                    if (tid == 0) { m.meta[5] = 2u; atomicOr(&g_sq_fault, 4u); }
                    break;
                }
                if (tid == 0) L.chg = 0u;
                __syncthreads();
                const uint32_t tag = 0x80000000u | it;
                for (uint32_t i0 = tid; i0 < nw; i0 += kFB * kThreads) {
                    int64_t p[kFB];
                    uint32_t sp[kFB];
                    float T[kFB], cur[kFB];
#pragma unroll
                    for (int u = 0; u < kFB; ++u) {
                        const uint32_t i = i0 + uint32_t(u) * kThreads;
                        const uint32_t x = i < nw ? (it == 0 ? i : wa[i]) : 0u;
                        sp[u] = seq + x;
                        p[u] = i < nw ? int64_t(m.logp[seq + x]) : int64_t(ew) + 1;
                    }
#pragma unroll
                    for (int u = 0; u < kFB; ++u) {
                        T[u] = fm_dist_seq<kInner>(st, m.t, p[u], ew, sp[u]);
                        cur[u] = m.t[p[u]];
                    }
#pragma unroll
                    for (int u = 0; u < kFB; ++u)
                        if (i0 + uint32_t(u) * kThreads < nw && T[u] != cur[u]) {
                            m.t[p[u]] = T[u];
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                const int64_t nq = p[u] + off[q];
                                const uint32_t sn = st[nq];
                                if (sn > sp[u] && sn != INF && atomicExch(&m.own[nq], tag) != tag)
                                    wb[atomicAdd(&L.chg, 1u)] = sn - seq;
                            }
                        }
                }
                sync_all();
                nw = L.chg;
                __syncthreads();
#ifdef OFD_SQ_PROF
                if (tid == 0) prof[pb + 6] += 1;
#endif
                uint32_t *tmp = wa;
                wa = wb;
                wb = tmp;
#ifdef OFD_BUCKET_TRACE
                nsw = it + 1;
#endif
                if (nw == 0) break;
            }
        }
        SQ_T(f5);
        SQ_ACC(pb + 4, f4, f5);
        for (uint32_t i = tid; i < npush; i += kThreads) m.logt[seq + i] = m.t[m.logp[seq + i]];
        seq += npush;
        sync_all();
        if (kInner && pub) publish_prog(m, seq, last_pub, false);
        SQ_T(f6);
        SQ_ACC(pb + 5, f5, f6);
#ifdef OFD_BUCKET_TRACE
        if (threadIdx.x == 0 && 8 * nbuckets + 8 < 4 * m.en) {  // inner at 8 en, outer at 20 en
            uint32_t *tr = m.rec + (kInner ? 8 : 20) * m.en + 8 * (nbuckets - 1);
            tr[0] = uint32_t((__builtin_amdgcn_s_memtime() - tb0) >> 4);
            tr[4] = uint32_t((tb1 - tb0) >> 4);
            tr[5] = uint32_t((tb2 - tb1) >> 4);
            tr[6] = uint32_t((tb3 - tb2) >> 4);
            tr[7] = uint32_t((tb4 - tb3) >> 4);
            tr[1] = n;
            tr[2] = npush;
            tr[3] = k | (nsw << 16);
            m.rec[(kInner ? 8 : 20) * m.en + 4 * m.en] = nbuckets;
        }
#endif
    }
    return seq;
}

// The outer march's push log and sort buffers (its own area: the pipelined
// fill records holes while the marches run).
__device__ __forceinline__ Img outer_view(const Img &m) {
    Img o = m;
    o.logp = m.olog;
    o.logt = reinterpret_cast<float *>(m.olog + m.en);
    o.k0 = reinterpret_cast<uint64_t *>(m.olog + 2 * m.en);
    o.k1 = o.k0 + m.en;
    return o;
}

// Two workgroups per image: blockIdx.y = 0 runs the outer march over the ring
// (icvCalcFMM(out, t, Out, negate = true)) and negates its distances,
// blockIdx.y = 1 the inner march over the holes (icvTeleaInpaintFMM's order).
// They touch disjoint pixels (ring pixels are not 4-adjacent to holes) and
// keep separate stamps, logs and sort buffers; the only value both read is
// the band's zero distance (band_t).
__global__ __launch_bounds__(kThreads) void sq_fmm_kernel(SqWs w, double bscale, int pub) {
    __shared__ FmmLds L;
    const Img m = image(w, blockIdx.x);
    const uint32_t nb = m.meta[0];
    uint32_t nbk = 0;
    uint64_t prof[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    // each march's duration on the constant-rate wall clock (meta[24] outer,
    // meta[25] inner; tools/seq_time.py) -- those words hold the large-bucket
    // probe clocks in OFD_SQ_PROF builds instead
    const uint64_t w0 = threadIdx.x == 0 ? wall_clock64() : 0;
    if (threadIdx.x == 0 && blockIdx.y == 1) put64(m.pipe + kPTFmm, w0);
    if (blockIdx.y == 0) {
        const Img o = outer_view(m);
        const uint32_t no = fmm_pass<false>(o, m.sO, nb, L, nbk, prof, bscale, false);
        for (uint32_t i = threadIdx.x; i < no; i += kThreads) {
            const uint32_t p = o.logp[i];
            m.t[p] = -m.t[p];
        }
        sync_all();
        // the ring's distances are final: publish (RECORD reads them)
        if (threadIdx.x == 0) {
            put64(m.pipe + kPTOut, wall_clock64());
            __hip_atomic_store(&m.pipe[kPOutDone], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (threadIdx.x == 0) {
            atomicAdd(&m.meta[4], nbk);
#ifndef OFD_SQ_PROF
            m.meta[24] = uint32_t(wall_clock64() - w0);
#endif
        }
        return;
    }
    const uint32_t ni = fmm_pass<true>(m, m.sI, nb, L, nbk, prof, bscale, pub != 0);
    {
        uint64_t last = 0;
        publish_prog(m, ni, last, true);  // (fmm_pass ended on a barrier after its last stores)
    }
    if (threadIdx.x == 0) {
        put64(m.pipe + kPTIn, wall_clock64());
        __hip_atomic_store(&m.pipe[kPInDone], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
#ifndef OFD_SQ_PROF
        m.meta[25] = uint32_t(wall_clock64() - w0);
#endif
        m.meta[1] = ni - nb;
        atomicAdd(&m.meta[4], nbk);
        for (int k = 0; k < 8; ++k) m.meta[8 + k] = uint32_t(k == 6 ? prof[k] : prof[k] >> 8);
#ifdef OFD_SQ_PROF
        for (int k = 0; k < 8; ++k) m.meta[24 + k] = uint32_t(k == 6 ? prof[8 + k] : prof[8 + k] >> 8);
#endif
    }
}

// ---------------------------------------------------------------- COUNT / COLOUR
// Window of a hole's colour: disk positions (a^2 + b^2 <= r^2) and their 3x3
// neighbours (gradients, cv2's border shifts) -- symmetric, so "q is in p's
// window" and "p is in q's window" coincide.
__device__ __forceinline__ bool in_window(int a, int b, int r) {
    const int a1 = max(abs(a) - 1, 0), b1 = max(abs(b) - 1, 0);
    return a1 * a1 + b1 * b1 <= r * r;
}

// Radius-3 window positions (patch offsets a, b in [-4, 4]): the disk and
// its 3x3 neighbourhood.
constexpr bool disk3(int a, int b) { return a * a + b * b <= 9; }
constexpr bool win3(int a, int b) {
    const int a1 = (a < 0 ? -a : a) - 1, b1 = (b < 0 ? -b : b) - 1;
    return (a1 < 0 ? 0 : a1) * (a1 < 0 ? 0 : a1) + (b1 < 0 ? 0 : b1) * (b1 < 0 ? 0 : b1) <= 9;
}
// The window positions a hole's colour actually reads when none of its disk
// pixels is on a border row / column (where cv2's gradient shifts by one):
// the disk and its 4-neighbours (cv2's gradients are central, forward or
// backward differences along x and y) -- 48 of win3's 60 neighbours; the 12
// others, (+-3, +-3), (+-4, +-1), (+-1, +-4), are read only near a border.
constexpr bool need3(int a, int b) {
    return disk3(a, b) || disk3(a + 1, b) || disk3(a - 1, b) || disk3(a, b + 1) || disk3(a, b - 1);
}

// pending[p] = holes of smaller stamp in p's window; level 0 = none
__global__ __launch_bounds__(256) void sq_count_kernel(SqWs w, int range) {
    const int j = blockIdx.x * 64 + (threadIdx.x & 63), i = blockIdx.y * 4 + (threadIdx.x >> 6);
    const Img m = image(w, blockIdx.z);
    if (i < 1 || j < 1 || i >= m.eh - 1 || j >= m.ew - 1) return;
    const int64_t p = int64_t(i) * m.ew + j;
    const uint32_t s = m.sI[p];
    if (s == 0u || s == INF) return;
    const int R = range + 1;
    uint32_t cnt = 0;
    for (int a = -R; a <= R; ++a) {
        const int y = i + a;
        if (y < 1 || y >= m.eh - 1) continue;
        for (int b = -R; b <= R; ++b) {
            const int x = j + b;
            if (x < 1 || x >= m.ew - 1 || !(a || b) || !in_window(a, b, range)) continue;
            const uint32_t sq = m.sI[int64_t(y) * m.ew + x];
            cnt += (sq != 0u && sq < s) ? 1u : 0u;
        }
    }
    m.own[p] = cnt;
    if (cnt == 0u) {
        uint32_t *front = reinterpret_cast<uint32_t *>(m.k0);
        front[atomicAdd(&m.meta[2], 1u)] = uint32_t(p);
    }
}

// cv2's Telea colour of padded hole (i, j) with stamp s, channel c (the
// oracle's telea_colour with INSIDE = "stamp >= s"): every value it reads is
// a pixel of smaller stamp (final) or a known pixel, or -- through cv2's
// border index shifts -- a later hole that still holds its input value.
__device__ __forceinline__ unsigned telea_colour_seq(const Img &m, const float *plane, int W, int i, int j, uint32_t s,
                                                     int range) {
    const int eh = m.eh, ew = m.ew;
    const uint32_t *st = m.sI;
    const float *t = m.t;
    auto IN = [&](int a, int b) -> bool { return st[int64_t(a) * ew + b] >= s; };
    auto TT = [&](int a, int b) -> float { return t[int64_t(a) * ew + b]; };
    auto smp = [&](int y, int x) -> int { return int(plane[int64_t(y) * W + x]); };
    float gtx, gty;
    const float tij = TT(i, j);
    if (!IN(i, j + 1))
        gtx = !IN(i, j - 1) ? (TT(i, j + 1) - TT(i, j - 1)) * 0.5f : (TT(i, j + 1) - tij);
    else
        gtx = !IN(i, j - 1) ? (tij - TT(i, j - 1)) : 0.f;
    if (!IN(i + 1, j))
        gty = !IN(i - 1, j) ? (TT(i + 1, j) - TT(i - 1, j)) * 0.5f : (TT(i + 1, j) - tij);
    else
        gty = !IN(i - 1, j) ? (tij - TT(i - 1, j)) : 0.f;
    float Ia = 0, Jx = 0, Jy = 0, sum = 1.0e-20f;
    for (int k = i - range; k <= i + range; ++k) {
        const int km = k - 1 + (k == 1), kp = k - 1 - (k == eh - 2);
        for (int l = j - range; l <= j + range; ++l) {
            const int lm = l - 1 + (l == 1), lp = l - 1 - (l == ew - 2);
            if (!(k > 0 && l > 0 && k < eh - 1 && l < ew - 1)) continue;
            if (IN(k, l) || (l - j) * (l - j) + (k - i) * (k - i) > range * range) continue;
            const float ry = float(i - k), rx = float(j - l);
            const float len2 = rx * rx + ry * ry;
            const float dst = float(1. / (double(len2) * sqrt(double(len2))));
            const float lev = float(1. / (1 + fabs(double(TT(k, l) - tij))));
            float dir = rx * gtx + ry * gty;
            if (fabs(double(dir)) <= 0.01) dir = 0.000001f;
            const float wgt = float(fabs(double(dst * lev * dir)));
            float gix, giy;
            if (!IN(k, l + 1))
                gix = !IN(k, l - 1) ? float(smp(km, lp + 1) - smp(km, lm - 1)) * 2.0f : float(smp(km, lp + 1) - smp(km, lm));
            else
                gix = !IN(k, l - 1) ? float(smp(km, lp) - smp(km, lm - 1)) : 0.f;
            if (!IN(k + 1, l))
                giy = !IN(k - 1, l) ? float(smp(kp + 1, lm) - smp(km - 1, lm)) * 2.0f : float(smp(kp + 1, lm) - smp(km, lm));
            else
                giy = !IN(k - 1, l) ? float(smp(kp, lm) - smp(km - 1, lm)) : 0.f;
            Ia += wgt * float(smp(km, lm));
            Jx -= wgt * (gix * rx);
            Jy -= wgt * (giy * ry);
            sum += wgt;
        }
    }
    const float sat = float(double(Ia / sum) + double(Jx + Jy) / (sqrt(double(Jx * Jx + Jy * Jy)) + double(1.0e-20f)) +
                            double(0.5f));
    return sat_u8(sat);
}

struct ColLds {
    uint32_t nnext;
};

// Any radius: one thread per hole, dependants released by atomic counters.
__global__ __launch_bounds__(kColThreads) void sq_colour_kernel(SqWs w, float *__restrict__ out, int C, int H, int W,
                                                             int64_t b0, int range) {
    __shared__ ColLds L;
    const int tid = threadIdx.x;
    const Img m = image(w, blockIdx.x);
    const int64_t HW = int64_t(H) * W;
    float *ob = out + (b0 + blockIdx.x) * int64_t(C) * HW;
    uint32_t *fa = reinterpret_cast<uint32_t *>(m.k0), *fb = fa + m.en;
    uint32_t *lsz = reinterpret_cast<uint32_t *>(m.k1);  // diagnostics: size of each level (tools/seq_time.py)
    uint32_t n = m.meta[2], levels = 0;
    const int R = range + 1;
    if (tid == 0) L.nnext = 0u;
    __syncthreads();
    while (n) {
        if (tid == 0 && levels < uint32_t(2 * m.en)) lsz[levels] = n;
        ++levels;
        for (uint32_t e = tid; e < n; e += kColThreads) {
            const int64_t p = fa[e];
            const int i = int(p / m.ew), j = int(p - int64_t(i) * m.ew);
            const uint32_t s = m.sI[p];
            for (int c = 0; c < C; ++c) {
                float *pl = ob + c * HW;
                pl[int64_t(i - 1) * W + (j - 1)] = float(telea_colour_seq(m, pl, W, i, j, s, range));
            }
            for (int a = -R; a <= R; ++a) {
                const int y = i + a;
                if (y < 1 || y >= m.eh - 1) continue;
                for (int b = -R; b <= R; ++b) {
                    const int x = j + b;
                    if (x < 1 || x >= m.ew - 1 || !(a || b) || !in_window(a, b, range)) continue;
                    const int64_t q = int64_t(y) * m.ew + x;
                    const uint32_t sq = m.sI[q];
                    if (sq > s && sq != INF && atomicSub(&m.own[q], 1u) == 1u) fb[atomicAdd(&L.nnext, 1u)] = uint32_t(q);
                }
            }
        }
        sync_all();
        n = L.nnext;
        __syncthreads();
        if (tid == 0) L.nnext = 0u;
        uint32_t *tmp = fa;
        fa = fb;
        fb = tmp;
        __syncthreads();
    }
    if (tid == 0) m.meta[3] = levels;
}

// Radius 3 (the reference's inpaintRange): a group of 16 lanes per hole, 64
// holes in flight per workgroup.  Lane g of a group owns disk positions g and
// g + 16 (cv2's raster order over the 29 positions of the r = 3 disk) and
// loads what they need -- stamps of the position and its 4-neighbours, its
// distance, and per channel the (up to 7) values cv2's gradient reads, with
// its border index shifts -- so the only cross-lane traffic is the ordered
// sums: cv2 adds the window's terms in (k, l) order, and so does the group,
// one shuffle per term.  Release: lanes own the 60 window positions 16 apart.
constexpr int kG = 16;
constexpr int kG16Threads = 1024;  // <= 128 VGPRs: four waves per SIMD
constexpr int kGroups = kG16Threads / kG;

constexpr int disk_count() {
    int n = 0;
    for (int a = -3; a <= 3; ++a)
        for (int b = -3; b <= 3; ++b) n += disk3(a, b) ? 1 : 0;
    return n;
}
constexpr int win_count() {
    int n = 0;
    for (int a = -4; a <= 4; ++a)
        for (int b = -4; b <= 4; ++b) n += (win3(a, b) && (a || b)) ? 1 : 0;
    return n;
}
constexpr int kDisk = disk_count();  // 29
constexpr int kWin = win_count();    // 60
static_assert(kDisk <= 2 * kG && kWin <= 4 * kG, "radius-3 window does not fit the lane group");

// d-th position (raster order) of the disk / of the window without its centre
__device__ __forceinline__ void disk_pos(int d, int &a, int &b) {
    int n = 0;
    a = b = 0;
    for (int u = -3; u <= 3; ++u)
        for (int v = -3; v <= 3; ++v)
            if (disk3(u, v)) {
                if (n == d) {
                    a = u;
                    b = v;
                }
                ++n;
            }
}
__device__ __forceinline__ void win_pos(int d, int &a, int &b) {
    int n = 0;
    a = b = 0;
    for (int u = -4; u <= 4; ++u)
        for (int v = -4; v <= 4; ++v)
            if (win3(u, v) && (u || v)) {
                if (n == d) {
                    a = u;
                    b = v;
                }
                ++n;
            }
}

constexpr int kChunkC = 3;  // channels whose values are loaded together (RGB in one round)

struct G16Lds {
    uint32_t nnext;
    float terms[kGroups][kChunkC][3][2 * kG];  // per group: Ia / Jx / Jy terms of each disk position
    float wts[kGroups][2 * kG];                // per group: weight of each disk position
};

__global__ __launch_bounds__(kG16Threads) void sq_colour_g16_kernel(SqWs w, float *__restrict__ out, int C, int H, int W,
                                                                   int64_t b0) {
    __shared__ G16Lds L;
    const int tid = threadIdx.x, g = tid / kG, gl = tid % kG;
    const Img m = image(w, blockIdx.x);
    const int eh = m.eh, ew = m.ew;
    const int64_t HW = int64_t(H) * W;
    float *ob = out + (b0 + blockIdx.x) * int64_t(C) * HW;
    uint32_t *fa = reinterpret_cast<uint32_t *>(m.k0), *fb = fa + m.en;
    uint32_t *lsz = reinterpret_cast<uint32_t *>(m.k1);
    // this lane's disk positions (slot 0, 1) and window positions (release)
    int da[2], db[2], wa[4], wb[4];
    bool dv[2], wv[4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        dv[k] = gl + kG * k < kDisk;
        disk_pos(gl + kG * k, da[k], db[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        wv[k] = gl + kG * k < kWin;
        win_pos(gl + kG * k, wa[k], wb[k]);
    }
    uint32_t n = m.meta[2], levels = 0;
    if (tid == 0) L.nnext = 0u;
    __syncthreads();
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)prof;
    auto clampi = [&](int y, int x) -> int64_t {
        return int64_t(min(max(y, 0), eh - 1)) * ew + min(max(x, 0), ew - 1);
    };
    while (n) {
        if (tid == 0 && levels < uint32_t(2 * m.en)) lsz[levels] = n;
        ++levels;
        SQ_T(l0);
        for (uint32_t e = g; e < n; e += kGroups) {
            SQ_T(c0);
            const int64_t p = fa[e];
            const int i = int(p / ew), j = int(p - int64_t(i) * ew);
            const uint32_t s = m.sI[p];
            // every load of the hole up front: the gradient's neighbours, this
            // lane's disk positions, and the window stamps for the release
            const uint32_t su = m.sI[p - ew], sd = m.sI[p + ew], sl = m.sI[p - 1], sr = m.sI[p + 1];
            const float tij = m.t[p], tu = m.t[p - ew], td = m.t[p + ew], tl = m.t[p - 1], tr = m.t[p + 1];
            uint32_t sc[2], sR[2], sL[2], sD[2], sU[2];
            float tk[2];
            bool inimg[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int y = i + da[k], x = j + db[k];
                inimg[k] = dv[k] && y > 0 && x > 0 && y < eh - 1 && x < ew - 1;
                sc[k] = m.sI[clampi(y, x)];
                sR[k] = m.sI[clampi(y, x + 1)];
                sL[k] = m.sI[clampi(y, x - 1)];
                sD[k] = m.sI[clampi(y + 1, x)];
                sU[k] = m.sI[clampi(y - 1, x)];
                tk[k] = m.t[clampi(y, x)];
            }
            uint32_t sw[4];
            int64_t qq[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int y = i + wa[k], x = j + wb[k];
                const bool ok = wv[k] && y > 0 && x > 0 && y < eh - 1 && x < ew - 1;
                qq[k] = clampi(y, x);
                sw[k] = m.sI[qq[k]];
                sw[k] = ok ? sw[k] : 0u;
            }
            SQ_T(c1);
            float gtx, gty;
            if (!(sr >= s))
                gtx = !(sl >= s) ? (tr - tl) * 0.5f : (tr - tij);
            else
                gtx = !(sl >= s) ? (tij - tl) : 0.f;
            if (!(sd >= s))
                gty = !(su >= s) ? (td - tu) * 0.5f : (td - tij);
            else
                gty = !(su >= s) ? (tij - tu) : 0.f;
            float wt[2];
            bool used[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                used[k] = inimg[k] && !(sc[k] >= s);
                const float ry = float(-da[k]), rx = float(-db[k]);
                const float len2 = rx * rx + ry * ry;
                const float dst = float(1. / (double(len2) * sqrt(double(len2))));
                const float lev = float(1. / (1 + fabs(double(tk[k] - tij))));
                float dir = rx * gtx + ry * gty;
                if (fabs(double(dir)) <= 0.01) dir = 0.000001f;
                wt[k] = used[k] ? float(fabs(double(dst * lev * dir))) : 0.f;
                L.wts[g][gl + kG * k] = wt[k];
            }
            SQ_T(c2);
            for (int c0 = 0; c0 < C; c0 += kChunkC) {
                const int nc = min(kChunkC, C - c0);
                // the values cv2's gradient reads at this lane's positions, every channel of the chunk
                float vv[kChunkC][2][7];
#pragma unroll
                for (int cc = 0; cc < kChunkC; ++cc) {
                    const float *pl = ob + int64_t(c0 + min(cc, nc - 1)) * HW;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int y = i + da[k], x = j + db[k];  // padded (k, l) of cv2's loop
                        const int k1 = y == 1, kE = y == eh - 2, l1 = x == 1, lE = x == ew - 2;
                        auto V = [&](int yy, int xx) -> float {  // unpadded read, clamped (unselected reads only)
                            return pl[int64_t(min(max(yy, 0), H - 1)) * W + min(max(xx, 0), W - 1)];
                        };
                        vv[cc][k][0] = V(y - 1 + k1, x - 1 + l1);  // (km, lm)
                        vv[cc][k][1] = V(y - 1 + k1, x - lE);      // (km, lp + 1)
                        vv[cc][k][2] = V(y - 1 + k1, x - 2 + l1);  // (km, lm - 1)
                        vv[cc][k][3] = V(y - 1 + k1, x - 1 - lE);  // (km, lp)
                        vv[cc][k][4] = V(y - kE, x - 1 + l1);      // (kp + 1, lm)
                        vv[cc][k][5] = V(y - 2 + k1, x - 1 + l1);  // (km - 1, lm)
                        vv[cc][k][6] = V(y - 1 - kE, x - 1 + l1);  // (kp, lm)
                    }
                }
                SQ_T(cv);
                SQ_ACC(2, c2, cv);
#pragma unroll
                for (int cc = 0; cc < kChunkC; ++cc)
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const bool nr = !(sR[k] >= s), nl = !(sL[k] >= s), nd = !(sD[k] >= s), nu = !(sU[k] >= s);
                        const float *v = vv[cc][k];
                        const float vs = v[0];
                        const float gix = nr ? (nl ? (v[1] - v[2]) * 2.0f : (v[1] - vs)) : (nl ? (v[3] - v[2]) : 0.f);
                        const float giy = nd ? (nu ? (v[4] - v[5]) * 2.0f : (v[4] - vs)) : (nu ? (v[6] - v[5]) : 0.f);
                        const float ry = float(-da[k]), rx = float(-db[k]);
                        L.terms[g][cc][0][gl + kG * k] = wt[k] * vs;
                        L.terms[g][cc][1][gl + kG * k] = wt[k] * (gix * rx);
                        L.terms[g][cc][2][gl + kG * k] = wt[k] * (giy * ry);
                    }
                // the group's lanes are one wave's: LDS order within it suffices
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                SQ_T(ct);
                SQ_ACC(7, cv, ct);
                if (gl < nc) {
                    // cv2's sums in its (k, l) order, one lane per channel.  An
                    // unused position's weight and terms are +-0: adding them
                    // leaves every sum unchanged except the sign of an exact
                    // zero, which the final expression cannot see.
                    const int cc = gl;
                    float sum = 1.0e-20f;
#pragma unroll
                    for (int d = 0; d < kDisk; ++d) sum += L.wts[g][d];
                    float Ia = 0.f, Jx = 0.f, Jy = 0.f;
#pragma unroll
                    for (int d = 0; d < kDisk; ++d) {
                        Ia += L.terms[g][cc][0][d];
                        Jx -= L.terms[g][cc][1][d];
                        Jy -= L.terms[g][cc][2][d];
                    }
                    const float sat = float(double(Ia / sum) +
                                            double(Jx + Jy) / (sqrt(double(Jx * Jx + Jy * Jy)) + double(1.0e-20f)) +
                                            double(0.5f));
                    ob[int64_t(c0 + cc) * HW + int64_t(i - 1) * W + (j - 1)] = float(sat_u8(sat));
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            SQ_T(c3);
            // release the holes of larger stamp whose window holds this one
            uint32_t old[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) old[k] = (sw[k] > s && sw[k] != INF) ? atomicSub(&m.own[qq[k]], 1u) : 0u;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (old[k] == 1u) fb[atomicAdd(&L.nnext, 1u)] = uint32_t(qq[k]);
            SQ_T(c4);
            SQ_ACC(3, c0, c1);
            SQ_ACC(4, c1, c2);
            SQ_ACC(5, c2, c3);
            SQ_ACC(6, c3, c4);
        }
        SQ_T(l1);
        sync_all();
        SQ_T(l2);
        SQ_ACC(0, l0, l1);
        SQ_ACC(1, l1, l2);
        n = L.nnext;
        __syncthreads();
        if (tid == 0) L.nnext = 0u;
        uint32_t *tmp = fa;
        fa = fb;
        fb = tmp;
        __syncthreads();
    }
    if (tid == 0) {
        m.meta[3] = levels;
        for (int k = 0; k < 8; ++k) m.meta[16 + k] = uint32_t(prof[k] >> 8);
    }
}

// ---------------------------------------------------------------- radius 3, C <= 3: records + LDS frontier
// What a hole's colour needs besides the colours themselves -- its 29 disk
// weights, the gradient formula at each disk position, the weight sum, and
// which later holes read it -- depends on the stamps and distances only, so
// RECORD computes it for every hole of the chunk at once (one thread per
// hole, no ordering).  COLOUR3 then walks the Kahn levels with one round of
// loads per level: a 16-byte record slice and the hole's 61-pixel window of
// packed uint8 colours (the shadow image), 8 lanes per hole, 128 holes in
// flight, the frontier in LDS (entries past kFrCap in global memory).  The
// release atomics are issued as soon as the record's dependants mask lands,
// so their round trip overlaps the colour arithmetic.
constexpr int kL3 = 8;                   // lanes per hole
constexpr int kSlots3 = 1024 / kL3;      // holes in flight per workgroup
constexpr int kVal3 = 61;                // window (disk dilated by 3x3) incl. the centre
constexpr int kTerm3 = 9 * kDisk;        // 3 channels x (Ia, Jx, Jy) x disk positions
constexpr int kFrCap = 1280;             // LDS frontier entries per buffer
// a hole's LDS slot stride: >= kTerm3 and = 8 (mod 64 banks), so the 8 holes
// x 8 lanes of a wave hit 64 distinct banks on lane-contiguous accesses
constexpr int kBufStride = (kTerm3 + 55) / 64 * 64 + 8;
static_assert(kBufStride >= kTerm3 && kBufStride % 64 == 8, "slot stride");


// e-th position (raster order) of the window including its centre
__device__ __forceinline__ void val_pos(int e, int &a, int &b) {
    int n = 0;
    a = b = 0;
    for (int u = -4; u <= 4; ++u)
        for (int v = -4; v <= 4; ++v)
            if (win3(u, v)) {
                if (n == e) {
                    a = u;
                    b = v;
                }
                ++n;
            }
}

// Record of padded hole (i, j) with stamp s (layout: word 4*l + k = weight of
// disk position l + 8k; word 32 + l/2, bits 16*(l&1) + 4k = gradient codes of
// that position (x in bits 0-1, y in bits 2-3); words 36-37 = dependants
// mask over win_pos order; word 38 = cv2's weight sum).  Also the Kahn
// counter (record index << 6 | earlier holes in the window) and level 0.
constexpr int kRecTH = 16;  // RECORD tile: 64 x kRecTH padded pixels per workgroup
#ifndef OFD_REC_MINW  // RECORD waves per SIMD the register budget must allow (168 VGPRs at 3, no spill)
#define OFD_REC_MINW 3
#endif

__global__ __launch_bounds__(256, OFD_REC_MINW) void sq_record3_kernel(SqWs w) {
    // Only the holes whose stamps lie in this round's window [lo, hi) (the
    // pacing kernel's snapshot; the whole log in the final round).  Pixels
    // beyond it may be written by the march while this kernel runs: a racy
    // stamp read gives INF or a stamp >= hi, both later than any hole
    // recorded here, and a racy distance is only read where its stamp says
    // it is not used.
    // The workgroup's 64 x kRecTH pixels with a 4-pixel halo (clamped to the
    // padded image) of stamps and distances in LDS: every window read below
    // is an LDS read.  The tile's holes (~a fifth of its pixels) are listed
    // first and dealt to the threads densely, so a wave's lanes all work
    // (one thread per pixel left ~4 of 5 lanes idle in every wave).
    constexpr int TR = kRecTH + 8, TC = 64 + 8;
    __shared__ uint32_t Ls[TR][TC];
    __shared__ float Lt[TR][TC];
    __shared__ uint16_t hl[64 * kRecTH];
    __shared__ uint32_t nh;
    const int i0 = int(blockIdx.y) * kRecTH - 4, j0 = int(blockIdx.x) * 64 - 4;
    const Img m = image(w, blockIdx.z);
    const int eh = m.eh, ew = m.ew;
    const uint32_t lo = m.pipe[kPLo], hi = m.pipe[kPHi];
    if (lo >= hi) return;  // uniform: nothing of this image in the window
    if (threadIdx.x == 0) nh = 0u;
    for (int e = threadIdx.x; e < TR * TC; e += 256) {
        const int r = e / TC, c = e - r * TC;
        const int64_t q = int64_t(min(max(i0 + r, 0), eh - 1)) * ew + min(max(j0 + c, 0), ew - 1);
        Ls[r][c] = m.sI[q];
        Lt[r][c] = m.t[q];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * kRecTH; e += 256) {
        const int li = 4 + e / 64, lj = 4 + (e & 63);
        const int i = i0 + li, j = j0 + lj;
        const uint32_t sv = Ls[li][lj];
        const bool hole = i >= 1 && j >= 1 && i < eh - 1 && j < ew - 1 && sv != 0u && sv >= lo && sv < hi;
        const uint64_t bal = __ballot(hole);
        uint32_t base = 0;
        if ((threadIdx.x & 63) == 0 && bal) base = atomicAdd(&nh, uint32_t(__popcll(bal)));
        base = __shfl(base, 0);
        if (hole) hl[base + __popcll(bal & ((uint64_t(1) << (threadIdx.x & 63)) - 1))] = uint16_t(e);
    }
    __syncthreads();
    for (uint32_t h = threadIdx.x; h < nh; h += 256) {
        const int e = hl[h];
        const int li = 4 + e / 64, lj = 4 + (e & 63);
        const int i = i0 + li, j = j0 + lj;
        const int64_t p = int64_t(i) * ew + j;
        auto S = [&](int y, int x) -> uint32_t { return Ls[y - i0][x - j0]; };   // |y - i|, |x - j| <= 4
        auto TT = [&](int y, int x) -> float { return Lt[y - i0][x - j0]; };
        const uint32_t s = Ls[li][lj];
        // records are indexed by padded pixel (the region holds en records), so
        // COLOUR3 can address a dependant's record without a lookup
        const uint32_t idx = uint32_t(p);
        // Kahn counter and dependants: window positions inside the image (the
        // tile's clamped halo holds the image's own pixels there).  A hole not
        // pushed yet (INF) is a later one: a dependant.  h depends on an
        // earlier q at offset o iff o is among the positions h's colour reads
        // (need3, or all of win3 for a hole within 4 of the padded border,
        // whose disk may reach a border row or column); the same predicate,
        // with q's position, decides whether a later q depends on h (the
        // position sets are symmetric) -- the counter and the releases agree.
        const auto near_border = [&](int y, int x) { return y <= 4 || x <= 4 || y >= eh - 5 || x >= ew - 5; };
        const bool hb = near_border(i, j);
        uint32_t cnt = 0;
        uint64_t dep = 0, emask = 0;  // emask: the earlier holes counted (the levels-free colour pass waits on them)
        int bit = 0;
#pragma unroll
        for (int a = -4; a <= 4; ++a)
#pragma unroll
            for (int b = -4; b <= 4; ++b) {
                if (!win3(a, b) || !(a || b)) continue;
                const int y = i + a, x = j + b;
                if (y >= 1 && x >= 1 && y < eh - 1 && x < ew - 1) {
                    const uint32_t q = S(y, x);
                    if (q != 0u && q < s && (need3(a, b) || hb)) {
                        ++cnt;
                        emask |= uint64_t(1) << bit;
                    }
                    if (q > s && (need3(a, b) || near_border(y, x))) dep |= uint64_t(1) << bit;
                }
                ++bit;
            }
        // cv2's distance gradient at the hole
        const uint32_t su = S(i - 1, j), sd = S(i + 1, j), sl = S(i, j - 1), sr = S(i, j + 1);
        const float tij = TT(i, j), tu = TT(i - 1, j), td = TT(i + 1, j), tl = TT(i, j - 1), tr = TT(i, j + 1);
        float gtx, gty;
        if (!(sr >= s))
            gtx = !(sl >= s) ? (tr - tl) * 0.5f : (tr - tij);
        else
            gtx = !(sl >= s) ? (tij - tl) : 0.f;
        if (!(sd >= s))
            gty = !(su >= s) ? (td - tu) * 0.5f : (td - tij);
        else
            gty = !(su >= s) ? (tij - tu) : 0.f;
        uint32_t r[kRecW];
#pragma unroll
        for (int k = 0; k < kRecW; ++k) r[k] = 0u;
        float sum = 1.0e-20f;
        int d = 0;
#pragma unroll
        for (int a = -3; a <= 3; ++a)
#pragma unroll
            for (int b = -3; b <= 3; ++b) {
                if (!disk3(a, b)) continue;
                const int y = i + a, x = j + b;
                const bool inimg = y > 0 && x > 0 && y < eh - 1 && x < ew - 1;
                const bool used = inimg && !(S(y, x) >= s);
                const float ry = float(-a), rx = float(-b);
                const float len2 = rx * rx + ry * ry;
                const float dst = float(1. / (double(len2) * sqrt(double(len2))));
                const float lev = float(1. / (1 + fabs(double(TT(y, x) - tij))));
                float dir = rx * gtx + ry * gty;
                if (fabs(double(dir)) <= 0.01) dir = 0.000001f;
                const float wt = used ? float(fabs(double(dst * lev * dir))) : 0.f;
                sum += wt;
                const bool nr = !(S(y, x + 1) >= s), nl = !(S(y, x - 1) >= s);
                const bool nd = !(S(y + 1, x) >= s), nu = !(S(y - 1, x) >= s);
                const uint32_t cx = nr ? (nl ? 0u : 1u) : (nl ? 2u : 3u);
                const uint32_t cy = nd ? (nu ? 0u : 1u) : (nu ? 2u : 3u);
                const int l = d % kL3, k = d / kL3;
                r[4 * l + k] = __float_as_uint(wt);
                r[32 + l / 2] |= (cx | (cy << 2)) << (16 * (l & 1) + 4 * k);
                ++d;
            }
        r[36] = uint32_t(dep);
        r[37] = uint32_t(dep >> 32);
        r[23] = uint32_t(emask);  // spare weight slots (disk positions 29 and 30 of lanes 5 and 6)
        r[27] = uint32_t(emask >> 32);
        r[38] = __float_as_uint(sum);
        uint4 *dstp = reinterpret_cast<uint4 *>(m.rec + size_t(idx) * kRecW);
#pragma unroll
        for (int k = 0; k < kRecW / 4; ++k) dstp[k] = make_uint4(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]);
        // Kahn counter: kK - cnt here, + 1 per release of an earlier hole
        // (COLOUR3, before or after this): ready at kK, whoever adds last
        // (cnt <= 60 < kK, so the releases alone never reach it).  No COLOUR3
        // runs while RECORD does (one stream orders the rounds), so the
        // releases so far are a plain read and the sum a plain store (a
        // returning atomic per hole cost ~10 ms per 64 images).
        const uint32_t rel = m.kc[p];
        m.kc[p] = kK - cnt + rel;
        if (rel == cnt) m.rq[atomicAdd(&m.meta[2], 1u)] = (uint64_t(idx) << 32) | uint64_t(p);
    }
}

struct C3Lds {
    uint32_t nnext[3];  // level l appends to nnext[l % 3]; reset two levels ahead (one barrier per level)
    uint32_t stop[3];   // level l's deadline verdict (thread 0, before the level's barrier; same rotation)
    uint64_t fr[2][kFrCap];
    float buf[kSlots3][kBufStride];  // per hole: the 9x9 colour grid (81 words), then the terms
    float res[kSlots3][9];       // per hole: chain results (Ia, Jx, Jy per channel)
#if OFD_C3_PF
    uint32_t dump[64];  // prefetch loads' discarded words
#endif
};

// Pipelined rounds are time-bounded: round e stops at a level boundary once
// the constant-rate clock passes t0 + (e + 2) * round_ticks (t0: the pacing
// origin; the next round's scheduled start) and leaves its next level in cy
// for round e + 1, so every image's chain keeps moving between rounds instead
// of each round lasting as long as its slowest image.  fin: no deadline.
// The colours do not depend on how the levels are grouped: a hole is
// coloured once all its earlier neighbours are, whichever round that is.
__global__ __launch_bounds__(1024) void sq_colour3_kernel(SqWs w, int C, int H, int W, int e, int fin,
                                                          uint64_t round_ticks) {
    __shared__ C3Lds L;
    const int tid = threadIdx.x, g = tid / kL3, gl = tid % kL3;
    const Img m = image(w, blockIdx.x);
    const int eh = m.eh, ew = m.ew;
    uint8_t *shb = reinterpret_cast<uint8_t *>(m.shd);
    // this lane's window loads, dependants bits and disk positions, as 9x9
    // grid cells (row-major, centre 40)
    // (packed per k: window load cell | dependant cell << 8 | disk cell << 16)
    int tb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int a, b;
        val_pos(gl + kL3 * k, a, b);
        tb[k] = (a + 4) * 9 + b + 4;
        win_pos(gl + kL3 * k, a, b);
        tb[k] |= ((a + 4) * 9 + b + 4) << 8;
        if (k < 4) {
            disk_pos(gl + kL3 * k, a, b);
            tb[k] |= ((a + 4) * 9 + b + 4) << 16;
        }
    }
#define VC(k) (tb[k] & 0xFF)
#define WC(k) ((tb[k] >> 8) & 0xFF)
#define DC(k) (tb[k] >> 16)
    // this round's first level: the frontier the round before left (cy),
    // then the ready queue's new entries (RECORD's holes whose earlier
    // neighbours are all coloured); entries past the LDS capacity go to fr3,
    // later levels' alternate between fr2 and fr3
    const uint32_t q0 = m.pipe[kPRqc], q1 = m.meta[2], nc = m.pipe[kPCarry];
    uint64_t *ga = m.fr3, *gb = m.fr2;
    int cur = 0;
    uint32_t n = nc + (q1 - q0), levels = 0, rounds = 0, small = 0;
    if (tid == 0 && n) {
        if (m.pipe[kPCRounds] == 0u) put64(m.pipe + kPTc0, wall_clock64());
        m.pipe[kPCRounds] += 1u;
    }
    for (uint32_t x = tid; x < n; x += 1024) {
        const uint64_t en = x < nc ? m.cy[x] : m.rq[q0 + (x - nc)];
        if (x < uint32_t(kFrCap))
            L.fr[0][x] = en;
        else
            ga[x] = en;
    }
    const uint64_t deadline =
        (fin || w.pipe[kPAllDone]) ? ~uint64_t(0)
            : (uint64_t(w.pipe[kPT0]) | (uint64_t(w.pipe[kPT0 + 1]) << 32)) + round_ticks * uint64_t(e + 2);
    if (tid == 0) L.nnext[0] = 0u;
    sync_all();  // (fr3's entries are read back by other waves)
    const int nch = 3 * C;
    int lv = 0;  // chains: (Ia, Jx, Jy) per channel
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)prof;
    bool stopped = false;
    while (n) {
        if (levels && L.stop[lv == 0 ? 2 : lv - 1]) {  // the level before passed the deadline (uniform)
            stopped = true;
            break;
        }
        ++levels;
        rounds += (n + kSlots3 - 1) / kSlots3;
        small += n <= uint32_t(kSlots3 / 2) ? 1u : 0u;
        // the counter the next level appends to: last read right after the
        // barrier that ended the level before the previous one
        if (tid == 0) L.nnext[lv == 2 ? 0 : lv + 1] = 0u;
        SQ_T(l0);
        for (uint32_t base = 0; base < n; base += kSlots3) {
            if (base + uint32_t(tid / 64) * (64 / kL3) >= n) continue;  // no hole of this round in this wave
            SQ_T(c0);
            // keep the lane tables opaque, so the compiler does not hoist
            // their derived offsets out of the loop (register pressure)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(tb[k]));
            const uint32_t e = base + g;
            const bool act = e < n;
            uint64_t ent = 0;
            if (act) ent = e < uint32_t(kFrCap) ? L.fr[cur][e] : ga[e];
            const uint32_t idx = uint32_t(ent >> 32), p = uint32_t(ent);
            const int i = int(p / uint32_t(ew)), j = int(p - uint32_t(i) * uint32_t(ew));
            // the level's one round of loads
            const uint32_t *rp = m.rec + size_t(idx) * kRecW;
            uint4 wq = make_uint4(0, 0, 0, 0), cq = wq, mq = wq;
            uint32_t v[8];
            if (act) {
                wq = *reinterpret_cast<const uint4 *>(rp + 4 * gl);
                cq = *reinterpret_cast<const uint4 *>(rp + 32);
                mq = *reinterpret_cast<const uint4 *>(rp + 36);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int y = min(max(i - 5 + VC(k) / 9, 0), H - 1), x = min(max(j - 5 + VC(k) % 9, 0), W - 1);
                    v[k] = (gl + kL3 * k < kVal3) ? m.shd[int64_t(y) * W + x] : 0u;
                }
            }
            SQ_T(c0a);
            float *bf = L.buf[g];
            uint32_t *gv = reinterpret_cast<uint32_t *>(bf);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (gl + kL3 * k < kVal3) gv[VC(k)] = v[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // release the later holes that read this one (their counters
            // reach zero only after this level's barrier is passed).  Issued
            // after the loads have landed, so no wait for the loads also
            // waits for these: their round trip overlaps the arithmetic.
            const uint64_t dep = uint64_t(mq.x) | (uint64_t(mq.y) << 32);
            uint32_t old[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                old[k] = 0;
                if (act && gl + kL3 * k < kWin && ((dep >> (gl + kL3 * k)) & 1u)) {
                    const int64_t q = int64_t(p) + int64_t(WC(k) / 9 - 4) * ew + (WC(k) % 9 - 4);
#if OFD_C3_PF
                    // the dependant's record (two 128-byte lines) towards this
                    // CU: a later level loads it (into a discarded LDS word)
                    const uint32_t *qr = m.rec + size_t(q) * kRecW;
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)qr,
                                                     (__attribute__((address_space(3))) void *)L.dump, 4, 0, 0);
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(qr + kRecW - 1),
                                                     (__attribute__((address_space(3))) void *)L.dump, 4, 0, 0);
#endif
                    old[k] = atomicAdd(&m.kc[q], 1u);
                }
            }
            // the holes whose last earlier neighbour this was join the next level
            auto append_ready = [&]() {
                // the returned counters stay opaque until here: otherwise the
                // compiler folds each into its compare at once and waits for
                // every atomic in turn (eight round trips per level, ~+35% time)
                asm volatile("" : "+v"(old[0]), "+v"(old[1]), "+v"(old[2]), "+v"(old[3]), "+v"(old[4]), "+v"(old[5]),
                             "+v"(old[6]), "+v"(old[7]));
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (old[k] + 1u == kK) {
                        const uint32_t f = atomicAdd(&L.nnext[lv], 1u);
                        const int64_t q = int64_t(p) + int64_t(WC(k) / 9 - 4) * ew + (WC(k) % 9 - 4);
                        const uint64_t en = (uint64_t(q) << 32) | uint64_t(q);
                        if (f < uint32_t(kFrCap))
                            L.fr[cur ^ 1][f] = en;
                        else
                            gb[f] = en;
                    }
            };
            SQ_T(c1);
            // this lane's terms (disk positions gl + 8k): channels 1 and 2 go
            // to LDS at once (past the grid), channel 0 waits in registers
            // until every lane of the hole is done with the grid
            const uint32_t wts[4] = {wq.x, wq.y, wq.z, wq.w};
            const uint32_t cw = (gl >> 1) == 0 ? cq.x : (gl >> 1) == 1 ? cq.y : (gl >> 1) == 2 ? cq.z : cq.w;
            const uint32_t codes = cw >> (16 * (gl & 1));
            float t0[4][3];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int a = DC(k) / 9 - 4, b = DC(k) % 9 - 4, y = i + a, x = j + b;
                const int k1 = y == 1, kE = y == eh - 2, l1 = x == 1, lE = x == ew - 2;
                auto G = [&](int ry, int rx) -> uint32_t {  // colour word at window offset (ry, rx), |ry|, |rx| <= 4
                    return gv[(ry + 4) * 9 + rx + 4];
                };
                const uint32_t w0 = G(a + k1, b + l1), w1 = G(a + k1, b + 1 - lE), w2 = G(a + k1, b - 1 + l1),
                               w3 = G(a + k1, b - lE), w4 = G(a + 1 - kE, b + l1), w5 = G(a - 1 + k1, b + l1),
                               w6 = G(a - kE, b + l1);
                const float wt = __uint_as_float(wts[k]);
                const uint32_t cx = (codes >> (4 * k)) & 3u, cy = (codes >> (4 * k + 2)) & 3u;
                // cv2's gradient cases as (A - B) * f, selected once for all channels:
                // code 0: (v1 - v2) * 2, 1: (v1 - v0), 2: (v3 - v2), 3: none ((v0 - v0) * 0 = +0)
                const uint32_t xa = cx <= 1u ? w1 : (cx == 2u ? w3 : w0), xb = (cx & 1u) ? w0 : w2;
                const uint32_t ya = cy <= 1u ? w4 : (cy == 2u ? w6 : w0), yb = (cy & 1u) ? w0 : w5;
                // gix * rx = (A - B) * (f * rx) exactly: integers below 2^24 (the
                // sign of an exact zero may differ, which no result can see)
                const float kx = (cx == 0u ? 2.0f : (cx == 3u ? 0.0f : 1.0f)) * float(-b);
                const float ky = (cy == 0u ? 2.0f : (cy == 3u ? 0.0f : 1.0f)) * float(-a);
                const bool live = gl + kL3 * k < kDisk;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    auto byte = [&](uint32_t q) -> int { return int((q >> (8 * c)) & 0xFFu); };
                    const float vs = float(byte(w0));
                    const float dx = float(byte(xa) - byte(xb)), dy = float(byte(ya) - byte(yb));
                    const float ta = wt * vs, tx = wt * (dx * kx), ty = wt * (dy * ky);
                    if (c == 0) {
                        t0[k][0] = ta;
                        t0[k][1] = tx;
                        t0[k][2] = ty;
                    } else if (live) {  // chains past 3 * C are never summed
                        bf[(3 * c) * kDisk + gl + kL3 * k] = ta;
                        bf[(3 * c + 1) * kDisk + gl + kL3 * k] = tx;
                        bf[(3 * c + 2) * kDisk + gl + kL3 * k] = ty;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (gl + kL3 * k < kDisk)
#pragma unroll
                    for (int q = 0; q < 3; ++q) bf[q * kDisk + gl + kL3 * k] = t0[k][q];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            SQ_T(c2);
            // cv2's sums in its (k, l) order: chains gl and gl + 8 side by side
            // (independent accumulators; Ia chains add, Jx / Jy chains subtract)
            {
                const int c1 = gl, c2 = gl + kL3;
                const bool has2 = c2 < nch;
                const float *t1 = bf + c1 * kDisk, *t2 = bf + (has2 ? c2 : c1) * kDisk;
                const float s1 = c1 % 3 == 0 ? 1.f : -1.f, s2 = c2 % 3 == 0 ? 1.f : -1.f;
                float a1 = 0.f, a2 = 0.f;
#pragma unroll
                for (int q = 0; q < kDisk; ++q) {
                    a1 += s1 * t1[q];  // x * +-1 is exact: acc + (-t) == acc - t
                    a2 += s2 * t2[q];
                }
                if (c1 < nch) L.res[g][c1] = a1;
                if (has2) L.res[g][c2] = a2;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            SQ_T(c3);
            if (act && gl < C) {
                const float sum = __uint_as_float(mq.z);
                const float Ia = L.res[g][3 * gl], Jx = L.res[g][3 * gl + 1], Jy = L.res[g][3 * gl + 2];
                const float sat = float(double(Ia / sum) +
                                        double(Jx + Jy) / (sqrt(double(Jx * Jx + Jy * Jy)) + double(1.0e-20f)) +
                                        double(0.5f));
                const unsigned u = sat_u8(sat);
                shb[4 * (int64_t(i - 1) * W + (j - 1)) + gl] = uint8_t(u);
            }
            append_ready();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            SQ_T(c4);
            SQ_ACC(2, c0, c0a);
            SQ_ACC(6, c0a, c1);
            SQ_ACC(3, c1, c2);
            SQ_ACC(4, c2, c3);
            SQ_ACC(5, c3, c4);
        }
        SQ_T(l1);
        if (tid == 0) L.stop[lv] = wall_clock64() >= deadline ? 1u : 0u;
        sync_all();
        SQ_T(l2);
        SQ_ACC(0, l0, l1);
        SQ_ACC(1, l1, l2);
        // one barrier per level: the next level writes the frontier buffer
        // and counter this one read (all reads done before the barrier) and
        // appends to a counter zeroed before it
        n = L.nnext[lv];
        lv = lv == 2 ? 0 : lv + 1;
        cur ^= 1;
        ga = gb;
        gb = gb == m.fr2 ? m.fr3 : m.fr2;
    }
    // a stopped round leaves its next level for the next round
    const uint32_t left = stopped ? n : 0u;
    for (uint32_t x = tid; x < left; x += 1024) m.cy[x] = x < uint32_t(kFrCap) ? L.fr[cur][x] : ga[x];
    if (tid == 0) {
        if (levels && !stopped) put64(m.pipe + kPTc1, wall_clock64());
        m.pipe[kPCarry] = left;
        m.pipe[kPRqc] = q1;
        m.meta[3] += levels;
        m.meta[6] += rounds;  // load rounds of kSlots3 holes (levels of more holes take several)
        m.meta[7] += small;   // levels of at most kSlots3 / 2 holes
        for (int k = 0; k < 8; ++k) m.meta[16 + k] = uint32_t(prof[k] >> 8);
    }
}
#undef VC
#undef WC
#undef DC


// COLOUR3 without levels (the default colour pass since round 5;
// ofd_inpaint_seq_set_colour(0) / OFD_SEQ_DF=0 select the level-synchronous
// COLOUR3 above): the ready holes sit in a
// queue (fr2, positions carried across rounds in kPQh / kPQt); each wave
// takes up to 8 of them, colours them with COLOUR3's per-hole code, and
// queues the holes its releases completed -- no workgroup barrier, so a
// hole starts as soon as its last earlier neighbour has released it.  The
// releases are issued before a hole's colour exists (their round trip
// overlaps the arithmetic), so a hole first waits for each earlier
// neighbour it reads to carry the coloured flag (byte 3 of its word: PREP
// sets it on kept pixels, the colour store on holes).  A wave leaves when
// the queue is empty and no wave holds a hole, or at the deadline (the
// queue is carried to the next round).  Every wait is bounded (fault 32).
#ifndef OFD_DF_WOFF  // levels-free pass: window-cell offsets from packed row / column bits
#define OFD_DF_WOFF 1
#endif
#ifndef OFD_DF_A32  // levels-free pass: per-image indices in 32 bits (no 64-bit multiply-adds)
#define OFD_DF_A32 1
#endif
#if OFD_DF_A32
#define IX32(e) uint32_t(e)
#else
#define IX32(e) int64_t(e)
#endif
#ifndef OFD_DF_SPIN  // levels-free pass: re-check only the still-missing cells while waiting
#define OFD_DF_SPIN 1
#endif
#ifndef OFD_DF_SLEEP  // ... and the wait's s_sleep between checks (64 clocks per unit)
#define OFD_DF_SLEEP 1
#endif
constexpr int kDfQ = 512;    // queue entries held in LDS (the rest in fr2)
template <int kThr>
struct C3DfLds {
    static constexpr int kCt = kThr >= 1024 ? 2048 : 1024;  // recent-colour table entries
    float buf[kThr / kL3][kBufStride];
    float res[kThr / kL3][9];
    uint64_t ct[kCt];  // recent colours: (position + 1) | word << 32, by position mod kCt
    uint64_t ring[kDfQ];  // queue entry y: (y + 1) | position << 32 at y mod kDfQ, or in fr2[y]
    uint32_t qh, qr, qp, inflight;
    uint32_t gbase;       // kMW: the shared-queue slots the round-end flush reserved
};
constexpr int kPQh = 52, kPQt = 53;  // pipe words: the queue's head and tail
// Several workgroups per image (kMW, ofd_inpaint_seq_set_multi): the image's
// ready holes sit in RECORD's rq (claimed by a CAS on kPRqc), in the
// workgroups' LDS queues, and in a shared queue in cy (a ring of en tagged
// granules, (position << 32) | (slot + 1), head kPGh / tail kPGt, device-scope
// atomics).  kPGo counts the holes queued in LDS or in the shared queue or
// being coloured, so a workgroup with nothing left leaves only when every
// workgroup of its image has nothing left either.
constexpr int kPGh = 54, kPGt = 55, kPGo = 56;
#ifndef OFD_MW_CAP  // kMW: LDS queue length past which a wave's new ready holes go to the shared queue
#define OFD_MW_CAP 16
#endif
#ifndef OFD_MW_THR  // kMW: threads per workgroup
#define OFD_MW_THR 512
#endif
static_assert(OFD_MW_THR <= 512, "kMW overflow slices are sized for at most 8 waves per workgroup");
#ifndef OFD_MW_APPEND_WAIT  // kMW: 1 = every append waits for its count to land (A/B)
#define OFD_MW_APPEND_WAIT 0
#endif
#ifndef OFD_MW_RELOAD  // kMW: a waiting hole re-reads a missing neighbour's word every this many tries
#define OFD_MW_RELOAD 2
#endif

template <int kThr, bool kMW>
__global__ __launch_bounds__(kThr) void sq_colour3df_kernel(SqWs w, int C, int H, int W, int e, int fin,
                                                            uint64_t round_ticks, int kw) {
    __shared__ C3DfLds<kThr> L;
    constexpr int kDfCt = C3DfLds<kThr>::kCt;
    const int tid = threadIdx.x, g = tid / kL3, gl = tid % kL3, lane = tid & 63;
    // kMW: kw workgroups per image, image-major (blocks b * kw .. b * kw + kw - 1)
    const int wr = kMW ? int(blockIdx.x) % kw : 0;
    const Img m = image(w, kMW ? int(blockIdx.x) / kw : int(blockIdx.x));
    // kMW: this workgroup's overflow slice of fr2 (LDS queue entries past kDfQ)
    const uint32_t ovf = kMW ? uint32_t(m.en / kw) : 0u, ovf0 = uint32_t(wr) * ovf;
    uint32_t *pw = m.pipe;
    const int eh = m.eh, ew = m.ew;
    const int wbias = 4 * ew + 4;
    (void)eh;
    (void)wbias;
    int tb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int a, b;
        val_pos(gl + kL3 * k, a, b);
        tb[k] = (a + 4) * 9 + b + 4;
        win_pos(gl + kL3 * k, a, b);
        tb[k] |= ((a + 4) * 9 + b + 4) << 8;
#if OFD_DF_WOFF
        tb[k] |= int((uint32_t(a + 4) << 24) | (uint32_t(b + 4) << 28));  // the window cell's row / column + 4
#endif
        if (k < 4) {
            disk_pos(gl + kL3 * k, a, b);
            tb[k] |= ((a + 4) * 9 + b + 4) << 16;
        }
    }
#define VC(k) (tb[k] & 0xFF)
#define WC(k) ((tb[k] >> 8) & 0xFF)
#define DC(k) ((tb[k] >> 16) & 0xFF)
#if OFD_DF_WOFF  // pixel offset of window cell WC(k): packed row / column, no division by 9
#define WOFF(k) (int((uint32_t(tb[k]) >> 24) & 15u) * ew + int(uint32_t(tb[k]) >> 28) - wbias)
#else
#define WOFF(k) ((WC(k) / 9 - 4) * ew + (WC(k) % 9 - 4))
#endif
    // the queue: carried entries, then RECORD's new ready holes (kMW: the
    // LDS queue starts empty; rq and the shared queue are claimed directly)
    const uint32_t q0 = m.pipe[kPRqc], q1 = m.meta[2], h0 = kMW ? 0u : m.pipe[kPQh], t0q = kMW ? 0u : m.pipe[kPQt];
    if constexpr (!kMW)
        for (uint32_t x = tid; x < q1 - q0; x += kThr) m.fr2[t0q + x] = m.rq[q0 + x];
    for (int x = tid; x < kDfCt; x += kThr) L.ct[x] = 0ull;
    for (int x = tid; x < kDfQ; x += kThr) L.ring[x] = 0ull;
    if (tid == 0) {
        L.qh = h0;
        L.qr = L.qp = kMW ? 0u : t0q + (q1 - q0);
        L.inflight = 0u;
        const bool work = kMW ? (q0 < q1 || __hip_atomic_load(pw + kPGo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
                              : h0 < t0q + (q1 - q0);
        if (work && wr == 0) {
            if (m.pipe[kPCRounds] == 0u) put64(m.pipe + kPTc0, wall_clock64());
            m.pipe[kPCRounds] += 1u;
        }
    }
    sync_all();
    const uint64_t deadline =
        (fin || w.pipe[kPAllDone]) ? ~uint64_t(0)
            : (uint64_t(w.pipe[kPT0]) | (uint64_t(w.pipe[kPT0 + 1]) << 32)) + round_ticks * uint64_t(e + 2);
    const uint64_t tstart = wall_clock64();
    const int nch = 3 * C;
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    (void)prof;
    uint32_t batches = 0;
    for (;;) {
        // take up to 8 entries: read their ring slots first, then claim them
        // with a CAS on the head -- a producer overwrites the slot of entry y
        // only once the head has passed y - kDfQ (its space check), so slots
        // read before a successful claim hold the claimed entries or stale tags
        uint32_t take = 0, qbase = 0;
        uint64_t se = 0;
        for (int t = 0; t < 64; ++t) {
            uint32_t h = 0, pq = 0;
            if (lane == 0) {
                h = __hip_atomic_load(&L.qh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                pq = __hip_atomic_load(&L.qp, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            h = __shfl(h, 0);
            pq = __shfl(pq, 0);
            if (h >= pq) break;  // (no provisional count while the queue is empty: the "all done" test sees 0)
            const uint32_t want = pq - h < 8u ? pq - h : 8u;
            if (uint32_t(lane) < want)
                se = __hip_atomic_load(&L.ring[(h + uint32_t(lane)) & uint32_t(kDfQ - 1)], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            asm volatile("" : "+v"(se));  // read before the claim
            uint32_t ok = 0;
            if (lane == 0) {
                atomicAdd(&L.inflight, 8u);  // before the take: no false "all done"
                if (atomicCAS(&L.qh, h, h + want) == h) {
                    ok = 1u;
                    atomicSub(&L.inflight, 8u - want);
                } else {
                    atomicSub(&L.inflight, 8u);
                }
            }
            if (__shfl(ok, 0)) {
                take = want;
                qbase = h;
                break;
            }
        }
        // kMW, nothing in the LDS queue: claim up to 8 holes of RECORD's rq,
        // else of the shared queue (src 1 / 2; 0 = the LDS queue)
        uint32_t src = 0;
        if constexpr (kMW) {
            if (take == 0u) {
                uint32_t tk = 0, qb = 0, sr = 0;
                if (lane == 0) {
                    // no provisional L.inflight here: the image's count kPGo
                    // covers a claimed batch until its end (idle waves adding
                    // to L.inflight while they poll kept their workgroup from
                    // ever seeing itself idle)
                    uint32_t c = __hip_atomic_load(pw + kPRqc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    // rq's holes are counted when claimed: 8 provisionally,
                    // returned before the claim, so no workgroup of the image
                    // sees rq drained and the count at 0 while this batch runs
                    const bool try_rq = c < q1;
                    if (try_rq) {
                        (void)__hip_atomic_fetch_add(pw + kPGo, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                    for (int t = 0; t < 64 && c < q1 && tk == 0u; ++t) {
                        const uint32_t want = q1 - c < 8u ? q1 - c : 8u;
                        const uint32_t o = atomicCAS(pw + kPRqc, c, c + want);
                        if (o == c) {
                            tk = want;
                            qb = c;
                            sr = 1u;
                        } else {
                            c = o;
                        }
                    }
                    if (try_rq && tk < 8u)
                        (void)__hip_atomic_fetch_sub(pw + kPGo, 8u - tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (tk == 0u) {
                        uint32_t gh = __hip_atomic_load(pw + kPGh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint32_t gt = __hip_atomic_load(pw + kPGt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        for (int t = 0; t < 64 && gh < gt && tk == 0u; ++t) {
                            const uint32_t want = gt - gh < 8u ? gt - gh : 8u;
                            const uint32_t o = atomicCAS(pw + kPGh, gh, gh + want);
                            if (o == gh) {
                                tk = want;
                                qb = gh;
                                sr = 2u;
                            } else {
                                gh = o;
                            }
                        }
                    }
                    if (tk) atomicAdd(&L.inflight, tk);  // the batch end's subtraction is uniform
                }
                take = __shfl(tk, 0);
                qbase = __shfl(qb, 0);
                src = __shfl(sr, 0);
            }
        }
        if (take == 0u) {
            uint32_t quit = 0;
            if (lane == 0) {
                const uint64_t now = wall_clock64();
                const uint32_t h = __hip_atomic_load(&L.qh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const uint32_t pq = __hip_atomic_load(&L.qp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const uint32_t inf = __hip_atomic_load(&L.inflight, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                bool none = h >= pq && inf == 0u;
                if (kMW && none)  // the image's other workgroups may still queue holes for the shared queue
                    none = __hip_atomic_load(pw + kPRqc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= q1 &&
                           __hip_atomic_load(pw + kPGo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
                quit = none || now >= deadline ? 1u : 0u;
                if (now - tstart > 400000000ull) {  // 4 s: cannot happen
                    atomicOr(&g_sq_fault, 32u);
#ifdef OFD_MW_DEBUG
                    if (kMW)
                        printf("MWDBG idle img %d wr %d fin %d h %u pq %u inf %u rqc %u q1 %u go %u gh %u gt %u\n",
                               int(blockIdx.x) / kw, wr, fin, h, pq, inf,
                               __hip_atomic_load(pw + kPRqc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), q1,
                               __hip_atomic_load(pw + kPGo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __hip_atomic_load(pw + kPGh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                               __hip_atomic_load(pw + kPGt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#endif
                    quit = 1u;
                }
            }
            if (__shfl(quit, 0)) break;
            __builtin_amdgcn_s_sleep(kMW ? 2 : 1);
            continue;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        SQ_T(c0);
        {
            // keep the lane tables opaque, so the compiler does not hoist
            // their derived offsets out of the loop (register pressure)
#pragma unroll
            for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(tb[k]));
            const bool act = uint32_t(g & 7) < take;  // the wave's 8 hole slots
            const uint32_t y = qbase + uint32_t(g & 7);
            uint64_t ent = __shfl(se, g & 7);
            if constexpr (kMW) {
                if (src == 1u) {
                    ent = act ? m.rq[y] : 0ull;  // RECORD's (pixel << 32 | pixel), written before this launch
                } else if (src == 2u) {
                    if (act) {  // the shared queue's granule: poll until its tag is the slot's
                        const uint32_t sl = y % uint32_t(m.en);
                        for (int t = 0;; ++t) {
                            ent = __hip_atomic_load(m.cy + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (uint32_t(ent) == y + 1u) break;
                            if (t > (1 << 22)) {  // cannot happen: a reserved slot is written right after
                                atomicOr(&g_sq_fault, 32u);
#ifdef OFD_MW_DEBUG
                                if (gl == 0) printf("MWDBG gqpoll wr %d y %u tag %u\n", wr, y, uint32_t(ent));
#endif
                                break;
                            }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                } else if (act && uint32_t(ent) != y + 1u) {
                    ent = m.fr2[ovf0 + y % ovf];  // not in the ring: this workgroup's overflow slice
                }
            } else if (act && uint32_t(ent) != y + 1u) {
                ent = m.fr2[y];  // not in the ring: fr2 (pixel << 32 | pixel)
            }
            const uint32_t p = uint32_t(ent >> 32), idx = p;
            const int i = int(p / uint32_t(ew)), j = int(p - uint32_t(i) * uint32_t(ew));
            // the level's one round of loads
            const uint32_t *rp = m.rec + size_t(idx) * kRecW;
            uint4 wq = make_uint4(0, 0, 0, 0), cq = wq, mq = wq;
            uint32_t v[8];
            if (act) {
                wq = *reinterpret_cast<const uint4 *>(rp + 4 * gl);
                cq = *reinterpret_cast<const uint4 *>(rp + 32);
                mq = *reinterpret_cast<const uint4 *>(rp + 36);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int y = min(max(i - 5 + VC(k) / 9, 0), H - 1), x = min(max(j - 5 + VC(k) % 9, 0), W - 1);
                    v[k] = (gl + kL3 * k < kVal3)
                               ? __hip_atomic_load(m.shd + IX32(y * W + x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                               : 0u;
                }
            }
            SQ_T(c0a);
            float *bf = L.buf[g];
            uint32_t *gv = reinterpret_cast<uint32_t *>(bf);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (gl + kL3 * k < kVal3) gv[VC(k)] = v[k];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // the earlier holes this one reads (RECORD's mask in the record's
            // spare weight words 23 and 27: lanes 5 and 6 of the hole) may
            // have released it before storing their colour: wait until each
            // one's word carries the coloured flag (byte 3), re-reading the
            // window past the vector L1
            {
                const int hl0 = (tid & 63) & ~(kL3 - 1);
                const uint32_t elo = __shfl(wq.w, hl0 + 5), ehi = __shfl(wq.w, hl0 + 6);
                const uint64_t em = act ? (uint64_t(elo) | (uint64_t(ehi) << 32)) : 0ull;
#if OFD_DF_SPIN
                // this lane's window cells whose earlier hole has no colour
                // yet; only those are looked up again (a waiting wave's issue
                // is taken from the waves that colour)
                uint32_t pend = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (gl + kL3 * k < kWin && ((em >> (gl + kL3 * k)) & 1u) && (gv[WC(k)] >> 24) == 0u) pend |= 1u << k;
                for (int tries = 0; __any(pend != 0u); ++tries) {
                    if (tries > (1 << 20)) {  // cannot happen: every released hole is being coloured
                        if (gl == 0) atomicOr(&g_sq_fault, 32u);
#ifdef OFD_MW_DEBUG
                        if (gl == 0) printf("MWDBG flagwait wr %d p %u pend %x\n", wr, p, pend);
#endif
                        break;
                    }
                    // the table entry may have been displaced, or (kMW) the
                    // neighbour coloured by another workgroup of the image
                    const bool reload = kMW ? (tries % OFD_MW_RELOAD) == OFD_MW_RELOAD - 1 : (tries & 7) == 7;
#pragma unroll
                    for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(tb[k]));  // no hoisted offsets (spills)
                    // every pending cell's lookup first (the table, else on a
                    // reload try the word itself: all reloads in flight at
                    // once), then the flags
                    uint32_t wvk[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        wvk[k] = 0u;
                        if (pend & (1u << k)) {
                            const uint32_t q = p + uint32_t(WOFF(k));
                            const uint64_t ce = __hip_atomic_load(&L.ct[q & uint32_t(kDfCt - 1)], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (uint32_t(ce) == q + 1u)
                                wvk[k] = uint32_t(ce >> 32);
                            else if (reload)  // an interior hole: no clamp
                                wvk[k] = __hip_atomic_load(
                                    m.shd + IX32((i - 5 + WC(k) / 9) * W + (j - 5 + WC(k) % 9)), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
                        }
                    }
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if ((pend & (1u << k)) && (wvk[k] >> 24) != 0u) {
                            gv[WC(k)] = wvk[k];
                            pend &= ~(1u << k);
                        }
                    if (!__any(pend != 0u)) break;
                    __builtin_amdgcn_s_sleep(OFD_DF_SLEEP);
                }
#else
                for (int tries = 0;; ++tries) {
                    bool miss = false;
#pragma unroll
                    for (int k = 0; k < 8; ++k) asm volatile("" : "+v"(tb[k]));  // no hoisted offsets (spills)
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (gl + kL3 * k < kWin && ((em >> (gl + kL3 * k)) & 1u) && (gv[WC(k)] >> 24) == 0u) {
                            // the workgroup's table of recent colours first
                            const uint32_t q = p + uint32_t(WOFF(k));
                            const uint64_t ce = __hip_atomic_load(&L.ct[q & uint32_t(kDfCt - 1)], __ATOMIC_RELAXED,
                                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (uint32_t(ce) == q + 1u)
                                gv[WC(k)] = uint32_t(ce >> 32);
                            else
                                miss = true;
                        }
                    if (!__any(miss)) break;
                    if (tries > (1 << 20)) {  // cannot happen: every released hole is being coloured
                        if (gl == 0) atomicOr(&g_sq_fault, 32u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    if ((tries & 7) != 7) continue;  // the table entry may have been displaced: re-read now and then
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int y = min(max(i - 5 + VC(k) / 9, 0), H - 1), x = min(max(j - 5 + VC(k) % 9, 0), W - 1);
                        if (act && gl + kL3 * k < kVal3)
                            gv[VC(k)] = __hip_atomic_load(m.shd + IX32(y * W + x), __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
#endif
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            // release the later holes that read this one (their counters
            // reach zero only after this level's barrier is passed).  Issued
            // after the loads have landed, so no wait for the loads also
            // waits for these: their round trip overlaps the arithmetic.
            const uint64_t dep = uint64_t(mq.x) | (uint64_t(mq.y) << 32);
            uint32_t old[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                old[k] = 0;
                if (act && gl + kL3 * k < kWin && ((dep >> (gl + kL3 * k)) & 1u)) {
                    const auto q = IX32(p + uint32_t(WOFF(k)));
#if OFD_C3_PF
                    // the dependant's record (two 128-byte lines) towards this
                    // CU: a later level loads it (into a discarded LDS word)
                    const uint32_t *qr = m.rec + size_t(q) * kRecW;
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)qr,
                                                     (__attribute__((address_space(3))) void *)L.dump, 4, 0, 0);
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(qr + kRecW - 1),
                                                     (__attribute__((address_space(3))) void *)L.dump, 4, 0, 0);
#endif
                    old[k] = atomicAdd(&m.kc[q], 1u);
                }
            }
            // the holes whose last earlier neighbour this was join the queue
            // (after this hole's colour is stored: the caller's order): slots
            // reserved with one LDS atomic per wave, written, then published
            // in reservation order
            auto append_ready = [&]() {
                asm volatile("" : "+v"(old[0]), "+v"(old[1]), "+v"(old[2]), "+v"(old[3]), "+v"(old[4]), "+v"(old[5]),
                             "+v"(old[6]), "+v"(old[7]));
                unsigned rmask = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) rmask |= (old[k] + 1u == kK ? 1u : 0u) << k;
                const uint32_t cnt = uint32_t(__popc(rmask));
                const int lane = tid & 63;
                // inclusive prefix of cnt (0..8) over the wave by bit planes:
                // four ballots instead of six dependent lane shuffles
                uint32_t incl = 0, tot = 0;
                {
                    const uint64_t upto = ~uint64_t(0) >> (63 - lane);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint64_t bal = __ballot((cnt >> k) & 1u);
                        incl += uint32_t(__popcll(bal & upto)) << k;
                        tot += uint32_t(__popcll(bal)) << k;
                    }
                }
                if (tot == 0u) return;  // wave-uniform
                uint32_t rb = 0, hq = 0, sp = 0;
                if (lane == 63) {
                    hq = __hip_atomic_load(&L.qh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if constexpr (kMW) {
                        // Holes for the shared queue are counted before any of
                        // them can be taken (the add has returned before the
                        // slots are published), so the image's count never
                        // misses a hole another workgroup could take.  Holes
                        // for this workgroup's LDS queue are held by it (it
                        // does not leave while its queue or a batch holds any),
                        // so their add need not land first: a count read too
                        // early can only make another workgroup leave sooner.
                        const uint32_t len = __hip_atomic_load(&L.qr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) - hq;
                        sp = len + tot > uint32_t(OFD_MW_CAP) ? 1u : 0u;
                        (void)__hip_atomic_fetch_add(pw + kPGo, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        rb = sp ? atomicAdd(pw + kPGt, tot) : atomicAdd(&L.qr, tot);
#if OFD_MW_APPEND_WAIT
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
                        if (sp) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
                    } else {
                        rb = atomicAdd(&L.qr, tot);
                    }
                }
                rb = __shfl(rb, 63);
                hq = __shfl(hq, 63);
                sp = __shfl(sp, 63);
                uint32_t f = rb + incl - cnt;
                bool glob = false;
                if (kMW && sp) {  // to the shared queue: tagged granules, no ordered publish
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (rmask & (1u << k)) {
                            const auto q = IX32(p + uint32_t(WOFF(k)));
                            __hip_atomic_store(m.cy + f % uint32_t(m.en), (uint64_t(q) << 32) | uint64_t(f + 1u),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            ++f;
                        }
                    return;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (rmask & (1u << k)) {
                        const auto q = IX32(p + uint32_t(WOFF(k)));
                        if (f - hq < uint32_t(kDfQ)) {  // the slot's previous entry (f - kDfQ) is claimed
                            __hip_atomic_store(&L.ring[f & uint32_t(kDfQ - 1)], (uint64_t(q) << 32) | uint64_t(f + 1u),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        } else {
                            m.fr2[kMW ? ovf0 + f % ovf : f] = (uint64_t(q) << 32) | uint64_t(q);
                            glob = true;
                        }
                        ++f;
                    }
                if (__any(glob)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the overflow's stores
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                SQ_T(cs0);
                if (lane == 0) {
                    for (int t = 0; __hip_atomic_load(&L.qp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != rb; ++t) {
                        if (t > (1 << 22)) {  // cannot happen: earlier reservations publish without waiting
                            atomicOr(&g_sq_fault, 32u);
#ifdef OFD_MW_DEBUG
                            printf("MWDBG publish wr %d rb %u qp %u\n", wr, rb, L.qp);
#endif
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    __hip_atomic_store(&L.qp, rb + tot, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                SQ_T(cs1);
                SQ_ACC(0, cs0, cs1);  // the ordered publish
            };
            SQ_T(c1);
            // this lane's terms (disk positions gl + 8k): channels 1 and 2 go
            // to LDS at once (past the grid), channel 0 waits in registers
            // until every lane of the hole is done with the grid
            const uint32_t wts[4] = {wq.x, wq.y, wq.z, wq.w};
            const uint32_t cw = (gl >> 1) == 0 ? cq.x : (gl >> 1) == 1 ? cq.y : (gl >> 1) == 2 ? cq.z : cq.w;
            const uint32_t codes = cw >> (16 * (gl & 1));
            float t0[4][3];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int a = DC(k) / 9 - 4, b = DC(k) % 9 - 4, y = i + a, x = j + b;
                const int k1 = y == 1, kE = y == eh - 2, l1 = x == 1, lE = x == ew - 2;
                auto G = [&](int ry, int rx) -> uint32_t {  // colour word at window offset (ry, rx), |ry|, |rx| <= 4
                    return gv[(ry + 4) * 9 + rx + 4];
                };
                const uint32_t w0 = G(a + k1, b + l1), w1 = G(a + k1, b + 1 - lE), w2 = G(a + k1, b - 1 + l1),
                               w3 = G(a + k1, b - lE), w4 = G(a + 1 - kE, b + l1), w5 = G(a - 1 + k1, b + l1),
                               w6 = G(a - kE, b + l1);
                const float wt = __uint_as_float(wts[k]);
                const uint32_t cx = (codes >> (4 * k)) & 3u, cy = (codes >> (4 * k + 2)) & 3u;
                // cv2's gradient cases as (A - B) * f, selected once for all channels:
                // code 0: (v1 - v2) * 2, 1: (v1 - v0), 2: (v3 - v2), 3: none ((v0 - v0) * 0 = +0)
                const uint32_t xa = cx <= 1u ? w1 : (cx == 2u ? w3 : w0), xb = (cx & 1u) ? w0 : w2;
                const uint32_t ya = cy <= 1u ? w4 : (cy == 2u ? w6 : w0), yb = (cy & 1u) ? w0 : w5;
                // gix * rx = (A - B) * (f * rx) exactly: integers below 2^24 (the
                // sign of an exact zero may differ, which no result can see)
                const float kx = (cx == 0u ? 2.0f : (cx == 3u ? 0.0f : 1.0f)) * float(-b);
                const float ky = (cy == 0u ? 2.0f : (cy == 3u ? 0.0f : 1.0f)) * float(-a);
                const bool live = gl + kL3 * k < kDisk;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    auto byte = [&](uint32_t q) -> int { return int((q >> (8 * c)) & 0xFFu); };
                    const float vs = float(byte(w0));
                    const float dx = float(byte(xa) - byte(xb)), dy = float(byte(ya) - byte(yb));
                    // Jx / Jy terms negated: their chains subtract, and acc + (-t)
                    // is acc - t exactly (as -1 * t), so every chain is a plain sum
                    const float ta = wt * vs, tx = -(wt * (dx * kx)), ty = -(wt * (dy * ky));
                    if (c == 0) {
                        t0[k][0] = ta;
                        t0[k][1] = tx;
                        t0[k][2] = ty;
                    } else if (live) {  // chains past 3 * C are never summed
                        bf[(3 * c) * kDisk + gl + kL3 * k] = ta;
                        bf[(3 * c + 1) * kDisk + gl + kL3 * k] = tx;
                        bf[(3 * c + 2) * kDisk + gl + kL3 * k] = ty;
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (gl + kL3 * k < kDisk)
#pragma unroll
                    for (int q = 0; q < 3; ++q) bf[q * kDisk + gl + kL3 * k] = t0[k][q];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            SQ_T(c2);
            // cv2's sums in its (k, l) order: chains gl and gl + 8 side by side
            // (independent accumulators; Ia chains add, Jx / Jy chains subtract)
            {
                const int c1 = gl, c2 = gl + kL3;
                const bool has2 = c2 < nch;
                const float *t1 = bf + c1 * kDisk, *t2 = bf + (has2 ? c2 : c1) * kDisk;
                float a1 = 0.f, a2 = 0.f;
#pragma unroll
                for (int q = 0; q < kDisk; ++q) {
                    a1 += t1[q];  // Jx / Jy terms are stored negated
                    a2 += t2[q];
                }
                if (c1 < nch) L.res[g][c1] = a1;
                if (has2) L.res[g][c2] = a2;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            SQ_T(cb);
#ifdef OFD_SQ_PROF
            asm volatile("" : "+v"(old[0]), "+v"(old[1]), "+v"(old[2]), "+v"(old[3]), "+v"(old[4]), "+v"(old[5]),
                         "+v"(old[6]), "+v"(old[7]));
#endif
            SQ_T(ca);
            // queue the holes this one's releases completed now, before its
            // colour exists: their loads overlap the rest of this hole (they
            // wait for its coloured flag)
            append_ready();
            SQ_T(c3);
            {
                unsigned u = 0;
                if (act && gl < C) {
                    const float sum = __uint_as_float(mq.z);
                    const float Ia = L.res[g][3 * gl], Jx = L.res[g][3 * gl + 1], Jy = L.res[g][3 * gl + 2];
                    const float sat = float(double(Ia / sum) +
                                            double(Jx + Jy) / (sqrt(double(Jx * Jx + Jy * Jy)) + double(1.0e-20f)) +
                                            double(0.5f));
                    u = sat_u8(sat);
                }
                // the hole's channels and the coloured flag in one word store
                const int hl0 = (tid & 63) & ~(kL3 - 1);
                const unsigned u1 = __shfl(u, hl0 + 1), u2 = __shfl(u, hl0 + 2);
                if (act && gl == 0) {
                    const uint32_t word = u | (u1 << 8) | (u2 << 16) | 0xFF000000u;
                    if constexpr (kMW)  // write-through (sc1): the other workgroups' sc1 polls see it
                        __hip_atomic_store(m.shd + (int64_t(i - 1) * W + (j - 1)), word, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    else
                        m.shd[int64_t(i - 1) * W + (j - 1)] = word;
                    __hip_atomic_store(&L.ct[p & uint32_t(kDfCt - 1)], (uint64_t(word) << 32) | uint64_t(p + 1u),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            SQ_T(c4);
            SQ_ACC(2, c0, c0a);
            SQ_ACC(6, c0a, c1);
            SQ_ACC(3, c1, c2);
            SQ_ACC(4, c2, cb);  // chains
            SQ_ACC(7, cb, ca);  // the release atomics' return
            SQ_ACC(1, ca, c3);  // the append
            SQ_ACC(5, c3, c4);
        }
        if (lane == 0) {
            // kMW: the image's count drops by this batch's holes, after the
            // batch's own additions have returned (append_ready waits for them)
            if (kMW) (void)__hip_atomic_fetch_sub(pw + kPGo, take, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicSub(&L.inflight, take);
        }
        ++batches;
        if (__shfl(lane == 0 ? (wall_clock64() >= deadline ? 1u : 0u) : 0u, 0)) break;  // the rest is carried
    }
    if (lane == 0) atomicAdd(&m.meta[6], batches);
    __syncthreads();
    if constexpr (kMW) {
        // the unclaimed entries of the LDS queue go to the shared queue for the
        // next round (still counted in kPGo)
        const uint32_t hq = L.qh, pq = L.qp;
        if (tid == 0 && pq > hq) L.gbase = atomicAdd(pw + kPGt, pq - hq);
        __syncthreads();
        const uint32_t gb = L.gbase;
        for (uint32_t y = hq + uint32_t(tid); y < pq; y += kThr) {
            const uint64_t v = L.ring[y & uint32_t(kDfQ - 1)];
            const uint32_t q = uint32_t(uint32_t(v) == y + 1u ? (v >> 32) : (m.fr2[ovf0 + y % ovf] >> 32));
            const uint32_t sl = gb + (y - hq);
            __hip_atomic_store(m.cy + sl % uint32_t(m.en), (uint64_t(q) << 32) | uint64_t(sl + 1u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0 && wr == 0 && pq <= hq &&
            __hip_atomic_load(pw + kPGo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
            put64(m.pipe + kPTc1, wall_clock64());
#ifdef OFD_SQ_PROF
        if (tid == 0 && wr == 0) {  // wave 0 of the image's first workgroup, all rounds
            for (int k = 0; k < 8; ++k) m.meta[16 + k] += uint32_t(prof[k] >> 8);
            m.meta[7] += batches;
        }
#endif
        return;
    }
    // the unclaimed entries still in the ring go to fr2 for the next round
    for (uint32_t y = L.qh + uint32_t(tid); y < L.qp; y += kThr) {
        const uint64_t v = L.ring[y & uint32_t(kDfQ - 1)];
        if (uint32_t(v) == y + 1u) m.fr2[y] = (v & 0xFFFFFFFF00000000ull) | (v >> 32);
    }
    if (tid == 0) {
        const uint32_t hq = L.qh, pq = L.qp;
        if (hq >= pq && q1 + t0q > h0) put64(m.pipe + kPTc1, wall_clock64());
        m.pipe[kPQh] = hq;
        m.pipe[kPQt] = pq;
        m.pipe[kPRqc] = q1;
#ifdef OFD_SQ_PROF
        for (int k = 0; k < 8; ++k) m.meta[16 + k] += uint32_t(prof[k] >> 8);  // wave 0's batches, all rounds
        m.meta[7] += batches;
#endif
    }
}
#undef VC
#undef WC
#undef DC
#undef WOFF

// Pacing of the pipelined fill's RECORD / COLOUR3 rounds (one workgroup).
// Round e first waits -- bounded by bound_ticks -- until round_ticks * (e + 1)
// after round 0 began, or until every image's two marches are done; then it
// snapshots each image's RECORD window [recdone, hi): hi is the inner march's
// published progress once its outer march is done (RECORD reads the ring's
// distances), else nothing.  fin: the marches have completed (stream order),
// no wait, the window runs to the end of the log.  Never waits on anything
// without a time bound, so a march that is not resident yet only delays.
__global__ __launch_bounds__(256) void sq_pace_kernel(SqWs w, int nimg, int e, int fin, uint64_t round_ticks,
                                                     uint64_t bound_ticks) {
    uint32_t *t0w = w.pipe + kPT0;  // image 0's pipe words hold the clock origin
    if (!fin) {
        if (threadIdx.x == 0) {
            const uint64_t now = wall_clock64();
            uint64_t t0 = now;
            if (e == 0) {
                t0w[0] = uint32_t(t0);
                t0w[1] = uint32_t(t0 >> 32);
            } else {
                t0 = uint64_t(t0w[0]) | (uint64_t(t0w[1]) << 32);
            }
            const uint64_t until = t0 + round_ticks * uint64_t(e + 1);
            for (;;) {
                const uint64_t tn = wall_clock64();
                if (tn >= until || tn - now >= bound_ticks) break;
                bool done = true;
                for (int b = 0; b < nimg && done; ++b) {
                    const uint32_t *pp = w.pipe + int64_t(b) * kPipe;
                    done = __hip_atomic_load(pp + kPInDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u &&
                           __hip_atomic_load(pp + kPOutDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
                }
                if (done) break;
                __builtin_amdgcn_s_sleep(64);
            }
        }
        __syncthreads();
    }
    // snapshot; and whether every march is done (each image's inner march
    // done before its progress is read, so hi is then its whole log): this
    // round then records every hole, and its colour pass runs to the end
    // (no deadline, no further round boundaries)
    int done = 1;
    for (int b = threadIdx.x; b < nimg; b += 256) {
        uint32_t *pp = w.pipe + int64_t(b) * kPipe;
        const uint32_t id = __hip_atomic_load(pp + kPInDone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t od = __hip_atomic_load(pp + kPOutDone, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t prog = __hip_atomic_load(pp + kPProg, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t lo = pp[kPRecDone];
        const uint32_t hi = (od != 0u && prog > lo) ? prog : lo;
        pp[kPLo] = lo;
        pp[kPHi] = hi;
        pp[kPRecDone] = hi;
        if (id == 0u || od == 0u) done = 0;
    }
    done = __syncthreads_and(done);
#ifndef OFD_SEQ_ALLDONE  // probe builds: 0 keeps every helper round's deadline (A/B)
#define OFD_SEQ_ALLDONE 1
#endif
    if (threadIdx.x == 0) w.pipe[kPAllDone] = (fin || (OFD_SEQ_ALLDONE && done)) ? 1u : 0u;
}

// The record path's result: every pixel's colours from the shadow image
// (kept pixels hold PREP's uint8 cast, holes their fill), as float32.
__global__ __launch_bounds__(256) void sq_unpack_kernel(SqWs w, float *__restrict__ out, int C, int64_t HW, int64_t b0) {
    const int64_t p = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (p >= HW) return;
    const uint32_t v = w.shd[int64_t(blockIdx.y) * w.hw + p];
    float *ob = out + (b0 + blockIdx.y) * int64_t(C) * HW + p;
    for (int c = 0; c < C; ++c) ob[int64_t(c) * HW] = float((v >> (8 * c)) & 0xFFu);
}


// The helper stream and events of the pipelined sequential fill (its
// RECORD / colour rounds beside the marches), one set per device, created on
// that device on first use.  A call uses the set of its stream's device
// (hipStreamGetDevice), so its rounds always run on the device that owns the
// workspace, image and output pointers, whichever device is current.
struct SeqHelpers {
    std::mutex mu;
    int device = -1;  // created for this device (-1: not yet)
    bool ok = false;
    hipStream_t stream[1] = {nullptr};
    hipEvent_t fork = nullptr, join[1] = {nullptr};
};
constexpr int kMaxSeqDevices = 64;

// The device a call on stream st runs on: the stream's own (the null stream's
// is the current device); -1 when it cannot be told.
int stream_device(hipStream_t st) {
    int dev = -1;
    if (hipStreamGetDevice(st, &dev) != hipSuccess) {
        (void)hipGetLastError();
        if (hipGetDevice(&dev) != hipSuccess) return -1;
    }
    return dev;
}

SeqHelpers *seq_helpers(int dev) {
    static SeqHelpers h[kMaxSeqDevices];
    static std::mutex mu;
    if (dev < 0 || dev >= kMaxSeqDevices) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    SeqHelpers &x = h[dev];
    if (x.device < 0) {
        int prev = -1;
        bool ok = hipGetDevice(&prev) == hipSuccess && (prev == dev || hipSetDevice(dev) == hipSuccess);
        ok = ok && hipEventCreateWithFlags(&x.fork, hipEventDisableTiming) == hipSuccess;
        for (int k = 0; k < 1 && ok; ++k)
            ok = hipStreamCreateWithFlags(&x.stream[k], hipStreamNonBlocking) == hipSuccess &&
                 hipEventCreateWithFlags(&x.join[k], hipEventDisableTiming) == hipSuccess;
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
        x.ok = ok;
        x.device = dev;
    }
    return &x;
}

// Pipelined radius-3 fill (ofd_inpaint_seq_set_pipeline): record / colour
// rounds on a helper stream beside the marches.  -1 = not set (OFD_SEQ_PIPE
// rounds, default 12; OFD_SEQ_PIPE_US per round, default 2000: 12 x 2 ms
// spans the marches of 64 images of 768 x 1024, 47.5 -> 43.0 ms a fill).
#ifndef OFD_SEQ_PIPE_DEFAULT
#define OFD_SEQ_PIPE_DEFAULT 12
#endif
#ifndef OFD_SEQ_PIPE_US_DEFAULT
#define OFD_SEQ_PIPE_US_DEFAULT 2000
#endif
int g_pipe_rounds = -1, g_pipe_us = -1;
int pipe_rounds_setting() {
    if (g_pipe_rounds < 0) {
        const char *e = getenv("OFD_SEQ_PIPE");
        g_pipe_rounds = e ? atoi(e) : OFD_SEQ_PIPE_DEFAULT;
        if (g_pipe_rounds < 0) g_pipe_rounds = 0;
        if (g_pipe_rounds > 256) g_pipe_rounds = 256;
    }
    return g_pipe_rounds;
}
int pipe_us_setting() {
    if (g_pipe_us < 0) {
        const char *e = getenv("OFD_SEQ_PIPE_US");
        g_pipe_us = e ? atoi(e) : OFD_SEQ_PIPE_US_DEFAULT;
        if (g_pipe_us < 1) g_pipe_us = 1;
    }
    return g_pipe_us;
}
// the colour pass: 1 = levels-free (sq_colour3df_kernel), 0 = level-synchronous
// COLOUR3; ofd_inpaint_seq_set_colour, default OFD_SEQ_DF (else 1)
int g_df_colour = [] {
    const char *e = getenv("OFD_SEQ_DF");
    return e ? (atoi(e) != 0 ? 1 : 0) : 1;
}();
// Workgroups per image of the levels-free colour pass (kMW: 256 threads
// each, sharing the image's queues; 1 = one 1024-thread workgroup, the
// single-CU pass).  ofd_inpaint_seq_set_multi, default OFD_SEQ_MW (else
// OFD_SEQ_MW_DEFAULT); images below kPipeMinPixels always take one.
#ifndef OFD_SEQ_MW_DEFAULT
#define OFD_SEQ_MW_DEFAULT 4
#endif
int g_seq_multi = [] {
    const char *e = getenv("OFD_SEQ_MW");
    const int v = e ? atoi(e) : OFD_SEQ_MW_DEFAULT;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
}();
int g_mw_force = 0;  // ofd_inpaint_seq_set_multi(k, 1): also below kPipeMinPixels (tests)
// images below this many pixels: marches too short to overlap (unless a
// test forces the pipeline with ofd_inpaint_seq_set_pipeline(rounds, us, 1))
int g_pipe_force = 0;
constexpr int64_t kPipeMinPixels = int64_t(1) << 18;

}  // namespace

unsigned ofd_sq_fault_read(int reset) {
    unsigned v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_sq_fault), sizeof(v)) != hipSuccess) return ~0u;
    if (reset) {
        const unsigned z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_sq_fault), &z, sizeof(z)) != hipSuccess) return ~0u;
    }
    return v;
}

extern "C" {

int ofd_inpaint_seq_helper_device(void *stream) {
    const int dev = stream_device(static_cast<hipStream_t>(stream));
    SeqHelpers *h = seq_helpers(dev);
    return h && h->ok ? h->device : -1;
}

int ofd_inpaint_seq_set_colour(int mode) {
    const int prev = g_df_colour;
    if (mode >= 0) g_df_colour = mode != 0 ? 1 : 0;
    return prev;
}

int ofd_inpaint_seq_set_multi(int workgroups, int force) {
    const int prev = g_seq_multi;
    if (workgroups >= 1) {
        g_seq_multi = workgroups > 16 ? 16 : workgroups;
        g_mw_force = force ? 1 : 0;
    }
    return prev;
}

int ofd_inpaint_seq_set_pipeline(int rounds, int round_us, int force) {
    const int prev = pipe_rounds_setting();
    (void)pipe_us_setting();
    if (rounds >= 0) g_pipe_rounds = rounds > 256 ? 256 : rounds;
    if (round_us == 0) {  // back to the default
        g_pipe_us = -1;
        (void)pipe_us_setting();
    }
    if (round_us >= 1) g_pipe_us = round_us;
    if (force >= 0) g_pipe_force = force ? 1 : 0;
    return prev;
}

size_t ofd_inpaint_seq_workspace_bytes(int64_t B, int64_t H, int64_t W) {
    if (B <= 0 || H <= 0 || W <= 0) return 0;
    return size_t(B) * per_image_bytes(H, W) + 8 * 256;
}

int ofd_inpaint_telea_seq_f32(const float *img, const float *valid, const float *collision, float *out, int64_t B,
                              int64_t C, int64_t H, int64_t W, int radius, void *workspace, size_t workspace_bytes,
                              void *stream) {
    if (B < 0 || C < 0 || H < 0 || W < 0) return OFD_FW_EINVAL;
    if (B * C * H * W == 0) return OFD_FW_OK;
    if (!img || !valid || !collision || !out) return OFD_FW_EINVAL;
    if (H < 2 || W < 2) return OFD_FW_EINVAL;
    const int64_t en = (H + 2) * (W + 2);
    if (en >= (int64_t(1) << 30)) return OFD_FW_ETOOBIG;  // ranks * 4 + direction fit 32 bits
    // the buckets' margin (a push lands >= 1/sqrt(2) above its popper, the
    // bucket is <= 0.7 wide) needs the float rounding of T well under 0.2:
    // T < H + W < 2^19 keeps its ulp at or below 2^-5
    if (H + W >= (int64_t(1) << 19)) return OFD_FW_ETOOBIG;
    const int r = radius < 1 ? 1 : (radius > kMaxRange ? kMaxRange : radius);
    if (!workspace || (reinterpret_cast<uintptr_t>(workspace) & 255u)) return OFD_FW_EWORKSPACE;
    const size_t pi = per_image_bytes(H, W), fixed = 8 * 256;
    if (workspace_bytes < fixed + pi) return OFD_FW_EWORKSPACE;
    int64_t G = int64_t((workspace_bytes - fixed) / pi);
    if (G > B) G = B;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // radius 3 with up to 3 channels (utils.inpaint's RGB call): the record
    // path; OFD_SEQ_COLOUR=g16 selects the one-pass colour kernel (A/B)
    static const bool force_g16 = [] {
        const char *e = getenv("OFD_SEQ_COLOUR");
        return e && e[0] == 'g';
    }();
    const bool rec3 = r == 3 && C <= 3 && en < (int64_t(1) << 26) && !force_g16;
    static const double wide = [] {  // OFD_SEQ_BUCKET=0.5 selects the narrow buckets (A/B)
        const char *e = getenv("OFD_SEQ_BUCKET");
        return e ? atof(e) : 0.7;
    }();
    const double bscale = (H + W < 8000 && wide > 0.0 && wide <= 0.7) ? 1.0 / wide : 2.0;
    // pipelined rounds (radius-3 path only; one group: the helper stream is the pipeline's)
    int rounds = (H * W >= kPipeMinPixels || g_pipe_force) ? pipe_rounds_setting() : 0;
    uint64_t pipe_ticks = 0;
    if (rounds > 0) {
        int dev = stream_device(st), khz = 0;
        if (dev < 0 || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
            khz = 100000;  // the MI355X's 100 MHz constant clock
        pipe_ticks = uint64_t(pipe_us_setting()) * uint64_t(khz) / 1000u;
    }
    const bool df_colour = g_df_colour != 0;
    // kMW: each workgroup's overflow slice of fr2 (en / mw entries) must hold
    // its LDS queue's worst case: kDfQ + OFD_MW_CAP + 8 waves x 480 new holes
    int mw = (df_colour && rec3 && (H * W >= kPipeMinPixels || g_mw_force)) ? g_seq_multi : 1;
    while (mw > 1 && en / mw < 4608) --mw;

    // one chunk of nb images (workspace w) on stream s
    auto run_chunk = [&](const SqWs &w, int64_t b0, int64_t nb, hipStream_t s) {
        hipLaunchKernelGGL(sq_prep_tile_kernel, dim3(unsigned((W + 63) / 64), unsigned((H + 15) / 16), unsigned(nb)),
                           dim3(256), 0, s, img, valid, collision, out, w, int(C), int(H), int(W), b0, rec3 ? 1 : 0);
        const dim3 bg(unsigned((w.ew + kBpTW - 1) / kBpTW), unsigned((w.eh + kBpTH - 1) / kBpTH), unsigned(nb));
        if (r + 1 <= kInitR) {  // INIT with bucket 0's push counts, one scan, the band log and pushes
            hipLaunchKernelGGL(sq_init_push_kernel, bg, dim3(256), 0, s, w, r);
            hipLaunchKernelGGL(sq_band3_scan_kernel, dim3(unsigned(nb)), dim3(kThreads), 0, s, w);
            hipLaunchKernelGGL(sq_band3_write_kernel, bg, dim3(256), 0, s, w);
        } else {
            if (r <= kInitR)
                hipLaunchKernelGGL(sq_init_tile_kernel,
                                   dim3(unsigned((w.ew + kInitTW - 1) / kInitTW), unsigned((w.eh + kInitTH - 1) / kInitTH),
                                        unsigned(nb)),
                                   dim3(256), 0, s, w, r);
            else
                hipLaunchKernelGGL(sq_init_kernel, dim3(unsigned((w.eh + 3) / 4), unsigned(nb)), dim3(256), 0, s, w, r);
            hipLaunchKernelGGL(sq_band_scan_kernel, dim3(unsigned(nb)), dim3(kThreads), 0, s, w);
            hipLaunchKernelGGL(sq_band_write_kernel, dim3(unsigned((w.eh + 3) / 4), unsigned(nb)), dim3(256), 0, s, w);
            hipLaunchKernelGGL(sq_band_push_count_kernel, bg, dim3(256), 0, s, w);
            hipLaunchKernelGGL(sq_band_push_scan_kernel, dim3(unsigned(nb), 2u), dim3(kThreads), 0, s, w);
            hipLaunchKernelGGL(sq_band_push_write_kernel, bg, dim3(256), 0, s, w);
        }
        const dim3 rgrid(unsigned((w.ew + 63) / 64), unsigned((w.eh + kRecTH - 1) / kRecTH), unsigned(nb));
        // kMW: the shared queues' granules are tagged by slot, which restarts
        // at 0 every fill -- clear the previous fill's tags
        if (rec3 && mw > 1) (void)hipMemsetAsync(w.cy, 0, size_t(nb) * size_t(w.en) * 8, s);
        auto round = [&](hipStream_t rs, int e, int fin) {  // one RECORD / COLOUR3 round
            hipLaunchKernelGGL(sq_pace_kernel, dim3(1), dim3(256), 0, rs, w, int(nb), e, fin, pipe_ticks, 4 * pipe_ticks);
            hipLaunchKernelGGL(sq_record3_kernel, rgrid, dim3(256), 0, rs, w);
            if (df_colour && mw > 1)
                hipLaunchKernelGGL((sq_colour3df_kernel<OFD_MW_THR, true>), dim3(unsigned(nb * mw)), dim3(OFD_MW_THR), 0, rs, w, int(C),
                                   int(H), int(W), e, fin, pipe_ticks, mw);
            else if (df_colour)
                hipLaunchKernelGGL((sq_colour3df_kernel<1024, false>), dim3(unsigned(nb)), dim3(1024), 0, rs, w, int(C),
                                   int(H), int(W), e, fin, pipe_ticks, 1);
            else
                hipLaunchKernelGGL(sq_colour3_kernel, dim3(unsigned(nb)), dim3(1024), 0, rs, w, int(C), int(H), int(W), e,
                                   fin, pipe_ticks);
        };
        // Pipelined (radius 3, C <= 3, large images): while the marches run
        // on s, a helper stream runs `rounds` RECORD / COLOUR3 rounds over the
        // holes the inner march has finished, so the colour chain overlaps
        // the march instead of following it; the final round on s (after the
        // marches) takes whatever is left.  Every round's result is the same:
        // counters are additive and the colour order is the Kahn order.
        SeqHelpers *hp = nullptr;
        if (rec3 && rounds > 0) {
            hp = seq_helpers(stream_device(s));
            if (hp && !hp->ok) hp = nullptr;
        }
        if (hp) {
            std::lock_guard<std::mutex> lk(hp->mu);
            (void)hipEventRecord(hp->fork, s);  // after BAND: the helper may start reading
            (void)hipStreamWaitEvent(hp->stream[0], hp->fork, 0);
            hipLaunchKernelGGL(sq_fmm_kernel, dim3(unsigned(nb), 2u), dim3(kThreads), 0, s, w, bscale, 1);
            for (int e = 0; e < rounds; ++e) round(hp->stream[0], e, 0);
            (void)hipEventRecord(hp->join[0], hp->stream[0]);
            (void)hipStreamWaitEvent(s, hp->join[0], 0);
        } else {
            hipLaunchKernelGGL(sq_fmm_kernel, dim3(unsigned(nb), 2u), dim3(kThreads), 0, s, w, bscale, 0);
        }
#ifdef OFD_BUCKET_TRACE
        return;  // probe: keep the record area (the inner march's bucket trace) for the host
#endif
        if (rec3) {
            round(s, 0, 1);
            hipLaunchKernelGGL(sq_unpack_kernel, dim3(unsigned((H * W + 255) / 256), unsigned(nb)), dim3(256), 0, s, w,
                               out, int(C), int64_t(H * W), b0);
            return;
        }
        hipLaunchKernelGGL(sq_count_kernel, dim3(unsigned((w.ew + 63) / 64), unsigned((w.eh + 3) / 4), unsigned(nb)),
                           dim3(256), 0, s, w, r);
        if (r == 3)
            hipLaunchKernelGGL(sq_colour_g16_kernel, dim3(unsigned(nb)), dim3(kG16Threads), 0, s, w, out, int(C), int(H),
                               int(W), b0);
        else
            hipLaunchKernelGGL(sq_colour_kernel, dim3(unsigned(nb)), dim3(kColThreads), 0, s, w, out, int(C), int(H),
                               int(W), b0, r);
    };
    const SqWs w = carve(workspace, G, H, W);
    for (int64_t b0 = 0; b0 < B; b0 += G) run_chunk(w, b0, B - b0 < G ? B - b0 : G, st);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

}  // extern "C"
