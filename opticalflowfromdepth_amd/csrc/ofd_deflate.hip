// ofd_deflate.hip -- MI355X (gfx950) DEFLATE encoder for the npz product.
//
// preprocess.py writes its product with np.savez_compressed (:446, :471-476):
// a zip of .npy members, each deflated by zlib on the host.  Per image that
// is 121 files and ~6.3 GB of float64 planes at 768x1024, and host zlib (one
// core per file) bounds the whole pipeline.  This file deflates the arrays on
// the GPU, where they already are, into streams any inflater (zlib, Python's
// zipfile, np.load) reads:
//
//   * every array is cut into 1 MiB SEGMENTS; each segment is one dynamic-
//     Huffman deflate block (literals only: 256 byte symbols + end-of-block,
//     no LZ77 matches -- f64 planes of f32 / integer values are dominated by
//     zero bytes, which a per-segment code prices at about one bit), closed
//     by an empty stored block (zlib's Z_SYNC_FLUSH marker 00 00 FF FF), so
//     every segment ends on a byte boundary and the segments concatenate;
//   * the array's stream ends with an empty final fixed block (03 00);
//   * CRC-32 (zlib's polynomial) of every array, for the zip headers.
//
// Kernels (all on the caller's stream, no host synchronisation):
//   HIST   one workgroup per 16 KiB chunk: the chunk's byte histogram (kept
//          per chunk and added into its segment's), and the chunk's CRC-32
//          (a table CRC per thread over 64 bytes, folded by x^(8n) mod P).
//   CODE   one workgroup per segment: the Huffman code lengths (max 15; the
//          frequencies are flattened and the tree rebuilt until it fits),
//          the canonical codes, the block header (code-length code, 257
//          literal / end lengths, one zero distance length), the segment's
//          size in bytes, every chunk's bit offset, the segment CRC.
//   SCAN   one thread per array: segment offsets, the array's size, its CRC,
//          the final block.
//   ENCODE one workgroup per chunk: per-thread bit counts, a block scan, then
//          every thread ORs its codes into the (zeroed) output with 32-bit
//          atomics; the chunk holding a segment's start writes the header,
//          the one holding its end the end-of-block code and FF FF.
//
// Plain HIP for gfx950.

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "ofd_deflate.h"
#include "ofd_fw.h"

namespace {

constexpr int kThr = 256;
constexpr int64_t kChunk = 16384;               // bytes per HIST / ENCODE workgroup
constexpr int kPerThr = int(kChunk / kThr);     // 64 bytes per thread
constexpr int64_t kSeg = int64_t(1) << 20;      // bytes per deflate block
constexpr int kChunksPerSeg = int(kSeg / kChunk);
constexpr int kSym = 257;                       // literals 0..255 + end of block
constexpr int kMaxLen = 15;
constexpr int kHdrWords = 80;                   // block header bits (<= 3+5+5+4+57+258*7 = 1880)
constexpr uint32_t kPoly = 0xEDB88320u;         // CRC-32, reflected

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// ---------------------------------------------------------------- CRC-32 algebra (zlib's multmodp / x2nmodp)
__host__ __device__ inline uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}

// x^(8 n) mod P: the operator that shifts a CRC past n more bytes
__host__ __device__ inline uint32_t x8nmodp(uint64_t n) {
    uint32_t p = 1u << 31;     // x^0
    uint32_t sq = 1u << 23;    // x^8
    while (n) {
        if (n & 1) p = multmodp(sq, p);
        sq = multmodp(sq, sq);
        n >>= 1;
    }
    return p;
}

// crc(A || B) from crc(A), crc(B) and |B|
__host__ __device__ inline uint32_t crc_combine(uint32_t ca, uint32_t cb, uint64_t lenb) {
    return multmodp(x8nmodp(lenb), ca) ^ cb;
}

struct Geo {        // one batch of `count` arrays of `each` bytes
    int64_t each;   // bytes per array
    int cpa;        // chunks per array
    int spa;        // segments per array
    int64_t bound;  // output slot per array
};

struct DWs {
    uint16_t *chist;   // [chunks][256]
    uint32_t *ccrc;    // [chunks]
    uint64_t *cbit;    // [chunks] bit offset of the chunk's first code from the segment start
    uint32_t *shist;   // [segs][256]  (zeroed per call)
    uint32_t *scode;   // [segs][257]  bit-reversed code | len << 24
    uint32_t *shdr;    // [segs][kHdrWords]
    uint32_t *shbits;  // [segs] header bits
    uint32_t *sbytes;  // [segs] segment bytes (header .. FF FF)
    uint32_t *scrc;    // [segs]
    uint64_t *soff;    // [segs] byte offset of the segment in its array's slot
};

size_t ws_bytes(int64_t count, int64_t each) {
    const int64_t cpa = (each + kChunk - 1) / kChunk, spa = (each + kSeg - 1) / kSeg;
    const size_t nc = size_t(count * cpa), ns = size_t(count * spa);
    return align256(nc * 512) + align256(nc * 4) + align256(nc * 8) + align256(ns * 1024) + align256(ns * 4 * kSym) +
           align256(ns * 4 * kHdrWords) + 4 * align256(ns * 4) + align256(ns * 8);
}

DWs carve(void *ws, int64_t count, const Geo &g) {
    const size_t nc = size_t(count) * g.cpa, ns = size_t(count) * g.spa;
    char *p = static_cast<char *>(ws);
    DWs w;
    w.chist = reinterpret_cast<uint16_t *>(p), p += align256(nc * 512);
    w.ccrc = reinterpret_cast<uint32_t *>(p), p += align256(nc * 4);
    w.cbit = reinterpret_cast<uint64_t *>(p), p += align256(nc * 8);
    w.shist = reinterpret_cast<uint32_t *>(p), p += align256(ns * 1024);
    w.scode = reinterpret_cast<uint32_t *>(p), p += align256(ns * 4 * kSym);
    w.shdr = reinterpret_cast<uint32_t *>(p), p += align256(ns * 4 * kHdrWords);
    w.shbits = reinterpret_cast<uint32_t *>(p), p += align256(ns * 4);
    w.sbytes = reinterpret_cast<uint32_t *>(p), p += align256(ns * 4);
    w.scrc = reinterpret_cast<uint32_t *>(p), p += align256(ns * 4);
    w.soff = reinterpret_cast<uint64_t *>(p);
    return w;
}

__device__ __forceinline__ void make_crc_table(uint32_t *T) {
    for (int k = threadIdx.x; k < 256; k += kThr) {
        uint32_t c = uint32_t(k);
        for (int b = 0; b < 8; ++b) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
        T[k] = c;
    }
}

// A thread's n <= 64 bytes at src + t0 as 16 little-endian words (bytes past
// n read as 0): four 16-byte loads when aligned and whole, else byte loads.
__device__ __forceinline__ void load64(const uint8_t *__restrict__ src, int t0, int n, uint32_t wd[16]) {
    const uint8_t *p = src + t0;
    if (n == kPerThr && (reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint4 v = reinterpret_cast<const uint4 *>(p)[q];
            wd[4 * q] = v.x;
            wd[4 * q + 1] = v.y;
            wd[4 * q + 2] = v.z;
            wd[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            uint32_t x = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (4 * q + r < n) x |= uint32_t(p[4 * q + r]) << (8 * r);
            wd[q] = x;
        }
    }
}

// ---------------------------------------------------------------- HIST
// chunk c = (array a, chunk k of the array); thread t owns bytes [64 t, 64 t + 64)
__global__ __launch_bounds__(kThr) void dfl_hist_kernel(const uint8_t *__restrict__ in, Geo g, DWs w) {
    __shared__ uint32_t T[256];
    __shared__ uint32_t H[256];
    __shared__ uint32_t C[kThr];
    const int c = blockIdx.x, a = c / g.cpa, k = c - a * g.cpa;
    const int64_t beg = int64_t(k) * kChunk, len = min(kChunk, g.each - beg);
    const uint8_t *src = in + int64_t(a) * g.each + beg;
    make_crc_table(T);
    H[threadIdx.x] = 0u;
    __syncthreads();
    const int t0 = threadIdx.x * kPerThr;
    const int n = int(min<int64_t>(kPerThr, max<int64_t>(len - t0, 0)));
    uint32_t wd[16];
    load64(src, t0, n, wd);
    uint32_t crc = 0xFFFFFFFFu, zeros = 0;
#pragma unroll
    for (int e = 0; e < kPerThr; ++e) {
        if (e < n) {
            const uint32_t b = (wd[e >> 2] >> (8 * (e & 3))) & 0xFFu;
            crc = T[(crc ^ b) & 0xFFu] ^ (crc >> 8);
            if (b == 0u)
                ++zeros;
            else
                atomicAdd(&H[b], 1u);
        }
    }
    crc = ~crc;
    // zero bytes dominate: one wave sum instead of 64 colliding LDS atomics per lane-step
    for (int d = 32; d > 0; d >>= 1) zeros += __shfl_xor(zeros, d);
    if ((threadIdx.x & 63) == 0 && zeros) atomicAdd(&H[0], zeros);
    C[threadIdx.x] = crc;
    __syncthreads();
    // fold the per-thread CRCs (thread t covers n_t bytes, all 64 but a ragged tail)
    for (int s = 1; s < kThr; s <<= 1) {
        if ((threadIdx.x & (2 * s - 1)) == 0 && threadIdx.x + s < kThr) {
            const int64_t lb = min<int64_t>(int64_t(s) * kPerThr, max<int64_t>(len - int64_t(threadIdx.x + s) * kPerThr, 0));
            if (lb > 0) C[threadIdx.x] = crc_combine(C[threadIdx.x], C[threadIdx.x + s], uint64_t(lb));
        }
        __syncthreads();
    }
    const int seg = a * g.spa + int(beg / kSeg);
    const uint32_t h = H[threadIdx.x];
    w.chist[int64_t(c) * 256 + threadIdx.x] = uint16_t(h);
    if (h) atomicAdd(&w.shist[int64_t(seg) * 256 + threadIdx.x], h);
    if (threadIdx.x == 0) w.ccrc[c] = len > 0 ? C[0] : 0u;
}

// ---------------------------------------------------------------- CODE
// Huffman code lengths (<= maxlen) of n <= 512 symbols with frequencies f[]
// (0 = absent), by thread 0 after a block-wide sort; the frequencies are
// flattened and the tree rebuilt until the deepest leaf fits.
struct HuffLds {
    uint64_t key[512];    // sorted (freq << 16 | symbol)
    uint32_t node[1024];  // internal node frequencies / parents
    uint32_t par[1024];
    uint8_t len[512];
};

__device__ void sort_keys(uint64_t *key) {  // 512 keys ascending, 256 threads
    for (int k = 2; k <= 512; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < 512; i += kThr) {
                const int l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const uint64_t x = key[i], y = key[l];
                    if ((x > y) == up) {
                        key[i] = y;
                        key[l] = x;
                    }
                }
            }
            __syncthreads();
        }
}

// lengths for symbols 0..n-1 into L.len; f[] in LDS, may be modified (flattening)
__device__ void huff_lengths(uint32_t *f, int n, int maxlen, HuffLds &L) {
    __shared__ int s_ok;
    for (;;) {
        for (int i = threadIdx.x; i < 512; i += kThr) {
            L.key[i] = (i < n && f[i]) ? (uint64_t(f[i]) << 16) | uint64_t(i) : ~0ull;
            if (i < n) L.len[i] = 0;
        }
        __syncthreads();
        sort_keys(L.key);
        if (threadIdx.x == 0) {
            int m = 0;
            while (m < 512 && L.key[m] != ~0ull) ++m;  // leaves, ascending
            // two-queue Huffman: leaves 0..m-1, internal nodes m..2m-2
            int i = 0, j = 0;
            for (int k = 0; k < m - 1; ++k) {
                uint32_t fx[2];
                int id[2];
                for (int r = 0; r < 2; ++r) {
                    const bool leaf = i < m && (j >= k || uint32_t(L.key[i] >> 16) <= L.node[j]);
                    if (leaf) {
                        fx[r] = uint32_t(L.key[i] >> 16);
                        id[r] = i++;
                    } else {
                        fx[r] = L.node[j];
                        id[r] = m + j++;
                    }
                }
                L.node[k] = fx[0] + fx[1];
                L.par[id[0]] = uint32_t(m + k);
                L.par[id[1]] = uint32_t(m + k);
            }
            // depths: root = node m + m - 2 at depth 0 (a lone leaf gets length 1)
            int deepest = 0;
            if (m == 1) {
                L.len[uint32_t(L.key[0]) & 0xFFFFu] = 1;
                deepest = 1;
            } else {
                L.node[m - 2] = 0;  // reuse: depth of internal node k
                for (int k = m - 3; k >= 0; --k) L.node[k] = L.node[L.par[m + k] - m] + 1;
                for (int q = 0; q < m; ++q) {
                    const int d = int(L.node[L.par[q] - m]) + 1;
                    L.len[uint32_t(L.key[q]) & 0xFFFFu] = uint8_t(d);
                    deepest = d > deepest ? d : deepest;
                }
            }
            s_ok = deepest <= maxlen;
        }
        __syncthreads();
        if (s_ok) return;
        for (int i = threadIdx.x; i < n; i += kThr)
            if (f[i]) f[i] = (f[i] + 1u) >> 1;  // flatten (stays >= 1) and rebuild
        __syncthreads();
    }
}

// canonical code of every symbol (RFC 1951 3.2.2), bit-reversed for LSB-first
// emission, as code | len << 24; by thread 0
__device__ void canonical(const uint8_t *len, int n, uint32_t *out) {
    uint32_t count[16] = {}, next[16];
    for (int s = 0; s < n; ++s) ++count[len[s]];
    count[0] = 0;
    uint32_t code = 0;
    for (int b = 1; b < 16; ++b) {
        code = (code + count[b - 1]) << 1;
        next[b] = code;
    }
    for (int s = 0; s < n; ++s) {
        const int l = len[s];
        uint32_t c = 0;
        if (l) {
            const uint32_t v = next[l]++;
            for (int b = 0; b < l; ++b) c |= ((v >> b) & 1u) << (l - 1 - b);
        }
        out[s] = c | (uint32_t(l) << 24);
    }
}

__device__ __forceinline__ void put_bits(uint32_t *buf, uint32_t &pos, uint32_t v, int n) {  // LSB first, n <= 16
    for (int b = 0; b < n; ++b, ++pos)
        if ((v >> b) & 1u) buf[pos >> 5] |= 1u << (pos & 31);
}

__global__ __launch_bounds__(kThr) void dfl_code_kernel(Geo g, DWs w) {
    __shared__ HuffLds L;
    __shared__ uint32_t f[512];
    __shared__ uint32_t code[kSym];
    __shared__ uint32_t hdr[kHdrWords];
    __shared__ uint32_t clf[19];
    __shared__ uint32_t clcode[19];
    __shared__ uint64_t cb[kChunksPerSeg];
    const int s = blockIdx.x, a = s / g.spa, k = s - a * g.spa;
    const int64_t sbeg = int64_t(k) * kSeg, slen = min(kSeg, g.each - sbeg);
    const int c0 = a * g.cpa + int(sbeg / kChunk), nch = int((slen + kChunk - 1) / kChunk);
    for (int i = threadIdx.x; i < 512; i += kThr) f[i] = i < 256 ? w.shist[int64_t(s) * 256 + i] : (i == 256 ? 1u : 0u);
    for (int i = threadIdx.x; i < kHdrWords; i += kThr) hdr[i] = 0u;
    __syncthreads();
    // the data's own frequencies are kept for the sizes below (f is flattened)
    const uint32_t fdata = threadIdx.x < 256 ? f[threadIdx.x] : 0u;
    huff_lengths(f, kSym, kMaxLen, L);
    if (threadIdx.x == 0) canonical(L.len, kSym, code);
    __syncthreads();
    // code-length code: frequencies of the 258 transmitted lengths (257 + one zero distance length)
    uint8_t litlen = threadIdx.x < kSym ? L.len[threadIdx.x] : 0;
    const uint8_t eob_len = L.len[256];
    __syncthreads();
    if (threadIdx.x < 19) clf[threadIdx.x] = 0u;
    __syncthreads();
    if (threadIdx.x < kSym) atomicAdd(&clf[litlen], 1u);
    if (threadIdx.x == 0) atomicAdd(&clf[0], 1u);  // the distance length
    if (threadIdx.x == 0) atomicAdd(&clf[L.len[256]], 1u);
    __syncthreads();
    // (symbol 256 is past the 256 threads above: counted by thread 0)
    huff_lengths(clf, 19, 7, L);
    if (threadIdx.x == 0) {
        canonical(L.len, 19, clcode);
        // block header: BFINAL 0, BTYPE 2 (dynamic), HLIT 257, HDIST 1, HCLEN
        static const int order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        int hclen = 19;
        while (hclen > 4 && L.len[order[hclen - 1]] == 0) --hclen;
        uint32_t pos = 0;
        put_bits(hdr, pos, 0u, 1);
        put_bits(hdr, pos, 2u, 2);
        put_bits(hdr, pos, 0u, 5);   // HLIT - 257
        put_bits(hdr, pos, 0u, 5);   // HDIST - 1
        put_bits(hdr, pos, uint32_t(hclen - 4), 4);
        for (int i = 0; i < hclen; ++i) put_bits(hdr, pos, L.len[order[i]], 3);
        for (int sy = 0; sy <= kSym; ++sy) {  // 257 literal / end lengths, then the distance length 0
            const uint32_t l = sy < kSym ? (code[sy] >> 24) : 0u;
            put_bits(hdr, pos, clcode[l] & 0xFFFFFFu, int(clcode[l] >> 24));
        }
        w.shbits[s] = pos;
    }
    __syncthreads();
    (void)eob_len;
    for (int i = threadIdx.x; i < kHdrWords; i += kThr) w.shdr[int64_t(s) * kHdrWords + i] = hdr[i];
    for (int i = threadIdx.x; i < kSym; i += kThr) w.scode[int64_t(s) * kSym + i] = code[i];
    // chunk bit counts from the chunk histograms (thread t: symbol t's length),
    // in order: each chunk's first code sits after the header and the chunks before it
    const uint32_t mylen = threadIdx.x < 256 ? (code[threadIdx.x] >> 24) : 0u;
    for (int q = 0; q < nch; ++q) {
        uint32_t bits = uint32_t(w.chist[int64_t(c0 + q) * 256 + threadIdx.x]) * mylen;
        for (int d = 32; d > 0; d >>= 1) bits += __shfl_xor(bits, d);
        if (threadIdx.x == 0) cb[q] = 0;
        __syncthreads();
        if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long *>(&cb[q]), (unsigned long long)bits);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint64_t acc = w.shbits[s];
        for (int q = 0; q < nch; ++q) {
            const uint64_t b = cb[q];
            w.cbit[c0 + q] = acc;
            acc += b;
        }
        acc += code[256] >> 24;                 // end of block
        acc += 3;                               // sync flush: an empty stored block's header ...
        const uint64_t bytes = (acc + 7) / 8 + 4;  // ... padded to a byte, LEN 0000, NLEN FFFF
        w.sbytes[s] = uint32_t(bytes);
        // segment CRC from its chunks' CRCs
        uint32_t crc = w.ccrc[c0];
        for (int q = 1; q < nch; ++q) {
            const int64_t lq = min(kChunk, slen - int64_t(q) * kChunk);
            crc = crc_combine(crc, w.ccrc[c0 + q], uint64_t(lq));
        }
        w.scrc[s] = crc;
    }
    (void)fdata;
}

// ---------------------------------------------------------------- SCAN
__global__ void dfl_scan_kernel(Geo g, DWs w, uint8_t *__restrict__ out, uint64_t *__restrict__ sizes,
                                uint32_t *__restrict__ crcs, int64_t count) {
    const int64_t a = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (a >= count) return;
    uint64_t off = 0;
    uint32_t crc = 0;
    for (int k = 0; k < g.spa; ++k) {
        const int64_t s = a * g.spa + k;
        w.soff[s] = off;
        off += w.sbytes[s];
        const int64_t lk = min(kSeg, g.each - int64_t(k) * kSeg);
        crc = k == 0 ? w.scrc[s] : crc_combine(crc, w.scrc[s], uint64_t(lk));
    }
    uint8_t *o = out + a * g.bound;
    o[off] = 0x03;  // final empty fixed block: BFINAL 1, BTYPE 1, end of block
    o[off + 1] = 0x00;
    sizes[a] = off + 2;
    crcs[a] = g.spa ? crc : 0u;
}

// ---------------------------------------------------------------- ENCODE
__device__ __forceinline__ void or_bits(uint32_t *o, uint64_t pos, uint64_t v, int n) {  // n <= 32, into zeroed memory
    const uint64_t wd = pos >> 5;
    const int sh = int(pos & 31);
    const uint64_t x = (v & ((n == 32) ? 0xFFFFFFFFull : ((1ull << n) - 1))) << sh;
    if (uint32_t(x)) atomicOr(o + wd, uint32_t(x));
    if (uint32_t(x >> 32)) atomicOr(o + wd + 1, uint32_t(x >> 32));
}

__global__ __launch_bounds__(kThr) void dfl_encode_kernel(const uint8_t *__restrict__ in, Geo g, DWs w,
                                                          uint8_t *__restrict__ out) {
    __shared__ uint32_t code[kSym];
    __shared__ uint32_t wsum[kThr / 64];
    const int c = blockIdx.x, a = c / g.cpa, k = c - a * g.cpa;
    const int64_t beg = int64_t(k) * kChunk, len = min(kChunk, g.each - beg);
    const int s = a * g.spa + int(beg / kSeg);
    for (int i = threadIdx.x; i < kSym; i += kThr) code[i] = w.scode[int64_t(s) * kSym + i];
    __syncthreads();
    const uint8_t *src = in + int64_t(a) * g.each + beg;
    const int t0 = threadIdx.x * kPerThr;
    const int n = int(min<int64_t>(kPerThr, max<int64_t>(len - t0, 0)));
    uint32_t wd[16];
    load64(src, t0, n, wd);
    auto byte = [&](int e) -> uint32_t { return (wd[e >> 2] >> (8 * (e & 3))) & 0xFFu; };
    uint32_t bits = 0;
#pragma unroll
    for (int e = 0; e < kPerThr; ++e)
        if (e < n) bits += code[byte(e)] >> 24;
    // exclusive scan of the bit counts over the workgroup
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = bits;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (int q = 0; q < wave; ++q) before += wsum[q];
    const uint64_t seg_bit0 = w.soff[s] * 8;
    const uint64_t pos = seg_bit0 + w.cbit[c] + before + incl - bits;
    uint32_t *o = reinterpret_cast<uint32_t *>(out + a * g.bound);  // slots are 256-byte aligned
    // The thread's codes, packed into 32-bit words: its first and last words
    // may hold its neighbours' bits too (atomic OR into the zeroed slot), the
    // words in between are its own (plain stores).
    if (bits) {
        const uint64_t w0 = pos >> 5, wl = (pos + bits - 1) >> 5;
        uint64_t acc = 0;
        int nacc = int(pos & 31);  // the first word's bits below the thread's start stay 0
        uint64_t wi = w0;
        auto emit = [&](uint32_t v) {
            if (wi == w0 || wi == wl)
                atomicOr(o + wi, v);
            else
                o[wi] = v;
            ++wi;
        };
#pragma unroll
        for (int e = 0; e < kPerThr; ++e) {
            if (e < n) {
                const uint32_t ce = code[byte(e)];
                acc |= uint64_t(ce & 0xFFFFFFu) << nacc;
                nacc += int(ce >> 24);
                if (nacc >= 32) {
                    emit(uint32_t(acc));
                    acc >>= 32;
                    nacc -= 32;
                }
            }
        }
        if (nacc > 0) emit(uint32_t(acc));
    }
    const int64_t sbeg = int64_t(beg / kSeg) * kSeg;
    if (threadIdx.x == 0 && beg == sbeg) {
        // the segment's first chunk: its block header
        const uint32_t hb = w.shbits[s];
        const uint32_t *h = w.shdr + int64_t(s) * kHdrWords;
        for (uint32_t q = 0; q * 32 < hb; ++q) {
            const int nb = int(min(32u, hb - q * 32));
            or_bits(o, seg_bit0 + uint64_t(q) * 32, h[q], nb);
        }
    }
    const int64_t slen = min(kSeg, g.each - sbeg);
    if (threadIdx.x == kThr - 1 && beg + len == sbeg + slen) {
        // the segment's last chunk: end of block, then the sync marker's FF FF
        const uint32_t ce = code[256];
        const uint64_t epos = seg_bit0 + w.cbit[c] + before + incl;
        or_bits(o, epos, ce & 0xFFFFFFu, int(ce >> 24));
        const uint64_t end = w.soff[s] + w.sbytes[s];  // byte after FF FF
        or_bits(o, (end - 2) * 8, 0xFFFFu, 16);
    }
}

}  // namespace

extern "C" {

size_t ofd_deflate_bound(int64_t bytes_each) {
    if (bytes_each < 0) return 0;
    const int64_t spa = (bytes_each + kSeg - 1) / kSeg;
    // <= 15 bits per byte, a header and the sync marker per segment, the final block
    return align256(size_t(bytes_each) * 2 + size_t(spa) * (kHdrWords * 4 + 16) + 64);
}

size_t ofd_deflate_workspace_bytes(int64_t count, int64_t bytes_each) {
    if (count <= 0 || bytes_each <= 0) return 0;
    return ws_bytes(count, bytes_each);
}

int ofd_deflate_batch(const void *in, int64_t count, int64_t bytes_each, void *out, uint64_t *sizes, uint32_t *crcs,
                      void *workspace, size_t workspace_bytes, void *stream) {
    if (count < 0 || bytes_each < 0) return OFD_FW_EINVAL;
    if (count == 0) return OFD_FW_OK;
    if (!out || !sizes || !crcs || (bytes_each > 0 && !in)) return OFD_FW_EINVAL;
    if (reinterpret_cast<uintptr_t>(out) & 255u) return OFD_FW_EALIGN;
    hipStream_t st = static_cast<hipStream_t>(stream);
    Geo g;
    g.each = bytes_each;
    g.cpa = int((bytes_each + kChunk - 1) / kChunk);
    g.spa = int((bytes_each + kSeg - 1) / kSeg);
    g.bound = int64_t(ofd_deflate_bound(bytes_each));
    if (int64_t(count) * g.cpa >= (int64_t(1) << 31)) return OFD_FW_ETOOBIG;
    hipError_t e = hipMemsetAsync(out, 0, size_t(count) * size_t(g.bound), st);
    if (e != hipSuccess) return int(e);
    if (bytes_each == 0) {  // an empty array: the final block alone
        hipLaunchKernelGGL(dfl_scan_kernel, dim3(unsigned((count + 255) / 256)), dim3(256), 0, st, g, DWs{},
                           static_cast<uint8_t *>(out), sizes, crcs, count);
        e = hipGetLastError();
        return e == hipSuccess ? OFD_FW_OK : int(e);
    }
    if (!workspace || workspace_bytes < ws_bytes(count, bytes_each) || (reinterpret_cast<uintptr_t>(workspace) & 255u))
        return OFD_FW_EWORKSPACE;
    const DWs w = carve(workspace, count, g);
    e = hipMemsetAsync(w.shist, 0, size_t(count) * g.spa * 1024, st);
    if (e != hipSuccess) return int(e);
    const unsigned nc = unsigned(count * g.cpa), ns = unsigned(count * g.spa);
    const uint8_t *src = static_cast<const uint8_t *>(in);
    uint8_t *dst = static_cast<uint8_t *>(out);
    hipLaunchKernelGGL(dfl_hist_kernel, dim3(nc), dim3(kThr), 0, st, src, g, w);
    hipLaunchKernelGGL(dfl_code_kernel, dim3(ns), dim3(kThr), 0, st, g, w);
    hipLaunchKernelGGL(dfl_scan_kernel, dim3(unsigned((count + 255) / 256)), dim3(256), 0, st, g, w, dst, sizes, crcs,
                       count);
    hipLaunchKernelGGL(dfl_encode_kernel, dim3(nc), dim3(kThr), 0, st, src, g, w, dst);
    e = hipGetLastError();
    return e == hipSuccess ? OFD_FW_OK : int(e);
}

}  // extern "C"
