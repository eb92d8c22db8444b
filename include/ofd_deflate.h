/*
 * ofd_deflate.h -- C ABI of the MI355X DEFLATE encoder for the npz product.
 *
 * Conventions as ofd_fw.h: plain pointers and sizes, gfx950 device pointers,
 * asynchronous on `stream` (a hipStream_t as void*); returns 0, an OFD_FW_E*
 * code (< 0) or a hipError_t (> 0).
 *
 * Replaces the host zlib of np.savez_compressed in preprocess.py:446 and
 * :471-476 (reference AegeanKI/OpticalFlowFromDepth @ 2024_08_07): the arrays
 * are deflated where they already are.  The streams are RFC 1951 raw deflate
 * (dynamic-Huffman literal blocks of 1 MiB, each closed by a sync marker, and
 * an empty final block), readable by any inflater -- zlib, Python's zipfile,
 * np.load; the compressed bytes differ from zlib's, the decompressed bytes
 * are the array's.
 */
#ifndef OFD_DEFLATE_H
#define OFD_DEFLATE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Output slot bytes per array of `bytes_each` bytes (an upper bound on one
 * stream, a multiple of 256). */
size_t ofd_deflate_bound(int64_t bytes_each);

/* Workspace bytes for ofd_deflate_batch(count, bytes_each). */
size_t ofd_deflate_workspace_bytes(int64_t count, int64_t bytes_each);

/* Deflate `count` arrays of `bytes_each` bytes laid out back to back at `in`
 * (device).  Array i's complete raw-deflate stream goes to
 * out + i * ofd_deflate_bound(bytes_each) (device, 256-byte aligned, count
 * slots; the call zeroes them first), its length in bytes to sizes[i] and the
 * CRC-32 (zlib's crc32) of its bytes to crcs[i] (both device arrays). */
int ofd_deflate_batch(const void *in, int64_t count, int64_t bytes_each, void *out, uint64_t *sizes, uint32_t *crcs,
                      void *workspace, size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* OFD_DEFLATE_H */
