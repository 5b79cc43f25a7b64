/*
 * cc_n5.h -- C ABI of the native N5 chunk codec (libcc_n5.so, host C++ + zlib, no GPU).
 *
 * Replaces z5py, which the reference reaches through elf.io.open_file
 * (cluster_tools/utils/volume_utils.py:21-22) for every ds[bb] read / write of the thresholded-
 * components path (block_components.py:151,180, write.py:185-202, merge_assignments.py:136-139).
 * N5 layout (byte-layout parity unpinned: no z5py-written file exists here): chunk file
 * <dataset>/<i_fastest>/.../<i_slowest>, big-endian header (u16 mode, u16 ndim, u32 dims fastest
 * first; mode 1 adds a u32 element count) and big-endian C-order payload, raw (compression 0) or
 * gzip (1, deflate `level`; reads accept gzip or zlib streams).
 *
 * Region [begin, end) (NULL = the whole dataset) of a dataset of `shape` / `chunks` (C order,
 * ndim 1..4), elem_size 1/2/4/8 bytes, host buffers in C order over the region.  The chunks a
 * call touches are coded on n_threads host threads.  Read: missing chunks read as 0.  Write:
 * partially covered chunks are read, merged and rewritten; skip_zero_chunks: an all-zero chunk
 * that has no file yet is not written (the reference never writes empty blocks).
 * Status 0 = ok, < 0 = error (message: cc_n5_last_error(), per thread).
 */
#ifndef CC_N5_H
#define CC_N5_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* "cc_n5 0.2 src=<hash>": src = SHA-256 prefix of the library sources (binary provenance) */
const char* cc_n5_version(void);
const char* cc_n5_last_error(void);
int cc_n5_read(const char* dataset_path, int ndim, const int64_t* shape, const int64_t* chunks, int elem_size,
               int compression, const int64_t* begin, const int64_t* end, void* out_host, int n_threads);
int cc_n5_write(const char* dataset_path, int ndim, const int64_t* shape, const int64_t* chunks, int elem_size,
                int compression, int level, const int64_t* begin, const int64_t* end, const void* in_host,
                int n_threads, int skip_zero_chunks);

#ifdef __cplusplus
}
#endif
#endif /* CC_N5_H */
