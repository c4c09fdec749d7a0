/*
 * hdxhash_debug.h — tuning hooks of libhdxhash.so (not part of the drop-in
 * boundary; used by scripts/ab_variants.py for interleaved A/B timing).
 */
#ifndef HDXHASH_DEBUG_H
#define HDXHASH_DEBUG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Select the hash kernel variant for subsequent launches in this process
 * (see hyperdex_amd/csrc/hdx_kernels.hip; -1 = automatic per schema);
 * returns the previous selection, or -2 for an unknown variant (nothing
 * changed). */
int hdxdbg_set_kernel_variant(int variant);
int hdxdbg_kernel_variant(void);
/* The variant hdx_hash_batch_device would launch for this schema and object
 * count (under the current selection), and the kernel's symbol as rocprofv3
 * reports it (*name; static string).  Returns -2 on a bad schema. */
int hdxdbg_kernel_for(const uint32_t* types, uint32_t attrs_sz, uint64_t n, const char** name);
/* HBM streaming probe: read `bytes` (a multiple of 4096) of device memory at
 * src in the hash kernels' access shape; write != 0 also stores one 8-byte
 * word per 64 bytes read into sink[bytes / 64] (the 1:8 write mix of the
 * 64-byte-attribute configs).  Asynchronous on `stream`.  bench.py reports the
 * rate as the practical ceiling beside the HBM3E spec. */
int hdxdbg_stream_probe(const void* src, uint64_t bytes, uint64_t* sink, int write, void* stream);

#ifdef __cplusplus
}
#endif

#endif
