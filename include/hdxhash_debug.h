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

#ifdef __cplusplus
}
#endif

#endif
