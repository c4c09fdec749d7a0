/*
 * hdxhash_debug.h — tuning hooks of libhdxhash.so (not part of the drop-in
 * boundary; used by scripts/ab_variants.py for interleaved A/B timing).
 */
#ifndef HDXHASH_DEBUG_H
#define HDXHASH_DEBUG_H

#ifdef __cplusplus
extern "C" {
#endif

/* Select the hash kernel variant for subsequent launches in this process
 * (see hyperdex_amd/csrc/hdx_kernels.hip; -1 = automatic per schema);
 * returns the previous selection, or -2 for an unknown variant (nothing
 * changed). */
int hdxdbg_set_kernel_variant(int variant);
int hdxdbg_kernel_variant(void);

#ifdef __cplusplus
}
#endif

#endif
