/*
 * hdxhash_debug.h — measurement and tuning hooks (not part of the drop-in
 * boundary).
 *
 * Both libraries: hdxdbg_kernel_for (which kernel the automatic policy runs),
 * hdxdbg_stream_probe (bench.py's practical HBM ceiling) and
 * hdxdbg_region_chunk_objects (tests/test_scale.py's chunk edges).
 * libhdxhash_dbg.so only (HDX_DEBUG_BUILD, hyperdex_amd/csrc/Makefile):
 * hdxdbg_set_kernel_variant / hdxdbg_kernel_variant, used by
 * scripts/ab_variants.py and the variant parity tests.  The product library
 * has no kernel selection and no environment switches.
 */
#ifndef HDXHASH_DEBUG_H
#define HDXHASH_DEBUG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* [debug library only] Select the hash kernel variant for subsequent launches in this process
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
/* [debug library only] The device set of hdx_init_mask from an explicit list
 * of HIP ordinals, repeats allowed (world 2+ on one GPU: host batches and
 * ungathered shards; a gather over a repeated device returns HDX_E_INVALID). */
int hdxdbg_init_devices(const int* devices, int n);
/* Objects per scratch chunk of the regions entry points when the caller
 * wants no coordinates (n objects of attrs_sz attributes; hdx_regions.hip). */
uint64_t hdxdbg_region_chunk_objects(uint64_t n, uint32_t attrs_sz);

#ifdef __cplusplus
}
#endif

#endif
