// hdx_internal.h — declarations shared by the kernels and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>
#include <vector>

#include "../../include/hdxhash.h"
#include "hdx_host_common.h"
#include "hdx_region_index.h"

namespace hdx {


// Kernel arguments, passed by value (kernarg segment).  codes[] holds the
// per-attribute dispatch class (hdx_device_hash.h CODE_*) for schemas of up
// to kKernargCodes attributes; wider schemas (up to HDX_MAX_ATTRS, the
// reference's u16 attrs_sz) run the wide kernels (hdx_wide.hip), which read
// the classes from codes_dev, a device copy (device_codes, hdx_capi.cpp).
constexpr uint32_t kKernargCodes = 256;
constexpr uint32_t kMaxSweepTables = 4;
constexpr uint32_t kWavePlanSlots = 128;  // BatchArgs::plan: two 64-slot passes
struct SweepTable {
    const uint64_t* index;  // interval index (NULL: scan lower/upper)
    const uint64_t* lower;
    const uint64_t* upper;
    const uint64_t* ids;
    uint64_t* out;
    uint32_t W, D, R, index_words;
    uint32_t lds_index, lds_ids;  // u64 offsets of the LDS copies (launch_hash_encoded)
    uint16_t attrs[16];
};

struct BatchArgs {
    const uint8_t* blob;
    const uint64_t* obj_base;
    const uint32_t* attr_len;
    uint64_t* coords;
    uint32_t* status;
    uint64_t n;
    uint32_t A;
    uint32_t uniform_code;  // the code every attribute shares, or 0xff if mixed
    double inv_A;           // 1.0 / A                       (finalize_args)
    uint32_t a_magic;       // ceil(2^31 / A): t / A == (t * a_magic) >> 31 for t * A < 2^31
    uint32_t pad_;
    const uint8_t* codes_dev;  // A > 128: the classes in device memory (the wide kernels)
    uint8_t codes[kKernargCodes];
    // fused region lookup (hash_regroup_regions_kernel): T tables, K whole
    // objects per wave, lds_tables u64 words of LDS table copies per workgroup
    uint32_t T, K, lds_tables, win_bytes;  // win_bytes: the staged kernels' LDS window (hdx_staged.hip)
    SweepTable t[kMaxSweepTables];
    // The wave-staged kernel's slot plan (hdx_wstage.h, PLAN; filled by its
    // launcher): every wave holds K objects of the same schema, so slot s of
    // any wave is attribute s % A of object s / A — j | o << 8 | code << 16,
    // code CODE_ZERO past the K objects.  Replaces per-slot division and the
    // code-table shuffle on the device.
    uint32_t plan[kWavePlanSlots];
};

hipError_t launch_hash_batch(const BatchArgs& args, hipStream_t stream);
// Wave-staged hash (hdx_wstage.hip): K whole objects per wave copied into an
// LDS window by DMA and hashed from LDS; form = passes / window size.
hipError_t launch_hash_wstage(const BatchArgs& args, hipStream_t stream, int form);  // debug library
// Its product form (hdx_wstage.hip): two passes per wave, head/tail hashing;
// A <= 128 (else hipErrorInvalidValue).
hipError_t launch_hash_wstage_product(const BatchArgs& args, hipStream_t stream);
hipError_t launch_hash_wstage_regions(const BatchArgs& args, hipStream_t stream);  // + args.T tables
// hash + lookup_region (args.T tables in args.t): one fused launch for A <=
// 128 below kRegionLookupMinObjects, else the hash and one lookup launch per
// table (hipErrorOutOfMemory when A > 128, coords is NULL and no scratch can
// be allocated)
hipError_t launch_hash_batch_regions(const BatchArgs& args, hipStream_t stream);
// The wide kernels (hdx_wide.hip): any A (args.codes_dev set).  Packed
// batches (the policy takes them for A > kKernargCodes) and stored objects
// (A > kWsweepMaxAttrs; coords != NULL).
hipError_t launch_hash_wide(const BatchArgs& args, hipStream_t stream);
struct EncodedArgs;
hipError_t launch_hash_sweep_wide(const EncodedArgs& a, hipStream_t stream);
// Debug library only (hdx_wide_dbg.hip): the wide sweep's retired forms.
hipError_t launch_sweep_wide_debug(const EncodedArgs& a, hipStream_t stream, int variant);
// Fills args.uniform_code from args.codes[0..A), and inv_A / a_magic from A.
void finalize_args(BatchArgs& args);
// Kernel variants (hdx_kernels.hip, variant_kernel_name): the automatic policy's
// choices and the alternatives scripts/ab_variants.py times against them.
hipError_t launch_hash_batch_variant(const BatchArgs& args, hipStream_t stream, int variant);
// The variant launch_hash_batch uses: -1 (the automatic policy) in the product
// library; libhdxhash_dbg.so (HDX_DEBUG_BUILD) adds a process-wide selection.
int hash_variant();
int set_hash_variant(int v);  // debug build only: -2 if unknown, else the previous selection
// Debug library only (hdx_kernels_dbg.hip): the retired A/B forms of the batch
// hash and of the fused hash + lookup.
hipError_t launch_debug_variant(const BatchArgs& args, hipStream_t stream, int variant);
hipError_t launch_fused_debug(const BatchArgs& args, hipStream_t stream, int variant);
// The variant launch_hash_batch would run for args, and its kernel's symbol.
int chosen_variant(const BatchArgs& args);
const char* variant_kernel_name(int v);

// Region lookup (hdx_regions.hip): table pointers are device memory owned by
// an hdx_region_table handle; attrs[] holds the subspace's attribute indices.
// index (may be NULL): the table's per-dimension interval index
// (hdx_regions.hip, region_index_build) of index_words u64, W mask words.
struct RegionArgs {
    const uint64_t* lower;   // [R*D]
    const uint64_t* upper;   // [R*D]
    const uint64_t* ids;     // [R]
    const uint64_t* index;
    uint32_t W, index_words;
    const uint64_t* coords;  // [n*A]
    uint64_t* out;           // [n]
    uint64_t n;
    uint32_t A, D, R;
    uint16_t attrs[16];
};

hipError_t launch_lookup_region(const RegionArgs& a, hipStream_t stream);

// Region ids by hash + one lookup launch per table instead of a fused kernel
// (hdx_regions.hip), for the VALU-bound hash kernels whose fused epilogue
// costs more than the coordinates' round trip through HBM — from
// kRegionLookupMinObjects objects (below, the one launch of the fused form
// wins: the daemon shim's batches).  hash(first, count, c) hashes objects
// [first, first + count) into c.  With coords, all n objects are hashed there
// first; without, chunks of at most kRegionChunkBytes of coordinates go
// through a stream-ordered scratch buffer (hipMallocAsync; each chunk pays a
// launch tail of ~0.01 ms: config 3b 4.59 / 3.72 / 3.52 ms with 16 / 64 /
// 256 MiB chunks, 3.47 unchunked, profiles/r3/ab_regions_by_lookup.jsonl).
// If that scratch cannot be allocated nothing is launched and *no_scratch is
// set: the caller then runs its fused form, which needs none.
// Debug variant 235: by lookup at any n, 64 MiB chunks (tests); 247: the
// same with the scratch allocation failing (the fallback).
using RegionHashFn = std::function<hipError_t(uint64_t first, uint64_t count, uint64_t* coords)>;
constexpr uint64_t kRegionChunkBytes = 2ull << 30;
constexpr uint64_t kRegionLookupMinObjects = 1ull << 20;
void trim_region_pools();  // hdx_regions.hip: release the regions scratch pools' cached memory
bool regions_by_lookup_pays(uint64_t n);
uint64_t regions_chunk_objects(uint64_t n, uint32_t A);
hipError_t regions_by_lookup(uint64_t n, uint32_t A, const SweepTable* t, uint32_t T, uint64_t* coords,
                             const RegionHashFn& hash, hipStream_t stream, bool* no_scratch);

// Several subspaces at once (the batcher's prev/this/next lookups): table t's
// region ids for object i go to out[t * out_stride + i].
constexpr uint32_t kMaxMultiTables = 16;
struct MultiRegionArgs {
    const uint64_t* coords;  // [n*A]
    uint64_t* out;
    uint64_t n, out_stride;
    uint32_t A, T;
    struct Table {
        const uint64_t* lower;
        const uint64_t* upper;
        const uint64_t* ids;
        const uint64_t* index;
        uint32_t W, index_words;
        uint32_t D, R;
        uint16_t attrs[16];
    } t[kMaxMultiTables];
};

hipError_t launch_lookup_regions_multi(const MultiRegionArgs& a, hipStream_t stream);

// Host: the interval index of a region table, hdx_region_index.h.

// Stored-object sweep (hdx_encoded.hip): device arrays.  T region tables
// (hdx_hash_encoded_regions_device): table t's region id of object i goes to
// t[t].out[i]; coords may then be NULL.
struct EncodedArgs {
    const uint8_t* keys;
    const uint64_t* key_off;
    const uint32_t* key_len;
    const uint8_t* vals;
    const uint64_t* val_off;
    const uint32_t* val_len;
    uint64_t* coords;
    uint64_t* versions;  // may be NULL
    uint32_t* status;    // may be NULL
    uint64_t n;
    uint32_t A;
    uint32_t a_magic;  // ceil(2^31 / A) (launch_hash_encoded fills it)
    uint32_t T, lds_tables;  // lds_tables: u64 words of the workgroup's table copies
    SweepTable t[kMaxSweepTables];
    const uint8_t* codes_dev;  // A > 128: the classes in device memory (the wide sweep)
    uint8_t codes[kKernargCodes];
    // numeric walk (launch_hash_encoded fills them): the attributes left to the
    // hash passes — the key and every STRING value attribute — in order
    uint8_t p2[kKernargCodes];
    uint32_t S, s_magic;  // how many; ceil(2^31 / S)
};

hipError_t launch_hash_encoded(const EncodedArgs& a, hipStream_t stream);
// hdx_gather.hip: n extents [src + src_off[i], +len[i]) written back to back at
// dst + dst_off[i] (src: device view of pinned host memory, or device memory;
// destination extents must not overlap).
hipError_t launch_gather_extents(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                                 const uint64_t* dst_off, uint8_t* dst, uint64_t n, hipStream_t stream);
// hdx_gather.hip: up to 8 contiguous copies of whole dwords (src: device
// views of pinned host memory, or device memory) by a kernel on `stream`.
hipError_t launch_copy_linear(const void* const* src, void* const* dst, const uint64_t* bytes, uint32_t count,
                              hipStream_t stream);
// The wave-staged sweep (hdx_wsweep.h): K objects per wave, keys and values
// copied into LDS by DMA, the walk and the hashing from LDS; coords != NULL,
// A <= 64 * passes (else hipErrorInvalidValue).  The product form, and (debug
// library) its A/B forms.
constexpr uint32_t kWsweepMaxAttrs = 128;
hipError_t launch_hash_wsweep_product(const EncodedArgs& a, hipStream_t stream);
hipError_t launch_hash_wsweep(const EncodedArgs& a, hipStream_t stream, int form);
// HBM streaming probe (hdx_synth.hip): read `bytes` (write = 1: plus one
// 8-byte store per 64 bytes read into sink[bytes / 64]).
hipError_t launch_stream_probe(const uint8_t* src, uint64_t bytes, uint64_t* sink, int write, hipStream_t s);

// Index-key encoding (hdx_index.hip): n values of one INT64 / FLOAT /
// TIMESTAMP_* attribute at blob + off[i], len[i] bytes; out holds n entries
// of 8 B (16 B for CODE_FLOAT).
struct IndexArgs {
    const uint8_t* blob;
    const uint64_t* off;
    const uint32_t* len;
    uint8_t* out;
    uint32_t* status;  // may be NULL
    uint64_t n;
    uint32_t code;     // CODE_INT64 or CODE_FLOAT (timestamps encode as int64)
};

hipError_t launch_index_encode(const IndexArgs& a, hipStream_t stream);

// Search pruning (hdx_index.hip) over one subspace's region table: m ranges
// that name a subspace attribute, in the order lookup_search visits them.
enum : uint8_t { SEARCH_NONE = 0, SEARCH_STRING_EQ = 1, SEARCH_ORDERED = 2 };
constexpr uint32_t kMaxSearchRanges = 16;  // one range per subspace dimension
struct SearchArgs {
    const uint64_t* lower;   // [R*D]
    const uint64_t* upper;   // [R*D]
    const uint64_t* hashes;  // [2*m]: hash of start, hash of end
    const uint8_t* replicas; // [R] 0 = region without replicas (skipped), or NULL = all have
    uint8_t* include;        // [R]
    uint32_t* cleared;       // set when the reference would clear the server list
    uint32_t R, D, m;
    uint8_t dim[kMaxSearchRanges];
    uint8_t kind[kMaxSearchRanges];
    uint8_t flags[kMaxSearchRanges];  // bit 0 has_start, bit 1 has_end
};

hipError_t launch_search_regions(const SearchArgs& a, hipStream_t stream);

struct SynthArgs {
    uint64_t seed;
    uint64_t first;
    uint64_t n;
    uint32_t A;
    uint32_t pad_;
    hdx_synth_rule rules[64];
};

hipError_t launch_synth_lengths(const SynthArgs& a, uint32_t* attr_len, hipStream_t s);
hipError_t launch_synth_fill(const SynthArgs& a, const uint64_t* obj_base, const uint32_t* attr_len,
                             uint8_t* blob, uint64_t bytes, hipStream_t s);

// keys (may be NULL): each key is also copied to keys + key_off[i]
hipError_t launch_synth_encode(const uint8_t* blob, const uint64_t* obj_base, const uint32_t* attr_len,
                               uint32_t A, uint64_t n, uint64_t first_version, const uint64_t* val_off,
                               uint8_t* vals, hipStream_t s, const uint64_t* key_off = nullptr,
                               uint8_t* keys = nullptr);

}  // namespace hdx
