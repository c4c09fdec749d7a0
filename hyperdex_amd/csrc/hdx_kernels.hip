// hdx_kernels.hip — batched hyperspace attribute hashing for gfx950.
//
// One launch hashes every attribute of n objects in the packed layout of
// include/hdxhash.h and writes coords[i*A + j] — hs[j] of the reference's
// hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68) for object i.
// The work unit is the (object, attribute) slot; 64 consecutive slots (one
// wave's worth) form a chunk.  Two kernels:
//   hash_chunk_kernel   — one wave per chunk, a single dependent chain;
//   hash_regroup_kernel — one wave per C chunks, descriptors in wave-private
//                         LDS, optionally counting-sorted by work class so a
//                         wave's lanes run the same CityHash regime.
// launch_hash_batch picks one per schema and size (auto_variant).  Variant ids
// are those of the round-1 A/B logs (profiles/r1/ab_*.jsonl); the ids of
// retired experiments (0-11, 13-17, 22-24, 27-29, 32-34, 36, 38, 39, 44-46,
// 50-53, 59: rounds-per-wave kernels, non-temporal loads, workgroup-barrier
// sorts, LDS-staged blocks, larger sort windows, occupancy caps, workgroup LDS
// windows with and without pipelining) are no longer built; their results are
// in DESIGN.md §4 and the logs.
// The kernel bodies and launch templates are in hdx_regroup.h; the retired
// experiments (debug library only) in hdx_kernels_dbg.hip.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "hdx_regroup.h"

#ifndef HDX_DEBUG_BUILD
#define HDX_DEBUG_BUILD 0
#endif

namespace hdx {

hipError_t launch_hash_batch_variant(const BatchArgs& args, hipStream_t stream, int variant) {
    switch (variant) {
        // the automatic policy's kernels (auto_variant)
        case 12: return launch_chunk<true>(args, stream);
        case 20: return launch_regroup<8, true, false>(args, stream);
        // 21 and 46: one wave per workgroup (round 5, profiles/r5/ab_wpb.jsonl: config 2 0.331 vs 0.336 ms,
        // mixed 2.18 vs 2.31; 25 and 12 keep four: 2.246 vs 2.302, 0.146 vs 0.147)
        case 21: return launch_regroup<4, true, false, true, false, false, false, 0, 1>(args, stream);
        case 25: return launch_regroup<16, true, false, false>(args, stream);
        case 44: return launch_regroup<2, true, true, true, true, false, true, 1>(args, stream);
        case 46: return launch_regroup<8, true, true, true, false, false, true, 1, 1>(args, stream);
        case 212: return launch_hash_wstage_product(args, stream);  // hdx_wstage.hip
        case 300: return launch_hash_wide(args, stream);            // hdx_wide.hip
        default:
#if HDX_DEBUG_BUILD
            return launch_debug_variant(args, stream, variant);  // hdx_kernels_dbg.hip
#else
            return hipErrorInvalidValue;
#endif
    }
}

static int auto_variant(const BatchArgs& args);

// The fused form follows the automatic policy's kind of pass shape with whole
// objects per wave, the tables looked up in a wave-uniform loop (UNI; one lane
// per (table, object) pair was 0.60 vs 0.47 ms on config 2): uniform strings 8
// unsorted chunks (the tables then fit in LDS beside the descriptors: 1.97 vs
// 2.66 ms with 16 chunks and the tables in global memory, config 3a), 2 below
// 32 M slots (config 1: 0.158 vs 0.178 ms with 8); numeric-heavy 4 unsorted;
// complex types 8 sorted; mixed strings (round 3) the wave-staged kernel and
// separate lookups, before that 3 sorted chunks with A4 loads (config 3b:
// 3.83 vs 4.26 ms with 2; profiles/r1/fused_batch_regions.jsonl,
// profiles/r2/ab_fused.jsonl).  A <= 128 (checked by the caller).
hipError_t launch_hash_batch_regions(const BatchArgs& args, hipStream_t stream) {
    if (args.n == 0) return hipSuccess;
    if (args.A > 128) {
        // wide schemas: the batch policy's hash (44, or the wide kernel above
        // 256 attributes), then one lookup launch per table
        const RegionHashFn hash = [&](uint64_t first, uint64_t count, uint64_t* c) {
            BatchArgs b = args;
            b.obj_base += first;
            b.attr_len += first * args.A;
            b.n = count;
            b.coords = c;
            b.T = 0;
            return launch_hash_batch(b, stream);
        };
        bool no_scratch = false;
        const hipError_t e = regions_by_lookup(args.n, args.A, args.t, args.T, args.coords, hash, stream, &no_scratch);
        return no_scratch ? hipErrorOutOfMemory : e;
    }
#if HDX_DEBUG_BUILD
    const int v = hash_variant();
    if (v >= 100 && v < 120) return launch_fused_debug(args, stream, v);  // hdx_kernels_dbg.hip
    if (v == 217) return launch_hash_wstage_regions(args, stream);
#endif
    switch (auto_variant(args)) {
        case 25: case 20: return launch_regroup_regions<8, false, false, false, 0, true>(args, stream);
        case 12: return launch_regroup_regions<2, false, false, false, 0, true>(args, stream);
        case 21: return launch_regroup_regions<4, false, false, false, 0, true>(args, stream);
        case 46: return launch_regroup_regions<8, true, false, true, 1, true>(args, stream);
        // mixed strings: the wave-staged kernel is VALU-bound, so a fused
        // epilogue costs more than the coordinates' round trip (config 3b,
        // 10 M objects, bench.py's two tables: fused 3.66 ms (debug 217),
        // hash + separate lookups 3.47; profiles/r3/ab_fused_batch.jsonl):
        // hash, then one lookup launch per table (chunked through scratch when
        // the caller wants no coordinates); small batches keep the one fused
        // launch (debug 217's kernel)
        case 212: {
            if (!regions_by_lookup_pays(args.n)) return launch_hash_wstage_regions(args, stream);
            const RegionHashFn hash = [&](uint64_t first, uint64_t count, uint64_t* c) {
                BatchArgs b = args;
                b.obj_base += first;
                b.attr_len += first * args.A;
                b.n = count;
                b.coords = c;
                b.T = 0;
                return launch_hash_wstage_product(b, stream);
            };
            bool no_scratch = false;
            const hipError_t e = regions_by_lookup(args.n, args.A, args.t, args.T, args.coords, hash, stream,
                                                   &no_scratch);
            return no_scratch ? launch_hash_wstage_regions(args, stream) : e;
        }
        default: return launch_regroup_regions<3, true, true, true, 1, true>(args, stream);
    }
}

// Automatic choice (interleaved A/B on one MI355X, profiles/r1/ab_variants_*.jsonl
// and profiles/r1/ab_a4_*.jsonl):
//  * schemas with timestamps or non-hashable attributes: regroup kernel with the
//    class sort, 8 chunks per wave, classes in ORDER 1 (46) — their diverse
//    paths dominate (mixed: 2.32 vs 2.49 ms in ORDER 0 (19), 3.48 for the
//    chunk kernel);
//  * mostly numerics: regroup unsorted, 4 chunks per wave, direct stores (21)
//    (config 2: 0.31 vs 0.42 ms);
//  * one code everywhere (all strings): regroup unsorted with 16 chunks per wave
//    and burst stores (25) when the grid keeps >= 64 K waves, 8 chunks (20) from
//    32 M slots (config 3a: 2.24 vs 2.38 ms), else the one-chunk kernel (12)
//    (config 1);
//  * otherwise (strings + int64/float, config 3b): the wave-staged kernel
//    (212, hdx_wstage.hip): each wave copies its 7 objects' span into LDS by
//    coalesced DMA, class-sorts the 119 slots and hashes them from LDS with
//    head/tail reads — 2.92 vs 3.32 ms for the gather kernel 44 (round 3,
//    profiles/r3/ab_wstage_ht.jsonl).  Up to round 2 this case ran 44: the
//    class sort over 2 chunks with dword-aligned loads (3.37 vs 3.43 ms in
//    ORDER 0 (38) and 4.22 for the chunk kernel — byte-misaligned 16-byte
//    loads had made the texture-address unit the bound).
//    Schemas of 129-256 attributes keep 44; wider ones (up to the reference's
//    65535) take the wide kernel (300, hdx_wide.hip), whose attribute classes
//    come from device memory.
static int auto_variant(const BatchArgs& args) {
    if (args.A > kKernargCodes) return 300;  // hdx_wide.hip
    uint32_t numeric = 0;
    bool complex_types = false;
    for (uint32_t j = 0; j < args.A; ++j) {
        const uint8_t c = args.codes[j];
        numeric += c >= CODE_INT64;
        complex_types |= c == CODE_ZERO || c >= CODE_TS_SECOND;
    }
    const uint64_t slots = args.n * args.A;
    if (complex_types) return 46;
    if (2 * numeric > args.A) return 21;
    if (args.uniform_code != 0xffu) {
        if (slots >= (64ull << 20)) return 25;
        if (slots >= (32ull << 20)) return 20;
        return 12;
    }
    return args.A <= 128 ? 212 : 44;
}

#if !HDX_DEBUG_BUILD
// The product library has no kernel selection: the automatic policy only
// (the debug library's selection is in hdx_kernels_dbg.hip).
int hash_variant() { return -1; }
#endif

void finalize_args(BatchArgs& args) {
    args.inv_A = 1.0 / (double)args.A;
    args.a_magic = (uint32_t)(((1ull << 31) + args.A - 1) / args.A);
    args.uniform_code = args.codes[0];
    for (uint32_t j = 1; j < std::min(args.A, kKernargCodes); ++j)
        if (args.codes[j] != args.codes[0]) args.uniform_code = 0xffu;
}

hipError_t launch_hash_batch(const BatchArgs& args, hipStream_t stream) {
    const int v = hash_variant();
    return launch_hash_batch_variant(args, stream, v < 0 ? auto_variant(args) : v);
}

int chosen_variant(const BatchArgs& args) {
    const int v = hash_variant();
    return v < 0 ? auto_variant(args) : v;
}

// The kernel symbol a variant launches, as rocprofv3 prints it.
const char* variant_kernel_name(int v) {
    switch (v) {
        case 12: return "void hdx::hash_chunk_kernel<true, false, 0, false>(hdx::BatchArgs)";
        case 30: return "void hdx::hash_chunk_kernel<true, true, 0, false>(hdx::BatchArgs)";
        case 31: return "void hdx::hash_chunk_kernel<true, false, 0, true>(hdx::BatchArgs)";
        case 18: return "void hdx::hash_regroup_kernel<4, true, true, true, false, false, false, 0, 4>(hdx::BatchArgs)";
        case 19: return "void hdx::hash_regroup_kernel<8, true, true, true, false, false, false, 0, 4>(hdx::BatchArgs)";
        case 20: return "void hdx::hash_regroup_kernel<8, true, false, true, false, false, false, 0, 4>(hdx::BatchArgs)";
        case 21: return "void hdx::hash_regroup_kernel<4, true, false, true, false, false, false, 0, 1>(hdx::BatchArgs)";
        case 25: return "void hdx::hash_regroup_kernel<16, true, false, false, false, false, false, 0, 4>(hdx::BatchArgs)";
        case 26: return "void hdx::hash_regroup_kernel<2, true, true, true, false, false, false, 0, 4>(hdx::BatchArgs)";
        case 35: return "void hdx::hash_regroup_kernel<2, true, true, true, true, false, false, 0, 4>(hdx::BatchArgs)";
        case 37: return "void hdx::hash_regroup_kernel<2, true, true, true, true, true, false, 0, 4>(hdx::BatchArgs)";
        case 38: return "void hdx::hash_regroup_kernel<2, true, true, true, true, false, true, 0, 4>(hdx::BatchArgs)";
        case 39: return "void hdx::hash_regroup_kernel<8, true, true, true, false, false, true, 0, 4>(hdx::BatchArgs)";
        case 44: return "void hdx::hash_regroup_kernel<2, true, true, true, true, false, true, 1, 4>(hdx::BatchArgs)";
        case 45: return "void hdx::hash_regroup_kernel<2, true, true, true, true, false, true, 2, 4>(hdx::BatchArgs)";
        case 46: return "void hdx::hash_regroup_kernel<8, true, true, true, false, false, true, 1, 1>(hdx::BatchArgs)";
        case 300: return "hdx::hash_wide_kernel(hdx::BatchArgs)";
        case 212: return "void hdx::hash_wstage_kernel<2, 8832u, 0, 6, 5, 0, false, true, true, true, false, 1, true, false, true, 1, true, true>(hdx::BatchArgs)";
        default: return "";
    }
}

}  // namespace hdx
