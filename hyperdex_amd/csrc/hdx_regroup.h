// hdx_regroup.h — the batch-hash kernels' bodies and launch templates, shared
// by the product translation unit (hdx_kernels.hip: the automatic policy's
// instantiations) and the debug library's experiment kernels
// (hdx_kernels_dbg.hip, libhdxhash_dbg.so only).  See hdx_kernels.hip and
// DESIGN.md §4 for the kernels; include/hdxhash.h for the layout.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_loads.h"
#include "hdx_region_lookup.h"

namespace hdx {

// ===========================================================================
// Chunk kernel (variant 12): one wave = one chunk of 64 consecutive
// (object, attribute) slots of the flattened n*A slot space — the layout's
// natural unit: a coalesced 256 B length load, 64 attributes hashed, one
// coalesced 512 B coordinate store.  A wave has a single dependent chain
// (lengths -> prefix sum -> addresses -> bytes -> hash -> store) and exits, so
// no store ever sits in front of a later load in the wave's vmcnt queue, and
// the hardware keeps up to 8 waves per SIMD issuing fresh loads.  An object
// that starts in an earlier chunk contributes a carry: the sum of its
// attribute lengths that precede this chunk (read back from lengths the
// neighbouring wave just pulled through L2).
// ===========================================================================

// SHAPE (debug variants only): 0 = the real kernel; 1 = its loads without the
// hash arithmetic (variant 40); 2 = its arithmetic without the byte loads
// (variant 41).  Shapes 1 and 2 write wrong coordinates: they bound the
// kernel's time by its memory and its VALU work.
template <bool NT_STORE, bool PIPE = false, int SHAPE = 0, bool A4 = false>
__global__ void __launch_bounds__(256)
hash_chunk_kernel(const BatchArgs args) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t A = args.A;
    const uint64_t nslots = args.n * A;
    const uint64_t q0 = wave * 64;
    if (q0 >= nslots) return;

    // this lane's slot -> (object il, attribute j)
    uint64_t i0;
    uint32_t j0;
    split_slot(q0, A, args.inv_A, i0, j0);
    const uint32_t t = j0 + (uint32_t)lane;
    const uint32_t di = div_small(t, args.a_magic);  // t < A + 64
    const uint32_t j = t - di * A;
    const uint64_t il = i0 + di;
    const bool valid = q0 + lane < nslots;

    // lengths of this chunk, the object bases, and the carry-in lengths
    const uint32_t L = valid ? args.attr_len[q0 + lane] : 0u;
    const uint64_t base = args.obj_base[valid ? il : i0];
    uint32_t carry = 0;
    for (uint32_t k = 0; k < j0; k += 64) {  // slots [q0 - j0, q0) belong to object i0
        const uint32_t idx = k + (uint32_t)lane;
        const uint32_t v = idx < j0 ? args.attr_len[q0 - j0 + idx] : 0u;
        carry += wave_sum_dpp(v);
    }
    uint32_t code;
    if (args.uniform_code != 0xffu) {
        code = args.uniform_code;
    } else {
        const uint32_t packed = reinterpret_cast<const uint32_t*>(args.codes)[lane];
        code = (__shfl(packed, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
    }

    const uint32_t Sx = wave_scan_dpp(L) - L;
    const int head = lane - (int)j;  // lane holding this object's attribute 0, if in this chunk
    const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
    const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
    const uint8_t* p = args.blob + base + off;

    const Blk blk = SHAPE == 2 ? fake_block(p, L)
                               : consume_any<A4>(issue_any<A4>(valid ? code : (uint32_t)CODE_ZERO, p, L));
    if (valid) {
        bool bad = false;
        const uint64_t h = SHAPE == 1 ? touch_blk(code, p, L, blk)
                                      : hash_blk<PIPE, SHAPE == 2, A4>(code, p, L, blk, bad);
        if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q0 + lane);
        else args.coords[q0 + lane] = h;
        if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
    }
}

// Work classes (the regroup kernel's sort key) and the 16-byte slot descriptor.
constexpr int kClasses = 8;

// ORDER 0: {numerics, <= 16 B}, 17..64 B, then > 64 B by loop blocks.
// ORDER 1: numerics, 33..64, <= 16, 17..32, then > 64 B by blocks (1, 2, 3, 4+):
//          puts the cheap 33..64-byte regime beside the numerics in the first
//          pass of a 2-chunk wave and the short-string regimes with the long ones.
// ORDER 2: numerics, <= 16, 17..32, 33..64, then > 64 B by blocks.
template <int ORDER = 0>
__device__ __forceinline__ uint32_t work_class(uint32_t code, uint32_t n, bool valid) {
    if constexpr (ORDER == 0) {
        if (!valid || code != CODE_STRING || n <= 16) return 0;
        if (n <= 64) return 1;
        const uint32_t b = (n - 1) >> 6;
        return b >= 6 ? 7u : 1u + b;
    } else {
        if (!valid || code != CODE_STRING) return 0;
        if (n > 64) {
            const uint32_t b = (n - 1) >> 6;
            return b >= 4 ? 7u : 3u + b;
        }
        if (ORDER == 1) return n > 32 ? 1u : n <= 16 ? 2u : 3u;
        return n <= 16 ? 1u : n <= 32 ? 2u : 3u;
    }
}
// ORDER 3 (the wave-staged kernel's head/tail hashing): strings of <= 64
// bytes first (33..64, <= 16, 17..32), then numerics / non-hashable / unused
// slots, then > 64 B by blocks: a 2-pass wave's second pass holds the long
// strings beside the cheapest regime.
__device__ __forceinline__ uint32_t work_class3(uint32_t code, uint32_t n, bool valid) {
    if (!valid || code != CODE_STRING) return 3;
    if (n > 64) {
        const uint32_t b = (n - 1) >> 6;
        return b >= 4 ? 7u : 3u + b;
    }
    return n > 32 ? 0u : n <= 16 ? 1u : 2u;
}

// work_class<1> without branches (selects only): a divergent if / else chain
// costs exec-mask bookkeeping on every lane of the wave (ORDER 4 of the
// wave-staged kernel, the sweep's BF form).
__device__ __forceinline__ uint32_t work_class1_bf(uint32_t code, uint32_t n, bool valid) {
    const uint32_t b = (n - 1) >> 6;
    const uint32_t longc = b >= 4 ? 7u : 3u + b;
    const uint32_t shortc = n > 32 ? 1u : n <= 16 ? 2u : 3u;
    const uint32_t c = n > 64 ? longc : shortc;
    return valid && code == CODE_STRING ? c : 0u;
}

// work_class<1> from a table: 3-bit classes indexed by ceil(min(n, 272) / 16)
// (0..17), one 64-bit shift instead of the comparison chain (ORDER 5 of the
// wave-staged kernel, with the slot plan).
constexpr uint64_t class1_table() {
    // idx: 0-1 <= 16 B (2), 2 17..32 (3), 3-4 33..64 (1), 5-8 one block (4),
    // 9-12 two (5), 13-16 three (6), 17 four or more (7)
    constexpr uint8_t c[18] = {2, 2, 3, 1, 1, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 6, 7};
    uint64_t t = 0;
    for (int i = 0; i < 18; ++i) t |= (uint64_t)c[i] << (3 * i);
    return t;
}
__device__ __forceinline__ uint32_t work_class1_tab(uint32_t code, uint32_t n, bool valid) {
    const uint32_t idx = (min(n, 272u) + 15u) >> 4;
    const uint32_t c = (uint32_t)(class1_table() >> (3 * idx)) & 7u;
    return valid && code == CODE_STRING ? c : 0u;
}

// Wave-local counting sort of a wave's NCH * 64 slots by work class into
// perm[] (slot | code << 8, pass t = perm[64 t .. 64 t + 63]); slots s >= ns
// are pads (hashed as CODE_ZERO, results unused).  A pass pays for the union
// of the CityHash regimes its lanes hold, so with GAP (NCH == 2) the class
// that would straddle the pass boundary is moved whole into the second pass
// when there are pads enough to fill the first pass's rest: that pass then
// skips the class's regime code (config 3b: the <= 16 / 17..32 regime;
// config 5's sweep: the first > 64-byte loop).  Without GAP (or without pads
// enough) pads follow the last class.  fence(): the wave's LDS fence.
// pos_out (may be NULL): each of the lane's NCH slots' position in perm.
template <int NCH, bool GAP, class Fence>
__device__ __forceinline__ void class_sort(uint32_t* cnt, uint16_t* perm, const uint32_t (&cls)[NCH],
                                           const uint32_t (&code)[NCH], uint32_t ns, Fence fence,
                                           uint32_t* pos_out = nullptr) {
    const int lane = threadIdx.x & 63;
    if (lane < kClasses) cnt[lane] = 0;
    fence();
#pragma unroll
    for (int c = 0; c < NCH; ++c)
        if ((uint32_t)(c * 64 + lane) < ns)
            __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    fence();
    uint32_t gap = 0, gap_at = 0;  // wave-uniform
    {
        const uint32_t k = lane < kClasses ? cnt[lane] : 0u;
        uint32_t start = wave_scan_dpp(k) - k;
        if constexpr (GAP && NCH == 2) {
            const uint64_t cross = __ballot(lane < kClasses && start < 64 && start + k > 64);
            if (cross) {
                const int x = (int)__builtin_ctzll(cross);
                const uint32_t sx = __builtin_amdgcn_readlane(start, x);
                if (64 - sx <= NCH * 64 - ns) {
                    gap = 64 - sx;
                    gap_at = sx;
                    if (lane >= x) start += gap;
                }
            }
        }
        if (lane < kClasses) cnt[lane] = start;
    }
    fence();
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        uint32_t pos;
        if (s < ns) {
            pos = __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        } else {
            const uint32_t p = s - ns;  // pad p: the first `gap` fill the first pass, the rest follow the classes
            pos = p < gap ? gap_at + p : ns + p;
        }
        perm[pos] = (uint16_t)(s | (code[c] << 8));
        if (pos_out) pos_out[c] = pos;
    }
    fence();
}


// ===========================================================================
// Regroup kernel (variants 18/19/26/35/37 sorted with C = 4/8/2/2/2; 20/21/25
// unsorted with C = 8/4/16): a wave owns C consecutive chunks (C*64
// slots).  Phase 1 computes every slot's {pointer, length, code} as the chunk
// kernel does (all C length loads issued at once; the carry chains from chunk
// to chunk in registers) and writes a 16-byte descriptor per slot into the
// wave's private LDS.  A counting sort by work class (ballot + popcount +
// mbcnt, wave-local: no workgroup barrier) yields a permutation.  Phase 2
// hashes C passes of 64 class-sorted slots — the next pass's descriptors and
// bytes are in flight while the current pass is hashed — and writes each
// coordinate over its (already consumed) descriptor.  Phase 3 stores the C
// chunks in slot order, one coalesced 512 B store each.  A wave whose C*64
// slots all share one class skips the permutation.
// ===========================================================================
template <int C, int WPB = 4>
struct RegroupLds {
    SlotDesc desc[WPB][C * 64];   // reused for the coordinates in phase 2
    uint16_t perm[WPB][C * 64];
    uint32_t cnt[WPB][kClasses];  // ASORT: per-class counters / cursors
};

// A4: dword-aligned loads (hdx_loads.h); PIPE: the > 64-byte loop keeps the
// next block in flight; ASORT: the class sort by LDS fetch-add instead of
// ballot / mbcnt per (class, chunk).
// REG (hash_regroup_regions_kernel): a wave owns K = args.K whole objects
// (K * A <= C * 64 slots) instead of C * 64 slots, parks every coordinate,
// looks its objects up in the args.T region tables (configuration::
// lookup_region, hdx_region_lookup.h; tbl = the workgroup's LDS copies) and
// stores coordinates only when args.coords is set.
template <int C, bool NT_STORE, bool SORT, bool DIRECT, bool A4, bool PIPE, bool ASORT, int ORDER, bool REG,
          bool UNI = false, bool REGD = false, bool QUAD = false, int LATE = 0, int DEFER = 0,
          class Lds = RegroupLds<C>>
__device__ __forceinline__ void regroup_body(const BatchArgs& args, Lds& lds, const uint64_t* tbl,
                                             uint64_t wave = ~0ull) {
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    SlotDesc* desc = lds.desc[w];
    uint16_t* perm = lds.perm[w];
    uint64_t* res = reinterpret_cast<uint64_t*>(desc);  // res[2*s] = first 8 bytes of desc[s]

    if (wave == ~0ull) wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + w;
    const uint32_t A = args.A;
    uint64_t qw, nslots, o_begin = 0, o_end = 0;  // nslots: end of this wave's slots
    if constexpr (REG) {
        o_begin = wave * args.K;
        if (o_begin >= args.n) return;
        o_end = min<uint64_t>(args.n, o_begin + args.K);
        qw = o_begin * A;
        nslots = o_end * A;
    } else {
        nslots = args.n * A;
        qw = wave * (uint64_t)(C * 64);
        if (qw >= nslots) return;  // no workgroup barrier anywhere: waves are independent
    }

    uint64_t i0;
    uint32_t j0;
    split_slot(qw, A, args.inv_A, i0, j0);
    uint32_t carry = 0;
    for (uint32_t k = 0; k < j0; k += 64) {
        const uint32_t idx = k + (uint32_t)lane;
        const uint32_t v = idx < j0 ? args.attr_len[qw - j0 + idx] : 0u;
        carry += wave_sum_dpp(v);
    }
    const uint64_t last_slot = nslots - 1;
    uint32_t Lraw[C];
#pragma unroll
    for (int c = 0; c < C; ++c) Lraw[c] = args.attr_len[min(qw + c * 64 + lane, last_slot)];
    uint32_t packed_codes = 0;
    if (args.uniform_code == 0xffu) packed_codes = reinterpret_cast<const uint32_t*>(args.codes)[lane];

    // ---- phase 1: descriptors + classes -------------------------------------
    // REGD (unsorted waves only): each lane keeps its C descriptors in
    // registers — pass t's slot t * 64 + lane is the lane's own chunk-t slot
    static_assert(!REGD || (!SORT && !REG), "register descriptors need slot-order passes");
    // DEFER (slot-order passes with direct stores only): the string slots are
    // queued (perm) in phase 1 and hashed together in their own passes — 1
    // string before the numeric passes, the first numeric pass's loads in
    // flight; 2 after them — so a numeric pass no longer runs a string regime
    // for the few key lanes among its numerics (config 2: 13 of 64).
    static_assert(DEFER == 0 || (!SORT && DIRECT && !REG && !REGD && !QUAD && LATE == 0),
                  "deferred strings need slot-order passes with direct stores");
    uint32_t nq = 0;  // wave-uniform: queued string slots
    SlotDesc dreg[REGD ? C : 1];
    uint32_t cls[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t t = j0 + (uint32_t)(c * 64 + lane);
        const uint32_t di = div_small(t, args.a_magic);  // t < A + 64 * C
        const uint32_t j = t - di * A;
        const bool valid = qw + c * 64 + lane < nslots;
        const uint64_t il = valid ? i0 + di : i0;
        const uint64_t base = args.obj_base[il];
        const uint32_t L = valid ? Lraw[c] : 0u;
        const uint32_t Sx = wave_scan_dpp(L) - L;
        const int head = lane - (int)j;
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
        carry = __builtin_amdgcn_readlane(off + L, 63);
        uint32_t code = args.uniform_code != 0xffu
                            ? args.uniform_code
                            : (__shfl(packed_codes, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
        if (!valid) code = CODE_ZERO;
        SlotDesc d;
        d.p = args.blob + base + off;
        d.n = L;
        d.code_slot = code | ((uint32_t)(c * 64 + lane) << 8);
        if constexpr (REGD) dreg[c] = d;
        else desc[c * 64 + lane] = d;
        cls[c] = work_class<ORDER>(code, L, valid);
        if constexpr (DEFER != 0) {
            const bool def = code == CODE_STRING;  // slots past the end are CODE_ZERO
            const uint64_t m = __ballot(def);
            if (def)
                perm[nq + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                    (uint16_t)(c * 64 + lane);
            nq += (uint32_t)__popcll(m);
        }
    }

    // ---- counting sort by class (wave-local) ---------------------------------
    const uint32_t c00 = __builtin_amdgcn_readfirstlane(cls[0]);
    bool uniform = true;
#pragma unroll
    for (int c = 0; c < C; ++c) uniform &= __all(cls[c] == c00);
    if (!SORT) uniform = true;
    if (!uniform) {
        if constexpr (ASORT) {
            // LDS fetch-add counting sort: per-class counts, an exclusive scan
            // into cursors (lane k holds class k), one fetch-add per slot
            uint32_t* cnt = lds.cnt[w];
            if (lane < kClasses) cnt[lane] = 0;
#pragma unroll
            for (int c = 0; c < C; ++c)
                __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            const uint32_t k = lane < kClasses ? cnt[lane] : 0u;
            const uint32_t start = wave_scan_dpp(k) - k;
            if (lane < kClasses) cnt[lane] = start;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint32_t pos = __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WAVEFRONT);
                perm[pos] = (uint16_t)(c * 64 + lane);
            }
        } else {
            uint32_t before = 0;  // slots of lower classes, then of this class in lower chunks
#pragma unroll
            for (int k = 0; k < kClasses; ++k) {
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const uint64_t m = __ballot(cls[c] == (uint32_t)k);
                    if (cls[c] == (uint32_t)k) {
                        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        perm[before + rank] = (uint16_t)(c * 64 + lane);
                    }
                    before += (uint32_t)__popcll(m);
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- phase 2: C class-homogeneous passes, next pass in flight ------------
    // A slot's coordinate overwrites the first 8 bytes of its own descriptor,
    // which exactly one lane has already read (each slot is in one pass).
    struct Pass {
        SlotDesc d;
        Raw blk;
    };
    auto load_pass = [&](int t, Pass& P) {
        const uint32_t s = uniform ? (uint32_t)(t * 64 + lane) : perm[t * 64 + lane];
        if constexpr (REGD) P.d = dreg[t];
        else P.d = desc[s];
        if constexpr (LATE != 0) {  // LATE 1: > 64-byte strings load their head with their first
            // block; LATE 2: only the one-block strings (65..128 bytes)
            const bool g64 = (P.d.code_slot & 0xffu) == CODE_STRING && P.d.n > 64 && (LATE == 1 || P.d.n <= 128);
            P.blk = issue_any<A4>(g64 ? (uint32_t)CODE_ZERO : P.d.code_slot & 0xffu, P.d.p, g64 ? 0u : P.d.n);
        } else if constexpr (DEFER != 0) {  // a queued string loads nothing here
            const bool def = (P.d.code_slot & 0xffu) == CODE_STRING;
            P.blk = issue_any<A4>(def ? (uint32_t)CODE_ZERO : P.d.code_slot & 0xffu, P.d.p, def ? 0u : P.d.n);
        } else {
            P.blk = issue_any<A4>(P.d.code_slot & 0xffu, P.d.p, P.d.n);
        }
    };
    bool bad = false;
    // the queued strings: one lane per string, every lane in the same regimes
    auto string_passes = [&]() {
        for (uint32_t b0 = 0; b0 < nq; b0 += 64) {
            const bool act = b0 + (uint32_t)lane < nq;
            const uint32_t s = act ? perm[b0 + lane] : 0u;
            const SlotDesc d = desc[s];
            const uint32_t code = act ? (uint32_t)CODE_STRING : (uint32_t)CODE_ZERO;
            const uint32_t n = act ? d.n : 0u;
            const Raw r = issue_any<A4>(code, d.p, n);
            const uint64_t h = hash_blk<PIPE, false, A4>(code, d.p, n, consume_any<A4>(r), bad);
            if (act) {
                if (NT_STORE) __builtin_nontemporal_store(h, args.coords + qw + s);
                else args.coords[qw + s] = h;
            }
        }
    };
    Pass P0, P1;
    load_pass(0, P0);
    if constexpr (DEFER == 1) string_passes();  // pass 0's numerics in flight meanwhile
#pragma unroll
    for (int t = 0; t < C; ++t) {
        Pass& cur = (t & 1) ? P1 : P0;
        Pass& nxt = (t & 1) ? P0 : P1;
        if (t + 1 < C) load_pass(t + 1, nxt);
        uint64_t h;
        if constexpr (LATE != 0) {
            static_assert(A4 && !PIPE, "the late head follows the A4 piece layout");
            const uint32_t cd = cur.d.code_slot & 0xffu;
            h = cd == CODE_STRING && cur.d.n > 64 && (LATE == 1 || cur.d.n <= 128) ? city_gt64_late(cur.d.p, cur.d.n)
                                                   : hash_blk<false, false, true>(cd, cur.d.p, cur.d.n,
                                                                                 consume_any<true>(cur.blk), bad);
        } else if constexpr (QUAD) {
            static_assert(A4, "the quad-cooperative loop follows the A4 piece layout");
            h = hash_blk_quad(cur.d.code_slot & 0xffu, cur.d.p, cur.d.n, consume_any<A4>(cur.blk), bad);
        } else if constexpr (DEFER != 0) {  // a queued string is hashed in its own pass
            const uint32_t cd = cur.d.code_slot & 0xffu;
            h = cd == CODE_STRING ? 0ull : hash_blk_nonstring<A4>(cd, cur.d.p, cur.d.n, consume_any<A4>(cur.blk), bad);
        } else {
            h = hash_blk<PIPE, false, A4>(cur.d.code_slot & 0xffu, cur.d.p, cur.d.n, consume_any<A4>(cur.blk), bad);
        }
        if (DIRECT && uniform && !REG) {  // pass t is chunk t in slot order: store straight to HBM
            const uint64_t q = qw + t * 64 + lane;
            if (q < nslots && !(DEFER != 0 && (cur.d.code_slot & 0xffu) == CODE_STRING)) {
                if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q);
                else args.coords[q] = h;
            }
        } else {
            res[2 * (cur.d.code_slot >> 8)] = h;
        }
    }
    if constexpr (DEFER == 2) string_passes();
    if (DIRECT && uniform && !REG) {
        if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    if constexpr (REG) {
        // ---- phase 2b: lookup_region, one lane per object --------------------
        // UNI: the tables in a wave-uniform loop (a table's fields are scalar
        // loads, its attrs uniform LDS offsets); else one lane per (table,
        // object) pair, each lane reading its own table's fields.
        const uint32_t K = args.K, nobj = (uint32_t)(o_end - o_begin);
        auto lookup_one = [&](const SweepTable& tb, uint32_t o) {
            const uint64_t* po = res + 2ull * o * A;
            const auto coord = [&](uint32_t d) { return po[2 * tb.attrs[d]]; };
            uint64_t id;
            if (tb.lds_index != 0xffffffffu) {
                id = lookup_indexed_fn(tbl + tb.lds_index, tb.W, tb.D, coord, tbl + tb.lds_ids);
            } else if (tb.index) {
                id = lookup_indexed_fn(tb.index, tb.W, tb.D, coord, tb.ids);
            } else {
                uint64_t h[kMaxLookupDims];
#pragma unroll
                for (uint32_t d = 0; d < kMaxLookupDims; ++d)
                    if (d < tb.D) h[d] = coord(d);
                id = lookup_scan(tb.lower, tb.upper, tb.ids, tb.R, tb.D, h);
            }
            tb.out[o_begin + o] = id;
        };
        if constexpr (UNI) {
            for (uint32_t t = 0; t < args.T; ++t)
                for (uint32_t o = lane; o < nobj; o += 64) lookup_one(args.t[t], o);
        } else {
            for (uint32_t k = lane; k < args.T * K; k += 64) {
                const uint32_t t = k / K, o = k - t * K;
                if (o < nobj) lookup_one(args.t[t], o);
            }
        }
        if (!args.coords) {
            if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
            return;
        }
    }

    // ---- phase 3: coalesced stores in slot order -----------------------------
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint64_t q = qw + c * 64 + lane;
        if (q < nslots) {
            const uint64_t h = res[2 * (c * 64 + lane)];
            if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q);
            else args.coords[q] = h;
        }
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// WPB: waves per workgroup (each with its own LDS; the workgroup keeps it all
// until its last wave ends).
template <int C, bool NT_STORE, bool SORT = true, bool DIRECT = true, bool A4 = false, bool PIPE = false,
          bool ASORT = false, int ORDER = 0, int WPB = 4>
__global__ void __launch_bounds__(64 * WPB)
hash_regroup_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C, WPB> lds;
    regroup_body<C, NT_STORE, SORT, DIRECT, A4, PIPE, ASORT, ORDER, false>(args, lds, nullptr);
}

// The regroup kernel with the string slots deferred to passes of their own
// (DEFER 1: first, 2: last; slot-order passes, direct stores).
template <int C, bool NT_STORE, bool A4, int DEFER, int WPB = 1>
__global__ void __launch_bounds__(64 * WPB)
hash_regroup_defer_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C, WPB> lds;
    regroup_body<C, NT_STORE, false, true, A4, false, false, 0, false, false, false, false, 0, DEFER>(args, lds,
                                                                                                   nullptr);
}

// hash + lookup_region in one launch (hdx_hash_batch_regions_device).  The
// workgroup first copies the indexed tables that fit into LDS (its only
// barrier, before any wave may leave).
template <int C, bool SORT, bool A4, bool ASORT, int ORDER, bool UNI>
__global__ void __launch_bounds__(256)
hash_regroup_regions_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C> lds;
    extern __shared__ __attribute__((aligned(16))) uint64_t tbl[];
    if (args.lds_tables) {
        for (uint32_t t = 0; t < args.T; ++t) {
            const SweepTable& tb = args.t[t];
            if (tb.lds_index == 0xffffffffu) continue;
            for (uint32_t k = threadIdx.x; k < tb.index_words; k += blockDim.x) tbl[tb.lds_index + k] = tb.index[k];
            for (uint32_t k = threadIdx.x; k < tb.R; k += blockDim.x) tbl[tb.lds_ids + k] = tb.ids[k];
        }
        __syncthreads();
    }
    regroup_body<C, true, SORT, true, A4, false, ASORT, ORDER, true, UNI>(args, lds, tbl);
}

template <int C, bool NT, bool SORT = true, bool DIRECT = true, bool A4 = false, bool PIPE = false,
          bool ASORT = false, int ORDER = 0, int WPB = 4>
inline hipError_t launch_regroup(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + WPB - 1) / WPB;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_kernel<C, NT, SORT, DIRECT, A4, PIPE, ASORT, ORDER, WPB>), dim3((uint32_t)blocks),
                       dim3(64 * WPB), 0, stream, args);
    return hipGetLastError();
}

template <int C, bool NT, bool A4, int DEFER, int WPB = 1>
inline hipError_t launch_regroup_defer(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + WPB - 1) / WPB;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_defer_kernel<C, NT, A4, DEFER, WPB>), dim3((uint32_t)blocks), dim3(64 * WPB), 0,
                       stream, args);
    return hipGetLastError();
}

template <bool NT, bool PIPE = false, int SHAPE = 0, bool A4 = false, int WPB = 4>
inline hipError_t launch_chunk(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + 63) / 64;
    const uint64_t blocks = (waves + WPB - 1) / WPB;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_chunk_kernel<NT, PIPE, SHAPE, A4>), dim3((uint32_t)blocks), dim3(64 * WPB), 0, stream, args);
    return hipGetLastError();
}

template <int C, bool SORT, bool A4, bool ASORT, int ORDER, bool UNI = false>
inline hipError_t launch_regroup_regions(BatchArgs args, hipStream_t stream, bool lds_ok = true) {
    // stage indexed tables in LDS while they fit in 16 KiB together and the
    // workgroup's LDS stays within 80 KiB (two workgroups per CU)
    uint32_t words = 0;
    const bool room = lds_ok && sizeof(RegroupLds<C>) + 16384 <= 81920;
    for (uint32_t t = 0; t < args.T; ++t) {
        SweepTable& tb = args.t[t];
        tb.lds_index = tb.lds_ids = 0xffffffffu;
        const uint32_t need = tb.index_words + tb.R;
        if (room && tb.index && (words + need) * 8 <= 16384) {
            tb.lds_index = words;
            tb.lds_ids = words + tb.index_words;
            words += (need + 1) & ~1u;
        }
    }
    args.lds_tables = words;
    args.K = (C * 64) / args.A;
    if (args.K == 0) return hipErrorInvalidValue;
    const uint64_t waves = (args.n + args.K - 1) / args.K;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_regions_kernel<C, SORT, A4, ASORT, ORDER, UNI>), dim3((uint32_t)blocks), dim3(256),
                       (size_t)words * 8, stream, args);
    return hipGetLastError();
}

}  // namespace hdx
