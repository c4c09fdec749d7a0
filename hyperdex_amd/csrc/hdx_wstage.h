// hdx_wstage.h — wave-staged batch hash for mixed variable-length schemas
// (config 3b's shape: strings of every CityHash regime beside int64/float).
//
// hdx_hash_batch_device's contract (include/hdxhash.h): coords[i*A + j] =
// hs[j] of hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68).
//
// Why this shape.  The gather kernels load every
// slot's bytes with per-lane 16-byte loads, one value per lane: each load
// instruction touches ~64 cache lines, and strings over 64 bytes (the CityHash
// loop) stream at ~4 TB/s even with no hash arithmetic (tools/lwbench.hip,
// profiles/r3/lwbench.jsonl: 4.05 TB/s lane-per-string on 65..195-byte
// strings).  Here one wave owns K whole objects, which a packed batch stores
// back to back: their bytes are one span, copied into a wave-private LDS window
// by coalesced LDS DMA (global_load_lds_dwordx4, 1 KiB per instruction), which
// streams at ~5.4 TB/s in the same probe.  Per wave:
//   1. the K object bases (+ the next group's first, so the DMA of
//      [base[o0], base[o0 + K]) goes out before the lengths are back) and the
//      K*A lengths, coalesced;
//   2. per-slot in-object offsets by a DPP prefix scan, object sizes, a check
//      that the objects are back to back and fit the window;
//   3. a wave-local counting sort of the slots by work class (ORDER 1 of
//      hdx_regroup.h: numerics, 33..64 B, <= 16 B, 17..32 B, > 64 B by loop
//      blocks), so a pass of 64 lanes runs few CityHash regimes;
//   4. s_waitcnt vmcnt(0) (the compiler does not order ds_read behind an LDS
//      DMA), then NCH passes hashing from LDS (hdx_lds_hash.h: dword reads +
//      v_alignbyte, the A4 arithmetic), each coordinate parked over its
//      consumed descriptor;
//   5. one coalesced non-temporal store of the K*A coordinates.
// A group whose objects are not back to back or do not fit the window is
// hashed from global memory instead (the A4 loads of hdx_loads.h), so every
// layout gives the reference's coordinates.  Four waves per workgroup, each
// with its own window: no workgroup barrier.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>

#include "hdx_lds_hash.h"
#include "hdx_region_lookup.h"
#include "hdx_regroup.h"

namespace hdx {
namespace {

typedef __attribute__((address_space(3))) void* lds_void_t;

template <int NCH, int WPB = 4, bool RD = false>
struct WStageMeta {
    uint64_t desc[WPB][NCH * 64];  // {offset u32, length u32}; then the slot's parked coordinate
    uint16_t perm[WPB][NCH * 64];  // slot | code << 8, in class order
    uint32_t cnt[WPB][kClasses];
};
// RD (descriptors in registers): no desc array
template <int NCH, int WPB>
struct WStageMeta<NCH, WPB, true> {
    uint16_t perm[WPB][NCH * 64];
    uint32_t cnt[WPB][kClasses];
    uint64_t desc[WPB][1];  // unused
};

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return pack64(__builtin_amdgcn_readlane((uint32_t)v, l), __builtin_amdgcn_readlane((uint32_t)(v >> 32), l));
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int l) {
    return pack64((uint32_t)__shfl((int)(uint32_t)v, l, 64), (uint32_t)__shfl((int)(uint32_t)(v >> 32), l, 64));
}
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

// One wave's group: K = args.K consecutive objects from o0, their bases,
// lengths, codes and work classes, and (staged) their span in `win`.
template <int NCH>
struct Group {
    uint64_t q0, mybase;
    uint32_t nobj, ns;
    bool staged;
    uint32_t L[NCH], code[NCH], cls[NCH];
    uint32_t doff[NCH];  // the slot's descriptor offset (desc[s]'s low word)
};

// Phases 1-3a: bases and lengths, the span's DMA into win (early when the
// next group's first object bounds it), in-object offsets, object sizes, the
// staged decision, and every slot's descriptor desc[s] = {offset, length}:
// the offset in `win` + win_off when staged, else in the object.  SHAPE 2
// (debug) skips the DMA.
// ADMA: the DMA as inline asm (dma_x4_asm), the code table loaded with the
// bases and lengths and waited for before the DMA goes out — nothing in
// phases 2-3 then waits for the DMA.
// NT: the bases, lengths and span loaded non-temporal (read once).
// PLAN: slot s's object, attribute and code from args.plan (the launcher's
// per-schema table) instead of a division and a code-table shuffle.
template <int NCH, uint32_t WB, int SHAPE, int ORDER = 1, bool ADMA = false, bool DL = false, bool NT = false,
          bool PLAN = false>
__device__ __forceinline__ Group<NCH> describe_group(const BatchArgs& args, uint64_t o0, uint8_t* win, uint32_t win_off,
                                                     uint64_t* desc) {
    const int lane = threadIdx.x & 63;
    const uint32_t A = args.A, K = args.K;
    Group<NCH> g;
    g.nobj = (uint32_t)min<uint64_t>(K, args.n - o0);
    g.ns = g.nobj * A;
    g.q0 = o0 * A;

    // ---- bases (lane nobj: the next group's first object) and lengths ------
    const bool has_next = o0 + K < args.n;
    const uint32_t nbase = g.nobj + (has_next ? 1u : 0u);
    const uint64_t mybase =
        (uint32_t)lane < nbase ? (NT ? __builtin_nontemporal_load(args.obj_base + o0 + lane) : args.obj_base[o0 + lane]) : 0;
    g.mybase = mybase;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        g.L[c] = s < g.ns ? (NT ? __builtin_nontemporal_load(args.attr_len + g.q0 + s) : args.attr_len[g.q0 + s]) : 0u;
    }
    uint32_t packed_codes = 0;
    uint32_t pw[NCH];
    if constexpr (PLAN) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) pw[c] = args.plan[c * 64 + lane];
        if constexpr (ADMA) {
#pragma unroll
            for (int c = 0; c < NCH; ++c) asm volatile("" ::"v"(pw[c]));  // loaded before the DMA is issued
        }
    } else if constexpr (ADMA) {
        packed_codes = reinterpret_cast<const uint32_t*>(args.codes)[lane];
        asm volatile("" ::"v"(packed_codes));  // its load completes before the DMA is issued
    }
    const uint64_t b0 = readlane64(mybase, 0);
    const uint64_t bnext = has_next ? readlane64(mybase, (int)g.nobj) : 0;
    const uint32_t lead = (uint32_t)((uintptr_t)(args.blob + b0) & 15);
    const uint8_t* s16 = args.blob + b0 - lead;
    // units 16-byte units from s16 -> win (units <= WB / 16); lanes past the
    // span write nothing: the window need not be whole KiB
    auto dma = [&](uint32_t units) {
        if constexpr (DL) dma_units16_loop<ADMA>(s16, win, units);
        else dma_units16<ADMA, NT>(s16, win, units);
    };
    // the span up to the next group's first object, before the lengths are back
    const bool early = has_next && bnext > b0 && lead + (bnext - b0) <= WB;
    if (early && SHAPE != 2) dma((lead + (uint32_t)(bnext - b0) + 15) >> 4);

    // ---- in-object offsets, codes, object sizes ----------------------------
    if constexpr (!ADMA && !PLAN) packed_codes = reinterpret_cast<const uint32_t*>(args.codes)[lane];
    uint32_t off[NCH], endv[NCH], obj[NCH];
    uint32_t carry = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        const uint32_t o = PLAN ? (pw[c] >> 8) & 0xffu : div_small(s, args.a_magic);
        const uint32_t j = PLAN ? pw[c] & 0xffu : s - o * A;
        obj[c] = o;
        const uint32_t Sx = wave_scan_dpp(g.L[c]) - g.L[c];
        const int head = lane - (int)j;
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        off[c] = head >= 0 ? Sx - head_sx : carry + Sx;
        carry = __builtin_amdgcn_readlane(off[c] + g.L[c], 63);
        const uint32_t cd = PLAN                          ? pw[c] >> 16
                            : args.uniform_code != 0xffu ? args.uniform_code
                                                         : (__shfl(packed_codes, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
        g.code[c] = s < g.ns ? cd : (uint32_t)CODE_ZERO;
        endv[c] = off[c] + g.L[c];
    }
    // lane o < nobj: its object's size = the end of its last attribute
    const uint32_t last_slot = (uint32_t)lane * A + A - 1;
    uint32_t mysize = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t v = (uint32_t)__shfl((int)endv[c], (int)(last_slot & 63), 64);
        if ((last_slot >> 6) == (uint32_t)c) mysize = v;
    }
    const uint64_t nextb = shfl64(mybase, (lane + 1) & 63);
    const bool runs = __all((uint32_t)lane >= g.nobj || (uint32_t)lane + 1 >= nbase || mybase + mysize == nextb);
    const uint64_t bend = readlane64(mybase + mysize, (int)g.nobj - 1);
    g.staged = runs && bend >= b0 && lead + (bend - b0) <= WB;
    if (g.staged && !early && SHAPE != 2) dma((lead + (uint32_t)(bend - b0) + 15) >> 4);  // the batch's last group
    const uint32_t rel = (uint32_t)(mybase - b0) + lead + win_off;  // lane o: its object's window offset (staged)

    // ---- descriptors and work classes ----------------------------------------
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        const uint32_t o = obj[c];
        const uint32_t orel = (uint32_t)__shfl((int)rel, (int)(o & 63), 64);
        const uint32_t doff = g.staged ? orel + off[c] : off[c];
        g.doff[c] = doff;
        if (desc) desc[s] = (uint64_t)doff | ((uint64_t)g.L[c] << 32);
        g.cls[c] = ORDER == 3   ? work_class3(g.code[c], g.L[c], s < g.ns)
                   : ORDER == 4 ? work_class1_bf(g.code[c], g.L[c], s < g.ns)
                   : ORDER == 5 ? work_class1_tab(g.code[c], g.L[c], s < g.ns)
                                : work_class<1>(g.code[c], g.L[c], s < g.ns);
    }
    return g;
}

// One slot: staged from the LDS window lw (desc offset), else from global
// memory at its object's base (lane o of mybase).  SHAPE 1 (debug): one LDS
// dword instead of the hash.
// HT: staged slots hashed by hash_slot_window (first / last 32 bytes, every
// regime from the same two reads; lw then points kFrontHT bytes before the
// window); HT 2 / 3: hash_slot_window's LOOP 2 / 3; HT 5: LOOP 2 with TNUM;
// HT 6: LOOP 4 with TNUM.
constexpr uint32_t kFrontHT = 32;
template <int SHAPE, int HT = 0, int W128 = 0, bool NUM2 = false>
__device__ __forceinline__ uint64_t hash_slot(const BatchArgs& args, ldsw_t lw, bool staged, uint64_t mybase,
                                              uint32_t s, uint32_t cd, uint64_t d, bool& bad) {
    const uint32_t doff = (uint32_t)d, dn = (uint32_t)(d >> 32);
    if (SHAPE == 1) return lw[doff >> 2] ^ dn;
    if (staged && HT)
        return hash_slot_window<W128, (HT == 6 ? 4 : HT >= 5 ? 2 : HT > 1 ? HT : 1), (HT >= 5), NUM2 && HT >= 5>(lw, cd, doff + kFrontHT,
                                                                                                  dn, bad);
    if (staged) return cd == CODE_STRING ? hash_string_lds(lw, doff, dn) : hash_numeric_lds(lw, cd, doff, dn, bad);
    const uint32_t o = div_small(s, args.a_magic);
    const uint64_t ob = shfl64(mybase, (int)(o & 63));
    const uint8_t* p = args.blob + ob + doff;
    return hash_blk<false, false, true>(cd, p, dn, consume_any<true>(issue_any<true>(cd, p, dn)), bad);
}

// NCH passes of 64 slots: K = min(floor(64 * NCH / A), KCAP, 63) objects per
// wave; WB-byte windows.  SHAPE (debug variants 207/208 only, WRONG
// coordinates): 1 = everything but the hash (one LDS dword per slot instead);
// 2 = no DMA (the hash runs on whatever the window holds).
// REGIONS (hdx_hash_batch_regions_device): the wave's objects are then looked
// up in the args.T region tables from their coordinates parked in LDS
// (lookup_tables_wave), coordinates stored only when args.coords is set.
// GAP: the class straddling the pass boundary moves whole into the second
// pass when pads allow (class_sort, hdx_regroup.h).  DL (debug): round 3's
// span copy, addresses and predicate per KiB (dma_units16_loop).  WPB: waves
// (each with its own window) per workgroup.  NT: the lengths, bases and span
// loaded non-temporal (read once).
// PLAN: the slot plan (describe_group); NUM2: numerics by selects, the
// schema holds strings, int64 and floats only (the launcher checks).
template <int NCH, uint32_t WB, int SHAPE = 0, int HT = 0, int ORDER = 1, int W128 = 0, bool REGIONS = false,
          bool GAP = false, bool ADMA = false, bool PU = true, bool DL = false, int WPB = 4, bool XS = false,
          bool RD = false, bool NT = false, int PRIO = 0, bool PLAN = false, bool NUM2 = false>
__global__ void __launch_bounds__(64 * WPB)
hash_wstage_kernel(const BatchArgs args) {
    // PRIO 1 (the product since round 5): the load phase at high wave
    // priority, the passes at low.  The schedules that lost (the reverse, the
    // stores high, the sort medium: profiles/r5/ab_priority.jsonl) are gone.
    static_assert(PRIO == 0 || PRIO == 1, "PRIO: 0 none, 1 loads high");
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(3);
    static_assert(NCH >= 1 && NCH <= 4 && WB % 16 == 0, "slot indices are 8 bits; windows whole DMA units");
    static_assert(!(RD && REGIONS), "the fused lookups read the coordinates parked in desc");
    constexpr uint32_t FRONT = HT ? kFrontHT : 0;
    // +64: dword over-reads past the span; HT: 32 bytes before it (short strings' tail reads)
    __shared__ __attribute__((aligned(16))) uint8_t win_all[WPB][FRONT + WB + 64];
    __shared__ WStageMeta<NCH, WPB, RD> meta;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    uint8_t* win = win_all[w] + FRONT;
    uint64_t* desc = RD ? nullptr : meta.desc[w];
    uint16_t* perm = meta.perm[w];
    uint32_t* cnt = meta.cnt[w];
    const ldsw_t lw = as_ldsw(win_all[w]);

    const uint64_t o0 = ((uint64_t)(XS ? xcd_block() : blockIdx.x) * WPB + w) * args.K;
    if (o0 >= args.n) return;  // no barrier anywhere: waves are independent
    const Group<NCH> g = describe_group<NCH, WB, SHAPE, ORDER, ADMA, DL, NT, PLAN>(args, o0, win, 0, desc);

    // ---- counting sort by work class (wave-local) --------------------------
    uint32_t pos[NCH];
    class_sort<NCH, GAP>(cnt, perm, g.cls, g.code, g.ns, wave_lds_fence, RD ? pos : nullptr);
    // every LDS-DMA of this wave must have landed before the window is read
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(0);

    if constexpr (RD) {
        // RD: descriptors and coordinates stay in registers.  Pass t's lane
        // reads its slot s's descriptor from lane s % 64's registers (set
        // s / 64) by ds_bpermute, and a coordinate goes back to its slot's
        // lane the same way (from the lane and pass its position in perm
        // names) — no desc array in LDS: 1 KiB less per wave.
        bool bad = false;
        uint64_t res[NCH];
#pragma unroll(PU ? NCH : 1)
        for (int t = 0; t < NCH; ++t) {
            const uint32_t e = perm[t * 64 + lane];
            const uint32_t s = e & 0xffu, src = s & 63u, set = s >> 6;
            uint32_t doff = 0, ln = 0;
#pragma unroll
            for (int c = 0; c < NCH; ++c) {
                const uint32_t d = (uint32_t)__shfl((int)g.doff[c], (int)src, 64);
                const uint32_t l = (uint32_t)__shfl((int)g.L[c], (int)src, 64);
                if (set == (uint32_t)c) {
                    doff = d;
                    ln = l;
                }
            }
            res[t] = hash_slot<SHAPE, HT, W128, NUM2>(args, lw, g.staged, g.mybase, s, e >> 8,
                                                (uint64_t)doff | ((uint64_t)ln << 32), bad);
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t p = pos[c], src = p & 63u, pass = p >> 6;
            uint64_t v = 0;
#pragma unroll
            for (int t = 0; t < NCH; ++t) {
                const uint64_t x = shfl64(res[t], (int)src);
                if (pass == (uint32_t)t) v = x;
            }
            const uint32_t s = (uint32_t)(c * 64 + lane);
            if (s < g.ns) __builtin_nontemporal_store(v, args.coords + g.q0 + s);
        }
        if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
        return;
    }

    // ---- NCH class-sorted passes, coordinates parked over their descriptors ---
    bool bad = false;
    // PU 0: the pass loop not unrolled (one copy of the hash code instead of NCH)
#pragma unroll(PU ? NCH : 1)
    for (int t = 0; t < NCH; ++t) {
        const uint32_t e = perm[t * 64 + lane];
        const uint32_t s = e & 0xffu;
        // (round 6: storing it straight to HBM from the pass instead, 64
        // scattered 8-byte stores per pass, measured 2.69 vs 2.44 ms)
        desc[s] = hash_slot<SHAPE, HT, W128, NUM2>(args, lw, g.staged, g.mybase, s, e >> 8, desc[s], bad);
    }
    wave_lds_fence();

    // ---- coalesced stores in slot order ------------------------------------
    if (!REGIONS || args.coords) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t s = (uint32_t)(c * 64 + lane);
            if (s < g.ns) __builtin_nontemporal_store(desc[s], args.coords + g.q0 + s);
        }
    }
    if constexpr (REGIONS)  // the window is free now: the lookups' scratch
        lookup_tables_wave(args.t, args.T, desc, args.A, g.nobj, o0, reinterpret_cast<uint64_t*>(win), wave_lds_fence);
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// Launch: K = floor(64 * NCH / A) whole objects per wave (at most 63), four
// independent waves per 256-thread workgroup, no workgroup barrier.
// The slot plan of BatchArgs::plan for K objects of A attributes.
inline void fill_wave_plan(BatchArgs& args) {
    for (uint32_t s = 0; s < kWavePlanSlots; ++s) {
        const uint32_t o = s / args.A, j = s % args.A;
        const uint32_t code = o < args.K ? args.codes[j] : (uint32_t)CODE_ZERO;
        args.plan[s] = (j & 0xffu) | (o & 0xffu) << 8 | code << 16;
    }
}
// Codes the NUM2 kernels handle: strings, int64 and floats.
inline bool num2_schema(const BatchArgs& args) {
    for (uint32_t j = 0; j < args.A && j < kKernargCodes; ++j)
        if (args.codes[j] != CODE_STRING && args.codes[j] != CODE_INT64 && args.codes[j] != CODE_FLOAT) return false;
    return args.A <= kKernargCodes;
}

template <int NCH, uint32_t WB, uint32_t KCAP = 63, int SHAPE = 0, int HT = 0, int ORDER = 1, int W128 = 0,
          bool REGIONS = false, bool GAP = false, bool ADMA = false, bool PU = true, bool DL = false, int WPB = 4,
          bool XS = false, bool RD = false, bool NT = false, int PRIO = 0, bool PLAN = false, bool NUM2 = false>
static hipError_t launch_wstage_t(BatchArgs args, hipStream_t stream) {
    // lane o holds object o's base and lane K the next group's first: K <= 63
    args.K = std::min<uint32_t>(std::min<uint32_t>((uint32_t)(64 * NCH) / args.A, KCAP), 63u);
    if (args.K == 0) return hipErrorInvalidValue;
    static_assert(!PLAN || NCH * 64 <= kWavePlanSlots, "the plan covers two passes");
    if (PLAN) fill_wave_plan(args);
    if (NUM2 && !num2_schema(args)) return hipErrorInvalidValue;
    const uint64_t waves = (args.n + args.K - 1) / args.K;
    const uint64_t blocks = (waves + WPB - 1) / WPB;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_wstage_kernel<NCH, WB, SHAPE, HT, ORDER, W128, REGIONS, GAP, ADMA, PU, DL, WPB, XS, RD, NT, PRIO,
                                           PLAN, NUM2>),
                       dim3((uint32_t)blocks), dim3(64 * WPB), 0, stream, args);
    return hipGetLastError();
}


}  // namespace hdx
