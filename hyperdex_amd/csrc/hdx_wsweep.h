// hdx_wsweep.h — the wave-staged reindex sweep:
// the kernel template and its launcher, shared by the product instantiation
// (hdx_wsweep.hip) and the A/B forms (hdx_wsweep_dbg.hip, debug library only).
//
// hdx_hash_encoded_device's contract (include/hdxhash.h): value i is
// [u64 BE version][u16 BE count]{[u32 BE len][bytes]}*count
// (daemon/datalayer_encodings.cc:139-166), decoded as decode_value does
// (:168-217) and re-hashed with its key (common/hash.cc:56-68).
//
// Why this shape.  The gather sweep (hdx_encoded.hip)
// walks every value's length prefixes from global memory — a chain of
// dependent loads that touches nearly every line of the value — and then
// gathers the attributes per lane, so the values cross the fabric twice
// (raw FETCH 1.2-1.4x the bytes) and every load instruction touches ~64
// lines.  Here one wave owns K consecutive stored objects, as the wave-staged
// batch kernel (hdx_wstage.h) does:
//   1. the K key and value offsets and lengths (+ the next object's offsets,
//      which bound the spans), coalesced;
//   2. the objects' keys and values — two spans for a packed store — copied
//      into the wave's LDS window by coalesced LDS DMA (keys first, values
//      after; a value span longer than the window is held in part);
//   3. the prefix walk, lane = object, from LDS (from global memory for a
//      value the window does not hold), writing a {window offset, length}
//      descriptor per attribute — the walk costs LDS latency, not HBM round
//      trips;
//   4. the wave's K*A slots counting-sorted by CityHash regime, hashed from
//      the window with head/tail reads (hash_slot_window, hdx_lds_hash.h) in
//      NCH passes, coordinates parked over their descriptors, one coalesced
//      store.
// A slot whose bytes are not in the window (unpacked layouts, the launch's
// last group, an oversized object) is hashed from global memory, sorted into a
// class of its own.  Each byte crosses HBM once.
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
typedef uint32_t __attribute__((aligned(1))) u32_u;
typedef uint64_t __attribute__((aligned(1))) u64_u;
typedef uint16_t __attribute__((aligned(1))) u16_u;

constexpr uint32_t kZero = 0xffffffffu;   // descriptor offset of a slot hashed as 0
constexpr uint32_t kGlobal = 0x80000000u; // descriptor length bit: hashed from global memory
constexpr uint32_t kFrontS = 32, kBackS = 64;

__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
    return pack64(__builtin_amdgcn_readlane((uint32_t)v, l), __builtin_amdgcn_readlane((uint32_t)(v >> 32), l));
}
__device__ __forceinline__ uint64_t sh64(uint64_t v, int l) {
    return pack64((uint32_t)__shfl((int)(uint32_t)v, l, 64), (uint32_t)__shfl((int)(uint32_t)(v >> 32), l, 64));
}
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// big-endian fields at byte p of global memory / at byte offset o of the window
__device__ __forceinline__ uint32_t g_be32(const uint8_t* p) {
    return __builtin_bswap32(*(const __attribute__((address_space(1))) u32_u*)p);
}
__device__ __forceinline__ uint64_t g_be64(const uint8_t* p) {
    return __builtin_bswap64(*(const __attribute__((address_space(1))) u64_u*)p);
}
__device__ __forceinline__ uint32_t g_be16(const uint8_t* p) {
    const uint16_t v = *(const __attribute__((address_space(1))) u16_u*)p;
    return (uint32_t)(uint16_t)((v >> 8) | (v << 8));
}
// The walk's big-endian reads at any byte offset: one misaligned ds_read_b32
// each (gfx950 serves them, replaying the misaligned part; the walk runs on
// 6 of 64 lanes, where that costs little, and saves the dword pair's address
// and v_alignbyte — the hash's 64-lane reads keep the aligned form).  DW: the
// dword pair + v_alignbyte (round 3; debug SHAPE 4).
typedef const __attribute__((address_space(3))) uint32_t __attribute__((aligned(1))) lds_ua32_t;
template <bool DW = false>
__device__ __forceinline__ uint32_t w_be32(ldsw_t w, uint32_t o) {
    if constexpr (DW) return lds_be32(w, o);
    else return __builtin_bswap32(*(lds_ua32_t*)((const __attribute__((address_space(3))) uint8_t*)w + o));
}
template <bool DW = false>
__device__ __forceinline__ uint64_t w_be64(ldsw_t w, uint32_t o) {
    return ((uint64_t)w_be32<DW>(w, o) << 32) | w_be32<DW>(w, o + 4);
}
template <bool DW = false>
__device__ __forceinline__ uint32_t w_be16(ldsw_t w, uint32_t o) { return w_be32<DW>(w, o) >> 16; }

// Sort classes: class 7 = hashed from global memory; > 64-byte strings with
// 3+ blocks share class 6; otherwise work_class<1>'s order (numerics and
// zero slots first).
__device__ __forceinline__ uint32_t sweep_class(uint32_t code, uint32_t n, bool zero, bool global) {
    if (zero) return 0;
    if (global) return 7;
    return std::min<uint32_t>(work_class<1>(code, n, true), 6u);
}
// ... with selects only (BF)
__device__ __forceinline__ uint32_t sweep_class_bf(uint32_t code, uint32_t n, bool zero, bool global) {
    const uint32_t c = std::min<uint32_t>(work_class1_bf(code, n, true), 6u);
    return zero ? 0u : global ? 7u : c;
}

// ... from the class table (work_class1_tab, NUM2 forms)
__device__ __forceinline__ uint32_t sweep_class_tab(uint32_t code, uint32_t n, bool zero, bool global) {
    const uint32_t c = std::min<uint32_t>(work_class1_tab(code, n, true), 6u);
    return zero ? 0u : global ? 7u : c;
}

__device__ __forceinline__ uint64_t hash_global(const uint8_t* p, uint32_t code, uint32_t n, bool& bad) {
    return hash_blk<false, false, true>(code, p, n, consume_any<true>(issue_any<true>(code, p, n)), bad);
}

// lane 0's offset (the group's first object)
__device__ __forceinline__ uint64_t k0_of(uint64_t off) { return rl64(off, 0); }

// copy [src, src + bytes) (src 16-byte aligned) to LDS dst: whole 16-byte
// units by LDS DMA, the last partial unit as dwords (a dword never crosses a
// page, so nothing past the span's last dword is read); ASM: inline-asm DMA
// (hdx_lds_hash.h; debug form 13 only — the sweep drains its copies right
// after issuing them, and the builtin measured faster)
template <bool ASM = false>
__device__ __forceinline__ void dma16(const void* src, void* dst) {
    if constexpr (ASM) dma_x4_asm(src, dst);
    else __builtin_amdgcn_global_load_lds(src, (lds_void_t)dst, 16, 0, 0);
}
template <bool ASM = false>
__device__ __forceinline__ void dma4(const void* src, void* dst) {
    if constexpr (ASM) dma_x1_asm(src, dst);
    else __builtin_amdgcn_global_load_lds(src, (lds_void_t)dst, 4, 0, 0);
}
template <bool ASM = false, bool DL = false>
__device__ __forceinline__ void copy_span(const uint8_t* src, uint8_t* dst, uint32_t bytes, int lane) {
    const uint32_t units = bytes >> 4;
    if constexpr (DL) dma_units16_loop<ASM>(src, dst, units);
    else dma_units16<ASM>(src, dst, units);
    const uint32_t tdw = ((bytes & 15) + 3) >> 2;
    if ((uint32_t)lane < tdw) dma4<ASM>(src + 16ull * units + 4 * lane, dst + 16 * units);
}

}  // namespace

// NCH passes of 64 slots; K = min(64 * NCH / A, KCAP) objects per wave; a
// WB-byte window per wave, four waves per workgroup, no workgroup barrier.
// REGIONS (hdx_hash_encoded_regions_device): every object is then looked up
// in the a.T region tables (configuration::lookup_region, hdx_region_lookup.h:
// the interval index, or the scan), lane = object, from the coordinates
// parked in LDS; coordinates are stored only when a.coords is set.
// GAP: the class straddling the pass boundary moves whole into the second
// pass when pads allow (class_sort, hdx_regroup.h).
// LOOP: hash_slot_window's; + 10: with TNUM.
// SHAPE (debug forms 7 / 8 / 19, WRONG coordinates): 3 = no copy and no walk,
// the hash on made-up descriptors (the compute alone); 1 = no hash (a slot's
// coordinate is its descriptor), 2 = no hash and no walk.  SHAPE 4 (debug
// form 22, correct coordinates): the walk's reads as round 3's dword pairs.
// NUM2 (round 6): a schema of strings, int64 and floats only — numerics by
// selects (hash_slot_window NUM2) and the class from the table.
template <int NCH, uint32_t WB, uint32_t KCAP, bool REGIONS = false, bool GAP = false, int SHAPE = 0, int LOOP = 1,
          bool ASM = false, bool PU = true, bool BF = false, bool RECS = true, bool KUNITS = true, bool DL = false,
          int WPB = 4, bool XS = false, int PRIO = 0, bool NUM2 = false>
__global__ void __launch_bounds__(64 * WPB)
hash_sweep_wstage_kernel(const EncodedArgs a) {
    // PRIO 4 (the product since round 5): loads high, the walk and the sort
    // medium, the passes low; the schedules that lost are gone
    // (profiles/r5/ab_priority.jsonl)
    static_assert(PRIO == 0 || PRIO == 4, "PRIO: 0 none, 4 the product's schedule");
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(3);
    constexpr uint32_t SL = NCH * 64;
    __shared__ __attribute__((aligned(16))) uint8_t win_all[WPB][kFrontS + WB + kBackS];
    __shared__ uint64_t desc_all[WPB][SL];   // {offset, length | kGlobal}; then the parked coordinate
    __shared__ uint16_t perm_all[WPB][SL];   // slot | code << 8, in class order
    __shared__ uint32_t cnt_all[WPB][kClasses];
    __shared__ __attribute__((aligned(4))) uint8_t codes_all[WPB][SL];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    uint8_t* win = win_all[w];
    const ldsw_t lw = as_ldsw(win);
    uint64_t* desc = desc_all[w];
    uint16_t* perm = perm_all[w];
    uint32_t* cnt = cnt_all[w];
    uint8_t* codes = codes_all[w];
    const uint32_t A = a.A;
    const uint32_t K = std::min<uint32_t>(SL / A, KCAP);
    const uint64_t o0 = ((uint64_t)(XS ? xcd_block() : blockIdx.x) * WPB + w) * K;
    if (o0 >= a.n) return;
    const uint32_t nobj = (uint32_t)std::min<uint64_t>(K, a.n - o0);
    const uint32_t ns = nobj * A;
    const bool has_next = o0 + nobj < a.n;

    // ---- offsets and lengths (lane nobj: the next object's offsets) ---------
    const bool lv = (uint32_t)lane < nobj || ((uint32_t)lane == nobj && has_next);
    const uint64_t koff = lv ? a.key_off[o0 + lane] : 0, voff = lv ? a.val_off[o0 + lane] : 0;
    const uint32_t klen = (uint32_t)lane < nobj ? a.key_len[o0 + lane] : 0u;
    const uint32_t vlen = (uint32_t)lane < nobj ? a.val_len[o0 + lane] : 0u;
    // the code table (4 bytes a lane: a per-lane index into the kernel
    // arguments would become serialized scalar loads)
    if ((uint32_t)lane * 4 < A && (uint32_t)lane * 4 < SL)
        reinterpret_cast<uint32_t*>(codes)[lane] = reinterpret_cast<const uint32_t*>(a.codes)[lane];

    // ---- records [key][value] back to back: one span ------------------------
    // A store whose entries keep each key right before its value (a LevelDB
    // block's adjacency; synth.make_encoded_device(layout="records")) is one
    // contiguous run of bytes per group: copied by one span DMA, keys and
    // values then both read from it.
    // (keys == vals, a wave-uniform test, gates the per-lane check: the other
    // layouts pay one scalar compare)
    uint64_t rend = 0;
    bool rspan = false;
    if (RECS && a.keys == a.vals) {
        const uint64_t knx = sh64(koff, (lane + 1) & 63);
        if (__all((uint32_t)lane >= nobj ||
                  (voff == koff + klen && ((uint32_t)lane + 1 >= nobj || knx == voff + vlen)))) {
            rend = rl64(voff + vlen, (int)nobj - 1);
            rspan = rend - k0_of(koff) + ((uintptr_t)(a.keys + k0_of(koff)) & 15) <= WB;
        }
    }

    // ---- else the keys, then the value span (whatever of it fits) -----------
    // Keys stored back to back (a key column) are one span, copied by 16-byte
    // LDS DMA; otherwise they are gathered dword by dword (a store keeps each
    // key in its own place).
    const uint64_t knext = sh64(koff, (lane + 1) & 63);
    const bool kruns = rspan || __all((uint32_t)lane + 1 >= nobj || koff + klen == knext);
    const uint64_t k0 = rl64(koff, 0);
    const uint32_t klead = (uint32_t)((uintptr_t)(a.keys + k0) & 15);
    uint32_t kdx = 0, kreg = 0;  // kdx: lane o's first dword in the gathered key region
    bool keys_in = false, kspan = false;
    const uint64_t v0 = rl64(voff, 0);
    uint32_t vlead = (uint32_t)((uintptr_t)(a.vals + v0) & 15), vheld = 0;
    const uint64_t kaddr = (uint64_t)(uintptr_t)(a.keys + koff);
    uint32_t kU = 0;  // keys gathered as 16-byte units: units per key slot
    if (rspan) {
        kspan = keys_in = true;  // kreg 0: the values lie in the same span
        vlead = klead + (uint32_t)(v0 - k0);
        vheld = klead + (uint32_t)(rend - k0);
        if (SHAPE != 3) copy_span<ASM, DL>(a.keys + k0 - klead, win + kFrontS, vheld, lane);
    } else {
        if (kruns) {
            const uint64_t kend = rl64(koff + klen, (int)nobj - 1);
            kspan = kend - k0 + klead <= WB / 4;
            keys_in = kspan;
            if (kspan) {
                kreg = (klead + (uint32_t)(kend - k0) + 15) & ~15u;
                if (SHAPE != 3) copy_span<ASM, DL>(a.keys + k0 - klead, win + kFrontS, klead + (uint32_t)(kend - k0), lane);
            }
        }
        // keys in their own places, as whole 16-byte units: lane o*U + k copies
        // unit k of key o (U = the most units a key of the group spans) with
        // one LDS DMA; key o lands at 16*U*o + (its address & 15)
        const uint32_t ku = (uint32_t)lane < nobj ? ((uint32_t)(kaddr & 15) + klen + 15) >> 4 : 0u;
        if (!kspan && KUNITS) {
            for (uint32_t o = 0; o < nobj; ++o) kU = std::max(kU, (uint32_t)__builtin_amdgcn_readlane(ku, (int)o));
            if (kU && nobj * kU <= 64 && 16 * nobj * kU <= WB / 4) {
                const uint32_t magic = (65536u + kU - 1) / kU;  // lane / kU for lane < 64, kU <= 64
                const uint32_t o = ((uint32_t)lane * magic) >> 16, k = (uint32_t)lane - o * kU;
                const uint64_t src = sh64(kaddr & ~15ull, (int)(o & 63)) + 16ull * k;
                const uint32_t uo = (uint32_t)__shfl((int)ku, (int)(o & 63), 64);
                if (o < nobj && k < uo && SHAPE != 3) dma16<ASM>((const void*)(uintptr_t)src, win + kFrontS);
                keys_in = true;
                kreg = 16 * nobj * kU;
            } else {
                kU = 0;
            }
        }
        if (!kspan && !kU) {
            // lane o < nobj: its key's dwords [kd, kd + kdw) from the key's dword floor
            const uint64_t kd = (uint64_t)(uintptr_t)(a.keys + koff) >> 2;
            const uint32_t kdw =
                (uint32_t)lane < nobj ? ((uint32_t)((uintptr_t)(a.keys + koff) & 3) + klen + 3) >> 2 : 0u;
            kdx = wave_scan_dpp(kdw) - kdw;
            const uint32_t td = __builtin_amdgcn_readlane(kdx + kdw, 63);
            keys_in = 4 * td <= WB / 4;
            kreg = keys_in ? (4 * td + 15) & ~15u : 0u;  // the values' region starts 16-byte aligned
            if (keys_in) {
                for (uint32_t u0 = 0; u0 < td; u0 += 64) {
                    const uint32_t u = u0 + (uint32_t)lane;
                    // the object whose key holds region dword u (a wave-uniform walk over <= 63 objects)
                    uint64_t src = 0;
                    for (uint32_t o = 0; o < nobj; ++o) {
                        const uint32_t x0 = __builtin_amdgcn_readlane(kdx, (int)o),
                                       xn = __builtin_amdgcn_readlane(kdw, (int)o);
                        if (u >= x0 && u < x0 + xn) src = 4 * (rl64(kd, (int)o) + (u - x0));
                    }
                    if (u < td) dma4<ASM>((const void*)(uintptr_t)src, win + kFrontS + 4 * u0);
                }
            }
        }
        const uint64_t vend = has_next ? rl64(voff, (int)nobj) : 0;
        vheld = has_next && vend >= v0 ? (uint32_t)std::min<uint64_t>(vlead + (vend - v0), WB - kreg) : 0u;
        if (vheld && SHAPE != 3) copy_span<ASM, DL>(a.vals + v0 - vlead, win + kFrontS + kreg, vheld, lane);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the compiler does not order ds_read after LDS DMA
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(2);  // the walk and sort at medium priority
    wave_fence();

    // ---- decode_value (datalayer_encodings.cc:168-217), lane = object --------
    bool bad = false, ok = false;
    uint64_t my_version = 0;  // stored with the coordinates (a store here would stall the LDS atomics' waits)
    if ((uint32_t)lane < nobj) {
        const uint32_t kw = kFrontS + (kspan ? klead + (uint32_t)(koff - k0)
                                       : kU   ? 16 * kU * (uint32_t)lane + (uint32_t)(kaddr & 15)
                                              : 4 * kdx + (uint32_t)(kaddr & 3));
        desc[lane * A] = keys_in ? ((uint64_t)kw | ((uint64_t)klen << 32)) : ((uint64_t)0 | ((uint64_t)(klen | kGlobal) << 32));
        const uint64_t vrel = voff - v0;
        const bool vin = voff >= v0 && vlead + vrel + vlen <= vheld;
        const uint32_t vw = kFrontS + kreg + vlead + (uint32_t)vrel;  // the value's window offset (vin)
        const uint8_t* vp = a.vals + voff;
        // the walk, reading the value from the window (vin) or global memory
        auto walk = [&](auto be16, auto be32, auto be64, uint32_t base, uint32_t gbit) {
            ok = vlen >= 10;
            uint64_t version = 0;
            if (ok) {
                version = be64(0);
                ok = be16(8) == A - 1;
            }
            uint32_t pos = 10;
            for (uint32_t k = 0; k + 1 < A; ++k) {
                uint32_t len = 0;
                if (ok) {
                    if (vlen - pos < 4) {
                        ok = false;
                    } else {
                        len = be32(pos);
                        pos += 4;
                        if (len > vlen - pos) ok = false;  // the reference does not check this (:201-213)
                    }
                }
                desc[lane * A + 1 + k] = ok ? ((uint64_t)(base + pos) | ((uint64_t)(len | gbit) << 32)) : (uint64_t)kZero;
                if (ok) pos += len;
            }
            return version;
        };
        uint64_t version;
        if (vin) {
            // branch-free from the window: each step's end pos_{k+1} = pos_k +
            // 4 + len_k only grows, and step k decodes iff pos_{k+1} <= vlen,
            // so the object decodes iff the last end does (lengths clamped to
            // WB >= vlen: no wrap, and a clamped one still fails).  Steps past
            // a failure read garbage (or 0 past the LDS allocation) and their
            // descriptors are reset below.
            version = w_be64<SHAPE == 4>(lw, vw);
            ok = vlen >= 10 && w_be16<SHAPE == 4>(lw, vw + 8) == A - 1;
            uint32_t pos = 10;
            uint64_t* dp = desc + lane * A + 1;
            if (SHAPE == 2 || SHAPE == 3) {  // debug shapes: no walk (descriptors of assorted lengths at the value's start)
                for (uint32_t k = 0; k + 1 < A; ++k) dp[k] = (uint64_t)(vw + 14) | ((uint64_t)((k * 37) & 127) << 32);
                pos = vlen;
            } else
#pragma unroll 4
            for (uint32_t k = 0; k + 1 < A; ++k) {
                const uint32_t len = std::min(w_be32<SHAPE == 4>(lw, vw + pos), WB);
                dp[k] = (uint64_t)(vw + pos + 4) | ((uint64_t)len << 32);
                pos += 4 + len;
            }
            ok = ok && pos <= vlen;
        } else
            version = walk([&](uint32_t o) { return g_be16(vp + o); }, [&](uint32_t o) { return g_be32(vp + o); },
                           [&](uint32_t o) { return g_be64(vp + o); }, 0u, kGlobal);
        if (!ok)  // undecodable: every coordinate of the object is 0
            for (uint32_t j = 0; j < A; ++j) desc[lane * A + j] = (uint64_t)kZero;
        my_version = ok ? version : 0;
    }
    const bool any_bad = __any((uint32_t)lane < nobj && !ok);
    wave_fence();

    // ---- counting sort of the slots by class (wave-local) -------------------
    uint32_t cls[NCH], cd[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        const bool valid = s < ns;
        const uint32_t j = s - div_small(s, a.a_magic) * A;
        if constexpr (BF) {  // unguarded loads: s < SL and j < A are always inside desc / codes
            const uint64_t d0 = desc[s];
            const uint32_t c0 = codes[j];
            const uint64_t d = valid ? d0 : (uint64_t)kZero;
            const bool zero = (uint32_t)d == kZero;
            const uint32_t ln = (uint32_t)(d >> 32);
            cd[c] = valid && !zero ? c0 : (uint32_t)CODE_ZERO;
            cls[c] = NUM2 ? sweep_class_tab(cd[c], ln & ~kGlobal, !valid || zero, (ln & kGlobal) != 0)
                          : sweep_class_bf(cd[c], ln & ~kGlobal, !valid || zero, (ln & kGlobal) != 0);
        } else {
            const uint64_t d = valid ? desc[s] : (uint64_t)kZero;
            const bool zero = (uint32_t)d == kZero;
            const uint32_t ln = (uint32_t)(d >> 32);
            cd[c] = valid && !zero ? (uint32_t)codes[j] : (uint32_t)CODE_ZERO;
            cls[c] = sweep_class(cd[c], ln & ~kGlobal, !valid || zero, (ln & kGlobal) != 0);
        }
    }
    class_sort<NCH, GAP>(cnt, perm, cls, cd, ns, wave_fence);
    if constexpr (PRIO == 4) __builtin_amdgcn_s_setprio(0);  // the passes low

    // ---- NCH class-sorted passes, coordinates parked over their descriptors ---
    // (PU 0: the loop not unrolled, one copy of the hash code instead of NCH)
#pragma unroll(PU ? NCH : 1)
    for (int t = 0; t < NCH; ++t) {
        const uint32_t e = perm[t * 64 + lane];
        const uint32_t s = e & 0xffu, code = e >> 8;
        const uint64_t d = desc[s];
        const uint32_t obj = div_small(s, a.a_magic);
        const uint32_t j = s - obj * A;
        const uint32_t off = (uint32_t)d, ln = (uint32_t)(d >> 32);
        // the object bases of slots hashed from global memory, by shuffle with
        // every lane active (a ds_bpermute from an inactive lane reads 0):
        // both, before any branch, and only when the pass has such a slot
        uint64_t ob = 0;
        if (__any(s < ns && off != kZero && (ln & kGlobal) != 0)) {
            const uint64_t kb = sh64(koff, (int)(obj & 63)), vb = sh64(voff, (int)(obj & 63));
            asm volatile("" ::"v"(kb), "v"(vb));
            ob = j == 0 ? kb : vb;
        }
        uint64_t h = 0;
        if (s < ns && off != kZero) {
            if (ln & kGlobal) h = hash_global((j == 0 ? a.keys : a.vals) + ob + off, code, ln & ~kGlobal, bad);
            else if (SHAPE == 1 || SHAPE == 2) h = d ^ lw[off >> 2];
            else h = hash_slot_window<false, (LOOP >= 10 ? LOOP - 10 : LOOP), (LOOP >= 10), NUM2 && LOOP >= 10>(
                lw, code, off, ln, bad);
        }
        desc[s] = h;
    }
    wave_fence();
    if (!REGIONS || a.coords) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t s = (uint32_t)(c * 64 + lane);
            if (s < ns) __builtin_nontemporal_store(desc[s], a.coords + o0 * A + s);
        }
    }
    if (a.versions && (uint32_t)lane < nobj) a.versions[o0 + lane] = my_version;
    if constexpr (REGIONS)  // the window is free now: the lookups' scratch
        lookup_tables_wave(a.t, a.T, desc, A, nobj, o0, reinterpret_cast<uint64_t*>(win), wave_fence);
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// Codes the NUM2 forms handle: strings, int64 and floats.
static bool num2_codes(const EncodedArgs& a) {
    if (a.A > kKernargCodes) return false;
    for (uint32_t j = 0; j < a.A; ++j)
        if (a.codes[j] != CODE_STRING && a.codes[j] != CODE_INT64 && a.codes[j] != CODE_FLOAT) return false;
    return true;
}

template <int NCH, uint32_t WB, uint32_t KCAP, bool REGIONS = false, bool GAP = false, int SHAPE = 0, int LOOP = 1,
          bool ASM = false, bool PU = true, bool BF = false, bool RECS = true, bool KUNITS = true, bool DL = false,
          int WPB = 4, bool XS = false, int PRIO = 0, bool NUM2 = false>
static hipError_t launch_wsweep_t(const EncodedArgs& a, hipStream_t stream) {
    const uint32_t K = std::min<uint32_t>(64 * NCH / a.A, KCAP);
    if (K == 0) return hipErrorInvalidValue;
    if (NUM2 && !num2_codes(a)) return hipErrorInvalidValue;
    const uint64_t waves = (a.n + K - 1) / K;
    const uint64_t blocks = (waves + WPB - 1) / WPB;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_sweep_wstage_kernel<NCH, WB, KCAP, REGIONS, GAP, SHAPE, LOOP, ASM, PU, BF, RECS, KUNITS, DL, WPB, XS, PRIO,
                                                 NUM2>),
                       dim3((uint32_t)blocks), dim3(64 * WPB), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
