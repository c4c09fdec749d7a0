// hdx_kernels_dbg.hip — the batch hash's retired A/B experiments (DESIGN.md
// §4.9), built into libhdxhash_dbg.so only (Makefile SRCS_DBG): occupancy
// caps, quad-cooperative loop loads, late heads, register descriptors, grid
// striding, the column, typed and workgroup-sorted kernels, the fused forms'
// alternatives, and the process-wide variant selection
// (hdxdbg_set_kernel_variant / HDX_KERNEL_VARIANT).  Every form here writes
// the reference's coordinates (except the named debug shapes 40 / 41, 57 / 58)
// and is parity-tested in tests/; none is reachable from the
// product library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

#include "hdx_regroup.h"

namespace hdx {

// Debug: the same kernel held to WPE waves per SIMD (amdgpu_waves_per_eu caps
// the VGPRs at 512 / WPE), for occupancy A/B (variants 140-147).
template <int WPE, int C, bool NT_STORE, bool SORT = true, bool DIRECT = true, bool A4 = false, bool PIPE = false,
          bool ASORT = false, int ORDER = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
hash_regroup_wpe_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C> lds;
    regroup_body<C, NT_STORE, SORT, DIRECT, A4, PIPE, ASORT, ORDER, false>(args, lds, nullptr);
}

// Debug: the sorted A4 kernel with the > 64-byte loop's loads quad-cooperative
// (variants 160/161: 2 / 4 chunks).
template <int C>
__global__ void __launch_bounds__(256)
hash_regroup_quad_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C> lds;
    regroup_body<C, true, true, true, true, false, true, 1, false, false, false, true>(args, lds, nullptr);
}

// Debug: variant 44 with each > 64-byte string's head (190), or each one-block
// string's (191), loaded with its first loop block instead of a pass ahead.
template <int C, int LATE>
__global__ void __launch_bounds__(256)
hash_regroup_late_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C> lds;
    regroup_body<C, true, true, true, true, false, true, 1, false, false, false, false, LATE>(args, lds, nullptr);
}

// Debug: unsorted waves with the descriptors in registers (variants 154/155).
template <int C, bool NT_STORE>
__global__ void __launch_bounds__(256)
hash_regroup_regd_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C> lds;
    regroup_body<C, NT_STORE, false, true, false, false, false, 0, false, false, true>(args, lds, nullptr);
}

// Debug: a fixed grid whose waves stride over the C * 64-slot windows
// (variants 150-152), against the one-window-per-wave launch.
template <int C, bool NT_STORE, bool SORT = true, bool DIRECT = true, bool A4 = false, bool PIPE = false,
          bool ASORT = false, int ORDER = 0>
__global__ void __launch_bounds__(256)
hash_regroup_stride_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C> lds;
    const uint64_t windows = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t stride = (uint64_t)gridDim.x * 4;
    for (uint64_t wv = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); wv < windows; wv += stride) {
        regroup_body<C, NT_STORE, SORT, DIRECT, A4, PIPE, ASORT, ORDER, false>(args, lds, nullptr, wv);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// ===========================================================================
// Column kernel (variants 90-92): one lane per object, the attributes walked
// in schema order.  For narrow schemas whose per-attribute work is the same on
// every lane (config 2: a 64-byte key and four int64; config 1), the type
// dispatch is wave-uniform (codes[j] is a kernel argument), no slot scan or
// descriptor is needed, and a value's loads are only the ones its type needs:
// a string's dword-aligned A4 pieces, a numeric's two dwords + one.  The
// next attribute's loads are in flight while the current one is hashed; the
// wave's 64 * A coordinates are parked in LDS and stored coalesced.
// ===========================================================================
template <int AMAX>
__global__ void __launch_bounds__(256)
hash_column_kernel(const BatchArgs args) {
    __shared__ uint64_t park[4][64 * AMAX];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint64_t i0 = ((uint64_t)blockIdx.x * 4 + w) * 64;
    if (i0 >= args.n) return;
    const uint32_t A = args.A;
    const uint32_t nobj = (uint32_t)min<uint64_t>(64, args.n - i0);
    const bool valid = (uint32_t)lane < nobj;
    const uint64_t i = i0 + (valid ? lane : 0);
    uint32_t L[AMAX], off[AMAX];
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < AMAX; ++j) L[j] = (j < (int)A && valid) ? args.attr_len[i * A + j] : 0u;
    const uint8_t* base = args.blob + args.obj_base[i];
#pragma unroll
    for (int j = 0; j < AMAX; ++j) {
        off[j] = run;
        run += L[j];
    }
    struct Att {
        Raw blk;
        uint32_t d0, d1, d2;
    };
    auto issue = [&](int j, Att& a) {
        const uint32_t code = args.codes[j];  // wave-uniform
        const uint8_t* p = base + off[j];
        if (code == CODE_STRING) {
            a.blk = issue_any<true>(CODE_STRING, valid ? p : g_zero_pad, L[j]);
        } else if (code != CODE_ZERO && L[j] == 8) {
            const uint8_t* q = dw_floor(p);
            a.d0 = gld4(q);
            a.d1 = gld4(q + 4);
            a.d2 = gld4(dw_floor(p + 7));
        }
    };
    bool bad = false;
    auto consume = [&](int j, Att& a) -> uint64_t {
        const uint32_t code = args.codes[j];
        const uint8_t* p = base + off[j];
        if (code == CODE_STRING)
            return hash_blk<false, false, true>(CODE_STRING, valid ? p : g_zero_pad, L[j], consume_any<true>(a.blk), bad);
        if (code == CODE_ZERO) return 0;
        if (L[j] == 8) {
            const uint32_t r = (uint32_t)(uintptr_t)p & 3;
            return hash_numeric(code, pack64(__builtin_amdgcn_alignbyte(a.d1, a.d0, r),
                                             __builtin_amdgcn_alignbyte(a.d2, a.d1, r)));
        }
        if (L[j] != 0) {
            bad = true;
            return 0;
        }
        return hash_numeric(code, 0);
    };
    Att P0, P1;
    issue(0, P0);
#pragma unroll
    for (int j = 0; j < AMAX; ++j) {
        if (j >= (int)A) break;
        Att& cur = (j & 1) ? P1 : P0;
        Att& nxt = (j & 1) ? P0 : P1;
        if (j + 1 < (int)A && j + 1 < AMAX) issue(j + 1, nxt);
        const uint64_t h = consume(j, cur);
        park[w][lane * A + j] = h;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t total = nobj * A;
    for (uint32_t t = (uint32_t)lane; t < total; t += 64)
        __builtin_nontemporal_store(park[w][t], args.coords + i0 * A + t);
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int AMAX>
static hipError_t launch_column(const BatchArgs& args, hipStream_t stream) {
    if (args.A > AMAX) return hipErrorInvalidValue;
    const uint64_t waves = (args.n + 63) / 64;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_column_kernel<AMAX>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

// ===========================================================================
// Typed regroup kernel (variants 70-73): the regroup kernel's wave-local class
// sort (ORDER 1), with the non-string slots (int64 / float / timestamps /
// non-hashable, class 0) taken out of the 64-lane passes: they are hashed in
// a lean loop of their own — two dword loads and two v_alignbyte per value,
// no descriptor-driven 16-byte pieces, no CityHash code in the loop — and
// only the strings, sorted by regime and loop count, fill the passes
// (DESIGN.md §4.9).  Config 3b measured 373 VALU per 128 numeric slots through
// the string-shaped passes (profiles/r2/regime_costs_v44.txt).
// ===========================================================================
template <int C>
struct TypedLds {
    SlotDesc desc[4][C * 64];
    uint16_t perm[4][C * 64];
    uint32_t cnt[4][kClasses];
};

template <int C>
__global__ void __launch_bounds__(256)
hash_typed_kernel(const BatchArgs args) {
    __shared__ TypedLds<C> lds;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    SlotDesc* desc = lds.desc[w];
    uint16_t* perm = lds.perm[w];
    uint64_t* res = reinterpret_cast<uint64_t*>(desc);  // res[2*s] = first 8 bytes of desc[s]

    const uint64_t wave = (uint64_t)blockIdx.x * 4 + w;
    const uint32_t A = args.A;
    const uint64_t nslots = args.n * A;
    const uint64_t qw = wave * (uint64_t)(C * 64);
    if (qw >= nslots) return;  // no workgroup barrier anywhere: waves are independent

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

    // ---- phase 1: descriptors + classes (ORDER 1: class 0 = every non-string)
    uint32_t cls[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t t = j0 + (uint32_t)(c * 64 + lane);
        const uint32_t di = div_small(t, args.a_magic);
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
        desc[c * 64 + lane] = d;
        cls[c] = work_class<1>(code, L, valid);
    }

    // ---- counting sort by class (LDS fetch-add, wave-local) -----------------
    const uint32_t c00 = __builtin_amdgcn_readfirstlane(cls[0]);
    bool uniform = true;
#pragma unroll
    for (int c = 0; c < C; ++c) uniform &= __all(cls[c] == c00);
    uint32_t n0;  // sorted positions [0, n0) hold the non-string slots
    if (!uniform) {
        uint32_t* cnt = lds.cnt[w];
        if (lane < kClasses) cnt[lane] = 0;
#pragma unroll
        for (int c = 0; c < C; ++c)
            __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint32_t k = lane < kClasses ? cnt[lane] : 0u;
        const uint32_t start = wave_scan_dpp(k) - k;
        n0 = __builtin_amdgcn_readlane(start + k, 0);
        if (lane < kClasses) cnt[lane] = start;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const uint32_t pos = __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WAVEFRONT);
            perm[pos] = (uint16_t)(c * 64 + lane);
        }
    } else {
        n0 = c00 == 0 ? (uint32_t)(C * 64) : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- phase 2: string passes (next pass in flight) and the non-string
    // slots; the first string pass's bytes and every non-string value are
    // requested before anything is consumed, so the wave waits on memory once
    const uint32_t npass = ((uint32_t)(C * 64) - n0 + 63) / 64;
    struct Pass {
        SlotDesc d;
        Raw blk;
    };
    auto load_pass = [&](int t, Pass& P) {
        const uint32_t k = n0 + (uint32_t)(t * 64 + lane);
        if (k < (uint32_t)(C * 64)) {
            P.d = desc[uniform ? k : perm[k]];
        } else {  // past the wave's slots: hashes the zero pad, never stored
            P.d.p = g_zero_pad;
            P.d.n = 0;
            P.d.code_slot = CODE_ZERO | (0xffffu << 8);
        }
        P.blk = issue_any<true>(P.d.code_slot & 0xffu, P.d.p, P.d.n);
    };
    Pass P0, P1;
    if (npass > 0) load_pass(0, P0);

    // non-string slots: descriptors and value dwords of every sub-pass first
    bool bad = false;
    uint32_t nslot[C], nd0[C], nd1[C], nd2[C], ncode[C], nlen[C], nsh[C];
#pragma unroll
    for (int u = 0; u < C; ++u) {
        const uint32_t k = (uint32_t)(u * 64 + lane);
        nslot[u] = 0xffffu;
        nd0[u] = nd1[u] = nd2[u] = 0;
        ncode[u] = CODE_ZERO;
        nlen[u] = 0;
        nsh[u] = 0;
        if ((uint32_t)(u * 64) < n0 && k < n0) {
            const uint32_t sl = uniform ? k : perm[k];
            const SlotDesc d = desc[sl];
            nslot[u] = sl;
            ncode[u] = d.code_slot & 0xffu;
            nlen[u] = d.n;
            if (ncode[u] != CODE_ZERO && d.n == 8) {
                const uint8_t* a = dw_floor(d.p);
                nsh[u] = (uint32_t)(uintptr_t)d.p & 3;
                nd0[u] = gld4(a);
                nd1[u] = gld4(a + 4);
                nd2[u] = gld4(dw_floor(d.p + 7));
            }
        }
    }
#pragma unroll
    for (int u = 0; u < C; ++u) {
        if (nslot[u] == 0xffffu) continue;
        uint64_t h = 0;
        if (ncode[u] != CODE_ZERO) {
            if (nlen[u] == 8) {
                h = hash_numeric(ncode[u], pack64(__builtin_amdgcn_alignbyte(nd1[u], nd0[u], nsh[u]),
                                                  __builtin_amdgcn_alignbyte(nd2[u], nd1[u], nsh[u])));
            } else if (nlen[u] == 0) {
                h = hash_numeric(ncode[u], 0);
            } else {
                bad = true;
            }
        }
        res[2 * nslot[u]] = h;
    }

    // strings
#pragma unroll
    for (int t = 0; t < C; ++t) {
        if ((uint32_t)t >= npass) break;
        Pass& cur = (t & 1) ? P1 : P0;
        Pass& nxt = (t & 1) ? P0 : P1;
        if ((uint32_t)t + 1 < npass) load_pass(t + 1, nxt);
        const uint64_t h = hash_blk<false, false, true>(cur.d.code_slot & 0xffu, cur.d.p, cur.d.n,
                                                        consume_any<true>(cur.blk), bad);
        const uint32_t s = cur.d.code_slot >> 8;
        if (s != 0xffffu) res[2 * s] = h;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- phase 3: coalesced stores in slot order ------------------------------
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint64_t q = qw + c * 64 + lane;
        if (q < nslots) __builtin_nontemporal_store(res[2 * (c * 64 + lane)], args.coords + q);
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int C>
static hipError_t launch_typed(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_typed_kernel<C>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

// ===========================================================================
// Workgroup-sorted kernel (variants 60-65): the class sort of the regroup
// kernel over the whole workgroup's 4 * C * 64 slots instead of one wave's
// C * 64.  A wave's share of the work and of the L2 working set is the same as
// a C-chunk regroup wave (C passes of 64 slots, one 8.7 KB window of config
// 3b per 2 chunks), but the sort window is four times larger, so far fewer
// passes mix CityHash regimes and > 64-byte loop counts:
//   phase 1  each wave describes its C chunks ({pointer, length, code} into
//            the workgroup's LDS, as the regroup kernel does) and counts its
//            slots per class (ballots);
//   barrier  per-class totals -> each wave's base in the class-sorted order;
//            every slot writes its local index at its sorted position;
//   barrier  passes of 64 sorted slots: static (wave w takes passes w, w+4,
//            ...) or dynamic (an LDS counter hands out passes, costliest
//            classes first); A4 loads with the next pass in flight; each
//            coordinate is stored straight to its slot (the workgroup's
//            4 * C * 64 coordinates are one contiguous 4-8 KB range, merged
//            in L2).
// ORDER 10: classes by falling cost (> 64 B by blocks 4+, 3, 2, 1; 17..32;
// <= 16; 33..64; numerics); ORDER 11: rising cost.
// ===========================================================================
constexpr int kWgClasses = 9;  // 8 work classes + the padding slots past the batch end

template <int ORDER>
__device__ __forceinline__ uint32_t wg_class(uint32_t code, uint32_t n, bool valid) {
    if (!valid) return 8;
    uint32_t k;  // 0 = cheapest .. 7 = costliest
    if (code != CODE_STRING) {
        k = 0;
    } else if (n > 64) {
        const uint32_t b = (n - 1) >> 6;
        k = b >= 4 ? 7u : 3u + b;
    } else {
        k = n > 32 ? 1u : n <= 16 ? 2u : 3u;
    }
    return ORDER == 10 ? 7u - k : k;
}

template <int C>
struct WgSortLds {
    SlotDesc desc[4 * C * 64];
    uint16_t perm[4 * C * 64];
    uint32_t cnt[4][kWgClasses + 1];
    uint32_t next;
};

template <int C, int ORDER, bool DYN, bool PARK = false, bool NOSORT = false>
__global__ void __launch_bounds__(256)
hash_wgsort_kernel(const BatchArgs args) {
    __shared__ WgSortLds<C> lds;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    constexpr uint32_t S = 4 * C * 64;  // slots per workgroup
    const uint32_t A = args.A;
    const uint64_t nslots = args.n * A;
    const uint64_t qg = (uint64_t)blockIdx.x * S;  // < nslots (grid sized by the host)
    const uint32_t nv = (uint32_t)min<uint64_t>(S, nslots - qg);  // valid slots of the workgroup
    const uint64_t qw = qg + (uint64_t)w * (C * 64);
    const bool wave_live = qw < nslots;  // trailing waves of the last workgroup have no slots

    // ---- phase 1: descriptors + classes (the regroup kernel's, per wave) ------
    uint32_t cls[C];
    if (wave_live) {
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
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const uint32_t t = j0 + (uint32_t)(c * 64 + lane);
            const uint32_t di = div_small(t, args.a_magic);
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
            d.code_slot = code;
            lds.desc[w * (C * 64) + c * 64 + lane] = d;
            cls[c] = wg_class<ORDER>(code, L, valid);
        }
    } else {
#pragma unroll
        for (int c = 0; c < C; ++c) cls[c] = 8;
    }
    // per-class counts of this wave and each slot's rank within them
    uint32_t rank[C];
    uint32_t mycnt = 0;  // lane k < kWgClasses: this wave's slots of class k
#pragma unroll
    for (int k = 0; k < kWgClasses; ++k) {
        uint32_t run = 0;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const uint64_t m = __ballot(cls[c] == (uint32_t)k);
            if (cls[c] == (uint32_t)k)
                rank[c] = run + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            run += (uint32_t)__popcll(m);
        }
        if (lane == k) mycnt = run;
    }
    if (lane < kWgClasses) lds.cnt[w][lane] = mycnt;
    if (DYN && threadIdx.x == 0) lds.next = 0;
    __syncthreads();

    // ---- sorted positions: class start + this wave's base within the class ----
    uint32_t base_k = 0;
    if (lane < kWgClasses) {
        uint32_t tot = 0, before = 0;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint32_t x = lds.cnt[v][lane];
            tot += x;
            before += v < w ? x : 0u;
        }
        base_k = before + (wave_scan_dpp(tot) - tot);  // lanes >= kWgClasses add 0 to the scan
    } else {
        (void)wave_scan_dpp(0u);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t me = w * (C * 64) + c * 64 + lane;
        const uint32_t pos = NOSORT ? me : __shfl(base_k, (int)cls[c], 64) + rank[c];
        lds.perm[pos] = (uint16_t)me;
    }
    __syncthreads();

    // ---- phase 2: class-homogeneous passes, next pass in flight --------------
    const uint32_t npass = (nv + 63) / 64;
    struct Pass {
        uint32_t s;  // local slot, or ~0u for a padding lane
        SlotDesc d;
        Raw blk;
    };
    auto load_pass = [&](uint32_t p, Pass& P) {
        const uint32_t idx = p * 64 + (uint32_t)lane;
        const bool act = p < npass && idx < nv;
        P.s = act ? (uint32_t)lds.perm[idx] : ~0u;
        if (act) {
            P.d = lds.desc[P.s];
        } else {
            P.d.p = g_zero_pad;
            P.d.n = 0;
            P.d.code_slot = CODE_ZERO;
        }
        P.blk = issue_any<true>(P.d.code_slot & 0xffu, P.d.p, P.d.n);
    };
    auto grab = [&](uint32_t t) -> uint32_t {
        if constexpr (DYN) {
            uint32_t p = 0;
            if (lane == 0) p = __hip_atomic_fetch_add(&lds.next, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return __builtin_amdgcn_readfirstlane(p);
        } else {
            return (uint32_t)w + 4 * t;
        }
    };
    bool bad = false;
    auto hash_store = [&](const Pass& P) {
        const uint64_t h = hash_blk<false, false, true>(P.d.code_slot & 0xffu, P.d.p, P.d.n,
                                                        consume_any<true>(P.blk), bad);
        if (P.s != ~0u) {
            if (PARK) reinterpret_cast<uint64_t*>(lds.desc)[2 * P.s] = h;  // over its consumed descriptor
            else args.coords[qg + P.s] = h;
        }
    };
    // two named register sets, unrolled by hand: a runtime-selected reference
    // to either would put both on scratch
    Pass P0, P1;
    uint32_t t = 0;
    uint32_t p0 = grab(t++);
    if (p0 < npass) load_pass(p0, P0);
    while (p0 < npass) {
        const uint32_t p1 = grab(t++);
        if (p1 < npass) load_pass(p1, P1);
        hash_store(P0);
        if (p1 >= npass) break;
        p0 = grab(t++);
        if (p0 < npass) load_pass(p0, P0);
        hash_store(P1);
    }
    if constexpr (PARK) {  // every coordinate parked: coalesced stores in slot order
        __syncthreads();
        const uint64_t* res = reinterpret_cast<const uint64_t*>(lds.desc);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const uint32_t sl = w * (C * 64) + c * 64 + lane;
            if (sl < nv) __builtin_nontemporal_store(res[2 * sl], args.coords + qg + sl);
        }
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int C, int ORDER, bool DYN, bool PARK = false, bool NOSORT = false>
static hipError_t launch_wgsort(const BatchArgs& args, hipStream_t stream) {
    const uint64_t S = 4 * C * 64;
    const uint64_t blocks = (args.n * args.A + S - 1) / S;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_wgsort_kernel<C, ORDER, DYN, PARK, NOSORT>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

template <int WPE, int C, bool NT, bool SORT = true, bool DIRECT = true, bool A4 = false, bool PIPE = false,
          bool ASORT = false, int ORDER = 0>
static hipError_t launch_regroup_wpe(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_wpe_kernel<WPE, C, NT, SORT, DIRECT, A4, PIPE, ASORT, ORDER>),
                       dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

// Debug: variant 44's kernel with unused dynamic LDS, so that at most
// wg_per_cu workgroups share a CU (fewer waves contending for the L1).
static hipError_t launch_44_wg_limit(const BatchArgs& args, hipStream_t stream, uint32_t wg_per_cu) {
    constexpr int C = 2;
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    const size_t dyn = 160 * 1024 / wg_per_cu - sizeof(RegroupLds<C>) - 1024;
    hipLaunchKernelGGL((hash_regroup_kernel<C, true, true, true, true, false, true, 1>), dim3((uint32_t)blocks),
                       dim3(256), dyn, stream, args);
    return hipGetLastError();
}

template <int C, int LATE>
static hipError_t launch_late(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_late_kernel<C, LATE>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

template <int C>
static hipError_t launch_quad(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_quad_kernel<C>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

template <int C>
static hipError_t launch_regd(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_regd_kernel<C, true>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

template <int C, bool NT, bool SORT = true, bool DIRECT = true, bool A4 = false, bool PIPE = false,
          bool ASORT = false, int ORDER = 0>
static hipError_t launch_regroup_stride(const BatchArgs& args, hipStream_t stream, uint32_t wg_per_cu) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = std::min<uint64_t>((waves + 3) / 4, 256ull * wg_per_cu);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL((hash_regroup_stride_kernel<C, NT, SORT, DIRECT, A4, PIPE, ASORT, ORDER>),
                       dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

// Debug-only variants of launch_hash_batch_variant (hdx_kernels.hip).
hipError_t launch_debug_variant(const BatchArgs& args, hipStream_t stream, int variant) {
    switch (variant) {
        // alternatives for interleaved A/B (scripts/ab_variants.py), bit-exact
        case 18: return launch_regroup<4, true>(args, stream);
        case 19: return launch_regroup<8, true>(args, stream);
        case 26: return launch_regroup<2, true>(args, stream);
        case 30: return launch_chunk<true, true>(args, stream);
        case 31: return launch_chunk<true, false, 0, true>(args, stream);
        case 35: return launch_regroup<2, true, true, true, true>(args, stream);
        case 37: return launch_regroup<2, true, true, true, true, true>(args, stream);
        case 38: return launch_regroup<2, true, true, true, true, false, true>(args, stream);
        case 39: return launch_regroup<8, true, true, true, false, false, true>(args, stream);
        case 45: return launch_regroup<2, true, true, true, true, false, true, 2>(args, stream);
        case 90: return args.A <= 2 ? launch_column<2>(args, stream) : args.A <= 5 ? launch_column<5>(args, stream)
                                                             : args.A <= 8 ? launch_column<8>(args, stream)
                                                                           : launch_hash_batch_variant(args, stream, 44);
        case 80: return launch_hash_staged(args, stream, 192, 16384);
        case 81: return launch_hash_staged(args, stream, 128, 12288);
        case 82: return launch_hash_staged(args, stream, 256, 20480);
        case 83: return launch_hash_staged(args, stream, 128, 10240);
        case 84: return launch_hash_staged(args, stream, 128, 9216);
        case 85: return launch_hash_staged(args, stream, 96, 7168);
        case 86: return launch_hash_staged(args, stream, 64, 5120);
        case 70: return launch_typed<2>(args, stream);
        case 71: return launch_typed<3>(args, stream);
        case 72: return launch_typed<4>(args, stream);
        case 73: return launch_typed<6>(args, stream);
        case 60: return launch_wgsort<2, 10, false>(args, stream);
        case 61: return launch_wgsort<2, 10, true>(args, stream);
        case 62: return launch_wgsort<2, 11, false>(args, stream);
        case 63: return launch_wgsort<4, 10, true>(args, stream);
        case 64: return launch_wgsort<1, 10, true>(args, stream);
        case 65: return launch_wgsort<3, 10, true>(args, stream);
        case 66: return launch_wgsort<2, 10, true, true>(args, stream);
        case 67: return launch_wgsort<2, 10, true, true, true>(args, stream);
        case 68: return launch_wgsort<1, 10, true, true>(args, stream);
        case 69: return launch_wgsort<4, 10, true, true>(args, stream);
        // occupancy A/B: 44 at 6 / 7 / 8 waves per SIMD, 21 at 8, 25 at 4 / 5, 46 at 5 / 6
        case 140: return launch_regroup_wpe<6, 2, true, true, true, true, false, true, 1>(args, stream);
        case 141: return launch_regroup_wpe<7, 2, true, true, true, true, false, true, 1>(args, stream);
        case 142: return launch_regroup_wpe<8, 2, true, true, true, true, false, true, 1>(args, stream);
        case 143: return launch_regroup_wpe<8, 4, true, false>(args, stream);
        case 144: return launch_regroup_wpe<4, 16, true, false, false>(args, stream);
        case 145: return launch_regroup_wpe<5, 16, true, false, false>(args, stream);
        case 146: return launch_regroup_wpe<5, 8, true, true, true, false, false, true, 1>(args, stream);
        case 147: return launch_regroup_wpe<6, 8, true, true, true, false, false, true, 1>(args, stream);
        case 190: return launch_late<2, 1>(args, stream);
        case 191: return launch_late<2, 2>(args, stream);
        case 180: return launch_44_wg_limit(args, stream, 2);
        case 181: return launch_44_wg_limit(args, stream, 3);
        case 182: return launch_44_wg_limit(args, stream, 4);
        case 160: return launch_quad<2>(args, stream);
        case 161: return launch_quad<4>(args, stream);
        case 154: return launch_regd<4>(args, stream);
        case 155: return launch_regd<8>(args, stream);
        // fixed grids striding over the windows: 21 and 44 at 4 / 8 workgroups per CU
        case 150: return launch_regroup_stride<4, true, false>(args, stream, 4);
        case 151: return launch_regroup_stride<4, true, false>(args, stream, 8);
        case 152: return launch_regroup_stride<2, true, true, true, true, false, true, 1>(args, stream, 4);
        case 153: return launch_regroup_stride<2, true, true, true, true, false, true, 1>(args, stream, 8);
        // wave-staged (hdx_wstage.hip): 200 2 passes / 10 KiB, 201 3 / 14 KiB, 202 2 / 8 KiB,
        // 203 1 / 5 KiB, 204 4 / 18 KiB, 205 2 / 8832 B, 206 = 205 with <= 6 objects
        case 200: case 201: case 202: case 203: case 204: case 205: case 206: case 207: case 208:
        case 209: case 210: case 211: case 213: case 214: case 215: case 216: case 218: case 219: case 239: case 240: case 241: case 242: case 244: case 245: case 246: case 248: case 249: case 255: {
            const hipError_t e = launch_hash_wstage(args, stream, variant - 200);
            return e == hipErrorInvalidValue ? launch_hash_batch_variant(args, stream, 44) : e;
        }
        // streamed (hdx_stream.hip): 220 16 waves / 2 x 63 KiB, 221 8 waves / 2 x 31 KiB, 222 16 / 2 x 60 KiB
        case 220: case 221: case 222: case 223: case 224: case 225: case 226: case 227: {
            const hipError_t e = launch_hash_stream(args, stream, variant - 220);
            return e == hipErrorInvalidValue ? launch_hash_batch_variant(args, stream, 44) : e;
        }
        // debug shapes: WRONG coordinates, debug library only
        case 40: return launch_chunk<true, false, 1>(args, stream);  // loads only
        case 41: return launch_chunk<true, false, 2>(args, stream);  // arithmetic only
        default: return hipErrorInvalidValue;
    }
}

// Debug library only: the fused forms for interleaved A/B (variants 100-119).
hipError_t launch_fused_debug(const BatchArgs& args, hipStream_t stream, int v) {
    switch (v) {
        case 100: return launch_regroup_regions<4, false, false, false, 0, false>(args, stream);
        case 101: return launch_regroup_regions<4, false, false, false, 0, true>(args, stream);
        case 102: return launch_regroup_regions<2, false, false, false, 0, true>(args, stream);
        case 103: return launch_regroup_regions<8, false, false, false, 0, true>(args, stream);
        case 104: return launch_regroup_regions<4, false, false, false, 0, true>(args, stream, false);
        case 105: return launch_regroup_regions<3, true, true, true, 1, false>(args, stream);
        case 106: return launch_regroup_regions<3, true, true, true, 1, true>(args, stream);
        case 107: return launch_regroup_regions<2, true, true, true, 1, true>(args, stream);
        case 108: return launch_regroup_regions<8, false, false, false, 0, false>(args, stream);
        case 109: return launch_regroup_regions<8, false, false, false, 0, true>(args, stream);
        case 110: return launch_regroup_regions<1, false, false, false, 0, true>(args, stream);
        case 111: return launch_regroup_regions<4, true, true, true, 1, true>(args, stream);
        default: return hipErrorInvalidValue;
    }
}

// Debug library only (libhdxhash_dbg.so): a process-wide kernel selection for
// interleaved A/B runs, from hdxdbg_set_kernel_variant or HDX_KERNEL_VARIANT.
// 33 / 43 / 47 / 48 select the stored-object sweep's alternative forms, 57 / 58
// its walk-only and loads-only debug shapes (hdx_encoded.hip).
static bool known_variant(int v) {
    switch (v) {
        case -1: case 12: case 18: case 19: case 20: case 21: case 25: case 26: case 30: case 31: case 35: case 37:
        case 38: case 39: case 44: case 45: case 46:
        case 60: case 61: case 62: case 63: case 64: case 65: case 66: case 67: case 68: case 69:
        case 70: case 71: case 72: case 73: case 80: case 81: case 82: case 83: case 84: case 85: case 86: case 90:
        case 95: case 96: case 97: case 98: case 99:
        case 100: case 101: case 102: case 103: case 104: case 105: case 106: case 107: case 108: case 109:
        case 110: case 111:  // fused hash + lookup_region forms (launch_fused_debug)
        case 140: case 141: case 142: case 143: case 144: case 145: case 146: case 147:
        case 150: case 151: case 152: case 153: case 154: case 155: case 160: case 161:
        case 170: case 171: case 172: case 173: case 174:  // the sweep's numeric walk (hdx_encoded.hip)
        case 180: case 181: case 182: case 190: case 191:
        case 200: case 201: case 202: case 203: case 204: case 205: case 206:  // wave-staged (hdx_wstage.hip)
        case 207: case 208:  // its debug shapes: no hash / no DMA (WRONG coordinates)
        case 209:  // <= 3 objects per wave (per-regime VALU on uniform batches)
        case 212: case 213: case 214: case 215: case 216:  // wave-staged, head/tail window hashing
        case 217:  // wave-staged with the fused region lookup (hdx_hash_batch_regions_device)
        case 218:  // debug shape of 212: no hash (WRONG coordinates)
        case 219:  // 212 without the pass-boundary gap (class_sort)
        case 239:  // 212 / 230 with the one-block > 64-byte loop (city_gt64_lds LOOP 1)
        case 240:  // 212 with the DMA as the builtin (describe_group ADMA off)
        case 241:  // debug shape of 212: no hash (WRONG coordinates)
        case 242:  // 212 with / 230 without one final mix16 for the > 64 and 8..32-byte regimes (LOOP 3)
        case 243:  // 230 with the DMA as inline asm
        case 244:  // 212 / 230 with the pass loop not unrolled
        case 245:  // 212 / 230 with the branchy work class (and, 230, guarded loads)
        case 246:  // 212 / 230 without TNUM (numerics read apart from the strings' tail)
        case 220: case 221: case 222:  // streamed (hdx_stream.hip)
        case 230: case 231: case 232: case 233: case 234:  // wave-staged sweep (hdx_wsweep.hip; 233: fused regions; 234: the gather sweep's fused regions)
        case 236:  // 230 without the pass-boundary gap
        case 237: case 238:  // 230's debug shapes: no hash / no hash, no walk (WRONG coordinates)
        case 235:  // regions by hash + separate lookups at any n, 64 MiB chunks (hdx_regions.hip)
        case 247:  // 235 with the scratch allocation failing: the fused fallback
        case 248:  // debug shape of 212: its LDS reads at conflict-free addresses (WRONG coordinates)
        case 249:  // debug shape of 212: no funnel shifts on its LDS reads (WRONG coordinates)
        case 250:  // the product sweep (230) without the record span
        case 251:  // ... and with round 3's dword-by-dword key gather
        case 252:  // debug shape of 250: no copy, no walk, the hash on made-up descriptors (WRONG coordinates)
        case 253: case 254:  // the product sweep's non-record / record forms with round 3's per-KiB span copy
        case 255:  // 212 with round 3's per-KiB span copy; the sweep with round 3's walk reads
        case 223: case 224: case 225: case 226: case 227:  // its debug shapes (WRONG coordinates)
        case 210: case 211:  // wave-staged, sorted over the workgroup
        case 40: case 41:
        case 33: case 43: case 47: case 48: case 49: case 57: case 58:  // stored-object sweep forms (hdx_encoded.hip)
            return true;
        default:
            return false;
    }
}

static int g_variant = [] {
    const char* e = getenv("HDX_KERNEL_VARIANT");
    return e && *e && known_variant(atoi(e)) ? atoi(e) : -1;
}();

int hash_variant() { return __atomic_load_n(&g_variant, __ATOMIC_RELAXED); }

int set_hash_variant(int v) {
    if (!known_variant(v)) return -2;
    return __atomic_exchange_n(&g_variant, v, __ATOMIC_RELAXED);
}

}  // namespace hdx
