// hdx_encoded_staged_dbg.hip — (debug library only: an A/B experiment)
// the reindex sweep with each group of stored
// objects staged in LDS (variants 95-98).
//
// Same contract as hash_encoded_kernel (hdx_encoded.hip): every value
// [u64 BE version][u16 BE count]{[u32 BE len][bytes]}*count
// (daemon/datalayer_encodings.cc:139-217) is decoded and its attributes and
// key hashed (common/hash.cc:56-68) into coords, row-major; an undecodable
// value gives zero coordinates, version 0 and HDX_E_BADENC.
//
// The gather sweep walks each value's length prefixes in global memory and
// then re-reads the values to hash them: the walk touches every line, the
// lines are evicted before the hash passes, so the values cross
// HBM twice.  Here one wave owns G objects:
//   1. per object its key and value chunks (16-byte units) are copied into a
//      wave-private LDS window by LDS DMA, object by object (lane = chunk;
//      per-lane sources, so any layout works) — the bytes cross HBM once;
//   2. lane = object walks its value's prefixes in LDS (dword-aligned
//      ds_read + v_alignbyte: no HBM round trip per prefix);
//   3. passes of 64 slots in slot order hash out of LDS (hdx_lds_hash.h) and
//      store their coordinates coalesced.
// A group that does not fit the window is walked and hashed from global
// memory in the same wave (identical results).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_lds_hash.h"
#include "hdx_loads.h"

namespace hdx {


namespace {

typedef uint32_t __attribute__((aligned(1))) eu32_u;
typedef uint64_t __attribute__((aligned(1))) eu64_u;
typedef uint16_t __attribute__((aligned(1))) eu16_u;

__device__ __forceinline__ uint32_t g_be32(const uint8_t* p) {
    return __builtin_bswap32(*(const __attribute__((address_space(1))) eu32_u*)p);
}
__device__ __forceinline__ uint64_t g_be64(const uint8_t* p) {
    return __builtin_bswap64(*(const __attribute__((address_space(1))) eu64_u*)p);
}
__device__ __forceinline__ uint32_t g_be16(const uint8_t* p) {
    const uint16_t v = *(const __attribute__((address_space(1))) eu16_u*)p;
    return (uint32_t)(uint16_t)((v >> 8) | (v << 8));
}

constexpr uint32_t kEZero = 0xffffffffu;

struct alignas(8) EDesc {
    uint32_t off;  // staged: byte offset in the window; global: offset in the value (key: 0)
    uint32_t len;
};

// Static LDS (a separate object from the window: descriptor work never waits
// for the window's DMA).
template <int G>
struct EncStagedMeta {
    EDesc desc[G * 32];      // A <= 32; then the parked coordinates (SORT)
    uint16_t perm[G * 32];   // SORT: slots in class order
    uint32_t cnt[8];
    uint64_t voff[G], koff[G];
    uint8_t codes[256];
};

}  // namespace

template <int G, bool SORT>
__global__ void __launch_bounds__(64)
hash_encoded_staged_kernel(const EncodedArgs a, uint32_t WB) {
    extern __shared__ __attribute__((aligned(16))) uint8_t win[];
    __shared__ EncStagedMeta<G> meta;
    static_assert(G <= 64, "G objects per wave");
    const ldsw_t w = as_ldsw(win);
    const int lane = threadIdx.x;
    const uint32_t A = a.A;
    const uint64_t o0 = (uint64_t)blockIdx.x * G;
    if (o0 >= a.n) return;
    const uint32_t nobj = (uint32_t)min<uint64_t>(G, a.n - o0);
    const bool mine = (uint32_t)lane < nobj;
    reinterpret_cast<uint32_t*>(meta.codes)[lane] = reinterpret_cast<const uint32_t*>(a.codes)[lane];

    // ---- metadata, chunk counts, window placement ------------------------------
    const uint64_t i = o0 + (mine ? lane : 0);
    const uint64_t voff = mine ? a.val_off[i] : 0, koff = mine ? a.key_off[i] : 0;
    const uint32_t vlen = mine ? a.val_len[i] : 0u, klen = mine ? a.key_len[i] : 0u;
    const uint8_t* vsrc = a.vals + voff;
    const uint8_t* ksrc = a.keys + koff;
    const uint32_t vlead = (uint32_t)((uintptr_t)vsrc & 15), klead = (uint32_t)((uintptr_t)ksrc & 15);
    // 16-byte units covering the key and the value (64-bit: a value may be huge)
    const uint64_t kch = mine ? ((uint64_t)klead + klen + 15) >> 4 : 0;
    const uint64_t vch = mine ? ((uint64_t)vlead + vlen + 15) >> 4 : 0;
    const uint64_t nch = kch + vch;
    const uint32_t nch32 = nch > 0xffffu ? 0xffffu : (uint32_t)nch;
    const uint32_t cstart = wave_scan_dpp(nch32) - nch32;  // object's first unit in the window
    const uint32_t total = __builtin_amdgcn_readlane(cstart + nch32, 63);
    const bool staged = __all(!mine || nch <= 0xffffu) && (uint64_t)total * 16 <= WB;
    if (mine) {
        meta.voff[lane] = voff;
        meta.koff[lane] = koff;
    }

    // ---- 1. keys + values -> LDS, object by object ------------------------------
    if (staged) {
        for (uint32_t o = 0; o < nobj; ++o) {
            const uint32_t ko = __builtin_amdgcn_readlane((uint32_t)kch, (int)o);
            const uint32_t no = __builtin_amdgcn_readlane(nch32, (int)o);
            const uint32_t st = __builtin_amdgcn_readlane(cstart, (int)o);
            const uint64_t ka = pack64(__builtin_amdgcn_readlane((uint32_t)(uintptr_t)(ksrc - klead), (int)o),
                                       __builtin_amdgcn_readlane((uint32_t)((uintptr_t)(ksrc - klead) >> 32), (int)o));
            const uint64_t va = pack64(__builtin_amdgcn_readlane((uint32_t)(uintptr_t)(vsrc - vlead), (int)o),
                                       __builtin_amdgcn_readlane((uint32_t)((uintptr_t)(vsrc - vlead) >> 32), (int)o));
            for (uint32_t c0 = 0; c0 < no; c0 += 64) {
                const uint32_t c = c0 + (uint32_t)lane;
                if (c < no) {
                    const uint64_t src = c < ko ? ka + 16ull * c : va + 16ull * (c - ko);
                    __builtin_amdgcn_global_load_lds((const void*)(uintptr_t)src,
                                                     (__attribute__((address_space(3))) void*)(win + 16 * (st + c0)),
                                                     16, 0, 0);
                }
            }
        }
        // the window is read below: every LDS-DMA of this wave must have landed
        // (the compiler does not order ds_read after global_load_lds by itself)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }

    // ---- 2. decode_value (datalayer_encodings.cc:168-217), lane = object --------
    bool ok = mine && vlen >= 10;
    uint64_t version = 0;
    EDesc* desc = meta.desc;
    if (staged) {
        const uint32_t kb = cstart * 16 + klead;               // key byte 0 in the window
        const uint32_t vb = (cstart + (uint32_t)kch) * 16 + vlead;  // value byte 0
        if (ok) version = ((uint64_t)lds_be32(w, vb) << 32) | lds_be32(w, vb + 4);
        ok = ok && (lds_be32(w, vb + 6) & 0xffffu) == A - 1;
        if (mine) desc[lane * A] = EDesc{kb, klen};
        uint32_t pos = 10;
        for (uint32_t k = 0; k + 1 < A; ++k) {
            uint32_t len = 0;
            if (ok) {
                if (vlen - pos < 4) {
                    ok = false;
                } else {
                    len = lds_be32(w, vb + pos);
                    pos += 4;
                    if (len > vlen - pos) ok = false;  // the reference does not check this (:201-213)
                }
            }
            if (mine) desc[lane * A + 1 + k] = EDesc{ok ? vb + pos : kEZero, ok ? len : 0u};
            if (ok) pos += len;
        }
    } else {
        if (ok) version = g_be64(vsrc);
        ok = ok && g_be16(vsrc + 8) == A - 1;
        if (mine) desc[lane * A] = EDesc{0u, klen};
        uint32_t pos = 10;
        for (uint32_t k = 0; k + 1 < A; ++k) {
            uint32_t len = 0;
            if (ok) {
                if (vlen - pos < 4) {
                    ok = false;
                } else {
                    len = g_be32(vsrc + pos);
                    pos += 4;
                    if (len > vlen - pos) ok = false;
                }
            }
            if (mine) desc[lane * A + 1 + k] = EDesc{ok ? pos : kEZero, ok ? len : 0u};
            if (ok) pos += len;
        }
    }
    if (mine && !ok)  // undecodable: every coordinate of the object is 0
        for (uint32_t j = 0; j < A; ++j) desc[lane * A + j] = EDesc{kEZero, 0u};
    if (mine && a.versions) a.versions[i] = ok ? version : 0;
    const bool any_bad = __any(mine && !ok);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- 3. passes of 64 slots ---------------------------------------------------
    // SORT: the non-string slots first (lean), then the strings by CityHash
    // regime and loop count (the regroup kernel's ORDER 1 classes), every
    // coordinate parked over its descriptor and stored in slot order; else
    // slot order with direct coalesced stores.
    const uint32_t ns = nobj * A;
    bool bad = false;
    uint64_t* out = a.coords + o0 * A;
    auto hash_slot = [&](uint32_t s) -> uint64_t {
        const uint32_t o = div_small(s, a.a_magic), j = s - o * A;
        const EDesc d = desc[s];
        const uint32_t code = meta.codes[j];
        if (d.off == kEZero) return 0;
        if (staged)
            return code == CODE_STRING ? hash_string_lds(w, d.off, d.len) : hash_numeric_lds(w, code, d.off, d.len, bad);
        const uint8_t* p = (j == 0 ? a.keys + meta.koff[o] : a.vals + meta.voff[o]) + d.off;
        return code == CODE_STRING
                   ? hash_blk<false, false, true>(CODE_STRING, p, d.len,
                                                  consume_any<true>(issue_any<true>(CODE_STRING, p, d.len)), bad)
                   : hash_numeric_slot(code, p, d.len, bad);
    };
    if constexpr (SORT) {
        uint32_t* cnt = meta.cnt;
        if (lane < 8) cnt[lane] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t cls[(G * 32 + 63) / 64];
#pragma unroll
        for (int c = 0; c < (G * 32 + 63) / 64; ++c) {
            const uint32_t s = (uint32_t)(c * 64 + lane);
            uint32_t k = 0;
            if (s < ns) {
                const uint32_t o = div_small(s, a.a_magic), j = s - o * A;
                const EDesc d = desc[s];
                const uint32_t n = d.len;
                if (meta.codes[j] == CODE_STRING && d.off != kEZero)
                    k = n > 64 ? (((n - 1) >> 6) >= 4 ? 7u : 3u + ((n - 1) >> 6)) : n > 32 ? 1u : n <= 16 ? 2u : 3u;
                __hip_atomic_fetch_add(&cnt[k], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            }
            cls[c] = k;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t kc = lane < 8 ? cnt[lane] : 0u;
        const uint32_t start = wave_scan_dpp(kc) - kc;
        if (lane < 8) cnt[lane] = start;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int c = 0; c < (G * 32 + 63) / 64; ++c) {
            const uint32_t s = (uint32_t)(c * 64 + lane);
            if (s < ns) {
                const uint32_t pos = __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WAVEFRONT);
                meta.perm[pos] = (uint16_t)s;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint64_t* parked = reinterpret_cast<uint64_t*>(desc);
        for (uint32_t t = (uint32_t)lane; t < ns; t += 64) {
            const uint32_t s = meta.perm[t];
            parked[s] = hash_slot(s);  // over its own, consumed, descriptor
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t s = (uint32_t)lane; s < ns; s += 64) __builtin_nontemporal_store(parked[s], out + s);
    } else {
        for (uint32_t s = (uint32_t)lane; s < ns; s += 64) __builtin_nontemporal_store(hash_slot(s), out + s);
    }
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int G, bool SORT>
static hipError_t launch_enc_staged_g(const EncodedArgs& a, uint32_t WB, hipStream_t stream) {
    if (a.A > 32) return hipErrorInvalidValue;
    const uint64_t waves = (a.n + G - 1) / G;
    if (waves > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_encoded_staged_kernel<G, SORT>), dim3((uint32_t)waves), dim3(64), WB, stream, a, WB);
    return hipGetLastError();
}

// G objects per wave (A <= 32), an LDS window of WB bytes; SORT: class-sorted
// passes with the coordinates parked in LDS.
hipError_t launch_hash_encoded_staged(const EncodedArgs& a, int G, uint32_t WB, bool sort, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    switch (G * 2 + (sort ? 1 : 0)) {
        case 4 * 2: return launch_enc_staged_g<4, false>(a, WB, stream);
        case 8 * 2: return launch_enc_staged_g<8, false>(a, WB, stream);
        case 7 * 2: return launch_enc_staged_g<7, false>(a, WB, stream);
        case 7 * 2 + 1: return launch_enc_staged_g<7, true>(a, WB, stream);
        case 3 * 2 + 1: return launch_enc_staged_g<3, true>(a, WB, stream);
        case 11 * 2 + 1: return launch_enc_staged_g<11, true>(a, WB, stream);
        case 15 * 2 + 1: return launch_enc_staged_g<15, true>(a, WB, stream);
        default: return hipErrorInvalidValue;
    }
}


}  // namespace hdx
