// hdx_encoded.hip — reindex sweep over stored objects.
//
// The daemon stores an object as a LevelDB value
//   [u64 BE version][u16 BE count]{[u32 BE len][bytes]}*count
// (daemon/datalayer_encodings.cc:139-166, decoded by decode_value :168-217)
// with the key kept in the LevelDB key.  The datalayer_indexer_thread sweep
// (daemon/datalayer_indexer_thread.cc:161-176) iterates resident objects,
// decodes each value and works per attribute; here every object is decoded
// and re-hashed (common/hash.cc:56-68) in one fused launch.
//
// One wave = 64 objects.  Phase 0: each lane touches its value's cache lines
// (one dword per 128 B, up to 4 KiB) so the parse that follows walks L2-hot
// lines.  Phase 1: each lane walks its value's length prefixes (a sequential
// chain, as in the reference) and writes one 8-byte {offset, length} slot
// descriptor per attribute into the wave's LDS, key first.  Phase 2: A passes
// of 64 slots in object-major order — adjacent lanes hash adjacent attributes
// of the same values — with the next pass's bytes in flight and one coalesced
// coordinate store per pass.  (A lane-per-object variant that overlaps the
// prefix chain with hashing and needs no LDS ran 1.35-1.5x slower.)  A value that does not decode into A-1 attributes lying
// inside its bytes yields zero coordinates and sets HDX_E_BADENC in status.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_loads.h"
#include "hdx_region_lookup.h"

namespace hdx {

typedef uint32_t __attribute__((aligned(1))) u32_u;
typedef uint64_t __attribute__((aligned(1))) u64_u;
typedef uint16_t __attribute__((aligned(1))) u16_u;

__device__ __forceinline__ uint32_t load_be32(const uint8_t* p) {
    return __builtin_bswap32(*(const __attribute__((address_space(1))) u32_u*)p);
}
__device__ __forceinline__ uint64_t load_be64(const uint8_t* p) {
    return __builtin_bswap64(*(const __attribute__((address_space(1))) u64_u*)p);
}
__device__ __forceinline__ uint32_t load_be16(const uint8_t* p) {
    const uint16_t v = *(const __attribute__((address_space(1))) u16_u*)p;
    return (uint32_t)(uint16_t)((v >> 8) | (v << 8));
}

// Compact slot descriptor: byte offset inside the object's value (or key, for
// attribute 0) and length; kZeroSlot marks a slot hashed as 0.
struct alignas(8) EncDesc {
    uint32_t off;
    uint32_t len;
};
constexpr uint32_t kZeroSlot = 0xffffffffu;

#ifndef HDX_DEBUG_BUILD
#define HDX_DEBUG_BUILD 0
#endif

// Debug library only: HDX_SWEEP_REGION_LDS=0 makes the fused sweep read the
// region tables from global memory instead of staging them in LDS (A/B runs).
static bool sweep_region_lds() {
#if HDX_DEBUG_BUILD
    static const bool v = [] {
        const char* e = getenv("HDX_SWEEP_REGION_LDS");
        return !(e && e[0] == '0');
    }();
    return v;
#else
    return true;
#endif
}
// Wave-private LDS: G object bases {value, key}, the code table, the pass
// attribute list (numeric walk only), descriptors.
__host__ __device__ constexpr size_t encoded_lds_per_wave(uint32_t A, uint32_t G = 64, bool NW = false) {
    return G * 16 + 256 + (NW ? 256 : 0) + (size_t)G * A * sizeof(EncDesc);
}

// G objects per wave (lanes G..63 idle in phase 1).  SHAPE (debug variants
// 57/58 only, wrong coordinates): 1 = the walk alone (no phase 2), 2 = phase
// 2's loads without the hash arithmetic.  REGIONS: a wave holds all of its
// objects' coordinates (G*A slots), so it also looks every object up in the
// T region tables (hdx_region_lookup.h) — phase 2 parks each coordinate over
// its consumed descriptor, phase 3 has one lane per object.
// NW (numeric walk): the walk hashes every non-string value attribute as it
// reads its prefix — the prefix and the 8 value bytes come from two loads
// issued together, the type is wave-uniform (one schema) — and parks the
// coordinate; the hash passes then cover only the key and the strings
// (a.p2), and the wave stores its G * A coordinates from LDS at the end.
// SPEC (with NW): a run of consecutive int64 / float / timestamp attributes is
// read in one round trip — every prefix and value at the position it has if
// the run's values are all 8 bytes — then checked in order; from the first
// prefix that is not 8 on, that lane reads the rest of the run one prefix at
// a time.  The prefix walk is a chain of dependent loads, and this takes
// R - 1 links out of it for a run of R fixed-size values.
template <bool TOUCH, bool A4 = false, int SHAPE = 0, int G = 64, bool REGIONS = false, bool NW = false,
          bool SPEC = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8)))
hash_encoded_kernel(const EncodedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const uint32_t A = a.A;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    // REGIONS: the tables' indexes and ids, one copy per workgroup, first
    uint64_t* tbl = reinterpret_cast<uint64_t*>(smem_raw);
    if constexpr (REGIONS) {
        for (uint32_t t = 0; t < a.T; ++t) {
            const SweepTable& tb = a.t[t];
            if (tb.lds_index == 0xffffffffu) continue;
            for (uint32_t k = threadIdx.x; k < tb.index_words; k += blockDim.x) tbl[tb.lds_index + k] = tb.index[k];
            for (uint32_t k = threadIdx.x; k < tb.R; k += blockDim.x) tbl[tb.lds_ids + k] = tb.ids[k];
        }
        __syncthreads();  // the kernel's only workgroup barrier (before any wave may exit)
    }
    // wave-private LDS: G object bases {value, key}, the code table, descriptors
    uint8_t* wsmem = smem_raw + (REGIONS ? (size_t)a.lds_tables * 8 : 0) + (size_t)w * encoded_lds_per_wave(A, G, NW);
    uint64_t* bases = reinterpret_cast<uint64_t*>(wsmem);           // [G][2]
    uint8_t* codes = wsmem + G * 16;                                 // [256]
    uint8_t* p2 = wsmem + G * 16 + 256;                              // [256] (NW only)
    EncDesc* desc = reinterpret_cast<EncDesc*>(wsmem + G * 16 + 256 + (NW ? 256 : 0));
    bool bad = false;
    const uint64_t o0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + w) * G;
    if (o0 >= a.n) return;  // no barrier after this point: waves are independent
    const uint32_t nobj = (uint32_t)min<uint64_t>(G, a.n - o0);
    const bool valid = (uint32_t)lane < nobj;
    const uint64_t i = o0 + (valid ? lane : 0);

    const uint64_t voff = valid ? a.val_off[i] : 0, koff = valid ? a.key_off[i] : 0;
    const uint32_t vlen = valid ? a.val_len[i] : 0u, klen = valid ? a.key_len[i] : 0u;
    const uint8_t* v = a.vals + voff;
    if (lane < G) {
        bases[2 * lane] = voff;
        bases[2 * lane + 1] = koff;
    }
    for (uint32_t j = lane; j < A; j += 64) codes[j] = a.codes[j];
    if constexpr (NW)
        for (uint32_t j = lane; j < a.S; j += 64) p2[j] = a.p2[j];

    // phase 0: pull the value's lines toward L2 (independent loads, consumed late)
    uint32_t sink = 0;
    if (TOUCH) {
        const uint32_t touch = vlen >= 4 ? min(vlen - 3, 4096u) : 0u;
        for (uint32_t off = 0; off < touch; off += 128)
            sink ^= *(const __attribute__((address_space(1))) u32_u*)(v + off);
    }

    // phase 1: decode_value (datalayer_encodings.cc:168-217) into descriptors
    bool ok = valid && vlen >= 10;
    const uint64_t version = ok ? load_be64(v) : 0;
    ok = ok && load_be16(v + 8) == A - 1;
    if (valid) desc[lane * A] = EncDesc{0u, klen};
    uint32_t pos = 10;
    uint64_t* parked = reinterpret_cast<uint64_t*>(desc);  // coordinate of slot s over desc[s]
    for (uint32_t k = 0; k + 1 < A; ++k) {
        uint32_t len = 0;
        const uint32_t cj = a.codes[k + 1];  // wave-uniform (scalar load)
        if (SPEC && cj >= CODE_INT64) {
            constexpr uint32_t kRun = 8;
            uint32_t R = 1;  // wave-uniform run length (scalar loop over the codes)
            while (R < kRun && k + 1 + R < A && a.codes[k + 1 + R] >= CODE_INT64) ++R;
            uint32_t hd[kRun];
            uint64_t bits[kRun];
#pragma unroll
            for (uint32_t m = 0; m < kRun; ++m) {
                const bool room = m < R && ok && vlen - pos >= 12 * (m + 1);
                hd[m] = room ? load_be32(v + pos + 12 * m) : 0u;
                bits[m] = room ? *(const __attribute__((address_space(1))) u64_u*)(v + pos + 12 * m + 4) : 0;
            }
            bool spec = true;
#pragma unroll
            for (uint32_t m = 0; m < kRun; ++m) {
                if (m >= R) break;
                const uint32_t cm = a.codes[k + 1 + m];
                uint64_t h = 0;
                if (ok) {
                    if (vlen - pos < 4) {
                        ok = false;
                    } else {
                        uint32_t lm;
                        uint64_t b;
                        if (spec && hd[m] == 8 && vlen - pos >= 12) {
                            lm = 8;
                            b = bits[m];
                        } else {  // off the predicted positions: one prefix at a time
                            spec = false;
                            lm = load_be32(v + pos);
                            b = lm == 8 && vlen - pos >= 12 ? *(const __attribute__((address_space(1))) u64_u*)(v + pos + 4)
                                                            : 0;
                        }
                        pos += 4;
                        if (lm > vlen - pos) ok = false;
                        else if (lm == 8) h = hash_numeric(cm, b);
                        else if (lm == 0) h = hash_numeric(cm, 0);
                        else bad = true;
                        if (ok) pos += lm;
                    }
                }
                if (valid) parked[lane * A + 1 + k + m] = ok ? h : 0;
            }
            k += R - 1;
            continue;
        }
        if (NW && cj != CODE_STRING) {
            uint64_t h = 0;
            if (ok) {
                if (vlen - pos < 4) {
                    ok = false;
                } else {
                    // the 8 value bytes are read with the prefix when the value has room for them
                    const bool room = vlen - pos >= 12;
                    len = load_be32(v + pos);
                    const uint64_t bits = room ? *(const __attribute__((address_space(1))) u64_u*)(v + pos + 4) : 0;
                    pos += 4;
                    if (len > vlen - pos) ok = false;
                    else if (cj == CODE_ZERO) h = 0;                  // datatype_info.cc:169-180
                    else if (len == 8) h = hash_numeric(cj, bits);
                    else if (len == 0) h = hash_numeric(cj, 0);
                    else bad = true;                                   // the reference asserts
                }
            }
            if (valid) parked[lane * A + 1 + k] = ok ? h : 0;
            if (ok) pos += len;
            continue;
        }
        if (ok) {
            if (vlen - pos < 4) {
                ok = false;
            } else {
                len = load_be32(v + pos);
                pos += 4;
                if (len > vlen - pos) ok = false;  // the reference does not check this (:201-213)
            }
        }
        if (valid) desc[lane * A + 1 + k] = EncDesc{ok ? pos : kZeroSlot, ok ? len : 0u};
        if (ok) pos += len;
    }
    if (valid && !ok)  // undecodable: every coordinate of the object is 0
        for (uint32_t j = 0; j < A; ++j) {
            if (NW && j > 0 && codes[j] != CODE_STRING) parked[lane * A + j] = 0;
            else desc[lane * A + j] = EncDesc{kZeroSlot, 0u};
        }
    if (valid && a.versions) a.versions[i] = ok ? version : 0;
    const bool any_bad = __any(valid && !ok);
    if (TOUCH) asm volatile("; touch sink %0" ::"v"(sink));  // keeps the phase-0 loads live
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    const uint32_t nslots = nobj * A;
    // phase 2: passes of 64 slots (slot s = object * A + attribute; NW: pass
    // slot q = object * S + its index in a.p2).  The object's bases and the attribute's code are
    // read from LDS, not from other lanes: in a partial pass the lanes past the
    // batch end are inactive, and a ds_bpermute from an inactive lane returns 0.
    constexpr bool PARK = REGIONS || NW;  // coordinates parked over their descriptors
    const uint32_t nq = NW ? nobj * a.S : nslots;
    const uint32_t npass = SHAPE == 1 ? 0 : (nq + 63) / 64;
    if (SHAPE == 1) {
        for (uint32_t s = lane; s < nslots; s += 64) a.coords[o0 * A + s] = desc[s].off;
        return;
    }
    uint64_t* out = a.coords ? a.coords + o0 * A : nullptr;
    struct Pass {
        const uint8_t* p;
        uint32_t n, code, s;
        Raw blk;
    };
    auto load_pass = [&](uint32_t t, Pass& P) {
        const uint32_t q = t * 64 + (uint32_t)lane;
        uint32_t s, obj, j;
        if constexpr (NW) {
            const uint32_t qq = min(q, nq - 1);
            obj = div_small(qq, a.s_magic);
            j = p2[qq - obj * a.S];
            s = obj * A + j;
        } else {
            s = min(q, nslots - 1);
            obj = div_small(s, a.a_magic);  // s < 64 * A
            j = s - obj * A;
        }
        const EncDesc d = desc[s];
        const uint64_t base = bases[2 * obj + (j == 0)];
        const bool zero = d.off == kZeroSlot || q >= nq;
        P.s = q < nq ? s : 0xffffffffu;
        P.code = zero ? (uint32_t)CODE_ZERO : (uint32_t)codes[j];
        P.n = zero ? 0u : d.len;
        P.p = zero ? g_zero_pad : (j == 0 ? a.keys : a.vals) + base + d.off;
        P.blk = issue_any<A4>(P.code, P.p, P.n);
    };
    Pass P0, P1;
    load_pass(0, P0);
    for (uint32_t t = 0;; t += 2) {
        if (t + 1 < npass) load_pass(t + 1, P1);
        {
            const uint64_t h = SHAPE == 2 ? touch_blk(P0.code, P0.p, P0.n, consume_any<A4>(P0.blk))
                                          : hash_blk<false, false, A4>(P0.code, P0.p, P0.n, consume_any<A4>(P0.blk), bad);
            if (P0.s != 0xffffffffu) {
                if (!PARK) __builtin_nontemporal_store(h, out + P0.s);
                else parked[P0.s] = h;
            }
        }
        if (t + 1 >= npass) break;
        if (t + 2 < npass) load_pass(t + 2, P0);
        {
            const uint64_t h = SHAPE == 2 ? touch_blk(P1.code, P1.p, P1.n, consume_any<A4>(P1.blk))
                                          : hash_blk<false, false, A4>(P1.code, P1.p, P1.n, consume_any<A4>(P1.blk), bad);
            if (P1.s != 0xffffffffu) {
                if (!PARK) __builtin_nontemporal_store(h, out + P1.s);
                else parked[P1.s] = h;
            }
        }
        if (t + 2 >= npass) break;
    }
    if constexpr (PARK) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (out)  // the wave's G * A coordinates, coalesced, in slot order
            for (uint32_t s = lane; s < nslots; s += 64) __builtin_nontemporal_store(parked[s], out + s);
    }
    if constexpr (REGIONS) {
        // phase 3: lane = object; configuration::lookup_region per table
        // the tables in a wave-uniform loop, one lane per object: a table's
        // fields are then scalar loads (one lane per (table, object) pair
        // read every field per lane: 0.60 vs 0.47 ms in the batch kernel's
        // fused form, config 2)
        for (uint32_t t = 0; t < a.T; ++t) {
            const SweepTable& tb = a.t[t];
            for (uint32_t o = lane; o < nobj; o += 64) {
                const uint64_t* po = parked + o * A;
                if (tb.lds_index != 0xffffffffu) {
                    tb.out[o0 + o] = lookup_indexed_fn(tbl + tb.lds_index, tb.W, tb.D,
                                                       [&](uint32_t d) { return po[tb.attrs[d]]; }, tbl + tb.lds_ids);
                    continue;
                }
                uint64_t h[kMaxLookupDims];
#pragma unroll
                for (uint32_t d = 0; d < kMaxLookupDims; ++d)
                    if (d < tb.D) h[d] = po[tb.attrs[d]];
                tb.out[o0 + o] = tb.index ? lookup_indexed(tb.index, tb.W, tb.D, h, tb.ids)
                                          : lookup_scan(tb.lower, tb.upper, tb.ids, tb.R, tb.D, h);
            }
        }
    }
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <bool TOUCH, bool A4, int SHAPE = 0, int G = 64, bool REGIONS = false, bool NW = false, bool SPEC = false>
static hipError_t launch_encoded(const EncodedArgs& a_in, hipStream_t stream) {
    EncodedArgs a = a_in;
    if constexpr (NW) {  // the attributes left to the hash passes: the key and every string
        a.S = 0;
        for (uint32_t j = 0; j < a.A; ++j)
            if (j == 0 || a.codes[j] == CODE_STRING) a.p2[a.S++] = (uint8_t)j;
        a.s_magic = (uint32_t)(((1ull << 31) + a.S - 1) / a.S);
    }
    // 4 waves per workgroup while they fit in 64 KiB of LDS (A <= 61 at G = 32), else 1
    const size_t per_wave = encoded_lds_per_wave(a.A, G, NW);
    const uint32_t waves_per_block = 4 * per_wave <= 65536 ? 4 : 1;
    const uint64_t waves = (a.n + G - 1) / G;
    uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_encoded_kernel<TOUCH, A4, SHAPE, G, REGIONS, NW, SPEC>), dim3((uint32_t)blocks), dim3(64 * waves_per_block),
                       waves_per_block * per_wave + (REGIONS ? (size_t)a.lds_tables * 8 : 0), stream, a);
    return hipGetLastError();
}

hipError_t launch_hash_encoded(const EncodedArgs& a_in, hipStream_t stream) {
    if (a_in.n == 0) return hipSuccess;
    EncodedArgs a = a_in;
    if (a.A > kWsweepMaxAttrs || hash_variant() == 301) {
        // wide schemas (hdx_wide.hip): the wide sweep, then one lookup launch
        // per table (debug variant 301: at any A)
        const RegionHashFn hash = [&](uint64_t first, uint64_t count, uint64_t* c) {
            EncodedArgs b = a;
            b.key_off += first;
            b.key_len += first;
            b.val_off += first;
            b.val_len += first;
            if (b.versions) b.versions += first;
            b.n = count;
            b.coords = c;
            b.T = 0;
            return launch_hash_sweep_wide(b, stream);
        };
        if (!a.T) return launch_hash_sweep_wide(a, stream);
        bool no_scratch = false;
        const hipError_t e = regions_by_lookup(a.n, a.A, a.t, a.T, a.coords, hash, stream, &no_scratch);
        return no_scratch ? hipErrorOutOfMemory : e;
    }
    a.a_magic = (uint32_t)(((1ull << 31) + a.A - 1) / a.A);
    // default: dword-aligned loads (5.49 vs 6.14 ms per 10 M config-3b objects,
    // profiles/r1/ab_a4_cfg5.jsonl), 32 objects per wave (5.05 vs 5.31 ms for
    // 64 (variant 47) and 5.88 for 16 (48), ab_cfg5_objects_per_wave.jsonl);
    // variant 43 = byte-addressed loads, 64 objects per wave, variant 33 adds
    // the phase-0 line touch to those (measured 11 % slower, r1u).
    // Retired (profiles/r1/ab_cfg5_*.jsonl): class-sorted passes over the whole
    // wave or over groups of 2 / 4 passes, 16 / 32 objects per wave, and a
    // lane-per-object walk-and-hash kernel — all slower
    if (a.T) {
        // the wave-staged sweep, then one lookup launch per table (chunked
        // through scratch when the caller wants no coordinates): 25.8 ms at
        // 50 M objects and the two tables of bench.py vs 27.3 for the gather
        // sweep's fused form (debug 234, and below kRegionLookupMinObjects)
        // and 28.5 for the wave-staged sweep with the lookup fused (debug 233:
        // its 6 objects per wave make the lookups' L2 round trips the wave's
        // tail; profiles/r3/ab_fused_sweep.jsonl, ab_regions_by_lookup.jsonl)
        if (a.A <= kWsweepMaxAttrs && regions_by_lookup_pays(a.n)) {
#if HDX_DEBUG_BUILD
            if (hash_variant() == 233) return launch_hash_wsweep_product(a, stream);
            if (hash_variant() != 234)
#endif
            {
                const RegionHashFn hash = [&](uint64_t first, uint64_t count, uint64_t* c) {
                    EncodedArgs b = a;
                    b.key_off += first;
                    b.key_len += first;
                    b.val_off += first;
                    b.val_len += first;
                    if (b.versions) b.versions += first;
                    b.n = count;
                    b.coords = c;
                    b.T = 0;
                    return launch_hash_wsweep_product(b, stream);
                };
                bool no_scratch = false;
                const hipError_t e = regions_by_lookup(a.n, a.A, a.t, a.T, a.coords, hash, stream, &no_scratch);
                if (!no_scratch) return e;
                // no scratch for the coordinates: the gather sweep's fused form below
            }
        }
        // stage each indexed table (index + ids) in LDS while they fit in 16 KiB together
        uint32_t words = 0;
        for (uint32_t t = 0; t < a.T; ++t) {
            SweepTable& tb = a.t[t];
            tb.lds_index = tb.lds_ids = 0xffffffffu;
            const uint32_t need = tb.index_words + tb.R;
            if (tb.index && sweep_region_lds() && (words + need) * 8 <= 16384) {
                tb.lds_index = words;
                tb.lds_ids = words + tb.index_words;
                words += (need + 1) & ~1u;  // keep 16-byte alignment
            }
        }
        a.lds_tables = words;
#if HDX_DEBUG_BUILD
        if (hash_variant() == 47) return launch_encoded<false, true, 0, 64, true>(a, stream);
#endif
        return launch_encoded<false, true, 0, 32, true>(a, stream);
    }
#if HDX_DEBUG_BUILD
    switch (hash_variant()) {
        case 43: return launch_encoded<false, false>(a, stream);
        case 33: return launch_encoded<true, false>(a, stream);
        case 57: return launch_encoded<false, true, 1>(a, stream);  // debug shape: the walk alone (WRONG coords)
        case 58: return launch_encoded<false, true, 2>(a, stream);  // debug shape: phase 2 loads only (WRONG coords)
        case 47: return launch_encoded<false, true, 0, 64>(a, stream);
        // numeric walk (non-string value attributes hashed during the walk): 32 / 64 objects per wave
        case 170: return launch_encoded<false, true, 0, 32, false, true>(a, stream);
        case 171: return launch_encoded<false, true, 0, 64, false, true>(a, stream);
        case 172: return launch_encoded<false, true, 0, 16, false, true>(a, stream);
        // ... plus runs of fixed-size values read in one round trip: 32 / 64 objects per wave
        case 173: return launch_encoded<false, true, 0, 32, false, true, true>(a, stream);
        case 174: return launch_encoded<false, true, 0, 64, false, true, true>(a, stream);
        case 48: return launch_encoded<false, true, 0, 16>(a, stream);
        // wave-staged (hdx_wsweep_dbg.hip): 230 6 objects / 2 passes, 231 7 objects, 232 11 objects / 3 passes,
        // 236 = 230 without the pass-boundary gap, 237 / 238 its debug shapes (no hash / no hash, no walk),
        // 239 = 230 with the one-block > 64-byte loop, 242 without the shared final mix16,
        // 243 with the DMA as inline asm, 244 with the pass loop not unrolled, 245 with the
        // branchy class, 246 without TNUM
        case 230: case 231: case 232: case 236: case 237: case 238: case 239: case 242: case 243: case 244: case 245: case 246: {
            const hipError_t e = launch_hash_wsweep(a, stream, hash_variant() - 230);
            if (e != hipErrorInvalidValue) return e;
            break;
        }
        case 256: case 257: case 258: case 259: case 270: case 271: case 272: case 273: {  // the product sweep with one / two waves per
            // workgroup, 7.75 KiB windows, four waves; 270: XCD-aware block order; 271: 7 objects per wave
            const int v = hash_variant();
            const hipError_t e = launch_hash_wsweep(a, stream, v == 270 ? 27 : v == 271 ? 28 : v == 272 ? 29 : v == 273 ? 30
                                                                                                     : v - 256 + 23);
            if (e != hipErrorInvalidValue) return e;
            break;
        }
        case 277: {  // the product sweep without wave priorities
            const hipError_t e = launch_hash_wsweep(a, stream, 31);
            if (e != hipErrorInvalidValue) return e;
            break;
        }
        case 313: case 314: case 315: {  // the product sweep's debug shapes: no hash / no hash, no walk / no copy, no walk
            const hipError_t e = launch_hash_wsweep(a, stream, hash_variant() - 313 + 38);
            if (e != hipErrorInvalidValue) return e;
            break;
        }
        case 298: {  // the product sweep before LOOP 4 (LOOP 13: two head reads per divergent pass)
            const hipError_t e = launch_hash_wsweep(a, stream, 37);
            if (e != hipErrorInvalidValue) return e;
            break;
        }
        case 250: case 251: case 252: case 253: case 254: case 255: {  // the product sweep without the record
            // span; 251 also with round 3's dword key gather; 252 its debug shape: no copy, no walk, the hash on
            // made-up descriptors; 253 / 254 the product's non-record / record forms with round 3's per-KiB span
            // copy; 255 the non-record form with round 3's walk reads (dword pairs + v_alignbyte)
            const hipError_t e = launch_hash_wsweep(a, stream, hash_variant() - 250 + 17);
            if (e != hipErrorInvalidValue) return e;
            break;
        }
        default: break;
    }
    // 49: the gather sweep (the product's sweep up to round 2), for A/B runs
    if (hash_variant() == 49) return launch_encoded<false, true, 0, 32>(a, stream);
#endif
    // the wave-staged sweep (hdx_wsweep.h): 4.65 vs 5.10 ms per 10 M
    // config-3b objects, 24.2 vs 25.1 ms at 50 M (profiles/r3/ab_wsweep.jsonl)
    if (a.coords) {
        const hipError_t e = launch_hash_wsweep_product(a, stream);
        if (e != hipErrorInvalidValue) return e;
    }
    return launch_encoded<false, true, 0, 32>(a, stream);
}

}  // namespace hdx
