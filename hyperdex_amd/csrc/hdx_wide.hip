// hdx_wide.hip — schemas wider than the packed-code kernels take.
//
// The reference's schema holds up to 65535 attributes (schema::attrs_sz is a
// u16, common/schema.h:49; hash() loops over all of them, common/hash.cc:
// 64-67; encode_value writes up to 65535, daemon/datalayer_encodings.cc:145).
// The product kernels keep each wave's attribute classes in one VGPR (256
// one-byte codes) or stage whole objects in an LDS window (128 slots), so
// wider schemas run here, with the classes in device memory (codes_dev):
//   hash_wide_kernel        — packed batches with A > 256: one wave per
//                             object, 64 attributes per step (lengths
//                             coalesced, a DPP scan plus a carry gives the
//                             offsets, each lane hashes its attribute from
//                             global memory with the A4 loads, one coalesced
//                             coordinate store);
//   sweep_wide_walk_kernel + sweep_wide_hash_kernel — stored objects with
//                             A > 128: a lane per object walks the value's
//                             [u32 BE len] chain, writing each attribute's
//                             {offset, length} where its coordinate goes; a
//                             wave per object then hashes 64 attributes a step (daemon/datalayer_encodings.cc:
//                             168-217, as the sweep of hdx_wsweep.hip: the header, the
//                             count == A - 1, every prefix and attribute inside
//                             the value, else zero coordinates, version 0 and
//                             HDX_E_BADENC).
// Such schemas are rare; these kernels are correct at any width and sized for
// that, not tuned.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_lds_hash.h"
#include "hdx_loads.h"
#include "hdx_regroup.h"

#ifndef HDX_DEBUG_BUILD
#define HDX_DEBUG_BUILD 0
#endif

namespace hdx {

typedef __attribute__((address_space(3))) void* lds_void_t;

namespace {
// the wave's LDS accesses ordered (the class sort's phases, a window's reuse)
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
}  // namespace

// One attribute from global memory, any class (hash_blk on the A4 pieces).
__device__ __forceinline__ uint64_t hash_one(uint32_t code, const uint8_t* p, uint32_t n, bool& bad) {
    const Raw r = issue_block_a4(code, p, n);
    return hash_blk<false, false, true>(code, p, n, funnel_raw(r), bad);
}

__global__ void __launch_bounds__(256) hash_wide_kernel(const BatchArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t A = a.A;
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < a.n; i += nwaves) {
        const uint8_t* obj = a.blob + a.obj_base[i];
        const uint32_t* len = a.attr_len + i * A;
        uint64_t* out = a.coords + i * A;
        uint32_t carry = 0;  // an object's attributes total < 4 GiB
        for (uint32_t j0 = 0; j0 < A; j0 += 64) {
            const uint32_t j = j0 + lane;
            const bool v = j < A;
            const uint32_t L = v ? len[j] : 0u;
            const uint32_t incl = wave_scan_dpp(L);
            const uint32_t off = carry + incl - L;
            carry += __builtin_amdgcn_readlane(incl, 63);
            const uint32_t code = v ? (uint32_t)a.codes_dev[j] : (uint32_t)CODE_ZERO;
            const uint64_t h = hash_one(code, obj + off, L, bad);
            if (v) out[j] = h;
        }
    }
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

hipError_t launch_hash_wide(const BatchArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    if (!a.codes_dev) return hipErrorInvalidValue;
    const uint64_t blocks = std::min<uint64_t>((a.n + 3) / 4, 1ull << 20);  // 4 objects per block, grid-stride
    hipLaunchKernelGGL(hash_wide_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

// Unaligned big-endian reads of the value header and prefixes: the dwords
// holding the first and last byte (never outside the value's pages).
__device__ __forceinline__ uint32_t be32_at(const uint8_t* p) {
    const uint32_t r = (uint32_t)(uintptr_t)p & 3;
    const uint32_t d0 = gld4(dw_floor(p)), d1 = gld4(dw_floor(p + 3));
    return __builtin_bswap32(__builtin_amdgcn_alignbyte(d1, d0, r));
}
__device__ __forceinline__ uint64_t be64_at(const uint8_t* p) {
    const uint32_t r = (uint32_t)(uintptr_t)p & 3;
    const uint8_t* a = dw_floor(p);
    const uint32_t d0 = gld4(a), d1 = gld4(a + 4), d2 = gld4(dw_floor(p + 7));
    return __builtin_bswap64(pack64(__builtin_amdgcn_alignbyte(d1, d0, r), __builtin_amdgcn_alignbyte(d2, d1, r)));
}

// Two launches (round 6).  A wave per object walking its value's prefix chain
// left 63 lanes idle behind one dependent read per attribute: from global
// memory A = 200 / 1000 ran at 0.09 of the HBM roofline, from an LDS window
// of the value at 0.13 (profiles/r6/wide_*.jsonl).  Here the walk is a lane
// per object — thousands of chains advance side by side, each step's read an
// L2 hit of the line the previous step touched — and writes each attribute's
// {offset, length} into its coordinate's place; the hash launch then reads
// them coalesced, a wave per object and 64 attributes per step, and
// overwrites them with the coordinates.
constexpr uint64_t kWideZero = ~0ull;  // a coordinate of 0 (the object does not decode)

// The walk reads each prefix with ONE unaligned dword load (gfx950 serves
// them): the chains of all objects advance together and HBM lines are the
// bound (a dword-pair read per step measured 1.42 ms for A = 200 at 200 k
// objects); an in-chain prefetch cannot help — loads complete in order, so
// the next step's wait would also wait out the prefetch — and eight chains
// per wave walking per-object 2 KiB LDS windows lose to the refills' latency
// (3.87 vs 2.52 ms, profiles/r6/ab_wide_walk.jsonl).
typedef uint32_t __attribute__((aligned(1))) u32_unaligned;

// G: descriptors buffered in registers and stored G at a time (G = 1: one
// store per step).  Stored one per step, a lane's 8-byte descriptors reach
// its row's lines ~16 steps apart, each as a partial write: WRITE_SIZE 1.29 GB
// for 0.32 GB of descriptors at A = 200 (profiles/r6/pmc_wide_walk.txt); G
// back-to-back stores fill 8 G contiguous bytes while the line is in L2.
template <uint32_t G>
__global__ void __launch_bounds__(256) sweep_wide_walk_kernel(const EncodedArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool badenc = false;
    if (i < a.n) {
        const uint32_t A = a.A;
        const uint8_t* v = a.vals + a.val_off[i];
        const uint32_t vlen = a.val_len[i];
        uint64_t* out = a.coords + i * A;
        // :174-192 version and count
        bool ok = vlen >= 10;
        uint64_t version = 0;
        if (ok) {
            version = be64_at(v);
            ok = (be32_at(v + 6) & 0xffffu) == A - 1;  // the u16 at bytes 8..9
        }
        uint32_t pos = 10;  // pos <= vlen throughout
        // :198-213, and every attribute inside the value
        for (uint32_t j0 = 1; ok && j0 < A; j0 += G) {
            uint64_t d[G];
#pragma unroll
            for (uint32_t k = 0; k < G; ++k) {
                d[k] = 0;
                if (ok && j0 + k < A) {
                    if (vlen - pos < 4) {
                        ok = false;
                    } else {
                        const uint32_t L =
                            __builtin_bswap32(*(const __attribute__((address_space(1))) u32_unaligned*)(v + pos));
                        pos += 4;
                        if (L > vlen - pos) {
                            ok = false;
                        } else {
                            d[k] = (uint64_t)pos | ((uint64_t)L << 32);
                            pos += L;
                        }
                    }
                }
            }
            if (!ok) break;
#pragma unroll
            for (uint32_t k = 0; k < G; ++k)
                if (j0 + k < A) out[j0 + k] = d[k];
        }
        out[0] = ok ? 0 : kWideZero;
        if (!ok) {
            for (uint32_t j = 1; j < A; ++j) out[j] = kWideZero;
            version = 0;
            badenc = true;
        }
        if (a.versions) a.versions[i] = version;
    }
    if (a.status && __any(badenc) && (threadIdx.x & 63) == 0) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
}

// 64 attributes per step in schema order.  SORT (debug 311): each window of
// 256 attributes counting-sorted by CityHash regime (class_sort,
// hdx_regroup.h) and hashed in 4 passes of 64, the window's descriptors all
// read (and kept in LDS) before any of its coordinates overwrites them —
// measured slower (A = 200: 2.27 vs 2.08 ms; A = 1000: 2.53 vs 2.13,
// profiles/r6/ab_wide_hash_sort.jsonl): the sort and the window's serial
// load -> sort -> passes chain cost more than the regimes it saves.
template <bool SORT>
__global__ void __launch_bounds__(256) sweep_wide_hash_kernel(const EncodedArgs a) {
    constexpr uint32_t W = 256;
    __shared__ uint64_t desc_all[SORT ? 4 : 1][SORT ? W : 1];
    __shared__ uint16_t perm_all[SORT ? 4 : 1][SORT ? W : 1];
    __shared__ uint32_t cnt_all[SORT ? 4 : 1][kClasses];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t A = a.A;
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + w; i < a.n; i += nwaves) {
        const uint8_t* v = a.vals + a.val_off[i];
        uint64_t* out = a.coords + i * A;
        if constexpr (SORT) {
            uint64_t* desc = desc_all[w];
            uint16_t* perm = perm_all[w];
            const uint8_t* kp = a.keys + a.key_off[i];
            const uint32_t klen = a.key_len[i];
            for (uint32_t w0 = 0; w0 < A; w0 += W) {
                const uint32_t ns = std::min(W, A - w0);
                uint32_t cls[4], cd[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint32_t s = (uint32_t)c * 64 + lane, j = w0 + s;
                    const bool in = s < ns;
                    const uint64_t d = in ? out[j] : kWideZero;
                    const bool zero = d == kWideZero;
                    const uint32_t L = zero ? 0u : j == 0 ? klen : (uint32_t)(d >> 32);
                    cd[c] = in && !zero ? (uint32_t)a.codes_dev[j] : (uint32_t)CODE_ZERO;
                    cls[c] = work_class1_bf(cd[c], L, true);
                    // the slot's byte address (48 bits) and length (16 bits; 0xffff:
                    // read it again in the pass)
                    const uint8_t* p = j == 0 ? kp : v + (uint32_t)d;
                    desc[s] = (uint64_t)(uintptr_t)p | ((uint64_t)std::min(L, 0xffffu) << 48);
                }
                class_sort<4, false>(cnt_all[w], perm, cls, cd, ns, wave_fence);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if ((uint32_t)t * 64 >= ns) break;
                    const uint32_t e = perm[t * 64 + lane];
                    const uint32_t s = e & 0xffu, code = e >> 8, j = w0 + s;
                    const bool in = s < ns;
                    const uint64_t d = desc[s];
                    uint32_t L = (uint32_t)(d >> 48);
                    const uint8_t* p = (const uint8_t*)(uintptr_t)(d & 0xffffffffffffull);
                    if (in && L == 0xffffu) L = j == 0 ? klen : (uint32_t)(out[j] >> 32);  // 64 KiB or more
                    const uint64_t h = hash_one(in ? code : (uint32_t)CODE_ZERO, p, in ? L : 0u, bad);
                    if (in) out[j] = h;
                }
                wave_fence();  // the window's LDS free for the next
            }
        } else {
            for (uint32_t j0 = 0; j0 < A; j0 += 64) {
                const uint32_t j = j0 + lane;
                const bool in = j < A;
                const uint64_t d = in ? out[j] : kWideZero;
                const bool zero = d == kWideZero;
                const uint8_t* p = j == 0 ? a.keys + a.key_off[i] : v + (uint32_t)d;
                const uint32_t L = zero ? 0u : j == 0 ? a.key_len[i] : (uint32_t)(d >> 32);
                const uint32_t code = in && !zero ? (uint32_t)a.codes_dev[j] : (uint32_t)CODE_ZERO;
                const uint64_t h = hash_one(code, p, L, bad);
                if (in) out[j] = h;
            }
        }
    }
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

#if HDX_DEBUG_BUILD
// A streaming form (round 6, late; debug variants 304-308, not the product):
// a wave per object streams
// its value through a two-chunk LDS ring by LDS DMA — chunk c + 1 in flight
// while the walk reads chunk c — and walks the prefix chain from LDS, the
// whole wave on the same (broadcast) address, the chain's position in scalar
// registers.  Every 64 attributes the wave hashes the batch it has walked,
// a lane per attribute from global memory (the lines the DMA has just brought
// through L2), and stores 64 coordinates.  Each value byte crosses HBM once
// and the walk pays LDS latency per attribute instead of an HBM round trip
// under the load of 200 k chains.  A jump past the prefetched chunk (an
// attribute longer than a chunk) loads the chunk the next prefix is in.
// Ring: chunk c (stream bytes [c CH, (c + 1) CH) of the value from its
// 16-byte floor) in half c & 1; the first dword of an even chunk also in the
// 16-byte pad after the ring, so a prefix read across the ring's end is one
// unaligned ds_read_b32.  An undecodable object (the checks of §4.4): the
// batches already stored are overwritten with zero coordinates, version 0,
// HDX_E_BADENC.
// Measured slower than the two launches above (w200: 3.35-3.55 vs 2.50 ms;
// its walk alone, debug shape 307, 3.39 ms): one chain per wave issues ~30
// scalar instructions per prefix, and a CU's scalar unit serves all of its
// waves — the walk is scalar-issue-bound where the lane-per-object walk puts
// 64 chains in each instruction (profiles/r6/ab_wide_stream.jsonl).
// SHAPE (debug forms, WRONG coordinates): 1 = no hash (a coordinate is its
// descriptor), 2 = no walk (made-up descriptors inside the value).
template <uint32_t CH, int SHAPE = 0>
__global__ void __launch_bounds__(64) sweep_wide_stream_kernel(const EncodedArgs a) {
    static_assert(CH >= 1024 && (CH & (CH - 1)) == 0, "CH: a power of two, at least 1 KiB");
    __shared__ __attribute__((aligned(16))) uint8_t ring[2 * CH + 16];
    const uint32_t lane = threadIdx.x;
    const uint64_t i = blockIdx.x;
    const uint32_t A = a.A;
    const uint8_t* v = a.vals + a.val_off[i];
    const uint32_t vlen = a.val_len[i];
    uint64_t* out = a.coords + i * A;
    const uint8_t* sb = (const uint8_t*)((uintptr_t)v & ~(uintptr_t)15);
    const uint32_t lead = (uint32_t)((uintptr_t)v & 15);
    const uint64_t S = (uint64_t)lead + vlen;  // stream bytes
    const uint64_t nch = (S + CH - 1) / CH;

    // chunk c into half c & 1: whole 16-byte units, the last partial unit as
    // dwords (never past the dword holding the value's last byte)
    uint64_t hold[2] = {~0ull, ~0ull};
    auto load = [&](uint64_t c) {
        uint8_t* dst = ring + (c & 1) * CH;
        const uint64_t u0 = c * (CH / 16), U = S >> 4;
        if (u0 < U) dma_units16<false>(sb + 16 * u0, dst, (uint32_t)std::min<uint64_t>(CH / 16, U - u0));
        const uint64_t tb = U * 16;
        const uint32_t td = ((uint32_t)(S & 15) + 3) >> 2;
        if (td && tb >= c * CH && tb < (c + 1) * CH && lane < td)
            __builtin_amdgcn_global_load_lds(sb + tb + 4 * lane, (lds_void_t)(dst + (tb - c * CH)), 4, 0, 0);
        if (!(c & 1) && lane == 0)  // the ring's wrap: an even chunk's first dword again after the ring
            __builtin_amdgcn_global_load_lds(sb + c * CH, (lds_void_t)(ring + 2 * CH), 4, 0, 0);
        hold[c & 1] = c;
    };
    // Stream bytes below `ready` have landed in the ring (and nothing the walk
    // still reads has been overwritten): the walk's steps check only that.  At
    // the edge: the chunks [t, t + 4) lies in are loaded if not held, waited
    // for, and the next chunk prefetched into the other half when it is dead.
    uint64_t ready = 0;
    auto advance = [&](uint64_t t) {
        const uint64_t c0 = t / CH, c1 = (t + 3) / CH;
        if (hold[c0 & 1] != c0 || hold[c1 & 1] != c1) {  // a jump: no DMA still in flight into a half reloaded
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (hold[c0 & 1] != c0) load(c0);
            if (hold[c1 & 1] != c1) load(c1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS DMA is not ordered before ds_read
        ready = std::min<uint64_t>(S, (c1 + 1) * CH);
        if (c1 == c0 && c0 + 1 < nch) load(c0 + 1);  // the other half is dead
    };
    auto ring_be32 = [&](uint64_t t) {
        const uint32_t r = (uint32_t)(t & (2 * CH - 1));
        return __builtin_amdgcn_readfirstlane(
            __builtin_bswap32(*(const __attribute__((address_space(3))) u32_unaligned*)(
                (const __attribute__((address_space(3))) uint8_t*)(lds_void_t)ring + r)));
    };
    if (nch) load(0);

    // :174-192 version and count
    bool ok = vlen >= 10;
    uint64_t version = 0;
    if (ok) {
        advance(lead);  // the header lies in chunk 0
        version = ((uint64_t)ring_be32(lead) << 32) | ring_be32(lead + 4);
        ok = (ring_be32(lead + 6) & 0xffffu) == A - 1;
    }
    uint32_t pos = 10;  // pos <= vlen throughout
    bool bad = false;
    for (uint32_t j0 = 0; j0 < A; j0 += 64) {
        const uint32_t jend = std::min(j0 + 64, A);
        uint32_t dpos = 0, dlen = 0;
        // :198-213, and every attribute inside the value
        for (uint32_t j = std::max(j0, 1u); ok && j < jend; ++j) {
            const uint64_t t = (uint64_t)lead + pos;
            if (vlen - pos < 4) {
                ok = false;
                break;
            }
            if (SHAPE != 2 && t + 4 > ready) advance(t);
            const uint32_t L = SHAPE == 2 ? std::min<uint32_t>(64, vlen - pos - 4) : ring_be32(t);
            pos += 4;
            if (L > vlen - pos) {
                ok = false;
                break;
            }
            if (lane == j - j0) {
                dpos = pos;
                dlen = L;
            }
            pos += L;
        }
        if (!ok) break;
        const uint32_t j = j0 + lane;
        const bool in = j < jend;
        const uint8_t* p = j == 0 ? a.keys + a.key_off[i] : v + dpos;
        const uint32_t L = j == 0 ? a.key_len[i] : dlen;
        const uint32_t code = in ? (uint32_t)a.codes_dev[j] : (uint32_t)CODE_ZERO;
        const uint64_t h = SHAPE == 1 ? (uint64_t)(uintptr_t)p ^ L : hash_one(code, p, L, bad);
        if (in) out[j] = h;
    }
    if (!ok) {
        for (uint32_t j = lane; j < A; j += 64) out[j] = 0;
        version = 0;
    }
    if (a.versions && lane == 0) a.versions[i] = version;
    if (a.status && lane == 0 && !ok) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the wave
}

template <uint32_t CH, int SHAPE = 0>
static hipError_t launch_sweep_wide_stream(const EncodedArgs& a, hipStream_t stream) {
    if (a.n > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((sweep_wide_stream_kernel<CH, SHAPE>), dim3((uint32_t)a.n), dim3(64), 0, stream, a);
    return hipGetLastError();
}

#endif  // HDX_DEBUG_BUILD

// The product: the walk, a lane per object from global memory, then the
// hash, a wave per object.
template <uint32_t G, bool SORT = false>
static hipError_t launch_sweep_wide_two(const EncodedArgs& a, hipStream_t stream) {
    const uint64_t walk_blocks = (a.n + 255) / 256;
    if (walk_blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sweep_wide_walk_kernel<G>, dim3((uint32_t)walk_blocks), dim3(256), 0, stream, a);
    const uint64_t blocks = std::min<uint64_t>((a.n + 3) / 4, 1ull << 20);  // 4 objects per block, grid-stride
    hipLaunchKernelGGL(sweep_wide_hash_kernel<SORT>, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_hash_sweep_wide(const EncodedArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    if (!a.codes_dev || !a.coords) return hipErrorInvalidValue;
#if HDX_DEBUG_BUILD
    switch (hash_variant()) {
        case 304: return launch_sweep_wide_stream<4096>(a, stream);
        case 305: return launch_sweep_wide_stream<2048>(a, stream);
        case 306: return launch_sweep_wide_stream<8192>(a, stream);
        case 307: return launch_sweep_wide_stream<4096, 1>(a, stream);  // debug shape: no hash
        case 308: return launch_sweep_wide_stream<4096, 2>(a, stream);  // debug shape: no walk
        case 309: return launch_sweep_wide_two<1>(a, stream);  // the walk's stores one per step
        case 310: return launch_sweep_wide_two<8>(a, stream);  // ... 8 at a time
        case 311: return launch_sweep_wide_two<16, true>(a, stream);  // the hash class-sorted per 256 attributes
        default: break;
    }
#endif
    return launch_sweep_wide_two<16>(a, stream);
}

}  // namespace hdx
