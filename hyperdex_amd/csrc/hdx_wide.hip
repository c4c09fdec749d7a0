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
#include "hdx_loads.h"

namespace hdx {

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
        for (uint32_t j = 1; ok && j < A; ++j) {
            if (vlen - pos < 4) {
                ok = false;
                break;
            }
            const uint32_t L = __builtin_bswap32(*(const __attribute__((address_space(1))) u32_unaligned*)(v + pos));
            pos += 4;
            if (L > vlen - pos) {
                ok = false;
                break;
            }
            out[j] = (uint64_t)pos | ((uint64_t)L << 32);
            pos += L;
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

__global__ void __launch_bounds__(256) sweep_wide_hash_kernel(const EncodedArgs a) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint32_t A = a.A;
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < a.n; i += nwaves) {
        const uint8_t* v = a.vals + a.val_off[i];
        uint64_t* out = a.coords + i * A;
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
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

hipError_t launch_hash_sweep_wide(const EncodedArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    if (!a.codes_dev || !a.coords) return hipErrorInvalidValue;
    const uint64_t walk_blocks = (a.n + 255) / 256;
    if (walk_blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sweep_wide_walk_kernel, dim3((uint32_t)walk_blocks), dim3(256), 0, stream, a);
    const uint64_t blocks = std::min<uint64_t>((a.n + 3) / 4, 1ull << 20);  // 4 objects per block, grid-stride
    hipLaunchKernelGGL(sweep_wide_hash_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
