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
//                             168-217, as the sweep of hdx_wsweep.h: the header, the
//                             count == A - 1, every prefix and attribute inside
//                             the value, else zero coordinates, version 0 and
//                             HDX_E_BADENC).
// Such schemas are rare; these kernels are correct at any width and sized for
// that, not tuned.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "hdx_regroup.h"
#include "hdx_wide.h"

#ifndef HDX_DEBUG_BUILD
#define HDX_DEBUG_BUILD 0
#endif

namespace hdx {

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

// Two launches (round 6).  A wave per object walking its value's prefix chain
// left 63 lanes idle behind one dependent read per attribute: from global
// memory A = 200 / 1000 ran at 0.09 of the HBM roofline, from an LDS window
// of the value at 0.13 (profiles/r6/wide_*.jsonl).  Here the walk is a lane
// per object — thousands of chains advance side by side, each step's read an
// L2 hit of the line the previous step touched — and writes each attribute's
// {offset, length} into its coordinate's place; the hash launch then reads
// them coalesced, a wave per object and 64 attributes per step, and
// overwrites them with the coordinates.  Measured slower and kept in the debug
// library (hdx_wide_dbg.hip): a wave per object streaming its value through an
// LDS ring (304-308), and one launch with a lane per object walking and
// hashing (312: 2.37 vs 2.08 ms at A = 200, 3.52 vs 2.11 at A = 1000 — too few
// chains in flight, profiles/r6/ab_wide_fused.jsonl).
//
// The walk reads each prefix with ONE unaligned dword load (gfx950 serves
// them): the chains of all objects advance together and HBM lines are the
// bound (a dword-pair read per step measured 1.42 ms for A = 200 at 200 k
// objects); an in-chain prefetch cannot help — loads complete in order, so
// the next step's wait would also wait out the prefetch — and eight chains
// per wave walking per-object 2 KiB LDS windows lose to the refills' latency
// (3.87 vs 2.52 ms, profiles/r6/ab_wide_walk.jsonl).

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
        case 304: case 305: case 306: case 307: case 308: case 312:  // hdx_wide_dbg.hip
            return launch_sweep_wide_debug(a, stream, hash_variant());
        case 309: return launch_sweep_wide_two<1>(a, stream);  // the walk's stores one per step
        case 310: return launch_sweep_wide_two<8>(a, stream);  // ... 8 at a time
        case 311: return launch_sweep_wide_two<16, true>(a, stream);  // the hash class-sorted per 256 attributes
        default: break;
    }
#endif
    return launch_sweep_wide_two<16>(a, stream);
}

}  // namespace hdx
