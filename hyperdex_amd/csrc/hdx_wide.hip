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
//   hash_sweep_wide_kernel  — stored objects with A > 128: one wave per
//                             object; the wave walks the value's [u32 BE len]
//                             chain from an LDS window of the value, 63-64
//                             attributes ahead, then hashes them (daemon/datalayer_encodings.cc:
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

// The walk reads the value's prefixes from a per-wave LDS window of the
// value's dwords (round 6; the walk from global memory paid an HBM round trip
// per attribute — A = 200 / 1000 ran at 0.09 of the HBM roofline,
// profiles/r6/wide_*.json): the window is refilled from the prefix the walk
// has reached whenever the next prefix is not inside it, with coalesced dword
// loads that stay inside the value's dwords.
constexpr uint32_t kWideWinDwords = 1024;  // 4 KiB per wave

__global__ void __launch_bounds__(64) hash_sweep_wide_kernel(const EncodedArgs a) {
    __shared__ uint32_t win[kWideWinDwords + 1];
    const uint32_t lane = threadIdx.x;
    const uint32_t A = a.A;
    bool bad = false, badenc = false;
    for (uint64_t i = blockIdx.x; i < a.n; i += gridDim.x) {
        const uint8_t* v = a.vals + a.val_off[i];
        const uint32_t vlen = a.val_len[i];
        uint64_t* out = a.coords + i * A;
        // :174-192 version and count (wave-uniform: every lane reads them)
        bool ok = vlen >= 10;
        uint64_t version = 0;
        if (ok) {
            version = be64_at(v);
            ok = (be32_at(v + 6) & 0xffffu) == A - 1;  // the u16 at bytes 8..9
        }
        const uint64_t vaddr = (uint64_t)(uintptr_t)v;
        const uint64_t vd1 = (vaddr + vlen + 3) >> 2;  // one past the value's last dword
        uint64_t wd = 0, wend = 0;                     // the window's dwords [wd, wend)
        auto refill = [&](uint32_t at) {               // the window from value byte `at`'s dword
            wd = (vaddr + at) >> 2;
            wend = std::min<uint64_t>(wd + kWideWinDwords, vd1);
            const uint32_t nd = (uint32_t)(wend - wd);
            const uint32_t* src = (const uint32_t*)(uintptr_t)(wd << 2);
            __builtin_amdgcn_wave_barrier();  // the previous window's reads are done (one wave)
            for (uint32_t d = lane; d < nd; d += 64) win[d] = src[d];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        uint32_t pos = 10;  // pos <= vlen throughout
        for (uint32_t j0 = 0; ok && j0 < A; j0 += 64) {
            const uint32_t jend = std::min(A, j0 + 64);
            // :198-213 — the wave walks this step's value attributes together
            // (every lane the same LDS reads: broadcasts); lane j - j0 keeps
            // attribute j's offset and length
            uint32_t my_off = 0, my_len = 0;
            for (uint32_t j = std::max(j0, 1u); j < jend; ++j) {
                if (vlen - pos < 4) { ok = false; break; }
                const uint64_t pa = vaddr + pos;
                if (((pa + 3) >> 2) >= wend || (pa >> 2) < wd) refill(pos);
                const uint32_t r = (uint32_t)(pa & 3), d = (uint32_t)((pa >> 2) - wd);
                const uint32_t L = __builtin_bswap32(__builtin_amdgcn_alignbyte(win[d + 1], win[d], r));
                pos += 4;
                if (L > vlen - pos) { ok = false; break; }
                if (lane == j - j0) {
                    my_off = pos;
                    my_len = L;
                }
                pos += L;
            }
            if (ok) {
                const uint32_t j = j0 + lane;
                if (j < A) {
                    const uint8_t* p = j == 0 ? a.keys + a.key_off[i] : v + my_off;
                    const uint32_t L = j == 0 ? a.key_len[i] : my_len;
                    out[j] = hash_one(a.codes_dev[j], p, L, bad);
                }
            }
        }
        if (!ok) {
            for (uint32_t j = lane; j < A; j += 64) out[j] = 0;
            version = 0;
            badenc = true;
        }
        if (a.versions && lane == 0) a.versions[i] = version;
    }
    if (a.status && lane == 0 && badenc) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

hipError_t launch_hash_sweep_wide(const EncodedArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    if (!a.codes_dev || !a.coords) return hipErrorInvalidValue;
    const uint64_t blocks = std::min<uint64_t>(a.n, 1ull << 20);
    hipLaunchKernelGGL(hash_sweep_wide_kernel, dim3((uint32_t)blocks), dim3(64), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
