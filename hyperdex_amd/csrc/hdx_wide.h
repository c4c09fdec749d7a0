// hdx_wide.h — helpers of the wide-schema kernels (hdx_wide.hip and the
// debug forms in hdx_wide_dbg.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_lds_hash.h"
#include "hdx_loads.h"

namespace hdx {

typedef __attribute__((address_space(3))) void* lds_void_t;

// the wave's LDS accesses ordered (the class sort's phases, a window's reuse)
__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One attribute from global memory, any class (hash_blk on the A4 pieces).
__device__ __forceinline__ uint64_t hash_one(uint32_t code, const uint8_t* p, uint32_t n, bool& bad) {
    const Raw r = issue_block_a4(code, p, n);
    return hash_blk<false, false, true>(code, p, n, funnel_raw(r), bad);
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

constexpr uint64_t kWideZero = ~0ull;  // a coordinate of 0 (the object does not decode)
typedef uint32_t __attribute__((aligned(1))) u32_unaligned;

}  // namespace hdx
