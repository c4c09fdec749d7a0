// hdx_device_hash.h — per-attribute hash arithmetic for gfx950 (device code).
//
// Bit-exact with the reference path:
//   CityHash64 v1.1            cityhash/city.cc:255-397 (+ Hash128to64, city.h:100-109)
//   ordered_encode_int64       common/ordered_encoding.cc:43-49
//   ordered_encode_double      common/ordered_encoding.cc:114-161
//   timestamp calendar hash    common/datatype_timestamp.cc:117-219
//
// Register-fed: the callers (hdx_kernels.hip) load the bytes; the 0..16-byte
// and > 64-byte CityHash regimes, which need the loads interleaved with the
// arithmetic, live there.  64-bit multiplies lower to v_mad_u64_u32 +
// v_mul_lo_u32; rotates to v_alignbit_b32; bswap to v_perm_b32.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_internal.h"

namespace hdx {

constexpr uint64_t K0 = 0xc3a5c85c97cb3127ULL;
constexpr uint64_t K1 = 0xb492b66fbe98f273ULL;
constexpr uint64_t K2 = 0x9ae16a3b2f90404fULL;
constexpr uint64_t KMUL = 0x9ddfea08eb382d69ULL;

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));


typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
// (lo, hi) -> u64 as a register pair (a shift-or would be rewritten into adds)
__device__ __forceinline__ uint64_t pack64(uint32_t lo, uint32_t hi) {
    const u32x2 t = {lo, hi};
    return __builtin_bit_cast(uint64_t, t);
}

// Rotate right by a constant 1..63 as two v_alignbit_b32 (the compiler's
// 64-bit funnel lowering takes three instructions).
__device__ __forceinline__ uint64_t ror(uint64_t v, int r) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    if (r >= 32) {
        const uint32_t t = lo; lo = hi; hi = t;
        r -= 32;
    }
    if (r == 0) return pack64(lo, hi);
    return pack64(__builtin_amdgcn_alignbit(hi, lo, r), __builtin_amdgcn_alignbit(lo, hi, r));
}
// v ^ (v >> 47): only the low word changes.
__device__ __forceinline__ uint64_t shiftmix(uint64_t v) {
    const uint32_t hi = (uint32_t)(v >> 32);
    return pack64((uint32_t)v ^ (hi >> 15), hi);
}
__device__ __forceinline__ uint64_t bswap(uint64_t v) { return __builtin_bswap64(v); }

// city.cc:268-276 (and Hash128to64 with mul = KMUL)
__device__ __forceinline__ uint64_t mix16(uint64_t u, uint64_t v, uint64_t mul) {
    uint64_t a = (u ^ v) * mul;
    a ^= a >> 47;
    uint64_t b = (v ^ a) * mul;
    b ^= b >> 47;
    return b * mul;
}

// city.cc:305-313, operands as two 16-byte vectors: lo = s[0,16), hi = s[n-16,n)
__device__ __forceinline__ uint64_t city_17to32(u64x2 lo, u64x2 hi, uint32_t n) {
    const uint64_t mul = K2 + 2ull * n;
    uint64_t a = lo.x * K1;
    uint64_t b = lo.y;
    uint64_t c = hi.y * mul;
    uint64_t d = hi.x * K2;
    return mix16(ror(a + b, 43) + ror(c, 30) + d, a + ror(b + K2, 18) + c, mul);
}

// city.cc:340-359: q0 = s[0,16), q1 = s[16,32), t0 = s[n-32,n-16), t1 = s[n-16,n)
__device__ __forceinline__ uint64_t city_33to64(u64x2 q0, u64x2 q1, u64x2 t0, u64x2 t1, uint32_t n) {
    const uint64_t mul = K2 + 2ull * n;
    uint64_t a = q0.x * K2;
    uint64_t b = q0.y;
    uint64_t c = t0.y;
    uint64_t d = t0.x;
    uint64_t e = q1.x * K2;
    uint64_t f = q1.y * 9;
    uint64_t g = t1.y;
    uint64_t h = t1.x * mul;
    uint64_t u = ror(a + g, 43) + (ror(b, 30) + c) * 9;
    uint64_t v = ((a + g) ^ d) + f + 1;
    uint64_t w = bswap((u + v) * mul) + h;
    uint64_t x = ror(e + f, 42) + c;
    uint64_t y = (bswap((v + w) * mul) + g) * mul;
    uint64_t z = e + f + c;
    a = bswap((x + z) * mul + y) + b;
    b = shiftmix((z + a) * mul + d + h) * mul;
    return b + x;
}

// city.cc:317-329: WeakHashLen32WithSeeds on four words
__device__ __forceinline__ void weak32(uint64_t w, uint64_t x, uint64_t y, uint64_t z,
                                       uint64_t a, uint64_t b, uint64_t& o0, uint64_t& o1) {
    a += w;
    b = ror(b + a + z, 21);
    uint64_t c = a;
    a += x;
    a += y;
    b += ror(a, 44);
    o0 = a + z;
    o1 = b + c;
}

// ordered_encoding.cc:43-49: x + (x >= 0 ? 2^63 : INT64_MIN) == x ^ 2^63 (mod 2^64)
__device__ __forceinline__ uint64_t encode_int64(uint64_t bits) { return bits ^ 0x8000000000000000ULL; }

// ordered_encoding.cc:114-161 on the bit pattern (no FP compare: NaN/inf/zero
// tested on fields, in the reference's order inf -> NaN -> zero -> finite).
__device__ __forceinline__ uint64_t encode_double(uint64_t bits) {
    const uint64_t FRAC = 0x000fffffffffffffULL;
    const uint64_t ex = (bits >> 52) & 0x7ff;
    if (ex == 0x7ff) {
        if ((bits & FRAC) == 0) return (bits >> 63) ? 0ULL : 0xfff0000000000002ULL;
        return 0xfff0000000000003ULL;
    }
    if ((bits << 1) == 0) return 0x8000000000000001ULL;
    if (bits >> 63) return (~bits & 0x7fffffffffffffffULL) + 1;  // sign'=0, exp^0x7ff, frac^mask, +1
    return (bits | 0x8000000000000000ULL) + 2;                     // sign'=1, +2
}

// encode_double without branches (the same cases, as selects): -bits for a
// negative finite x (~bits & 0x7fff... + 1), bits + 2^63 + 2 for a positive
// one, then ±0, ±inf and NaN override in the reference's precedence.
__device__ __forceinline__ uint64_t encode_double_sel(uint64_t bits) {
    const uint64_t EXP = 0x7ff0000000000000ULL;
    const uint64_t mag = bits & 0x7fffffffffffffffULL;
    const bool neg = (int64_t)bits < 0;
    uint64_t r = neg ? 0 - bits : bits + 0x8000000000000002ULL;
    r = mag == 0 ? 0x8000000000000001ULL : r;
    const uint64_t special = mag == EXP ? (neg ? 0ULL : 0xfff0000000000002ULL) : 0xfff0000000000003ULL;
    return mag >= EXP ? special : r;
}

// datatype_timestamp.cc:117-219 for granularity G (0..5 = second..month).
// TABLE_* (:131-136) visits digit G, G-1, .., 0, then G+1 .. 6; the running
// divisor y_i = floor(y_{i-1} / I[T[i]]) from y = UINT64_MAX depends only on G,
// so with G a template parameter the whole chain folds to constants.
constexpr uint64_t TS_I[6] = {60, 60, 24, 7, 4, 12};

template <uint32_t G>
__device__ __forceinline__ uint64_t hash_timestamp_g(uint64_t t) {
    // :198 — u64 -> f64 (round to nearest), IEEE division, truncation to u64.
    uint64_t x = (uint64_t)((double)t / 1000000.0);
    uint64_t d[7];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        d[i] = x % TS_I[i];
        x /= TS_I[i];
    }
    d[6] = x;
    uint64_t y = ~0ULL, h = 0;
#pragma unroll
    for (uint32_t i = 0; i < 6; ++i) {
        const uint32_t k = i <= G ? G - i : i;
        y /= TS_I[k];
        h += d[k] * y;
    }
    return h + d[6];
}

__device__ __forceinline__ uint64_t hash_timestamp(uint32_t g, uint64_t t) {
    switch (g) {
        case 0: return hash_timestamp_g<0>(t);
        case 1: return hash_timestamp_g<1>(t);
        case 2: return hash_timestamp_g<2>(t);
        case 3: return hash_timestamp_g<3>(t);
        case 4: return hash_timestamp_g<4>(t);
        default: return hash_timestamp_g<5>(t);
    }
}

}  // namespace hdx
