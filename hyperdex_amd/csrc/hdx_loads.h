// hdx_loads.h — loads and register-fed hashing shared by the hash kernels
// (hdx_kernels.hip, hdx_encoded.hip).  Device code only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"

namespace hdx {

// One slot's work: where its bytes are, how many, and its dispatch code (low
// byte) | slot index within the wave's window << 8.
struct alignas(16) SlotDesc {
    const uint8_t* p;
    uint32_t n;
    uint32_t code_slot;  // code | slot << 8
};

// int64 / float / timestamp from their 8-byte little-endian bit pattern.
__device__ __forceinline__ uint64_t hash_numeric(uint32_t code, uint64_t bits) {
    if (code == CODE_INT64) return encode_int64(bits);
    if (code == CODE_FLOAT) return encode_double(bits);
    return hash_timestamp(code - CODE_TS_SECOND, bits);
}

// ===========================================================================
// Loads and register-fed hashing.
//
// Every lane issues exactly four 16-byte loads per slot, unconditionally, at
// per-lane addresses chosen by the attribute's regime (unused slots point at
// a 64-byte zero pad), so the load stream is straight-line code and the
// compiler's counted s_waitcnt can keep independent loads in flight:
//   string  > 64 B : s[n-64,n) in four pieces (the tail block CityHash starts with)
//   string 33..64 B: s[0,32) and s[n-32,n)
//   string 16..32 B: s[0,16) and s[n-16,n)
//   string  1..15 B, int64/float/timestamp: the aligned 16-byte chunks holding
//                    the first and last byte — a load never leaves the pages
//                    the value lives in, so short values at the very end of a
//                    buffer are read safely — then a funnel shift (v_alignbyte)
//                    recovers the value's bytes in registers.
// ===========================================================================
static __device__ __attribute__((aligned(64))) uint8_t g_zero_pad[64];  // per code object

// 16-byte load through an explicit global (addrspace 1) pointer at any
// alignment: keeps the access a global_load_dwordx4 (never flat_, whose
// out-of-order completion would force full vmcnt/lgkmcnt drains).
typedef u64x2 __attribute__((aligned(1))) u64x2_u;
typedef const __attribute__((address_space(1))) u64x2_u* gvec_ptr;
__device__ __forceinline__ u64x2 gld16(const uint8_t* p) { return *(gvec_ptr)p; }

struct Blk {
    u64x2 v0, v1, v2, v3;
};

__device__ __forceinline__ Blk issue_block(uint32_t code, const uint8_t* p, uint32_t n) {
    const uint8_t* D = g_zero_pad;
    const bool str = code == CODE_STRING;
    const bool shortv = (str && n > 0 && n < 16) || (code >= CODE_INT64 && n == 8);
    const uint8_t* lo = p - ((uintptr_t)p & 15);  // pointer arithmetic keeps provenance
    const uint8_t* hi = (p + n - 1) - ((uintptr_t)(p + n - 1) & 15);
    const bool g64 = str && n > 64, g32 = str && n > 32 && n <= 64, g16 = str && n >= 16 && n <= 32;
    const uint8_t* a0 = g64 ? p + n - 64 : (g32 || g16) ? p : shortv ? lo : D;
    const uint8_t* a1 = g64 ? p + n - 48 : g32 ? p + 16 : g16 ? p + n - 16 : shortv ? hi : D;
    const uint8_t* a2 = g64 || g32 ? p + n - 32 : D;
    const uint8_t* a3 = g64 || g32 ? p + n - 16 : D;
    Blk b;
    b.v0 = gld16(a0);
    b.v1 = gld16(a1);
    b.v2 = gld16(a2);
    b.v3 = gld16(a3);
    return b;
}

__device__ __forceinline__ uint32_t dw(const u64x2& v, int k) {
    return (uint32_t)((k & 2 ? v.y : v.x) >> (32 * (k & 1)));
}
__device__ __forceinline__ uint32_t pick4(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return q == 0 ? a : q == 1 ? b : q == 2 ? c : d;
}

// Bytes [sh, sh+16) of the 32-byte concatenation c0 || c1 (sh in 0..15).
__device__ __forceinline__ u64x2 window16(const u64x2& c0, const u64x2& c1, uint32_t sh) {
    const uint32_t d0 = dw(c0, 0), d1 = dw(c0, 1), d2 = dw(c0, 2), d3 = dw(c0, 3);
    const uint32_t d4 = dw(c1, 0), d5 = dw(c1, 1), d6 = dw(c1, 2), d7 = dw(c1, 3);
    const uint32_t q = sh >> 2, r = sh & 3;
    const uint32_t e0 = pick4(q, d0, d1, d2, d3), e1 = pick4(q, d1, d2, d3, d4);
    const uint32_t e2 = pick4(q, d2, d3, d4, d5), e3 = pick4(q, d3, d4, d5, d6);
    const uint32_t e4 = pick4(q, d4, d5, d6, d7);
    const uint32_t o0 = __builtin_amdgcn_alignbyte(e1, e0, r), o1 = __builtin_amdgcn_alignbyte(e2, e1, r);
    const uint32_t o2 = __builtin_amdgcn_alignbyte(e3, e2, r), o3 = __builtin_amdgcn_alignbyte(e4, e3, r);
    u64x2 w;
    w.x = ((uint64_t)o1 << 32) | o0;
    w.y = ((uint64_t)o3 << 32) | o2;
    return w;
}

// Bytes [sh, sh+8) of c0 || c1.
__device__ __forceinline__ uint64_t window8(const u64x2& c0, const u64x2& c1, uint32_t sh) {
    const uint32_t d0 = dw(c0, 0), d1 = dw(c0, 1), d2 = dw(c0, 2), d3 = dw(c0, 3);
    const uint32_t d4 = dw(c1, 0), d5 = dw(c1, 1);
    const uint32_t q = sh >> 2, r = sh & 3;
    const uint32_t e0 = pick4(q, d0, d1, d2, d3), e1 = pick4(q, d1, d2, d3, d4);
    const uint32_t e2 = pick4(q, d2, d3, d4, d5);
    return ((uint64_t)__builtin_amdgcn_alignbyte(e2, e1, r) << 32) | __builtin_amdgcn_alignbyte(e1, e0, r);
}

// city.cc:278-301 with the (up to) 16 string bytes in registers.
__device__ __forceinline__ uint64_t city_le16_reg(const u64x2& w, uint32_t n) {
    const uint64_t mul = K2 + 2ull * n;
    const uint32_t d0 = (uint32_t)w.x, d1 = (uint32_t)(w.x >> 32);
    const uint32_t d2 = (uint32_t)w.y, d3 = (uint32_t)(w.y >> 32);
    if (n >= 8) {
        // b = bytes [n-8, n): shift by t = n-8 in 0..8
        const uint32_t t = n - 8, q = t >> 2, r = t & 3;
        const uint32_t e0 = q == 0 ? d0 : q == 1 ? d1 : d2;
        const uint32_t e1 = q == 0 ? d1 : q == 1 ? d2 : d3;
        const uint32_t e2 = q == 0 ? d2 : d3;
        const uint64_t b = ((uint64_t)__builtin_amdgcn_alignbyte(e2, e1, r) << 32) |
                           __builtin_amdgcn_alignbyte(e1, e0, r);
        const uint64_t a = w.x + K2;
        const uint64_t c = ror(b, 37) * mul + a;
        const uint64_t d = (ror(a, 25) + b) * mul;
        return mix16(c, d, mul);
    }
    if (n >= 4) {
        const uint64_t a = d0;
        const uint32_t b = __builtin_amdgcn_alignbyte(d1, d0, n - 4);
        return mix16(n + (a << 3), b, mul);
    }
    if (n > 0) {
        const uint32_t y = (d0 & 0xff) + (((d0 >> (8 * (n >> 1))) & 0xff) << 8);
        const uint32_t z = n + (((d0 >> (8 * (n - 1))) & 0xff) << 2);
        return shiftmix((uint64_t)y * K2 ^ (uint64_t)z * K0) * K2;
    }
    return K2;
}

// city.cc:361-397 for n > 64 with the tail block in registers; the first
// 64-byte block is loaded up front (its first word is Fetch64(s) of :380).
// PIPE: block k+1 is in flight while block k is mixed (the last iteration
// re-reads its own block, so the loads stay unconditional).
template <bool PIPE>
__device__ __forceinline__ uint64_t city_gt64_reg(const uint8_t* s, uint32_t n, const Blk& t) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    u64x2 b0 = gld16(s), b1 = gld16(s + 16), b2 = gld16(s + 32), b3 = gld16(s + 48);
    x = x * K1 + b0.x;
    const uint32_t blocks = (n - 1) >> 6;
    const uint8_t* last = s + 64 * (blocks - 1);
    for (uint32_t k = 0;;) {
        u64x2 n0, n1, n2, n3;
        const uint8_t* ns = s + 64 < last ? s + 64 : last;
        if (PIPE) {
            n0 = gld16(ns); n1 = gld16(ns + 16); n2 = gld16(ns + 32); n3 = gld16(ns + 48);
        }
        x = ror(x + y + v0 + b0.y, 37) * K1;
        y = ror(y + v1 + b3.x, 42) * K1;
        x ^= w1;
        y += v0 + b2.y;
        z = ror(z + w0, 33) * K1;
        uint64_t nv0, nv1, nw0, nw1;
        weak32(b0.x, b0.y, b1.x, b1.y, v1 * K1, x + w0, nv0, nv1);
        weak32(b2.x, b2.y, b3.x, b3.y, z + w1, y + b1.x, nw0, nw1);
        v0 = nv0; v1 = nv1; w0 = nw0; w1 = nw1;
        const uint64_t tt = z; z = x; x = tt;
        if (++k == blocks) break;
        s = ns;
        if (PIPE) {
            b0 = n0; b1 = n1; b2 = n2; b3 = n3;
        } else {
            b0 = gld16(s); b1 = gld16(s + 16); b2 = gld16(s + 32); b3 = gld16(s + 48);
        }
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

template <bool PIPE = false>
__device__ __forceinline__ uint64_t hash_blk(uint32_t code, const uint8_t* p, uint32_t n, const Blk& b,
                                             bool& bad) {
    const uint32_t sh = (uint32_t)(uintptr_t)p & 15;
    if (code == CODE_STRING) {
        if (n > 64) return city_gt64_reg<PIPE>(p, n, b);
        if (n > 32) return city_33to64(b.v0, b.v1, b.v2, b.v3, n);
        if (n > 16) return city_17to32(b.v0, b.v1, n);
        return city_le16_reg(n == 16 ? b.v0 : window16(b.v0, b.v1, sh), n);
    }
    if (code == CODE_ZERO) return 0;
    uint64_t bits = 0;
    if (n == 8) {
        bits = window8(b.v0, b.v1, sh);
    } else if (n != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}

// Inclusive wave64 prefix sum on DPP (row_shr within 16-lane rows, then the
// row_bcast:15 / row_bcast:31 carries across rows).
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}

}  // namespace hdx
