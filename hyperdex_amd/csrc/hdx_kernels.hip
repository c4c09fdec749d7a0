// hdx_kernels.hip — batched hyperspace attribute hashing for gfx950.
//
// One launch hashes every attribute of n objects in the packed layout of
// include/hdxhash.h and writes coords[i*A + j] — hs[j] of the reference's
// hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68) for object i.
// The work unit is the (object, attribute) slot; 64 consecutive slots (one
// wave's worth) form a chunk.  Two kernels:
//   hash_chunk_kernel   — one wave per chunk, a single dependent chain;
//   hash_regroup_kernel — one wave per C chunks, descriptors in wave-private
//                         LDS, optionally counting-sorted by work class so a
//                         wave's lanes run the same CityHash regime.
// launch_hash_batch picks one per schema and size (auto_variant).  Variant ids
// are those of the round-1 A/B logs (profiles/r1/ab_variants_*.jsonl); the ids
// of retired experiments (0-11, 13-17: a rounds-per-wave kernel with and
// without software pipelining, non-temporal loads, a workgroup-barrier sort,
// early touching of long strings) are no longer built; their results are in
// DESIGN.md §4.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"

namespace hdx {

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
__device__ __attribute__((aligned(64))) uint8_t g_zero_pad[64];

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
    for (uint32_t k = 0;;) {
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
        s += 64;
        b0 = gld16(s); b1 = gld16(s + 16); b2 = gld16(s + 32); b3 = gld16(s + 48);
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

__device__ __forceinline__ uint64_t hash_blk(uint32_t code, const uint8_t* p, uint32_t n, const Blk& b,
                                             bool& bad) {
    const uint32_t sh = (uint32_t)(uintptr_t)p & 15;
    if (code == CODE_STRING) {
        if (n > 64) return city_gt64_reg(p, n, b);
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

// ===========================================================================
// Chunk kernel (variant 12): one wave = one chunk of 64 consecutive
// (object, attribute) slots of the flattened n*A slot space — the layout's
// natural unit: a coalesced 256 B length load, 64 attributes hashed, one
// coalesced 512 B coordinate store.  A wave has a single dependent chain
// (lengths -> prefix sum -> addresses -> bytes -> hash -> store) and exits, so
// no store ever sits in front of a later load in the wave's vmcnt queue, and
// the hardware keeps up to 8 waves per SIMD issuing fresh loads.  An object
// that starts in an earlier chunk contributes a carry: the sum of its
// attribute lengths that precede this chunk (read back from lengths the
// neighbouring wave just pulled through L2).
// ===========================================================================

// Wave-uniform slot -> (object, attribute) split without a 64-bit integer
// divide: q < 2^53, so the f64 quotient is off by at most one; fix it up.
__device__ __forceinline__ void split_slot(uint64_t q, uint32_t A, uint64_t& i0, uint32_t& j0) {
    uint64_t i = (uint64_t)((double)q * (1.0 / (double)A));
    int64_t rem = (int64_t)(q - i * A);
    if (rem < 0) { --i; rem += A; }
    if (rem >= (int64_t)A) { ++i; rem -= A; }
    i0 = i;
    j0 = (uint32_t)rem;
}

__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
    return __builtin_amdgcn_readlane(wave_scan_dpp(v), 63);
}

template <bool NT_STORE>
__global__ void __launch_bounds__(256)
hash_chunk_kernel(const BatchArgs args) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t A = args.A;
    const uint64_t nslots = args.n * A;
    const uint64_t q0 = wave * 64;
    if (q0 >= nslots) return;

    // this lane's slot -> (object il, attribute j)
    uint64_t i0;
    uint32_t j0;
    split_slot(q0, A, i0, j0);
    const uint32_t t = j0 + (uint32_t)lane;
    const uint32_t di = t / A;  // small: t < A + 64
    const uint32_t j = t - di * A;
    const uint64_t il = i0 + di;
    const bool valid = q0 + lane < nslots;

    // lengths of this chunk, the object bases, and the carry-in lengths
    const uint32_t L = valid ? args.attr_len[q0 + lane] : 0u;
    const uint64_t base = args.obj_base[valid ? il : i0];
    uint32_t carry = 0;
    for (uint32_t k = 0; k < j0; k += 64) {  // slots [q0 - j0, q0) belong to object i0
        const uint32_t idx = k + (uint32_t)lane;
        const uint32_t v = idx < j0 ? args.attr_len[q0 - j0 + idx] : 0u;
        carry += wave_sum_dpp(v);
    }
    uint32_t code;
    if (args.uniform_code != 0xffu) {
        code = args.uniform_code;
    } else {
        const uint32_t packed = reinterpret_cast<const uint32_t*>(args.codes)[lane];
        code = (__shfl(packed, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
    }

    const uint32_t Sx = wave_scan_dpp(L) - L;
    const int head = lane - (int)j;  // lane holding this object's attribute 0, if in this chunk
    const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
    const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
    const uint8_t* p = args.blob + base + off;

    const Blk blk = issue_block(valid ? code : (uint32_t)CODE_ZERO, p, L);
    if (valid) {
        bool bad = false;
        const uint64_t h = hash_blk(code, p, L, blk, bad);
        if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q0 + lane);
        else args.coords[q0 + lane] = h;
        if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
    }
}

// Work classes (the regroup kernel's sort key) and the 16-byte slot descriptor.
constexpr int kClasses = 8;

__device__ __forceinline__ uint32_t work_class(uint32_t code, uint32_t n, bool valid) {
    if (!valid || code != CODE_STRING || n <= 16) return 0;
    if (n <= 64) return 1;
    const uint32_t b = (n - 1) >> 6;
    return b >= 6 ? 7u : 1u + b;
}

struct alignas(16) SlotDesc {
    const uint8_t* p;
    uint32_t n;
    uint32_t code_slot;  // code | slot << 8
};

// ===========================================================================
// Regroup kernel (variants 18-22: 18/19 sorted with C = 4/8; 20/21/22 unsorted,
// C = 8/4/16): a wave owns C consecutive chunks (C*64
// slots).  Phase 1 computes every slot's {pointer, length, code} as the chunk
// kernel does (all C length loads issued at once; the carry chains from chunk
// to chunk in registers) and writes a 16-byte descriptor per slot into the
// wave's private LDS.  A counting sort by work class (ballot + popcount +
// mbcnt, wave-local: no workgroup barrier) yields a permutation.  Phase 2
// hashes C passes of 64 class-sorted slots — the next pass's descriptors and
// bytes are in flight while the current pass is hashed — and writes each
// coordinate over its (already consumed) descriptor.  Phase 3 stores the C
// chunks in slot order, one coalesced 512 B store each.  A wave whose C*64
// slots all share one class skips the permutation.
// ===========================================================================
template <int C>
struct RegroupLds {
    SlotDesc desc[4][C * 64];   // reused for the coordinates in phase 2
    uint16_t perm[4][C * 64];
};

template <int C, bool NT_STORE, bool SORT = true, bool DIRECT = true>
__global__ void __launch_bounds__(256)
hash_regroup_kernel(const BatchArgs args) {
    __shared__ RegroupLds<C> lds;
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
    split_slot(qw, A, i0, j0);
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

    // ---- phase 1: descriptors + classes -------------------------------------
    uint32_t cls[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint32_t t = j0 + (uint32_t)(c * 64 + lane);
        const uint32_t di = t / A;
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
        cls[c] = work_class(code, L, valid);
    }

    // ---- counting sort by class (wave-local) ---------------------------------
    const uint32_t c00 = __builtin_amdgcn_readfirstlane(cls[0]);
    bool uniform = true;
#pragma unroll
    for (int c = 0; c < C; ++c) uniform &= __all(cls[c] == c00);
    if (!SORT) uniform = true;
    if (!uniform) {
        uint32_t before = 0;  // slots of lower classes, then of this class in lower chunks
#pragma unroll
        for (int k = 0; k < kClasses; ++k) {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const uint64_t m = __ballot(cls[c] == (uint32_t)k);
                if (cls[c] == (uint32_t)k) {
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    perm[before + rank] = (uint16_t)(c * 64 + lane);
                }
                before += (uint32_t)__popcll(m);
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- phase 2: C class-homogeneous passes, next pass in flight ------------
    // A slot's coordinate overwrites the first 8 bytes of its own descriptor,
    // which exactly one lane has already read (each slot is in one pass).
    struct Pass {
        SlotDesc d;
        Blk blk;
    };
    auto load_pass = [&](int t, Pass& P) {
        const uint32_t s = uniform ? (uint32_t)(t * 64 + lane) : perm[t * 64 + lane];
        P.d = desc[s];
        P.blk = issue_block(P.d.code_slot & 0xffu, P.d.p, P.d.n);
    };
    bool bad = false;
    Pass P0, P1;
    load_pass(0, P0);
#pragma unroll
    for (int t = 0; t < C; ++t) {
        Pass& cur = (t & 1) ? P1 : P0;
        Pass& nxt = (t & 1) ? P0 : P1;
        if (t + 1 < C) load_pass(t + 1, nxt);
        const uint64_t h = hash_blk(cur.d.code_slot & 0xffu, cur.d.p, cur.d.n, cur.blk, bad);
        if (DIRECT && uniform) {  // pass t is chunk t in slot order: store straight to HBM
            const uint64_t q = qw + t * 64 + lane;
            if (q < nslots) {
                if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q);
                else args.coords[q] = h;
            }
        } else {
            res[2 * (cur.d.code_slot >> 8)] = h;
        }
    }
    if (DIRECT && uniform) {
        if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- phase 3: coalesced stores in slot order -----------------------------
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const uint64_t q = qw + c * 64 + lane;
        if (q < nslots) {
            const uint64_t h = res[2 * (c * 64 + lane)];
            if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q);
            else args.coords[q] = h;
        }
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int C, bool NT, bool SORT = true, bool DIRECT = true>
static hipError_t launch_regroup(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_kernel<C, NT, SORT, DIRECT>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

template <bool NT>
static hipError_t launch_chunk(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + 63) / 64;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_chunk_kernel<NT>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

hipError_t launch_hash_batch_variant(const BatchArgs& args, hipStream_t stream, int variant) {
    switch (variant) {
        case 12: return launch_chunk<true>(args, stream);
        case 18: return launch_regroup<4, true>(args, stream);
        case 19: return launch_regroup<8, true>(args, stream);
        case 20: return launch_regroup<8, true, false>(args, stream);
        case 21: return launch_regroup<4, true, false>(args, stream);
        case 22: return launch_regroup<16, true, false>(args, stream);
        case 23: return launch_regroup<8, true, false, false>(args, stream);
        case 24: return launch_regroup<4, true, false, false>(args, stream);
        case 25: return launch_regroup<16, true, false, false>(args, stream);
        default: return hipErrorInvalidValue;
    }
}

static constexpr int kDefaultVariant = -1;  // automatic
static bool known_variant(int v) { return v == -1 || v == 12 || (v >= 18 && v <= 25); }

static int g_variant = [] {
    const char* e = getenv("HDX_KERNEL_VARIANT");
    return e && *e ? atoi(e) : kDefaultVariant;
}();

// Automatic choice (interleaved A/B on one MI355X, profiles/r1/ab_variants_*.jsonl):
//  * schemas with timestamps or non-hashable attributes: regroup kernel with the
//    class sort, 8 chunks per wave (19) — their diverse paths dominate (mixed: -26 %);
//  * mostly numerics: regroup unsorted, 4 chunks per wave, direct stores (21)
//    (config 2: 0.31 vs 0.42 ms);
//  * one code everywhere (all strings): regroup unsorted with 16 chunks per wave
//    and burst stores (25) when the grid keeps >= 64 K waves, 8 chunks (20) from
//    32 M slots (config 3a: 2.24 vs 2.38 ms), else the one-chunk kernel (12)
//    (config 1);
//  * otherwise (strings + int64/float, config 3b): one-chunk kernel (12).
static int auto_variant(const BatchArgs& args) {
    uint32_t numeric = 0;
    bool complex_types = false;
    for (uint32_t j = 0; j < args.A; ++j) {
        const uint8_t c = args.codes[j];
        numeric += c >= CODE_INT64;
        complex_types |= c == CODE_ZERO || c >= CODE_TS_SECOND;
    }
    const uint64_t slots = args.n * args.A;
    if (complex_types) return 19;
    if (2 * numeric > args.A) return 21;
    if (args.uniform_code != 0xffu) {
        if (slots >= (64ull << 20)) return 25;
        if (slots >= (32ull << 20)) return 20;
    }
    return 12;
}

int hash_variant() { return __atomic_load_n(&g_variant, __ATOMIC_RELAXED); }

int set_hash_variant(int v) {
    if (!known_variant(v)) return -2;
    return __atomic_exchange_n(&g_variant, v, __ATOMIC_RELAXED);
}

void finalize_args(BatchArgs& args) {
    args.uniform_code = args.codes[0];
    for (uint32_t j = 1; j < args.A; ++j)
        if (args.codes[j] != args.codes[0]) args.uniform_code = 0xffu;
}

hipError_t launch_hash_batch(const BatchArgs& args, hipStream_t stream) {
    const int v = hash_variant();
    return launch_hash_batch_variant(args, stream, v < 0 ? auto_variant(args) : v);
}

}  // namespace hdx
