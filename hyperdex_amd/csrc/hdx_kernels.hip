// hdx_kernels.hip — batched hyperspace attribute hashing for gfx950.
//
// One launch hashes every attribute of n objects in the packed layout of
// include/hdxhash.h and writes coords[i*A + j] — the reference's
// hs[j] of hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68) for
// object i.
//
// Work decomposition:
//   * one wave64 owns 64 consecutive objects and walks their 64*A attributes
//     in A rounds of 64 consecutive (object, attr) slots, so every attr_len
//     load and every coords store is one coalesced 256 B / 512 B access;
//   * a lane's byte offset inside its object is a wave-wide prefix sum of the
//     round's lengths plus a carry from the previous round;
//   * each lane hashes one attribute: type dispatch through an LDS code table,
//     strings read as 16 B vectors straight from HBM.
// Software pipelining (template flags, A/B-able through launch_hash_batch_variant):
//   PF_LEN  — round r+1's lengths are loaded while round r is hashed;
//   BASE_RF — the wave's 64 obj_base values live in one VGPR (lane l = object
//             o0+l) and are fetched per round by ds_bpermute, not by a load;
//   PF_STR  — round r+1's first string block (up to 64 B, regime-dependent)
//             is loaded before round r is hashed;
//   NT_STORE — coordinates stored with the non-temporal hint.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"

namespace hdx {

// Inclusive wave64 prefix sum (u32, modular).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t hash_numeric(uint32_t code, uint64_t bits) {
    if (code == CODE_INT64) return encode_int64(bits);
    if (code == CODE_FLOAT) return encode_double(bits);
    return hash_timestamp(code - CODE_TS_SECOND, bits);
}

__device__ __forceinline__ uint64_t hash_attr(uint32_t code, const uint8_t* p, uint32_t len,
                                              bool& bad) {
    if (code == CODE_STRING) return cityhash64(p, len);
    if (code == CODE_ZERO) return 0;
    // int64 / float / timestamp: 0 or 8 bytes (datatype_*::unpack)
    uint64_t bits = 0;
    if (len == 8) {
        bits = ld8(p);
    } else if (len != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}

// Prefetched first block of a string attribute (PF_STR):
//   17..32 B: v0 = s[0,16),   v3 = s[n-16,n)
//   33..64 B: v0..v1 = s[0,32), v2..v3 = s[n-32,n)
//   > 64 B  : v0..v3 = s[n-64,n) (the tail block the long path starts with)
//   <= 16 B and non-strings load at use.
struct StrBlock {
    u64x2 v0, v1, v2, v3;
};

__device__ __forceinline__ void prefetch_block(uint32_t code, const uint8_t* s, uint32_t n, StrBlock& b) {
    if (code != CODE_STRING || n <= 16) return;
    if (n > 64) {
        b.v0 = ld16(s + n - 64);
        b.v1 = ld16(s + n - 48);
        b.v2 = ld16(s + n - 32);
        b.v3 = ld16(s + n - 16);
        return;
    }
    b.v0 = ld16(s);
    b.v3 = ld16(s + n - 16);
    if (n > 32) {
        b.v1 = ld16(s + 16);
        b.v2 = ld16(s + n - 32);
    }
}

// city_gt64 with the tail block already in registers.
__device__ __forceinline__ uint64_t city_gt64_tail(const uint8_t* s, uint32_t n, const StrBlock& t) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    x = x * K1 + ld8(s);
    uint32_t blocks = (n - 1) >> 6;
    for (uint32_t k = 0; k < blocks; ++k, s += 64) {
        const u64x2 b0 = ld16(s), b1 = ld16(s + 16), b2 = ld16(s + 32), b3 = ld16(s + 48);
        x = ror(x + y + v0 + b0.y, 37) * K1;
        y = ror(y + v1 + b3.x, 42) * K1;
        x ^= w1;
        y += v0 + b2.y;
        z = ror(z + w0, 33) * K1;
        uint64_t nv0, nv1, nw0, nw1;
        weak32(b0.x, b0.y, b1.x, b1.y, v1 * K1, x + w0, nv0, nv1);
        weak32(b2.x, b2.y, b3.x, b3.y, z + w1, y + b1.x, nw0, nw1);
        v0 = nv0; v1 = nv1; w0 = nw0; w1 = nw1;
        uint64_t tt = z; z = x; x = tt;
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

__device__ __forceinline__ uint64_t hash_attr_pf(uint32_t code, const uint8_t* p, uint32_t n,
                                                 const StrBlock& b, bool& bad) {
    if (code == CODE_STRING) {
        if (n <= 16) return city_le16(p, n);
        if (n <= 32) return city_17to32(b.v0, b.v3, n);
        if (n <= 64) return city_33to64(b.v0, b.v1, b.v2, b.v3, n);
        return city_gt64_tail(p, n, b);
    }
    return hash_attr(code, p, n, bad);
}

template <bool PF_LEN, bool BASE_RF, bool PF_STR, bool NT_STORE>
__global__ void __launch_bounds__(256)
hash_batch_kernel(const BatchArgs args) {
    __shared__ uint8_t codes[HDX_MAX_ATTRS];
    for (uint32_t j = threadIdx.x; j < args.A; j += blockDim.x) codes[j] = args.codes[j];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t o0 = wave * 64;
    if (o0 >= args.n) return;
    const uint32_t nobj = (uint32_t)min<uint64_t>(64, args.n - o0);
    const uint32_t A = args.A;
    const uint32_t qA = 64 / A, rA = 64 % A;

    const uint32_t* lens = args.attr_len + o0 * A;
    uint64_t* out = args.coords + o0 * A;
    const uint64_t* bases = args.obj_base + o0;
    uint64_t my_base = 0;
    if (BASE_RF) my_base = (uint32_t)lane < nobj ? bases[lane] : 0;

    // slot q = 64*r + lane  ->  (object il = q / A, attribute j = q % A)
    uint32_t il = (uint32_t)lane / A;
    uint32_t j = (uint32_t)lane % A;
    uint32_t carry = 0;
    bool bad = false;

    // round state: L, offset, pointer, code (+ prefetched block)
    auto load_len = [&](uint32_t r, uint32_t il_, uint32_t) -> uint32_t {
        return il_ < nobj ? lens[r * 64 + lane] : 0u;
    };
    auto locate = [&](uint32_t L, uint32_t il_, uint32_t j_, uint32_t& carry_) -> const uint8_t* {
        const uint32_t S = wave_inclusive_scan(L, lane);
        const uint32_t Sx = S - L;
        const int head = lane - (int)j_;
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        const uint32_t off = head >= 0 ? Sx - head_sx : carry_ + Sx;
        carry_ = __shfl(off + L, 63, 64);
        uint64_t base;
        if (BASE_RF) {
            const int src = il_ < 64 ? (int)il_ : 0;
            const uint32_t lo = __shfl((uint32_t)my_base, src, 64);
            const uint32_t hi = __shfl((uint32_t)(my_base >> 32), src, 64);
            base = ((uint64_t)hi << 32) | lo;
        } else {
            base = il_ < nobj ? bases[il_] : 0;
        }
        return args.blob + base + off;
    };
    auto advance = [&](uint32_t& il_, uint32_t& j_) {
        j_ += rA;
        il_ += qA;
        if (j_ >= A) {
            j_ -= A;
            ++il_;
        }
    };

    uint32_t L = load_len(0, il, j);
    const uint8_t* p = locate(L, il, j, carry);
    uint32_t code = codes[j];
    StrBlock blk;
    if (PF_STR && il < nobj) prefetch_block(code, p, L, blk);
    uint32_t Lnext = 0;
    uint32_t il_n = il, j_n = j;
    advance(il_n, j_n);
    if (PF_LEN && A > 1) Lnext = load_len(1, il_n, j_n);

    for (uint32_t r = 0; r < A; ++r) {
        const bool valid = il < nobj;
        // next round's lengths / address / first block, issued before this round's hash
        uint32_t Ln = 0, code_n = 0;
        const uint8_t* pn = nullptr;
        StrBlock blk_n;
        const bool more = r + 1 < A;
        if (more) {
            Ln = PF_LEN ? Lnext : 0;
            if (PF_STR) {
                if (!PF_LEN) Ln = load_len(r + 1, il_n, j_n);
                pn = locate(Ln, il_n, j_n, carry);
                code_n = codes[j_n];
                if (il_n < nobj) prefetch_block(code_n, pn, Ln, blk_n);
            }
            if (PF_LEN && r + 2 < A) {
                uint32_t il2 = il_n, j2 = j_n;
                advance(il2, j2);
                Lnext = load_len(r + 2, il2, j2);
            }
        }
        if (valid) {
            const uint64_t h = PF_STR ? hash_attr_pf(code, p, L, blk, bad) : hash_attr(code, p, L, bad);
            if (NT_STORE) __builtin_nontemporal_store(h, out + r * 64 + lane);
            else out[r * 64 + lane] = h;
        }
        if (!more) break;
        // rotate round state
        if (PF_STR) {
            p = pn;
            code = code_n;
            blk = blk_n;
        } else {
            if (!PF_LEN) Ln = load_len(r + 1, il_n, j_n);
            p = locate(Ln, il_n, j_n, carry);
            code = codes[j_n];
        }
        L = Ln;
        il = il_n;
        j = j_n;
        advance(il_n, j_n);
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// ===========================================================================
// Software-pipelined kernel (variants 7/8).
//
// Every lane issues exactly four 16-byte loads per round, unconditionally, at
// per-lane addresses chosen by the attribute's regime (unused slots point at
// a 64-byte zero pad), so the load stream is straight-line code and the
// compiler's counted s_waitcnt lets round r+1's bytes and round r+2's lengths
// be in flight while round r is hashed:
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
template <bool NT = false>
__device__ __forceinline__ u64x2 gld16(const uint8_t* p) {
    if (NT) return __builtin_nontemporal_load((gvec_ptr)p);
    return *(gvec_ptr)p;
}

struct Blk {
    u64x2 v0, v1, v2, v3;
};

template <bool NTL = false>
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
    b.v0 = gld16<NTL>(a0);
    b.v1 = gld16<NTL>(a1);
    b.v2 = gld16<NTL>(a2);
    b.v3 = gld16<NTL>(a3);
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
template <bool NTL = false>
__device__ __forceinline__ uint64_t city_gt64_reg(const uint8_t* s, uint32_t n, const Blk& t) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    u64x2 b0 = gld16<NTL>(s), b1 = gld16<NTL>(s + 16), b2 = gld16<NTL>(s + 32), b3 = gld16<NTL>(s + 48);
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
        b0 = gld16<NTL>(s); b1 = gld16<NTL>(s + 16); b2 = gld16<NTL>(s + 32); b3 = gld16<NTL>(s + 48);
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

template <bool NTL = false>
__device__ __forceinline__ uint64_t hash_blk(uint32_t code, const uint8_t* p, uint32_t n, const Blk& b,
                                             bool& bad) {
    const uint32_t sh = (uint32_t)(uintptr_t)p & 15;
    if (code == CODE_STRING) {
        if (n > 64) return city_gt64_reg<NTL>(p, n, b);
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

template <bool NT_STORE, int MIN_WAVES, bool NT_LOAD>
__global__ void __launch_bounds__(256, MIN_WAVES)
hash_pipelined_kernel(const BatchArgs args) {
    __shared__ uint8_t codes[HDX_MAX_ATTRS];
    for (uint32_t j = threadIdx.x; j < args.A; j += blockDim.x) codes[j] = args.codes[j];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t o0 = wave * 64;
    if (o0 >= args.n) return;
    const uint32_t nobj = (uint32_t)min<uint64_t>(64, args.n - o0);
    const uint32_t A = args.A;
    const uint32_t qA = 64 / A, rA = 64 % A;
    const uint32_t last = nobj * A - 1;  // last valid slot of this wave

    const uint32_t* lens = args.attr_len + o0 * A;
    uint64_t* out = args.coords + o0 * A;
    const uint64_t my_base = args.obj_base[o0 + min<uint32_t>((uint32_t)lane, nobj - 1)];

    uint32_t il = (uint32_t)lane / A, j = (uint32_t)lane % A;
    uint32_t carry = 0;
    bool bad = false;

    auto advance = [&](uint32_t& il_, uint32_t& j_) {
        j_ += rA;
        il_ += qA;
        if (j_ >= A) {
            j_ -= A;
            ++il_;
        }
    };
    // unconditional, clamped length load for round r
    auto load_len = [&](uint32_t r) -> uint32_t { return lens[min(r * 64 + (uint32_t)lane, last)]; };
    auto locate = [&](uint32_t Lraw, uint32_t il_, uint32_t j_, uint32_t& L) -> const uint8_t* {
        L = il_ < nobj ? Lraw : 0u;
        const uint32_t Sx = wave_scan_dpp(L) - L;
        const int head = lane - (int)j_;
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
        carry = __builtin_amdgcn_readlane(off + L, 63);
        const int src = il_ < nobj ? (int)il_ : 0;
        const uint32_t blo = __shfl((uint32_t)my_base, src, 64);
        const uint32_t bhi = __shfl((uint32_t)(my_base >> 32), src, 64);
        return args.blob + (((uint64_t)bhi << 32) | blo) + off;
    };

    // Two round states used ping-pong (loop unrolled by two) so that data still
    // in flight is never copied between registers.
    struct Round {
        const uint8_t* p;
        uint32_t L, code, il, j, Lraw_next;
        Blk blk;
    };
    // prologue: round 0 located; round 1 lengths and round 0 bytes in flight
    Round S0, S1;
    S0.il = il;
    S0.j = j;
    S0.p = locate(load_len(0), il, j, S0.L);
    S0.code = codes[j];
    S0.Lraw_next = load_len(1);
    S0.blk = issue_block<NT_LOAD>(S0.code, S0.p, S0.L);

    // Hash round r held in `cur`; first locate round r+1 into `nxt` and put its
    // bytes (and round r+2's lengths) in flight.  The prefetch is unconditional
    // (past the last round every lane is invalid, so its loads hit the zero pad):
    // no conditionally-assigned register survives into the next step.
    auto step = [&](Round& cur, Round& nxt, uint32_t r) {
        nxt.il = cur.il;
        nxt.j = cur.j;
        advance(nxt.il, nxt.j);
        nxt.p = locate(cur.Lraw_next, nxt.il, nxt.j, nxt.L);
        nxt.code = codes[nxt.j < A ? nxt.j : 0];
        nxt.Lraw_next = load_len(r + 2);
        nxt.blk = issue_block<NT_LOAD>(nxt.code, nxt.p, nxt.L);
        if (cur.il < nobj) {
            const uint64_t h = hash_blk<NT_LOAD>(cur.code, cur.p, cur.L, cur.blk, bad);
            if (NT_STORE) __builtin_nontemporal_store(h, out + r * 64 + lane);
            else out[r * 64 + lane] = h;
        }
    };
    for (uint32_t r = 0;; r += 2) {
        step(S0, S1, r);
        if (r + 1 >= A) break;
        step(S1, S0, r + 1);
        if (r + 2 >= A) break;
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <bool NT, int MIN_WAVES = 1, bool NTL = false>
static hipError_t launch_pipe(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n + 63) / 64;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_pipelined_kernel<NT, MIN_WAVES, NTL>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

// ===========================================================================
// Chunk kernel (variants 11/12): one wave = one chunk of 64 consecutive
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

// Touch the first dword of loop blocks 0..2 of a > 64-byte string while the
// tail block is in flight, so the CityHash loop's block loads (city.cc:383-394)
// find their lines in L2 instead of paying one HBM latency per block.  Clamped
// to the string; the values are folded into `sink`, consumed by an empty
// asm use placed after the hash, so the loads stay live and tracked by the
// compiler's counted waits without being waited for early.
__device__ __forceinline__ uint32_t touch_blocks(uint32_t code, const uint8_t* p, uint32_t n) {
    if (!(code == CODE_STRING && n > 64)) p = g_zero_pad, n = 65;
    const uint32_t last = (n - 1) & ~63u;  // start of the last loop block's successor region
    const uint32_t o1 = min(64u, last - 64u), o2 = min(128u, last - 64u);
    typedef const __attribute__((address_space(1))) uint32_t* gu32p;
    return *(gu32p)(p) ^ *(gu32p)(p + o1) ^ *(gu32p)(p + o2);
}

template <bool NT_STORE, bool NT_LOAD, bool TOUCH = false>
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

    const Blk blk = issue_block<NT_LOAD>(valid ? code : (uint32_t)CODE_ZERO, p, L);
    uint32_t sink = 0;
    if (TOUCH) sink = touch_blocks(valid ? code : (uint32_t)CODE_ZERO, p, L);
    if (valid) {
        bool bad = false;
        uint64_t h = hash_blk<NT_LOAD>(code, p, L, blk, bad);
        if (TOUCH) asm volatile("; touch sink %0" ::"v"(sink));  // keeps the touch loads live, late
        if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q0 + lane);
        else args.coords[q0 + lane] = h;
        if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
    }
}

template <bool NT, bool NTL = false, bool TOUCH = false>
static hipError_t launch_chunk(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + 63) / 64;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_chunk_kernel<NT, NTL, TOUCH>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

// ===========================================================================
// Binned chunk kernel (variant 15/16): the chunk kernel at workgroup scope
// (4 waves = 256 consecutive slots) with the slots regrouped by work class
// before hashing, so that a wave's lanes run the same CityHash regime and the
// same number of 64-byte loop blocks instead of the union of all of them.
//   class 0: numeric, non-hashable, empty and <= 16-byte strings (cheap paths)
//   class 1: 17..64-byte strings
//   class 1+b: strings of b = ceil(len/64)-1 loop blocks (b = 1..5), 6+ -> 7
// A counting sort in LDS (ballot + mbcnt ranks, per-wave class counts)
// places a 16-byte descriptor {pointer, length, code, slot} per slot; every
// wave hashes 64 consecutive sorted descriptors and writes its coordinates
// back to LDS by slot, and the workgroup stores them in slot order (one
// coalesced 512 B store per wave).  Workgroups whose 256 slots all fall into
// one class skip the sort.
// ===========================================================================
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

template <bool NT_STORE>
__global__ void __launch_bounds__(256)
hash_binned_kernel(const BatchArgs args) {
    __shared__ SlotDesc desc[256];
    __shared__ uint64_t res[256];
    __shared__ uint32_t counts[4][kClasses];
    __shared__ uint32_t wave_cls[4];

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + w;
    const uint32_t A = args.A;
    const uint64_t nslots = args.n * A;
    const uint64_t q0 = wave * 64;
    const bool live = q0 < nslots;  // wave-uniform: a dead wave still joins the barriers

    uint32_t L = 0, code = CODE_ZERO;
    const uint8_t* p = g_zero_pad;
    bool valid = false;
    if (live) {
        uint64_t i0;
        uint32_t j0;
        split_slot(q0, A, i0, j0);
        const uint32_t t = j0 + (uint32_t)lane;
        const uint32_t di = t / A;
        const uint32_t j = t - di * A;
        const uint64_t il = i0 + di;
        valid = q0 + lane < nslots;
        L = valid ? args.attr_len[q0 + lane] : 0u;
        const uint64_t base = args.obj_base[valid ? il : i0];
        uint32_t carry = 0;
        for (uint32_t k = 0; k < j0; k += 64) {
            const uint32_t idx = k + (uint32_t)lane;
            const uint32_t v = idx < j0 ? args.attr_len[q0 - j0 + idx] : 0u;
            carry += wave_sum_dpp(v);
        }
        if (args.uniform_code != 0xffu) {
            code = args.uniform_code;
        } else {
            const uint32_t packed = reinterpret_cast<const uint32_t*>(args.codes)[lane];
            code = (__shfl(packed, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
        }
        const uint32_t Sx = wave_scan_dpp(L) - L;
        const int head = lane - (int)j;
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
        p = args.blob + base + off;
        if (!valid) code = CODE_ZERO;
    }

    // ---- classify; skip the sort when the workgroup is one class ----------
    const uint32_t cls = work_class(code, L, valid);
    const uint32_t c0 = __builtin_amdgcn_readfirstlane(cls);
    const bool wave_uniform = __all(cls == c0);
    if (lane == 0) wave_cls[w] = live ? (wave_uniform ? c0 : 0xffu) : 0xfeu;
    uint32_t my_count = 0;
#pragma unroll
    for (int c = 0; c < kClasses; ++c) {
        const uint64_t m = __ballot(cls == (uint32_t)c);
        if ((uint32_t)c == cls) my_count = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == c) counts[w][c] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    uint32_t wc = 0xffu;
    bool one_class = true;
    for (int k = 0; k < 4; ++k) {
        const uint32_t x = wave_cls[k];
        if (x == 0xfeu) continue;
        if (x == 0xffu || (wc != 0xffu && x != wc)) one_class = false;
        wc = x;
    }

    bool bad = false;
    uint64_t h = 0;
    if (one_class) {
        const Blk blk = issue_block(code, p, L);
        if (valid) h = hash_blk(code, p, L, blk, bad);
    } else {
        // sorted position = (slots of lower classes) + (this class in lower waves) + rank
        uint32_t pos = my_count;
        for (int c = 0; c < kClasses; ++c) {
            const uint32_t tot = counts[0][c] + counts[1][c] + counts[2][c] + counts[3][c];
            if ((uint32_t)c < cls) pos += tot;
        }
        for (int k = 0; k < 4; ++k)
            if (k < w) pos += counts[k][cls];
        SlotDesc d;
        d.p = p;
        d.n = L;
        d.code_slot = code | ((uint32_t)threadIdx.x << 8);
        desc[pos] = d;
        __syncthreads();
        const SlotDesc e = desc[threadIdx.x];
        const uint32_t ecode = e.code_slot & 0xffu, eslot = e.code_slot >> 8;
        const Blk blk = issue_block(ecode, e.p, e.n);
        const uint64_t eh = hash_blk(ecode, e.p, e.n, blk, bad);
        res[eslot] = eh;
        __syncthreads();
        h = res[threadIdx.x];
    }
    if (valid) {
        if (NT_STORE) __builtin_nontemporal_store(h, args.coords + q0 + lane);
        else args.coords[q0 + lane] = h;
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <bool NT>
static hipError_t launch_binned(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + 63) / 64;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_binned_kernel<NT>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

// ===========================================================================
// Regroup kernel (variants 18/19): a wave owns C consecutive chunks (C*64
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

template <int C, bool NT_STORE, bool SORT = true>
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
        res[2 * (cur.d.code_slot >> 8)] = h;
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

template <int C, bool NT, bool SORT = true>
static hipError_t launch_regroup(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n * args.A + C * 64 - 1) / (C * 64);
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_regroup_kernel<C, NT, SORT>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

template <bool A_, bool B_, bool C_, bool D_ = false>
static hipError_t launch_t(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n + 63) / 64;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_batch_kernel<A_, B_, C_, D_>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

hipError_t launch_hash_batch_variant(const BatchArgs& args, hipStream_t stream, int variant) {
    switch (variant) {
        case 0: return launch_t<false, false, false>(args, stream);
        case 1: return launch_t<true, false, false>(args, stream);
        case 2: return launch_t<true, true, false>(args, stream);
        case 3: return launch_t<true, true, true>(args, stream);
        case 4: return launch_t<false, true, true>(args, stream);
        case 5: return launch_t<true, true, false, true>(args, stream);
        case 6: return launch_t<true, true, true, true>(args, stream);
        case 7: return launch_pipe<false>(args, stream);
        case 8: return launch_pipe<true>(args, stream);
        case 9: return launch_pipe<true, 5>(args, stream);
        case 10: return launch_pipe<true, 6>(args, stream);
        case 11: return launch_chunk<false>(args, stream);
        case 12: return launch_chunk<true>(args, stream);
        case 13: return launch_chunk<true, true>(args, stream);
        case 14: return launch_pipe<true, 1, true>(args, stream);
        case 15: return launch_binned<false>(args, stream);
        case 16: return launch_binned<true>(args, stream);
        case 17: return launch_chunk<true, false, true>(args, stream);
        case 18: return launch_regroup<4, true>(args, stream);
        case 19: return launch_regroup<8, true>(args, stream);
        case 20: return launch_regroup<8, true, false>(args, stream);
        case 21: return launch_regroup<4, true, false>(args, stream);
        case 22: return launch_regroup<16, true, false>(args, stream);
        default: return hipErrorInvalidValue;
    }
}

// -1 = automatic: the chunk kernel (12) unless most attributes are
// fixed-size numerics, where the 64-objects-per-wave pipelined kernel (8)
// amortises its per-wave setup better (scripts/ab_variants.py).
static constexpr int kDefaultVariant = -1;
static constexpr int kMaxVariant = 22;

static int g_variant = [] {
    const char* e = getenv("HDX_KERNEL_VARIANT");
    return e && *e ? atoi(e) : kDefaultVariant;
}();

// Automatic choice (interleaved A/B on one MI355X, profiles/r1/ab_variants_*.jsonl):
//  * schemas with timestamps or non-hashable attributes: regroup kernel with the
//    class sort (19) — their expensive/diverse paths dominate (mixed: -26 %);
//  * mostly numerics: multi-chunk, 4 chunks per wave (21) (config 2);
//  * one code everywhere (all strings): multi-chunk without sort, 16 or 8
//    chunks per wave when the grid stays >= 64 K waves (22/20) (config 3a),
//    else the one-chunk kernel (12) (config 1);
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
        if (slots >= (64ull << 20)) return 22;
        if (slots >= (32ull << 20)) return 20;
    }
    return 12;
}

int hash_variant() { return __atomic_load_n(&g_variant, __ATOMIC_RELAXED); }

int set_hash_variant(int v) {
    if (v < -1 || v > kMaxVariant) return -2;
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
