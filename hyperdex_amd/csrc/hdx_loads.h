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
// 128 bytes: a quad-cooperative loop load (ld64_quad) of a lane with no block
// reads 64 bytes + one dword here
static __device__ __attribute__((aligned(64))) uint8_t g_zero_pad[128];  // per code object

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

// ---------------------------------------------------------------------------
// Dword-aligned form (A4).  A 16-byte load at a byte-misaligned address costs
// the texture-address unit about twice an aligned one (tools/gldbench.hip:
// 4.37 vs 5.45 TB/s, TA 97 % busy), and packed variable-length values are
// byte-misaligned three times in four.  A4 loads every piece at the dword
// floor of its address, plus the dword after it, and funnel-shifts the bytes
// into place with v_alignbyte (4 VALU per 16 bytes).  Pieces, as issue_block's
// but with the 16..32-byte and short / numeric regimes in slots 1 and 3:
//   P0 P1 | P2 P3, P1's next dword E1, P3's next dword E3,
//   shift ra for P0/P1 (contiguous: P0's next dword is P1's first), rb for P2/P3.
// Every dword loaded holds at least one byte of the value (or is in the zero
// pad), so no load leaves the value's pages.
// ---------------------------------------------------------------------------
struct Raw {
    Blk b;
    uint32_t e1, e3, ra, rb;
};

__device__ __forceinline__ uint32_t gld4(const uint8_t* p) {
    return *(const __attribute__((address_space(1))) uint32_t*)p;
}
__device__ __forceinline__ const uint8_t* dw_floor(const uint8_t* p) { return p - ((uintptr_t)p & 3); }

// Piece offsets of the A4 form, from the value's base (or from the zero pad
// when the slot has no bytes to read: any = false), as 32-bit arithmetic;
// pl = the base's low address bits.  Shared by the global-memory form
// (issue_block_a4); the retired LDS-window kernels read the window with it.
struct A4Offsets {
    int32_t o0, o1, o2, o3, e1, e3;  // dword-aligned piece starts and next dwords
    uint32_t ra, rb;
    bool any;
};

__device__ __forceinline__ A4Offsets a4_offsets(uint32_t code, uint32_t pl_, uint32_t n) {
    const bool str = code == CODE_STRING;
    const bool shortv = (str && n > 0 && n < 16) || (code >= CODE_INT64 && n == 8);
    const bool g64 = str && n > 64, g32 = str && n > 32 && n <= 64, g16 = str && n >= 16 && n <= 32;
    const bool big = g64 || g32;
    A4Offsets o;
    o.any = big || g16 || shortv;
    const uint32_t pl = o.any ? pl_ : 0u;
    const int32_t lo = -(int32_t)(pl & 15u);                          // 16-aligned chunk of byte 0
    const int32_t hi = (int32_t)(((pl + n - 1u) & ~15u) - pl);       // ... of byte n-1
    const int32_t x1 = g64 ? (int32_t)n - 48 : g32 ? 16 : g16 ? 0 : shortv ? lo : 0;
    const int32_t x3 = big || g16 ? (int32_t)n - 16 : shortv ? hi : 0;
    const int32_t x0 = big ? x1 - 16 : x1;  // g64: n-64, g32: 0; else a repeat of piece 1
    const int32_t x2 = big ? x3 - 16 : x3;
    o.ra = (pl + (uint32_t)x1) & 3u;  // piece 0 shares piece 1's alignment, piece 2 piece 3's
    o.rb = (pl + (uint32_t)x3) & 3u;
    // the dword after piece 1 (3) is the one holding its last byte when the
    // piece is misaligned; else unused, and that dword is still a value byte's
    o.e1 = x1 + 15 - (int32_t)((pl + (uint32_t)x1 + 15u) & 3u);
    o.e3 = x3 + 15 - (int32_t)((pl + (uint32_t)x3 + 15u) & 3u);
    o.o0 = x0 - (int32_t)o.ra;
    o.o1 = x1 - (int32_t)o.ra;
    o.o2 = x2 - (int32_t)o.rb;
    o.o3 = x3 - (int32_t)o.rb;
    return o;
}

__device__ __forceinline__ Raw issue_block_a4(uint32_t code, const uint8_t* p, uint32_t n) {
    const A4Offsets o = a4_offsets(code, (uint32_t)(uintptr_t)p, n);
    const uint8_t* base = o.any ? p : g_zero_pad;  // the zero pad is 64-byte aligned
    Raw r;
    r.ra = o.ra;
    r.rb = o.rb;
    r.b.v0 = gld16(base + o.o0);
    r.b.v1 = gld16(base + o.o1);
    r.b.v2 = gld16(base + o.o2);
    r.b.v3 = gld16(base + o.o3);
    r.e1 = gld4(base + o.e1);
    r.e3 = gld4(base + o.e3);
    return r;
}

// Bytes [r, r+16) of the 20 bytes v || next (r in 0..3).
__device__ __forceinline__ u64x2 funnel16(const u64x2& v, uint32_t next, uint32_t r) {
    const uint32_t d0 = (uint32_t)v.x, d1 = (uint32_t)(v.x >> 32), d2 = (uint32_t)v.y, d3 = (uint32_t)(v.y >> 32);
    u64x2 w;
    w.x = pack64(__builtin_amdgcn_alignbyte(d1, d0, r), __builtin_amdgcn_alignbyte(d2, d1, r));
    w.y = pack64(__builtin_amdgcn_alignbyte(d3, d2, r), __builtin_amdgcn_alignbyte(next, d3, r));
    return w;
}

__device__ __forceinline__ Blk funnel_raw(const Raw& r) {
    Blk b;
    b.v0 = funnel16(r.b.v0, (uint32_t)r.b.v1.x, r.ra);
    b.v1 = funnel16(r.b.v1, r.e1, r.ra);
    b.v2 = funnel16(r.b.v2, (uint32_t)r.b.v3.x, r.rb);
    b.v3 = funnel16(r.b.v3, r.e3, r.rb);
    return b;
}

// issue / consume in either form: A4 = dword-aligned pieces, funnelled when
// consumed (so the next pass's loads stay in flight); else issue_block's.
template <bool A4>
__device__ __forceinline__ Raw issue_any(uint32_t code, const uint8_t* p, uint32_t n) {
    if constexpr (A4) {
        return issue_block_a4(code, p, n);
    } else {
        Raw r;
        r.b = issue_block(code, p, n);
        r.e1 = r.e3 = r.ra = r.rb = 0;
        return r;
    }
}
template <bool A4>
__device__ __forceinline__ Blk consume_any(const Raw& r) {
    if constexpr (A4) return funnel_raw(r);
    else return r.b;
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
    w.x = pack64(o0, o1);
    w.y = pack64(o2, o3);
    return w;
}

// Bytes [sh, sh+8) of c0 || c1.
__device__ __forceinline__ uint64_t window8(const u64x2& c0, const u64x2& c1, uint32_t sh) {
    const uint32_t d0 = dw(c0, 0), d1 = dw(c0, 1), d2 = dw(c0, 2), d3 = dw(c0, 3);
    const uint32_t d4 = dw(c1, 0), d5 = dw(c1, 1);
    const uint32_t q = sh >> 2, r = sh & 3;
    const uint32_t e0 = pick4(q, d0, d1, d2, d3), e1 = pick4(q, d1, d2, d3, d4);
    const uint32_t e2 = pick4(q, d2, d3, d4, d5);
    return pack64(__builtin_amdgcn_alignbyte(e1, e0, r), __builtin_amdgcn_alignbyte(e2, e1, r));
}

// city.cc:278-301 with the (up to) 16 string bytes in registers.  The
// 8..16-byte and 4..7-byte cases both end in HashLen16(u, v, mul) (:283-296),
// so their operands are chosen first and one HashLen16 serves both (a wave
// holding both lengths runs one instead of two).
__device__ __forceinline__ uint64_t city_le16_reg(const u64x2& w, uint32_t n) {
    const uint64_t mul = K2 + 2ull * n;
    const uint32_t d0 = (uint32_t)w.x, d1 = (uint32_t)(w.x >> 32);
    const uint32_t d2 = (uint32_t)w.y, d3 = (uint32_t)(w.y >> 32);
    uint64_t u, v;
    if (n >= 8) {
        // b = bytes [n-8, n): shift by t = n-8 in 0..8
        const uint32_t t = n - 8, q = t >> 2, r = t & 3;
        const uint32_t e0 = q == 0 ? d0 : q == 1 ? d1 : d2;
        const uint32_t e1 = q == 0 ? d1 : q == 1 ? d2 : d3;
        const uint32_t e2 = q == 0 ? d2 : d3;
        const uint64_t b = pack64(__builtin_amdgcn_alignbyte(e1, e0, r), __builtin_amdgcn_alignbyte(e2, e1, r));
        const uint64_t a = w.x + K2;
        u = ror(b, 37) * mul + a;
        v = (ror(a, 25) + b) * mul;
    } else {
        u = n + ((uint64_t)d0 << 3);
        v = __builtin_amdgcn_alignbyte(d1, d0, (n - 4) & 3);
    }
    const uint64_t h = mix16(u, v, mul);
    if (n >= 4) return h;
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
// FAKE (debug variant 41 only): the loop's loads are replaced by values made
// from the address, so a kernel built with it runs the arithmetic alone.
template <bool FAKE>
__device__ __forceinline__ u64x2 ld16(const uint8_t* s) {
    if constexpr (FAKE) {
        u64x2 v;
        v.x = (uint64_t)(uintptr_t)s;
        v.y = v.x * 3;
        return v;
    } else {
        return gld16(s);
    }
}

// One 64-byte loop block at s: four 16-byte loads, or (A4) four at the dword
// floor of s plus the dword after them, funnel-shifted by s & 3.  Every loop
// block ends at least one byte before the value does, so the extra dword
// holds value bytes.
struct Blk64 {
    Blk b;
    uint32_t e;
};
template <bool A4, bool FAKE>
__device__ __forceinline__ Blk64 ld64(const uint8_t* s) {
    Blk64 r;
    const uint8_t* a = A4 ? dw_floor(s) : s;
    r.b.v0 = ld16<FAKE>(a);
    r.b.v1 = ld16<FAKE>(a + 16);
    r.b.v2 = ld16<FAKE>(a + 32);
    r.b.v3 = ld16<FAKE>(a + 48);
    r.e = A4 && !FAKE ? gld4(a + 64) : 0u;
    return r;
}
template <bool A4>
__device__ __forceinline__ Blk use64(const Blk64& r, uint32_t sh) {
    if constexpr (!A4) {
        return r.b;
    } else {
        Blk b;
        b.v0 = funnel16(r.b.v0, (uint32_t)r.b.v1.x, sh);
        b.v1 = funnel16(r.b.v1, (uint32_t)r.b.v2.x, sh);
        b.v2 = funnel16(r.b.v2, (uint32_t)r.b.v3.x, sh);
        b.v3 = funnel16(r.b.v3, r.e, sh);
        return b;
    }
}

template <bool PIPE, bool FAKE = false, bool A4 = false>
__device__ __forceinline__ uint64_t city_gt64_reg(const uint8_t* s, uint32_t n, const Blk& t) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    const uint32_t sh = (uint32_t)(uintptr_t)s & 3;
    Blk cur = use64<A4>(ld64<A4, FAKE>(s), sh);
    u64x2 b0 = cur.v0, b1 = cur.v1, b2 = cur.v2, b3 = cur.v3;
    x = x * K1 + b0.x;
    const uint32_t blocks = (n - 1) >> 6;
    const uint8_t* last = s + 64 * (blocks - 1);
    for (uint32_t k = 0;;) {
        Blk64 nx;
        const uint8_t* ns = s + 64 < last ? s + 64 : last;
        if (PIPE) nx = ld64<A4, FAKE>(ns);
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
        if (!PIPE) nx = ld64<A4, FAKE>(s);
        cur = use64<A4>(nx, sh);
        b0 = cur.v0; b1 = cur.v1; b2 = cur.v2; b3 = cur.v3;
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

// ---------------------------------------------------------------------------
// Quad-cooperative loop loads.  The address unit's cost follows the distinct
// 128-byte lines a wave-instruction touches (tools/tabench.hip: 6.9 ns per
// instruction per CU for 1 KiB contiguous, 49 ns for 64 lanes in 64 lines,
// L2-resident), and a lane-per-value 64-byte block costs four 16-byte loads
// that each touch a line per lane.  Here the four lanes of a quad load each
// other's blocks: in round j every lane of the quad reads its 16-byte piece
// (lane & 3) of lane j's block, so one instruction touches 16 blocks (16-32
// lines) instead of 64; a 4 x 4 transpose over the quad (two butterfly
// stages of DPP quad_perm + v_cndmask) then gives each lane its own block.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int J>
__device__ __forceinline__ const uint8_t* qbcast_ptr(const uint8_t* a) {
    const uint64_t v = (uint64_t)(uintptr_t)a;
    return (const uint8_t*)(uintptr_t)pack64(qperm<J * 0x55>((uint32_t)v), qperm<J * 0x55>((uint32_t)(v >> 32)));
}
// One butterfly stage over dword t of the element pair (m, mm = m ^ D):
// the lane with bit D clear takes its partner's X[m] as its X[mm], the lane
// with bit D set takes its partner's X[mm] as its X[m].
template <int CTRL>
__device__ __forceinline__ void qswap(uint32_t& xm, uint32_t& xmm, bool hi) {
    const uint32_t recv = qperm<CTRL>(hi ? xm : xmm);
    xm = hi ? recv : xm;
    xmm = hi ? xmm : recv;
}
__device__ __forceinline__ void qswap16(u64x2& a, u64x2& b, bool hi, bool d1) {
    uint32_t a0 = (uint32_t)a.x, a1 = (uint32_t)(a.x >> 32), a2 = (uint32_t)a.y, a3 = (uint32_t)(a.y >> 32);
    uint32_t b0 = (uint32_t)b.x, b1 = (uint32_t)(b.x >> 32), b2 = (uint32_t)b.y, b3 = (uint32_t)(b.y >> 32);
    if (d1) {  // partner lane ^ 1: quad_perm [1, 0, 3, 2]
        qswap<0xB1>(a0, b0, hi); qswap<0xB1>(a1, b1, hi); qswap<0xB1>(a2, b2, hi); qswap<0xB1>(a3, b3, hi);
    } else {   // partner lane ^ 2: quad_perm [2, 3, 0, 1]
        qswap<0x4E>(a0, b0, hi); qswap<0x4E>(a1, b1, hi); qswap<0x4E>(a2, b2, hi); qswap<0x4E>(a3, b3, hi);
    }
    a.x = pack64(a0, a1); a.y = pack64(a2, a3);
    b.x = pack64(b0, b1); b.y = pack64(b2, b3);
}
// The 64 bytes at dword-aligned a (and the dword after them) of every lane;
// the whole wave must be active (quad partners read each other's addresses).
__device__ __forceinline__ Blk64 ld64_quad(const uint8_t* a) {
    const uint32_t i = threadIdx.x & 3;
    Blk64 r;
    r.b.v0 = gld16(qbcast_ptr<0>(a) + 16 * i);
    r.b.v1 = gld16(qbcast_ptr<1>(a) + 16 * i);
    r.b.v2 = gld16(qbcast_ptr<2>(a) + 16 * i);
    r.b.v3 = gld16(qbcast_ptr<3>(a) + 16 * i);
    r.e = gld4(a + 64);
    // lane i now holds piece i of the quad's blocks 0..3: transpose
    const bool b1 = (i & 2) != 0, b0 = (i & 1) != 0;
    qswap16(r.b.v0, r.b.v2, b1, false);
    qswap16(r.b.v1, r.b.v3, b1, false);
    qswap16(r.b.v0, r.b.v1, b0, true);
    qswap16(r.b.v2, r.b.v3, b0, true);
    return r;
}

// city_gt64_reg with the loop's block loads quad-cooperative: called by the
// whole wave (every lane takes part in the loads); g64 lanes get the hash.
__device__ __forceinline__ uint64_t city_gt64_quad(const uint8_t* s, uint32_t n, const Blk& t, bool g64) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    const uint32_t blocks = g64 ? (n - 1) >> 6 : 0u;
    const uint32_t sh = g64 ? (uint32_t)(uintptr_t)s & 3 : 0u;
    for (uint32_t k = 0; __builtin_amdgcn_ballot_w64(k < blocks) != 0; ++k) {
        const bool act = k < blocks;
        const Blk64 raw = ld64_quad(act ? dw_floor(s + 64 * k) : g_zero_pad);
        if (act) {
            const Blk cur = use64<true>(raw, sh);
            const u64x2 b0 = cur.v0, b1 = cur.v1, b2 = cur.v2, b3 = cur.v3;
            if (k == 0) x = x * K1 + b0.x;
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
        }
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

// city_gt64_reg (A4) with the head pieces loaded here, back to back with the
// first loop block — not a pass ahead — so that the L1 merges their requests
// for the lines they share (debug variant 190).
__device__ __forceinline__ uint64_t city_gt64_late(const uint8_t* p, uint32_t n) {
    const Raw r = issue_block_a4(CODE_STRING, p, n);
    const Blk64 b0 = ld64<true, false>(p);
    const Blk t = funnel_raw(r);
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    const uint32_t sh = (uint32_t)(uintptr_t)p & 3;
    Blk cur = use64<true>(b0, sh);
    x = x * K1 + cur.v0.x;
    const uint32_t blocks = (n - 1) >> 6;
    const uint8_t* s = p;
    for (uint32_t k = 0;;) {
        const u64x2 b_0 = cur.v0, b_1 = cur.v1, b_2 = cur.v2, b_3 = cur.v3;
        x = ror(x + y + v0 + b_0.y, 37) * K1;
        y = ror(y + v1 + b_3.x, 42) * K1;
        x ^= w1;
        y += v0 + b_2.y;
        z = ror(z + w0, 33) * K1;
        uint64_t nv0, nv1, nw0, nw1;
        weak32(b_0.x, b_0.y, b_1.x, b_1.y, v1 * K1, x + w0, nv0, nv1);
        weak32(b_2.x, b_2.y, b_3.x, b_3.y, z + w1, y + b_1.x, nw0, nw1);
        v0 = nv0; v1 = nv1; w0 = nw0; w1 = nw1;
        const uint64_t tt = z; z = x; x = tt;
        if (++k == blocks) break;
        s += 64;
        cur = use64<true>(ld64<true, false>(s), sh);
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

// A4: the block comes from issue_block_a4 (16..32-byte, short and numeric
// pieces in slots 1 and 3).
template <bool PIPE = false, bool FAKE = false, bool A4 = false>
__device__ __forceinline__ uint64_t hash_blk(uint32_t code, const uint8_t* p, uint32_t n, const Blk& b,
                                             bool& bad) {
    const uint32_t sh = (uint32_t)(uintptr_t)p & 15;
    const u64x2& f = A4 ? b.v1 : b.v0;  // first piece of the 16..32-byte / short regimes
    const u64x2& g = A4 ? b.v3 : b.v1;  // second piece
    if (code == CODE_STRING) {
        if (n > 64) return city_gt64_reg<PIPE, FAKE, A4>(p, n, b);
        if (n > 32) return city_33to64(b.v0, b.v1, b.v2, b.v3, n);
        if (n > 16) return city_17to32(f, g, n);
        return city_le16_reg(n == 16 ? f : window16(f, g, sh), n);
    }
    if (code == CODE_ZERO) return 0;
    uint64_t bits = 0;
    if (n == 8) {
        bits = window8(f, g, sh);
    } else if (n != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}

// hash_blk for a slot that is not a string (numerics, timestamps, non-hashable).
template <bool A4 = false>
__device__ __forceinline__ uint64_t hash_blk_nonstring(uint32_t code, const uint8_t* p, uint32_t n, const Blk& b,
                                                       bool& bad) {
    if (code == CODE_ZERO) return 0;
    const uint32_t sh = (uint32_t)(uintptr_t)p & 15;
    uint64_t bits = 0;
    if (n == 8) {
        bits = window8(A4 ? b.v1 : b.v0, A4 ? b.v3 : b.v1, sh);
    } else if (n != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}

// hash_blk (A4) with the > 64-byte loop quad-cooperative: called by the whole
// wave; the loop runs, wave-uniformly, while any lane has a block left.
__device__ __forceinline__ uint64_t hash_blk_quad(uint32_t code, const uint8_t* p, uint32_t n, const Blk& b,
                                                  bool& bad) {
    const bool g64 = code == CODE_STRING && n > 64;
    uint64_t hg = 0;
    if (__builtin_amdgcn_ballot_w64(g64) != 0) hg = city_gt64_quad(p, n, b, g64);
    const uint32_t sh = (uint32_t)(uintptr_t)p & 15;
    if (code == CODE_STRING) {
        if (n > 64) return hg;
        if (n > 32) return city_33to64(b.v0, b.v1, b.v2, b.v3, n);
        if (n > 16) return city_17to32(b.v1, b.v3, n);
        return city_le16_reg(n == 16 ? b.v1 : window16(b.v1, b.v3, sh), n);
    }
    if (code == CODE_ZERO) return 0;
    uint64_t bits = 0;
    if (n == 8) {
        bits = window8(b.v1, b.v3, sh);
    } else if (n != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}

// A numeric (or non-hashable) slot on its own: the dwords holding its first
// and last byte (never outside the value's pages) and two v_alignbyte —
// instead of a string slot's four 16-byte pieces.  Never called on strings.
__device__ __forceinline__ uint64_t hash_numeric_slot(uint32_t code, const uint8_t* p, uint32_t n, bool& bad) {
    if (code == CODE_ZERO) return 0;
    uint64_t bits = 0;
    if (n == 8) {
        const uint8_t* a = dw_floor(p);
        const uint32_t r = (uint32_t)(uintptr_t)p & 3;
        const uint32_t d0 = gld4(a), d1 = gld4(a + 4), d2 = gld4(dw_floor(p + 7));
        bits = pack64(__builtin_amdgcn_alignbyte(d1, d0, r), __builtin_amdgcn_alignbyte(d2, d1, r));
    } else if (n != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}

// Debug shapes (variants 40/41).  touch_blk: the loads a slot's
// hash issues (its block plus every > 64-byte loop block), folded by XOR, no
// hash arithmetic.  fake_block: a block made from the address, no loads.
__device__ __forceinline__ uint64_t touch_blk(uint32_t code, const uint8_t* p, uint32_t n, const Blk& b) {
    uint64_t h = b.v0.x ^ b.v0.y ^ b.v1.x ^ b.v1.y ^ b.v2.x ^ b.v2.y ^ b.v3.x ^ b.v3.y;
    if (code == CODE_STRING && n > 64) {
        const uint32_t blocks = (n - 1) >> 6;
        for (uint32_t k = 0; k < blocks; ++k) {
            const u64x2 a0 = gld16(p + 64 * k), a1 = gld16(p + 64 * k + 16);
            const u64x2 a2 = gld16(p + 64 * k + 32), a3 = gld16(p + 64 * k + 48);
            h ^= a0.x ^ a0.y ^ a1.x ^ a1.y ^ a2.x ^ a2.y ^ a3.x ^ a3.y;
        }
    }
    return h;
}

__device__ __forceinline__ Blk fake_block(const uint8_t* p, uint32_t n) {
    Blk b;
    b.v0 = ld16<true>(p);
    b.v1 = ld16<true>(p + n);
    b.v2 = ld16<true>(p + 2 * n);
    b.v3 = ld16<true>(p + 3 * n);
    return b;
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

// t / A for small t (t * A < 2^31) by the host's ceil(2^31 / A).
__device__ __forceinline__ uint32_t div_small(uint32_t t, uint32_t a_magic) {
    return (uint32_t)(((uint64_t)t * a_magic) >> 31);
}

// Wave-uniform slot -> (object, attribute) split without a 64-bit integer
// divide: q < 2^53, so the f64 quotient by the host's 1/A is off by at most
// one; fix it up.
__device__ __forceinline__ void split_slot(uint64_t q, uint32_t A, double inv_A, uint64_t& i0, uint32_t& j0) {
    uint64_t i = (uint64_t)((double)q * inv_A);
    int64_t rem = (int64_t)(q - i * A);
    if (rem < 0) { --i; rem += A; }
    if (rem >= (int64_t)A) { ++i; rem -= A; }
    i0 = i;
    j0 = (uint32_t)rem;
}

// XCD-aware block order: the dispatcher deals workgroups round-robin over
// the 8 XCDs (block b to XCD b % 8), each with its own L2.  Renumbering so
// that each XCD's blocks take one contiguous run of the logical order keeps
// neighbouring groups — which share the cache lines at their span edges — on
// one L2.  A bijection on [0, gridDim.x).
__device__ __forceinline__ uint32_t xcd_block() {
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t per = nb >> 3, rem = nb & 7, x = b & 7, k = b >> 3;
    return x < rem ? x * (per + 1) + k : rem * (per + 1) + (x - rem) * per + k;
}

__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t v) {
    return __builtin_amdgcn_readlane(wave_scan_dpp(v), 63);
}

}  // namespace hdx
