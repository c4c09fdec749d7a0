// hdx_lds_hash.h — hashing slots whose bytes are staged in LDS (device code).
//
// The staged kernels (hdx_staged.hip) copy a group of objects' bytes into a
// wave-private LDS window with coalesced LDS DMA (global_load_lds_dwordx4:
// 1 KiB per wave-instruction, 8 cache lines, instead of 64 lines for a
// per-lane gather), then hash out of LDS.  Every LDS read here is a
// dword-aligned ds_read_b32 / ds_read2_b32 through an address-space-3 pointer
// (a misaligned wide LDS read is replayed; a generic pointer would become a
// flat load that waits on every outstanding global load), and the bytes are
// funnel-shifted into place with v_alignbyte exactly as the dword-aligned
// global form (A4, hdx_loads.h) does, so the arithmetic is shared:
// CityHash64 v1.1 (cityhash/city.cc:278-397), the ordered encodings and the
// timestamp hash (hdx_device_hash.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_loads.h"

namespace hdx {

typedef const __attribute__((address_space(3))) uint32_t* ldsw_t;  // LDS dwords
typedef __attribute__((address_space(3))) uint32_t* ldsw_mut_t;

__device__ __forceinline__ ldsw_t as_ldsw(const void* p) { return (ldsw_t)p; }

// LDS DMA (global_load_lds_dwordx4 / _dword: lane l's 16 / 4 bytes from src
// to dst + 16 l / 4 l, dst wave-uniform into M0) as inline asm.  The
// compiler's wait insertion does not see these, so it neither drains them
// before an unrelated load's use, nor before the first LDS atomic or read of
// the wave's metadata (it cannot tell those from the window), nor again after
// the kernel's own drain (then waiting on any store issued since).  The
// kernels wait for them themselves (s_waitcnt vmcnt(0) before the window is
// read).  Any wait the compiler emits for its own loads still covers them
// (vmcnt counts in issue order), at worst waiting longer.
// An SALU write of M0 needs one wait state before an LDS-DMA reads it (the
// s_nop 0 the compiler puts after its own M0 writes).
__device__ __forceinline__ uint32_t lds_addr_s(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)p);
}
__device__ __forceinline__ void dma_x4_asm(const void* src, const void* dst) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_addr_s(dst))
                 : "memory", "m0");
}
__device__ __forceinline__ void dma_x1_asm(const void* src, const void* dst) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(lds_addr_s(dst))
                 : "memory", "m0");
}

// round 3's span copy (debug forms): both addresses and the predicate per KiB
template <bool ASM>
__device__ __forceinline__ void dma_units16_loop(const uint8_t* src, void* dst, uint32_t units) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t u0 = 0; u0 < units; u0 += 64) {
        const uint32_t u = u0 + lane;
        if (u < units) {
            if constexpr (ASM) dma_x4_asm(src + 16ull * u, (uint8_t*)dst + 16 * u0);
            else __builtin_amdgcn_global_load_lds((const void*)(src + 16ull * u),
                                                  (__attribute__((address_space(3))) void*)((uint8_t*)dst + 16 * u0), 16, 0, 0);
        }
    }
}

// A span copy: `units` 16-byte units from src (16-byte aligned) to LDS dst,
// lane l copying units l, l + 64, ...  The instruction's immediate offset
// applies to both the global and the LDS address, so one VGPR address and
// one M0 serve four wave-instructions (4 KiB); only the last, partial 1 KiB
// is predicated (round 3's loop recomputed both addresses and the predicate
// for every KiB: ~6 VALU + ~8 SALU each).  ASM: inline asm (not seen by the
// compiler's waits), else the builtin.
// NT: the loads non-temporal (the `nt` policy bit: the span is read once).
#define HDX_DMA_ASM(NTS, OFFS) "s_mov_b32 m0, %1\n\ts_nop 0\n\t" OFFS(NTS)
#define HDX_DMA1(NTS) "global_load_lds_dwordx4 %0, off" NTS
#define HDX_DMA2(NTS) HDX_DMA1(NTS) "\n\tglobal_load_lds_dwordx4 %0, off offset:1024" NTS
#define HDX_DMA3(NTS) HDX_DMA2(NTS) "\n\tglobal_load_lds_dwordx4 %0, off offset:2048" NTS
#define HDX_DMA4(NTS) HDX_DMA3(NTS) "\n\tglobal_load_lds_dwordx4 %0, off offset:3072" NTS
#define HDX_DMA_EMIT(N)                                                                                      \
    do {                                                                                                     \
        if constexpr (NT) asm volatile(HDX_DMA_ASM(" nt", HDX_DMA##N)::"v"(p), "s"(m0) : "memory", "m0"); \
        else asm volatile(HDX_DMA_ASM("", HDX_DMA##N)::"v"(p), "s"(m0) : "memory", "m0");                  \
    } while (0)
template <bool ASM, bool NT = false>
__device__ __forceinline__ void dma_units16(const uint8_t* src, void* dst, uint32_t units) {
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass cannot instantiate the VGPR / SGPR constraints
    constexpr int POL = NT ? 2 : 0;  // the builtin's cache-policy operand: nt
    const uint32_t lane = threadIdx.x & 63;
    const uint8_t* p = src + 16 * lane;
    uint32_t m0 = lds_addr_s(dst);
    auto at = [&](uint32_t a) { return (__attribute__((address_space(3))) void*)(uintptr_t)a; };
    uint32_t full = __builtin_amdgcn_readfirstlane(units >> 6);
    for (; full >= 4; full -= 4) {
        if constexpr (ASM)
            HDX_DMA_EMIT(4);
        else {
            __builtin_amdgcn_global_load_lds(p, at(m0), 16, 0, POL);
            __builtin_amdgcn_global_load_lds(p, at(m0), 16, 1024, POL);
            __builtin_amdgcn_global_load_lds(p, at(m0), 16, 2048, POL);
            __builtin_amdgcn_global_load_lds(p, at(m0), 16, 3072, POL);
        }
        p += 4096;
        m0 += 4096;
    }
    if (full) {
        if constexpr (ASM) {
            if (full == 1) HDX_DMA_EMIT(1);
            else if (full == 2) HDX_DMA_EMIT(2);
            else HDX_DMA_EMIT(3);
        } else {
            __builtin_amdgcn_global_load_lds(p, at(m0), 16, 0, POL);
            if (full >= 2) __builtin_amdgcn_global_load_lds(p, at(m0), 16, 1024, POL);
            if (full >= 3) __builtin_amdgcn_global_load_lds(p, at(m0), 16, 2048, POL);
        }
        p += 1024 * full;
        m0 += 1024 * full;
    }
    if (lane < (units & 63)) {
        if constexpr (ASM)
            HDX_DMA_EMIT(1);
        else
            __builtin_amdgcn_global_load_lds(p, at(m0), 16, 0, POL);
    }
#endif
}
#undef HDX_DMA_EMIT

// 16 bytes at a dword-aligned LDS address as one ds_read_b128 (gfx950 serves
// dword-aligned b128 reads; the compiler emits them for 4-byte-aligned
// vectors).  W128 forms below read 4 dwords per instruction instead of 2.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef u32x4_t __attribute__((aligned(4))) u32x4_a4;
__device__ __forceinline__ u32x4_t lds_q(ldsw_t d) { return *(const __attribute__((address_space(3))) u32x4_a4*)d; }

// little-endian u32 at byte offset b of the window (any alignment)
__device__ __forceinline__ uint32_t lds_u32(ldsw_t w, uint32_t b) {
    const ldsw_t d = w + (b >> 2);
    return __builtin_amdgcn_alignbyte(d[1], d[0], b & 3);
}
__device__ __forceinline__ uint32_t lds_be32(ldsw_t w, uint32_t b) { return __builtin_bswap32(lds_u32(w, b)); }

// the 16 bytes at dword-aligned byte offset o
__device__ __forceinline__ u64x2 lds16(ldsw_t w, int32_t o) {
    const ldsw_t d = w + (o >> 2);
    u64x2 v;
    v.x = pack64(d[0], d[1]);
    v.y = pack64(d[2], d[3]);
    return v;
}

// A slot's A4 pieces (a4_offsets' layout, hdx_loads.h) out of the window;
// a slot with nothing to read reads the window's first dwords.
__device__ __forceinline__ Blk lds_block_a4(ldsw_t w, uint32_t code, uint32_t off, uint32_t n) {
    const A4Offsets o = a4_offsets(code, off, n);
    const int32_t base = o.any ? (int32_t)off : 0;
    Raw r;
    r.ra = o.ra;
    r.rb = o.rb;
    r.b.v0 = lds16(w, base + o.o0);
    r.b.v1 = lds16(w, base + o.o1);
    r.b.v2 = lds16(w, base + o.o2);
    r.b.v3 = lds16(w, base + o.o3);
    r.e1 = w[(base + o.e1) >> 2];
    r.e3 = w[(base + o.e3) >> 2];
    return funnel_raw(r);
}

// One 64-byte CityHash loop block at byte offset s: the 17 dwords from its
// dword floor, funnel-shifted (every loop block ends before the value does).
__device__ __forceinline__ Blk lds_block64(ldsw_t w, uint32_t s) {
    const ldsw_t d = w + (s >> 2);
    Blk64 b;
    b.b.v0.x = pack64(d[0], d[1]);
    b.b.v0.y = pack64(d[2], d[3]);
    b.b.v1.x = pack64(d[4], d[5]);
    b.b.v1.y = pack64(d[6], d[7]);
    b.b.v2.x = pack64(d[8], d[9]);
    b.b.v2.y = pack64(d[10], d[11]);
    b.b.v3.x = pack64(d[12], d[13]);
    b.b.v3.y = pack64(d[14], d[15]);
    b.e = d[16];
    return use64<true>(b, s & 3);
}

// Debug shapes (WRONG coordinates): W128 == 2 (variant 248) the same reads at
// addresses whose 32 lanes of a half-wave fall on 32 distinct banks — what
// the per-lane byte offsets' bank conflicts cost; W128 == 3 (249) the reads
// at the dword floor with no funnel shift — what the v_alignbyte cost.
__device__ __forceinline__ ldsw_t conflict_free(ldsw_t w, uint32_t o) {
    return w + (((o >> 2) & ~1023u) | (uint32_t)(threadIdx.x & 31));
}

__device__ __forceinline__ Blk lds_block64_w128(ldsw_t w, uint32_t s) {
    const ldsw_t d = w + (s >> 2);
    const u32x4_t q0 = lds_q(d), q1 = lds_q(d + 4), q2 = lds_q(d + 8), q3 = lds_q(d + 12);
    Blk64 b;
    b.b.v0.x = pack64(q0.x, q0.y);
    b.b.v0.y = pack64(q0.z, q0.w);
    b.b.v1.x = pack64(q1.x, q1.y);
    b.b.v1.y = pack64(q1.z, q1.w);
    b.b.v2.x = pack64(q2.x, q2.y);
    b.b.v2.y = pack64(q2.z, q2.w);
    b.b.v3.x = pack64(q3.x, q3.y);
    b.b.v3.y = pack64(q3.z, q3.w);
    b.e = d[16];
    return use64<true>(b, s & 3);
}

// city.cc:361-397 for n > 64: the tail block t in registers, the loop blocks
// read from the window (city_gt64_reg's arithmetic).
// LOOP 1: one block per trip, the next block read at its end (its registers
// then copied into the current block's, and x / z swapped by copies: ~9
// v_mov_b64 a trip); LOOP 2: two blocks per trip, the block after next read
// into the other register set before the current one is hashed, and x / z
// trading roles instead of places — no copies.  A read past the string's last
// block stays inside the LDS allocation or reads 0; its data are never used.
__device__ __forceinline__ void city_loop_step(uint64_t& x, uint64_t& y, uint64_t& z, uint64_t& v0, uint64_t& v1,
                                               uint64_t& w0, uint64_t& w1, const Blk& b) {
    x = ror(x + y + v0 + b.v0.y, 37) * K1;
    y = ror(y + v1 + b.v3.x, 42) * K1;
    x ^= w1;
    y += v0 + b.v2.y;
    z = ror(z + w0, 33) * K1;
    uint64_t nv0, nv1, nw0, nw1;
    weak32(b.v0.x, b.v0.y, b.v1.x, b.v1.y, v1 * K1, x + w0, nv0, nv1);
    weak32(b.v2.x, b.v2.y, b.v3.x, b.v3.y, z + w1, y + b.v1.x, nw0, nw1);
    v0 = nv0; v1 = nv1; w0 = nw0; w1 = nw1;
    // std::swap(z, x) is the caller's (LOOP 2: the next step gets them swapped)
}

// ... up to its last mix16: the result is mix16(u, v, KMUL) (LOOP 3 shares
// that mix16 with the <= 32-byte regimes' own, hash_slot_window).
template <int W128 = 0, int LOOP = 1>
__device__ __forceinline__ void city_gt64_lds_uv(ldsw_t w, uint32_t off, uint32_t n, const Blk& t, uint64_t& u,
                                                 uint64_t& v) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    const uint32_t blocks = (n - 1) >> 6;
    auto rd = [&](uint32_t o) {
        if constexpr (W128 == 2) return lds_block64(conflict_free(w, o), o & 3);
        else if constexpr (W128 == 3) return lds_block64(w + (o >> 2), 0);
        else return W128 ? lds_block64_w128(w, o) : lds_block64(w, o);
    };
    if constexpr (LOOP >= 2) {
        Blk ba = rd(off);
        x = x * K1 + ba.v0.x;
        for (uint32_t k = 0;;) {
            const Blk bb = rd(off + 64 * (k + 1));
            city_loop_step(x, y, z, v0, v1, w0, w1, ba);  // leaves x and z swapped: z is x now
            if (++k == blocks) {
                const uint64_t tt = z; z = x; x = tt;
                break;
            }
            ba = rd(off + 64 * (k + 1));
            city_loop_step(z, y, x, v0, v1, w0, w1, bb);  // roles traded back
            if (++k == blocks) break;
        }
    } else {
        Blk b = rd(off);
        x = x * K1 + b.v0.x;
        for (uint32_t k = 0;;) {
            city_loop_step(x, y, z, v0, v1, w0, w1, b);
            const uint64_t tt = z; z = x; x = tt;
            if (++k == blocks) break;
            b = rd(off + 64 * k);
        }
    }
    u = mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z;
    v = mix16(v1, w1, KMUL) + x;
}
template <int W128 = 0, int LOOP = 1>
__device__ __forceinline__ uint64_t city_gt64_lds(ldsw_t w, uint32_t off, uint32_t n, const Blk& t) {
    uint64_t u, v;
    city_gt64_lds_uv<W128, LOOP>(w, off, n, t, u, v);
    return mix16(u, v, KMUL);
}

// hash(type, slice) of a string slot at byte offset off of the window
// (hash_blk's regimes on the A4 piece layout).
__device__ __forceinline__ uint64_t hash_string_lds(ldsw_t w, uint32_t off, uint32_t n) {
    const Blk b = lds_block_a4(w, CODE_STRING, off, n);
    if (n > 64) return city_gt64_lds(w, off, n, b);
    if (n > 32) return city_33to64(b.v0, b.v1, b.v2, b.v3, n);
    if (n > 16) return city_17to32(b.v1, b.v3, n);
    return city_le16_reg(n == 16 ? b.v1 : window16(b.v1, b.v3, off & 15), n);
}

// A numeric (or non-hashable) slot at byte offset off of the window: the
// dwords holding its first and last byte, two v_alignbyte.
__device__ __forceinline__ uint64_t hash_numeric_lds(ldsw_t w, uint32_t code, uint32_t off, uint32_t n, bool& bad) {
    if (code == CODE_ZERO) return 0;
    uint64_t bits = 0;
    if (n == 8) {
        const ldsw_t d = w + (off >> 2);
        const uint32_t r = off & 3;
        const uint32_t d0 = d[0], d1 = d[1], d2 = w[(off + 7) >> 2];
        bits = pack64(__builtin_amdgcn_alignbyte(d1, d0, r), __builtin_amdgcn_alignbyte(d2, d1, r));
    } else if (n != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}

// 32 bytes at window byte offset o (any alignment): q[k] = bytes [o+8k, o+8k+8)
struct Q32 {
    uint64_t q0, q1, q2, q3;
};
template <int W128 = 0>
__device__ __forceinline__ Q32 lds_read32(ldsw_t w, uint32_t o) {
    const ldsw_t d = W128 == 2 ? conflict_free(w, o) : w + (o >> 2);
    const uint32_t r = W128 == 3 ? 0 : o & 3;
    uint32_t x[9];
    if constexpr (W128 == 1) {
        const u32x4_t a = lds_q(d), b = lds_q(d + 4);
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
        x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
        x[8] = d[8];
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) x[i] = d[i];
    }
    Q32 q;
    q.q0 = pack64(__builtin_amdgcn_alignbyte(x[1], x[0], r), __builtin_amdgcn_alignbyte(x[2], x[1], r));
    q.q1 = pack64(__builtin_amdgcn_alignbyte(x[3], x[2], r), __builtin_amdgcn_alignbyte(x[4], x[3], r));
    q.q2 = pack64(__builtin_amdgcn_alignbyte(x[5], x[4], r), __builtin_amdgcn_alignbyte(x[6], x[5], r));
    q.q3 = pack64(__builtin_amdgcn_alignbyte(x[7], x[6], r), __builtin_amdgcn_alignbyte(x[8], x[7], r));
    return q;
}
__device__ __forceinline__ uint64_t lds_read8(ldsw_t w, uint32_t o) {
    const ldsw_t d = w + (o >> 2);
    const uint32_t r = o & 3;
    const uint32_t x0 = d[0], x1 = d[1], x2 = d[2];
    return pack64(__builtin_amdgcn_alignbyte(x1, x0, r), __builtin_amdgcn_alignbyte(x2, x1, r));
}

// city.cc:278-301 (HashLen0to16) from s[0,8) and s[n-8,n).
__device__ __forceinline__ uint64_t city_le16_ht(uint64_t h0, uint64_t t3, uint32_t n) {
    const uint64_t mul = K2 + 2ull * n;
    if (n >= 8) {
        const uint64_t a = h0 + K2;
        return mix16(ror(t3, 37) * mul + a, (ror(a, 25) + t3) * mul, mul);
    }
    if (n >= 4) return mix16(n + ((h0 & 0xffffffffull) << 3), t3 >> 32, mul);
    if (n > 0) {
        const uint32_t d0 = (uint32_t)h0;
        const uint32_t y = (d0 & 0xff) + (((d0 >> (8 * (n >> 1))) & 0xff) << 8);
        const uint32_t z = n + ((uint32_t)(t3 >> 56) << 2);
        return shiftmix((uint64_t)y * K2 ^ (uint64_t)z * K0) * K2;
    }
    return K2;
}

// hash(type, slice) of a slot whose bytes start at window byte offset off,
// from its first and last 32 bytes (two reads that serve every regime:
// HashLen0to16 / 17to32 / 33to64 / the > 64-byte tail block) and, over 64
// bytes, the loop blocks.  The window needs 32 readable bytes before off
// (s[n-32, n) of a short string) and 36 after the value's end.
// A string slot from its last 32 bytes t (already read) and, as its regime
// needs, its first 32 and its loop blocks (hash_slot_window's string side).
template <int W128 = 0, int LOOP = 1>
__device__ __forceinline__ uint64_t hash_string_window(ldsw_t w, uint32_t off, uint32_t n, const Q32& t) {
    const u64x2 t01 = {t.q0, t.q1}, t23 = {t.q2, t.q3};
    if constexpr (LOOP >= 4) {
        // LOOP 3's shared final mix16 (also for 4..7-byte strings) with one head
        // read for both sides of the regime branch: s[n-64, n-32) over 64 bytes,
        // else s[0, 32)
        const Q32 h = lds_read32<W128>(w, n > 64 ? off + n - 64 : off);
        uint64_t u, v, mul;
        if (n > 64) {
            Blk b;
            b.v0 = u64x2{h.q0, h.q1};
            b.v1 = u64x2{h.q2, h.q3};
            b.v2 = t01;
            b.v3 = t23;
            city_gt64_lds_uv<W128, 2>(w, off, n, b, u, v);
            mul = KMUL;
        } else {
            if (n > 32) return city_33to64(u64x2{h.q0, h.q1}, u64x2{h.q2, h.q3}, t01, t23, n);
            if (n < 4) return city_le16_ht(h.q0, t.q3, n);
            mul = K2 + 2ull * n;
            if (n > 16) {  // city.cc:305-313 (city_17to32)
                const uint64_t a = h.q0 * K1, b = h.q1, c = t.q3 * mul, d = t.q2 * K2;
                u = ror(a + b, 43) + ror(c, 30) + d;
                v = a + ror(b + K2, 18) + c;
            } else if (n >= 8) {  // city.cc:281-286 (city_le16_ht, n >= 8)
                const uint64_t a = h.q0 + K2;
                u = ror(t.q3, 37) * mul + a;
                v = (ror(a, 25) + t.q3) * mul;
            } else {  // city.cc:287-291 (4 <= n < 8): Fetch32(s) and Fetch32(s + n - 4)
                u = n + ((h.q0 & 0xffffffffull) << 3);
                v = t.q3 >> 32;
            }
        }
        return mix16(u, v, mul);
    } else if constexpr (LOOP >= 3) {
        uint64_t u, v, mul;
        if (n > 64) {
            const Q32 q = lds_read32<W128>(w, off + n - 64);
            Blk b;
            b.v0 = u64x2{q.q0, q.q1};
            b.v1 = u64x2{q.q2, q.q3};
            b.v2 = t01;
            b.v3 = t23;
            city_gt64_lds_uv<W128, 2>(w, off, n, b, u, v);
            mul = KMUL;
        } else {
            const Q32 h = lds_read32<W128>(w, off);  // s[0, 32): the back pad covers n < 32
            if (n > 32) return city_33to64(u64x2{h.q0, h.q1}, u64x2{h.q2, h.q3}, t01, t23, n);
            if (n < 8) return city_le16_ht(h.q0, t.q3, n);
            mul = K2 + 2ull * n;
            if (n > 16) {  // city.cc:305-313 (city_17to32)
                const uint64_t a = h.q0 * K1, b = h.q1, c = t.q3 * mul, d = t.q2 * K2;
                u = ror(a + b, 43) + ror(c, 30) + d;
                v = a + ror(b + K2, 18) + c;
            } else {  // city.cc:281-286 (city_le16_ht, n >= 8)
                const uint64_t a = h.q0 + K2;
                u = ror(t.q3, 37) * mul + a;
                v = (ror(a, 25) + t.q3) * mul;
            }
        }
        return mix16(u, v, mul);
    }
    // one read serves both sides of the regime branch (a pass holding long and
    // short strings runs both): s[n-64, n-32) over 64 bytes, else s[0, 32)
    // (the back pad covers n < 32)
    const Q32 h = lds_read32<W128>(w, n > 64 ? off + n - 64 : off);
    if (n > 64) {
        Blk b;
        b.v0 = u64x2{h.q0, h.q1};
        b.v1 = u64x2{h.q2, h.q3};
        b.v2 = t01;
        b.v3 = t23;
        return city_gt64_lds<W128, (LOOP > 2 ? 2 : LOOP)>(w, off, n, b);
    }
    const u64x2 h01 = {h.q0, h.q1};
    if (n > 32) return city_33to64(h01, u64x2{h.q2, h.q3}, t01, t23, n);
    if (n > 16) return city_17to32(h01, t23, n);
    return city_le16_ht(h.q0, t.q3, n);
}

// LOOP: city_gt64_lds's; LOOP 3 = LOOP 2 with one final mix16 shared by the
// > 64-byte regime and the 8..32-byte ones (a pass holding both runs it once);
// LOOP 4 = LOOP 3 with one head read for both sides of the regime branch.
// TNUM: every slot reads its last 32 bytes before the type dispatch, and an
// 8-byte numeric takes its value from them (q3) — one read for the numeric
// and string lanes of a pass instead of two.
// NUM2: the schema's codes are STRING / INT64 / FLOAT only (pads CODE_ZERO):
// numerics by selects (encode_int64 / encode_double_sel), no timestamp code.
template <int W128 = 0, int LOOP = 1, bool TNUM = false, bool NUM2 = false>
__device__ __forceinline__ uint64_t hash_slot_window(ldsw_t w, uint32_t code, uint32_t off, uint32_t n, bool& bad) {
    if constexpr (NUM2) {
        static_assert(TNUM, "NUM2 takes the numeric from the tail read");
        const Q32 t = lds_read32<W128>(w, off + n - 32);  // the front pad covers n < 32
        if (code == CODE_STRING) return hash_string_window<W128, LOOP>(w, off, n, t);
        const bool num = code != CODE_ZERO;
        bad |= num && n != 8 && n != 0;
        const uint64_t bits = n == 8 ? t.q3 : 0;
        const uint64_t h = code == CODE_FLOAT ? encode_double_sel(bits) : encode_int64(bits);
        return num && (n == 8 || n == 0) ? h : 0;
    }
    if constexpr (TNUM) {
        if (code == CODE_ZERO) return 0;
        const Q32 t = lds_read32<W128>(w, off + n - 32);  // the front pad covers n < 32
        if (code != CODE_STRING) {
            if (n != 8 && n != 0) {
                bad = true;
                return 0;
            }
            return hash_numeric(code, n == 8 ? t.q3 : 0);
        }
        return hash_string_window<W128, LOOP>(w, off, n, t);
    }
    if (code == CODE_STRING)
        return hash_string_window<W128, LOOP>(w, off, n, lds_read32<W128>(w, off + n - 32));  // front pad: n < 32
    if (code == CODE_ZERO) return 0;
    uint64_t bits = 0;
    if (n == 8) {
        bits = lds_read8(w, off);
    } else if (n != 0) {
        bad = true;
        return 0;
    }
    return hash_numeric(code, bits);
}


}  // namespace hdx
