// hdx_encoded_staged.hip — the reindex sweep
// with each group of stored objects staged in LDS (variant 64 family).
//
// Same contract as hash_encoded_kernel (hdx_encoded.hip): decode every value
// [u64 BE version][u16 BE count]{[u32 BE len][bytes]}
// (daemon/datalayer_encodings.cc:139-217) and hash its attributes and the key
// (common/hash.cc:56-68) into coords, row-major.
//
// Why a second shape.  The lane-per-object walk of hash_encoded_kernel is a
// chain of dependent HBM loads (one per length prefix, ~68 bytes apart, so it
// touches every line of every value); covering its latency takes ~500 objects
// in flight per CU, which is more than the CU's L2 share, so the hash passes
// that follow re-read every value from HBM.  Here one wave
// owns G consecutive objects at a time:
//   1. their keys and values, when each forms one contiguous run (the packed
//      layout the sweep is fed) and fits the wave's LDS window, are copied
//      into LDS with coalesced 16-byte LDS DMA (global_load_lds_dwordx4) —
//      every HBM line crosses the fabric once, in one round trip;
//   2. lanes 0..G-1 walk their value's length prefixes in LDS (a chain of LDS
//      reads, not HBM round trips) and write one {LDS offset, length}
//      descriptor per slot;
//   3. passes of 64 slots in slot (= coordinate) order hash from LDS — dword
//      reads funnel-shifted with v_alignbyte, as the A4 global form — and
//      store each pass's coordinates with one coalesced store.
// A group that is not contiguous or does not fit is walked and hashed from
// global memory (the A4 loads of hdx_loads.h) in the same wave, so any layout
// is handled; the staged and global forms give identical coordinates.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_loads.h"

namespace hdx {

namespace {

typedef uint32_t __attribute__((aligned(1))) u32_u;
typedef uint64_t __attribute__((aligned(1))) u64_u;
typedef uint16_t __attribute__((aligned(1))) u16_u;

__device__ __forceinline__ uint32_t gload_be32(const uint8_t* p) {
    return __builtin_bswap32(*(const __attribute__((address_space(1))) u32_u*)p);
}
__device__ __forceinline__ uint64_t gload_be64(const uint8_t* p) {
    return __builtin_bswap64(*(const __attribute__((address_space(1))) u64_u*)p);
}
__device__ __forceinline__ uint32_t gload_be16(const uint8_t* p) {
    const uint16_t v = *(const __attribute__((address_space(1))) u16_u*)p;
    return (uint32_t)(uint16_t)((v >> 8) | (v << 8));
}

// ---------------------------------------------------------------------------
// Reading bytes from the LDS window (16-byte aligned base, so a byte offset's
// alignment mod 16 is its global address's): dword reads, funnel-shifted.
// ---------------------------------------------------------------------------
// the little-endian u32 at byte offset b (any alignment)
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* w, uint32_t b) {
    const uint32_t* d = w + (b >> 2);
    return __builtin_amdgcn_alignbyte(d[1], d[0], b & 3);
}
__device__ __forceinline__ uint32_t lds_be32(const uint32_t* w, uint32_t b) { return __builtin_bswap32(lds_u32(w, b)); }

__device__ __forceinline__ u64x2 lds16(const uint32_t* w, int32_t byte_off) {
    const uint32_t* d = w + (byte_off >> 2);
    u64x2 v;
    v.x = pack64(d[0], d[1]);
    v.y = pack64(d[2], d[3]);
    return v;
}

// The A4 pieces of a slot at byte offset off of the window (a4_offsets'
// layout; a slot with nothing to read points at offset 0).
template <bool FAKE = false>
__device__ __forceinline__ Blk lds_block_a4(const uint32_t* w, uint32_t code, uint32_t off, uint32_t n) {
    if constexpr (FAKE) {
        Blk b;
        b.v0 = u64x2{off * 0x9e3779b97f4a7c15ull, n};
        b.v1 = u64x2{off ^ n, off + 3};
        b.v2 = u64x2{off * 7, n * 5};
        b.v3 = u64x2{off + n, off - n};
        return b;
    }
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

// One 64-byte loop block at byte offset s of the window (17 dwords from the
// dword floor; every loop block ends before the value does).
template <bool FAKE = false>
__device__ __forceinline__ Blk lds_block64(const uint32_t* w, uint32_t s) {
    if constexpr (FAKE) {
        Blk b;
        b.v0 = u64x2{s * 0x9e3779b97f4a7c15ull, s};
        b.v1 = u64x2{s ^ 77, s + 3};
        b.v2 = u64x2{s * 7, s * 5};
        b.v3 = u64x2{s + 11, s - 1};
        return b;
    }
    const uint32_t* d = w + (s >> 2);
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

// city.cc:361-397 for n > 64: the tail block t in registers, the loop blocks
// read from the window (city_gt64_reg's arithmetic).
template <bool FAKE = false>
__device__ __forceinline__ uint64_t city_gt64_lds(const uint32_t* w, uint32_t off, uint32_t n, const Blk& t) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    const uint32_t blocks = (n - 1) >> 6;
    Blk b = lds_block64<FAKE>(w, off);
    x = x * K1 + b.v0.x;
    for (uint32_t k = 0;;) {
        x = ror(x + y + v0 + b.v0.y, 37) * K1;
        y = ror(y + v1 + b.v3.x, 42) * K1;
        x ^= w1;
        y += v0 + b.v2.y;
        z = ror(z + w0, 33) * K1;
        uint64_t nv0, nv1, nw0, nw1;
        weak32(b.v0.x, b.v0.y, b.v1.x, b.v1.y, v1 * K1, x + w0, nv0, nv1);
        weak32(b.v2.x, b.v2.y, b.v3.x, b.v3.y, z + w1, y + b.v1.x, nw0, nw1);
        v0 = nv0; v1 = nv1; w0 = nw0; w1 = nw1;
        const uint64_t tt = z; z = x; x = tt;
        if (++k == blocks) break;
        b = lds_block64<FAKE>(w, off + 64 * k);
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

// hash_blk (A4 piece layout) with the > 64-byte loop reading the window.
template <bool FAKE = false>
__device__ __forceinline__ uint64_t hash_blk_lds(const uint32_t* w, uint32_t code, uint32_t off, uint32_t n,
                                                 const Blk& b, bool& bad) {
    const uint32_t sh = off & 15;
    if (code == CODE_STRING) {
        if (n > 64) return city_gt64_lds<FAKE>(w, off, n, b);
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

__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
    return pack64(__builtin_amdgcn_readfirstlane((uint32_t)v), __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)));
}

// the regroup kernel's work classes in ORDER 1 (hdx_kernels.hip work_class):
// numerics, 33..64, <= 16, 17..32, then > 64 B by loop blocks
__device__ __forceinline__ uint32_t work_class1(uint32_t code, uint32_t n) {
    if (code != CODE_STRING) return 0;
    if (n > 64) {
        const uint32_t b = (n - 1) >> 6;
        return b >= 4 ? 7u : 3u + b;
    }
    return n > 32 ? 1u : n <= 16 ? 2u : 3u;
}

struct alignas(8) SDesc {
    uint32_t off;  // staged: byte offset in the window; global: offset in the value (key)
    uint32_t len;
};
constexpr uint32_t kZero = 0xffffffffu;

}  // namespace

// Per-wave LDS: the window (+16 bytes: dword reads may run one dword past a
// full window), G descriptor rows of A slots, G {value, key} bases, codes.
__host__ __device__ constexpr size_t staged_lds_bytes(uint32_t A, uint32_t G, uint32_t WB) {
    return WB + 16 + (size_t)G * A * sizeof(SDesc) + (size_t)G * 16 + 256;
}

namespace {

// One object's metadata per lane (lanes < objects in the group).
struct GroupMeta {
    uint64_t voff, koff;
    uint32_t vlen, klen;
};

// Where a group's bytes are and whether they are staged (wave-uniform).
struct GroupSpan {
    const uint8_t* vsrc;  // 16-byte aligned start of the values' cover
    const uint8_t* ksrc;  // ... of the keys' cover
    uint64_t vfirst, kfirst;
    uint32_t vsh, ksh, vunits, units, nobj;
    uint32_t staged;
};

// lane + 1's value (lane 63 reads its own)
__device__ __forceinline__ uint64_t shfl_next64(uint64_t v, int lane) {
    const int src = (lane < 63 ? lane + 1 : lane) << 2;
    return pack64((uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)v),
                  (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(v >> 32)));
}

template <int G>
__device__ __forceinline__ GroupMeta load_meta(const EncodedArgs& a, uint64_t g, int lane) {
    GroupMeta m{0, 0, 0u, 0u};
    const uint64_t i = g * G + (uint64_t)lane;
    if (lane < G && i < a.n) {
        m.voff = a.val_off[i];
        m.koff = a.key_off[i];
        m.vlen = a.val_len[i];
        m.klen = a.key_len[i];
    }
    return m;
}

// The group's values and keys are staged when each forms one contiguous run
// (object o+1 starts where object o ends) and both covers fit the window.
template <int G, int WB>
__device__ __forceinline__ GroupSpan make_span(const EncodedArgs& a, const GroupMeta& m, uint64_t g, int lane) {
    GroupSpan s;
    const uint64_t o0 = g * G;
    s.nobj = (uint32_t)min<uint64_t>(G, a.n - o0);
    const uint64_t vnext = shfl_next64(m.voff + m.vlen, lane), knext = shfl_next64(m.koff + m.klen, lane);
    s.vfirst = readfirstlane64(m.voff);
    s.kfirst = readfirstlane64(m.koff);
    const int last = (int)s.nobj - 1;
    const uint64_t vend = pack64(__builtin_amdgcn_readlane((uint32_t)(m.voff + m.vlen), last),
                                 __builtin_amdgcn_readlane((uint32_t)((m.voff + m.vlen) >> 32), last));
    const uint64_t kend = pack64(__builtin_amdgcn_readlane((uint32_t)(m.koff + m.klen), last),
                                 __builtin_amdgcn_readlane((uint32_t)((m.koff + m.klen) >> 32), last));
    const bool runs = __all(!(lane + 1 < (int)s.nobj) || (vnext == m.voff + m.vlen && knext == m.koff + m.klen));
    s.vsh = (uint32_t)((uintptr_t)(a.vals + s.vfirst) & 15);
    s.ksh = (uint32_t)((uintptr_t)(a.keys + s.kfirst) & 15);
    const uint64_t vbytes = (s.vsh + (vend - s.vfirst) + 15) & ~15ull;
    const uint64_t kbytes = (s.ksh + (kend - s.kfirst) + 15) & ~15ull;
    s.staged = runs && vbytes + kbytes <= (uint64_t)WB;
    s.vsrc = a.vals + s.vfirst - s.vsh;
    s.ksrc = a.keys + s.kfirst - s.ksh;
    s.vunits = s.staged ? (uint32_t)(vbytes >> 4) : 0u;
    s.units = s.staged ? (uint32_t)((vbytes + kbytes) >> 4) : 0u;
    return s;
}

// Every 16-byte unit of the covers, values then keys, in flight at once
// (unit k*64 + lane in r[k]); a unit holds at least one value / key byte.
template <int U>
__device__ __forceinline__ void issue_window(const GroupSpan& s, u64x2 (&r)[U], int lane) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint32_t u = (uint32_t)(k * 64 + lane);
        if (u < s.units) {
            const uint8_t* src = u < s.vunits ? s.vsrc + 16ull * u : s.ksrc + 16ull * (u - s.vunits);
            r[k] = *(const __attribute__((address_space(1))) u64x2*)src;
        }
    }
}

template <int U>
__device__ __forceinline__ void store_window(const GroupSpan& s, const u64x2 (&r)[U], uint32_t* win, int lane) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint32_t u = (uint32_t)(k * 64 + lane);
        if (u < s.units) *reinterpret_cast<u64x2*>(&win[u * 4]) = r[k];
    }
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

// A persistent wave walks groups g = blockIdx.x, + gridDim.x, ...; while it
// decodes and hashes group g out of LDS, group g+1's bytes are in flight into
// registers (they go to LDS at the top of the next iteration) and group g+2's
// metadata is loading, so each wave keeps one group of HBM reads outstanding
// at all times and the hash arithmetic hides them.
// MODE (debug variants 67-70, wrong coordinates): 1 = the slot reads from
// LDS without the hash arithmetic, 2 = the arithmetic on made-up blocks,
// 3 = no prefix walk (made-up descriptors), 4 = no hash passes.
template <int G, int WB, int MODE = 0, int WPE = 1>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
hash_encoded_pipe_kernel(const EncodedArgs a, uint64_t ngroups) {
    static_assert(G <= 64 && WB % 1024 == 0 && WB < 65536, "group shape");
    constexpr int U = WB / 1024;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const uint32_t A = a.A;
    const int lane = threadIdx.x;
    uint32_t* win = reinterpret_cast<uint32_t*>(smem_raw);
    SDesc* desc = reinterpret_cast<SDesc*>(smem_raw + WB + 16);
    uint64_t* bases = reinterpret_cast<uint64_t*>(smem_raw + WB + 16 + (size_t)G * A * sizeof(SDesc));
    uint8_t* codes = reinterpret_cast<uint8_t*>(bases + 2 * G);
    uint64_t g = blockIdx.x;
    if (g >= ngroups) return;  // every wave below runs its loop to ngroups: no barriers
    reinterpret_cast<uint32_t*>(codes)[lane] = reinterpret_cast<const uint32_t*>(a.codes)[lane];  // all 256 codes

    uint32_t bad = 0, any_bad = 0;
    GroupMeta m = load_meta<G>(a, g, lane);
    GroupSpan s = make_span<G, WB>(a, m, g, lane);
    u64x2 r[U];
    issue_window<U>(s, r, lane);
    // No load result crosses the loop's back edge except r (never copied): a
    // register copy of an in-flight load would wait for every older load.
    uint64_t ph[4] = {0, 0, 0, 0}, tp = __builtin_amdgcn_s_memtime();
    for (;;) {
        // group g's bytes -> LDS (the previous group's reads of the window are done)
        if (s.staged) store_window<U>(s, r, win, lane);
        const uint64_t gn = g + gridDim.x;
        const bool more = gn < ngroups;
        const GroupMeta mn = load_meta<G>(a, more ? gn : g, lane);  // consumed below, after the walk
        wave_lds_sync();

        if (MODE == 5) { const uint64_t t = __builtin_amdgcn_s_memtime(); ph[0] += t - tp; tp = t; }
        // ---- decode_value (datalayer_encodings.cc:168-217), lane = object --
        const uint64_t o0 = g * G;
        const bool valid = (uint32_t)lane < s.nobj;
        bool ok = valid && m.vlen >= 10;
        uint64_t version = 0;
        if (MODE == 3) {  // no walk: every slot a fixed 64-byte string inside the window
            for (uint32_t k = 0; k < A; ++k)
                if (valid) desc[lane * A + k] = SDesc{(uint32_t)(lane * 1024 + k * 64) % (WB - 256), 64u};
        } else if (s.staged) {
            const uint32_t vs = s.vsh + (uint32_t)(m.voff - s.vfirst);                     // value byte 0
            const uint32_t ks = s.vunits * 16 + s.ksh + (uint32_t)(m.koff - s.kfirst);   // key byte 0
            if (ok) version = ((uint64_t)lds_be32(win, vs) << 32) | lds_be32(win, vs + 4);
            ok = ok && (lds_be32(win, vs + 6) & 0xffffu) == A - 1;
            if (valid) desc[lane * A] = SDesc{ks, m.klen};
            uint32_t pos = 10;
            for (uint32_t k = 0; k + 1 < A; ++k) {
                uint32_t len = 0;
                if (ok) {
                    if (m.vlen - pos < 4) {
                        ok = false;
                    } else {
                        len = lds_be32(win, vs + pos);
                        pos += 4;
                        if (len > m.vlen - pos) ok = false;  // the reference does not check this (:201-213)
                    }
                }
                if (valid) desc[lane * A + 1 + k] = SDesc{ok ? vs + pos : kZero, ok ? len : 0u};
                if (ok) pos += len;
            }
        } else {
            const uint8_t* v = a.vals + m.voff;
            if (valid) {
                bases[2 * lane] = m.voff;
                bases[2 * lane + 1] = m.koff;
            }
            if (ok) version = gload_be64(v);
            ok = ok && gload_be16(v + 8) == A - 1;
            if (valid) desc[lane * A] = SDesc{0u, m.klen};
            uint32_t pos = 10;
            for (uint32_t k = 0; k + 1 < A; ++k) {
                uint32_t len = 0;
                if (ok) {
                    if (m.vlen - pos < 4) {
                        ok = false;
                    } else {
                        len = gload_be32(v + pos);
                        pos += 4;
                        if (len > m.vlen - pos) ok = false;
                    }
                }
                if (valid) desc[lane * A + 1 + k] = SDesc{ok ? pos : kZero, ok ? len : 0u};
                if (ok) pos += len;
            }
        }
        if (valid && !ok)  // undecodable: every coordinate of the object is 0
            for (uint32_t j = 0; j < A; ++j) desc[lane * A + j] = SDesc{kZero, 0u};
        if (valid && a.versions) a.versions[o0 + lane] = ok ? version : 0;
        any_bad |= __any(valid && !ok) ? 1u : 0u;
        if (MODE == 5) { const uint64_t t = __builtin_amdgcn_s_memtime(); ph[1] += t - tp; tp = t; }
        // group g+1: its span, and its bytes in flight while group g is hashed
        GroupSpan sn = make_span<G, WB>(a, mn, more ? gn : g, lane);
        if (!more) sn.units = 0;
        issue_window<U>(sn, r, lane);
        wave_lds_sync();

        if (MODE == 5) { const uint64_t t = __builtin_amdgcn_s_memtime(); ph[2] += t - tp; tp = t; }
        // ---- passes of 64 slots in coordinate order -------------------------
        const uint32_t nslots = s.nobj * A;
        uint64_t* out = a.coords + o0 * A;
        for (uint32_t t = 0; MODE != 4 && t * 64 < nslots; ++t) {
            const uint32_t sl0 = t * 64 + (uint32_t)lane;
            const bool live = sl0 < nslots;
            const uint32_t sl = live ? sl0 : nslots - 1;
            const uint32_t obj = div_small(sl, a.a_magic), j = sl - obj * A;
            const SDesc d = desc[sl];
            const bool zero = d.off == kZero || !live;
            const uint32_t code = zero ? (uint32_t)CODE_ZERO : (uint32_t)codes[j];
            const uint32_t n = zero ? 0u : d.len;
            uint64_t h;
            bool pbad = false;
            if (s.staged) {
                const uint32_t off = zero ? 0u : d.off;
                if (MODE == 1) {
                    const Blk b = lds_block_a4(win, code, off, n);
                    h = b.v0.x ^ b.v1.y ^ b.v2.x ^ b.v3.y;
                    if (code == CODE_STRING && n > 64)
                        for (uint32_t k = 0; k < (n - 1) >> 6; ++k) {
                            const Blk c = lds_block64(win, off + 64 * k);
                            h ^= c.v0.x ^ c.v1.y ^ c.v2.x ^ c.v3.y;
                        }
                } else {
                    h = hash_blk_lds<MODE == 2>(win, code, off, n, lds_block_a4<MODE == 2>(win, code, off, n), pbad);
                }
            } else {
                const uint8_t* p = zero ? g_zero_pad
                                        : (j == 0 ? a.keys : a.vals) + bases[2 * obj + (j == 0)] + d.off;
                h = hash_blk<false, false, true>(code, p, n, funnel_raw(issue_block_a4(code, p, n)), pbad);
            }
            bad |= pbad ? 1u : 0u;
            if (live) __builtin_nontemporal_store(h, out + sl0);
        }
        if (MODE == 5) { const uint64_t t = __builtin_amdgcn_s_memtime(); ph[3] += t - tp; tp = t; }
        if (!more) break;
        wave_lds_sync();  // this group's reads of desc / window precede the next group's writes
        g = gn;
        m = mn;
        s = sn;
    }
    if (MODE == 5 && lane == 0 && a.versions)  // debug: shader cycles per phase, summed over the wave's groups
        for (int k = 0; k < 4; ++k) a.versions[a.n + 4ull * blockIdx.x + k] = ph[k];
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// Ping-pong form (variants 74/75): the metadata of group g+1 is loaded one
// whole iteration ahead into one of two register sets used alternately (no
// copy of an in-flight load), and SORT hashes each staged group's slots in
// work-class order (the regroup kernel's LDS fetch-add counting sort) with
// the coordinates parked over their descriptors and stored in slot order.
template <int G, int WB, bool SORT>
__global__ void __launch_bounds__(64) hash_encoded_pp_kernel(const EncodedArgs a, uint64_t ngroups) {
    static_assert(G <= 64 && WB % 1024 == 0 && WB < 65536, "group shape");
    constexpr int U = WB / 1024;
    constexpr int kCls = 8;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const uint32_t A = a.A;
    const int lane = threadIdx.x;
    uint32_t* win = reinterpret_cast<uint32_t*>(smem_raw);
    SDesc* desc = reinterpret_cast<SDesc*>(smem_raw + WB + 16);
    uint64_t* bases = reinterpret_cast<uint64_t*>(smem_raw + WB + 16 + (size_t)G * A * sizeof(SDesc));
    uint8_t* codes = reinterpret_cast<uint8_t*>(bases + 2 * G);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(codes + 256);
    uint16_t* perm = reinterpret_cast<uint16_t*>(cnt + 16);
    uint64_t g = blockIdx.x;
    if (g >= ngroups) return;  // every wave below runs its loop to ngroups: no barriers
    reinterpret_cast<uint32_t*>(codes)[lane] = reinterpret_cast<const uint32_t*>(a.codes)[lane];

    uint32_t bad = 0, any_bad = 0;
    GroupMeta mA = load_meta<G>(a, g, lane);
    GroupSpan s = make_span<G, WB>(a, mA, g, lane);
    u64x2 r[U];
    issue_window<U>(s, r, lane);
    GroupMeta mB = load_meta<G>(a, g + gridDim.x < ngroups ? g + gridDim.x : g, lane);

    // X = group g's metadata (loaded), Y = group g+1's (in flight)
    auto body = [&](GroupMeta& X, const GroupMeta& Y) -> bool {
        if (s.staged) store_window<U>(s, r, win, lane);
        const uint64_t gn = g + gridDim.x;
        const bool more = gn < ngroups;
        GroupSpan sn = make_span<G, WB>(a, Y, more ? gn : g, lane);
        if (!more) sn.units = 0;
        issue_window<U>(sn, r, lane);
        wave_lds_sync();

        const uint64_t o0 = g * G;
        const bool valid = (uint32_t)lane < s.nobj;
        bool ok = valid && X.vlen >= 10;
        uint64_t version = 0;
        if (s.staged) {
            const uint32_t vs = s.vsh + (uint32_t)(X.voff - s.vfirst);
            const uint32_t ks = s.vunits * 16 + s.ksh + (uint32_t)(X.koff - s.kfirst);
            if (ok) version = ((uint64_t)lds_be32(win, vs) << 32) | lds_be32(win, vs + 4);
            ok = ok && (lds_be32(win, vs + 6) & 0xffffu) == A - 1;
            if (valid) desc[lane * A] = SDesc{ks, X.klen};
            uint32_t pos = 10;
            for (uint32_t k = 0; k + 1 < A; ++k) {
                uint32_t len = 0;
                if (ok) {
                    if (X.vlen - pos < 4) {
                        ok = false;
                    } else {
                        len = lds_be32(win, vs + pos);
                        pos += 4;
                        if (len > X.vlen - pos) ok = false;  // the reference does not check this (:201-213)
                    }
                }
                if (valid) desc[lane * A + 1 + k] = SDesc{ok ? vs + pos : kZero, ok ? len : 0u};
                if (ok) pos += len;
            }
        } else {
            const uint8_t* v = a.vals + X.voff;
            if (valid) {
                bases[2 * lane] = X.voff;
                bases[2 * lane + 1] = X.koff;
            }
            if (ok) version = gload_be64(v);
            ok = ok && gload_be16(v + 8) == A - 1;
            if (valid) desc[lane * A] = SDesc{0u, X.klen};
            uint32_t pos = 10;
            for (uint32_t k = 0; k + 1 < A; ++k) {
                uint32_t len = 0;
                if (ok) {
                    if (X.vlen - pos < 4) {
                        ok = false;
                    } else {
                        len = gload_be32(v + pos);
                        pos += 4;
                        if (len > X.vlen - pos) ok = false;
                    }
                }
                if (valid) desc[lane * A + 1 + k] = SDesc{ok ? pos : kZero, ok ? len : 0u};
                if (ok) pos += len;
            }
        }
        if (valid && !ok)
            for (uint32_t j = 0; j < A; ++j) desc[lane * A + j] = SDesc{kZero, 0u};
        if (valid && a.versions) a.versions[o0 + lane] = ok ? version : 0;
        any_bad |= __any(valid && !ok) ? 1u : 0u;
        // group g+2's metadata into X (dead now), a whole iteration ahead
        const uint64_t g2 = gn + gridDim.x;
        X = load_meta<G>(a, g2 < ngroups ? g2 : g, lane);
        wave_lds_sync();

        const uint32_t nslots = s.nobj * A;
        const uint32_t npass = (nslots + 63) / 64;
        uint64_t* out = a.coords + o0 * A;
        const bool sorted = SORT && s.staged;
        if (sorted) {
            // counting sort of the group's slots by work class
            if (lane < kCls) cnt[lane] = 0;
            wave_lds_sync();
            for (uint32_t t = 0; t < npass; ++t) {
                const uint32_t sl = t * 64 + (uint32_t)lane;
                if (sl < nslots) {
                    const SDesc d = desc[sl];
                    const uint32_t j = sl - div_small(sl, a.a_magic) * A;
                    const uint32_t c = d.off == kZero ? 0u : work_class1(codes[j], d.len);
                    __hip_atomic_fetch_add(&cnt[c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                }
            }
            wave_lds_sync();
            const uint32_t k = lane < kCls ? cnt[lane] : 0u;
            const uint32_t start = wave_scan_dpp(k) - k;
            if (lane < kCls) cnt[lane] = start;
            wave_lds_sync();
            for (uint32_t t = 0; t < npass; ++t) {
                const uint32_t sl = t * 64 + (uint32_t)lane;
                if (sl < nslots) {
                    const SDesc d = desc[sl];
                    const uint32_t j = sl - div_small(sl, a.a_magic) * A;
                    const uint32_t c = d.off == kZero ? 0u : work_class1(codes[j], d.len);
                    const uint32_t p = __hip_atomic_fetch_add(&cnt[c], 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WAVEFRONT);
                    perm[p] = (uint16_t)sl;
                }
            }
            wave_lds_sync();
        }
        uint64_t* parked = reinterpret_cast<uint64_t*>(desc);
        for (uint32_t t = 0; t < npass; ++t) {
            const uint32_t q = t * 64 + (uint32_t)lane;
            const bool live = q < nslots;
            const uint32_t sl = !live ? nslots - 1 : sorted ? (uint32_t)perm[q] : q;
            const uint32_t obj = div_small(sl, a.a_magic), j = sl - obj * A;
            const SDesc d = desc[sl];
            const bool zero = d.off == kZero || !live;
            const uint32_t code = zero ? (uint32_t)CODE_ZERO : (uint32_t)codes[j];
            const uint32_t n = zero ? 0u : d.len;
            uint64_t h;
            bool pbad = false;
            if (s.staged) {
                const uint32_t off = zero ? 0u : d.off;
                h = hash_blk_lds(win, code, off, n, lds_block_a4(win, code, off, n), pbad);
            } else {
                const uint8_t* p = zero ? g_zero_pad
                                        : (j == 0 ? a.keys : a.vals) + bases[2 * obj + (j == 0)] + d.off;
                h = hash_blk<false, false, true>(code, p, n, funnel_raw(issue_block_a4(code, p, n)), pbad);
            }
            bad |= pbad ? 1u : 0u;
            if (live) {
                if (sorted) parked[sl] = h;  // over its own (consumed) descriptor
                else __builtin_nontemporal_store(h, out + q);
            }
        }
        if (sorted) {
            wave_lds_sync();
            for (uint32_t t = 0; t < npass; ++t) {
                const uint32_t q = t * 64 + (uint32_t)lane;
                if (q < nslots) __builtin_nontemporal_store(parked[q], out + q);
            }
        }
        wave_lds_sync();  // this group's LDS reads precede the next group's writes
        s = sn;
        g = gn;
        return more;
    };
    while (body(mA, mB) && body(mB, mA)) {
    }
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int G, int WB, bool SORT>
static hipError_t launch_pp(const EncodedArgs& a, hipStream_t stream) {
    const uint64_t ngroups = (a.n + G - 1) / G;
    const size_t lds = staged_lds_bytes(a.A, G, WB) + 64 + (size_t)G * a.A * 2;
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hash_encoded_pp_kernel<G, WB, SORT>, 64, lds);
    if (e != hipSuccess) return e;
    const uint64_t resident = (uint64_t)max(cus, 1) * (uint64_t)max(per_cu, 1);
    const uint64_t blocks = ngroups < resident ? ngroups : resident;
    hipLaunchKernelGGL((hash_encoded_pp_kernel<G, WB, SORT>), dim3((uint32_t)blocks), dim3(64), lds, stream, a,
                       ngroups);
    return hipGetLastError();
}

template <int G, int WB, int MODE = 0, int WPE = 1>
static hipError_t launch_pipe(const EncodedArgs& a, hipStream_t stream) {
    const uint64_t ngroups = (a.n + G - 1) / G;
    const size_t lds = staged_lds_bytes(a.A, G, WB);
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hash_encoded_pipe_kernel<G, WB, MODE, WPE>, 64, lds);
    if (e != hipSuccess) return e;
    const uint64_t resident = (uint64_t)max(cus, 1) * (uint64_t)max(per_cu, 1);
    const uint64_t blocks = ngroups < resident ? ngroups : resident;
    if (getenv("HDX_DEBUG_LAUNCH"))
        fprintf(stderr, "hash_encoded_pipe_kernel<%d, %d>: %d CUs x %d blocks/CU, %llu blocks, %zu B LDS\n", G, WB,
                cus, per_cu, (unsigned long long)blocks, lds);
    hipLaunchKernelGGL((hash_encoded_pipe_kernel<G, WB, MODE, WPE>), dim3((uint32_t)blocks), dim3(64), lds, stream, a, ngroups);
    return hipGetLastError();
}

// variant 64: 7 objects per group, 10 KiB window; 65: 3 / 4 KiB; 66: 11 / 15 KiB
hipError_t launch_hash_encoded_staged(const EncodedArgs& a, hipStream_t stream, int variant) {
    if (a.n == 0) return hipSuccess;
    switch (variant) {
        case 65: return launch_pipe<3, 4096>(a, stream);
        case 66: return launch_pipe<11, 15360>(a, stream);
        case 67: return launch_pipe<7, 10240, 1>(a, stream);
        case 68: return launch_pipe<7, 10240, 2>(a, stream);
        case 69: return launch_pipe<7, 10240, 3>(a, stream);
        case 70: return launch_pipe<7, 10240, 4>(a, stream);
        case 74: return launch_pp<7, 10240, true>(a, stream);
        case 75: return launch_pp<7, 10240, false>(a, stream);
        case 72: return launch_pipe<7, 10240, 0, 4>(a, stream);
        case 73: return launch_pipe<7, 10240, 0, 5>(a, stream);
        case 71: return launch_pipe<7, 10240, 5>(a, stream);  // versions must hold n + 4 * blocks entries
        default: return launch_pipe<7, 10240>(a, stream);
    }
}

}  // namespace hdx
