// hdx_window.hip — the workgroup-window hash kernel (variants 50-53).
//
// Same contract as the kernels of hdx_kernels.hip: hashes every (object,
// attribute) slot of the packed layout (include/hdxhash.h) into coords —
// hs[j] of hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68).
//
// Why a different shape.  On schemas that mix numerics with strings of
// varied length (config 3b) a wave executes the union of the CityHash regimes
// its 64 lanes take, so the per-lane kernels are VALU-bound; sorting slots by
// regime fixes that only if the sorted passes do not gather their bytes from
// all over a large window (lines fetched twice).  Here a
// workgroup of 4 waves owns S consecutive slots:
//   A. every wave computes its slots' addresses, codes and work classes (as the
//      chunk kernel does) and the byte range they span;          [barrier 1]
//   B. when the workgroup's bytes fit the LDS window (and are near each other,
//      as packed batches are), they are copied into LDS with coalesced
//      global_load_lds_dwordx4 (16-byte aligned, every HBM line read once),
//      while the waves counting-sort the S slots by class into a permutation;
//                                                                [barrier 2]
//   C. every wave hashes S/256 class-homogeneous passes of 64 slots, reading
//      the bytes from LDS as dwords (a byte-misaligned wide LDS read is
//      replayed; dword reads are not) funnel-shifted with v_alignbyte exactly
//      as the A4 global form, and stores each coordinate to its slot.
// A workgroup whose bytes do not fit (long values, scattered objects) hashes
// its slots from global memory in slot order instead (the chunk kernel's
// path with A4 loads), so any layout is handled.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_loads.h"

namespace hdx {

constexpr int kWinClasses = kClasses10;

template <int S, int WIN>
struct WinLds {
    uint32_t win[WIN / 4 + 8];  // staged bytes from wbase (16-byte aligned)
    uint32_t desc[S];           // byte offset in win | length << 16
    uint16_t perm[S];
    uint8_t code[S];
    uint64_t lo[4], hi[4];      // per wave: [lowest first byte, highest end) of its slots
    uint32_t cnt[4][kWinClasses];  // per wave: slots of each class
    uint32_t cur[4][kWinClasses];  // per wave: next position of each class
    uint32_t ok[4];
};

// ---------------------------------------------------------------------------
// Reading a slot's bytes from the LDS window: the A4 pieces of hdx_loads.h at
// byte offset `off` (whose alignment mod 16 is the global address's, the
// window base being 16-byte aligned), as dword reads.
// ---------------------------------------------------------------------------
__device__ __forceinline__ u64x2 pack64x2(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    u64x2 v;
    v.x = pack64(a, b);
    v.y = pack64(c, d);
    return v;
}

__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
    return pack64(__builtin_amdgcn_readfirstlane((uint32_t)v), __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)));
}

__device__ __forceinline__ u64x2 lds16(const uint32_t* w, int32_t byte_off) {
    const uint32_t* d = w + (byte_off >> 2);
    u64x2 v;
    v.x = pack64(d[0], d[1]);
    v.y = pack64(d[2], d[3]);
    return v;
}

__device__ __forceinline__ Blk lds_block_a4(const uint32_t* w, uint32_t code, uint32_t off, uint32_t n) {
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

// One 64-byte loop block at byte offset s of the window.
__device__ __forceinline__ Blk lds_block64(const uint32_t* w, uint32_t s) {
    const uint32_t* d = w + (s >> 2);
    const uint32_t r = s & 3;
    Blk64 b;
    b.b.v0 = pack64x2(d[0], d[1], d[2], d[3]);
    b.b.v1 = pack64x2(d[4], d[5], d[6], d[7]);
    b.b.v2 = pack64x2(d[8], d[9], d[10], d[11]);
    b.b.v3 = pack64x2(d[12], d[13], d[14], d[15]);
    b.e = d[16];
    return use64<true>(b, r);
}

// city.cc:361-397 for n > 64 with the tail block in registers and the loop
// blocks read from the window (city_gt64_reg's arithmetic).
__device__ __forceinline__ uint64_t city_gt64_lds(const uint32_t* w, uint32_t off, uint32_t n, const Blk& t) {
    const u64x2 e0 = t.v0, e1 = t.v1, e2 = t.v2, e3 = t.v3;
    uint64_t x = e1.y;
    uint64_t y = e3.x + e0.y;
    uint64_t z = mix16(e1.x + n, e2.y, KMUL);
    uint64_t v0, v1, w0, w1;
    weak32(e0.x, e0.y, e1.x, e1.y, n, z, v0, v1);
    weak32(e2.x, e2.y, e3.x, e3.y, y + K1, x, w0, w1);
    const uint32_t blocks = (n - 1) >> 6;
    Blk b = lds_block64(w, off);
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
        b = lds_block64(w, off + 64 * k);
    }
    return mix16(mix16(v0, w0, KMUL) + shiftmix(y) * K1 + z, mix16(v1, w1, KMUL) + x, KMUL);
}

// hash_blk (A4 piece layout) with the > 64-byte loop reading the window.
__device__ __forceinline__ uint64_t hash_blk_lds(const uint32_t* w, uint32_t code, uint32_t off, uint32_t n,
                                                 const Blk& b, bool& bad) {
    const uint32_t sh = off & 15;
    if (code == CODE_STRING) {
        if (n > 64) return city_gt64_lds(w, off, n, b);
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

// NOHASH (debug variant 59 only): the passes read their descriptors and
// bytes but skip the hash arithmetic (wrong coordinates) — the overhead side.
template <int S, int WIN, bool NOHASH = false>
__global__ void __launch_bounds__(256)
hash_window_kernel(const BatchArgs args) {
    static_assert(S % 256 == 0 && WIN % 16 == 0 && WIN < 65536, "window shape");
    constexpr int R = S / 256;  // chunks (and passes) per wave
    __shared__ __attribute__((aligned(16))) WinLds<S, WIN> L;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint32_t A = args.A;
    const uint64_t nslots = args.n * A;
    const uint64_t qwg = (uint64_t)blockIdx.x * S;
    const uint64_t qw = qwg + (uint64_t)w * (R * 64);
    const bool live = qw < nslots;  // waves past the batch end still take part in the barriers

    // ---- A: addresses, codes, classes --------------------------------------
    const uint8_t* P[R];
    uint32_t Ln[R], Cd[R], Cl[R];
    bool need[R];
    uint64_t i0 = 0;
    uint32_t j0 = 0, carry = 0;
    if (live) {
        split_slot(qw, A, i0, j0);
        for (uint32_t k = 0; k < j0; k += 64) {  // slots [qw - j0, qw) belong to object i0
            const uint32_t idx = k + (uint32_t)lane;
            const uint32_t v = idx < j0 ? args.attr_len[qw - j0 + idx] : 0u;
            carry += wave_sum_dpp(v);
        }
    }
    uint32_t packed_codes = 0;
    if (args.uniform_code == 0xffu) packed_codes = reinterpret_cast<const uint32_t*>(args.codes)[lane];
    const uint64_t last_slot = nslots - 1;
#pragma unroll
    for (int c = 0; c < R; ++c) {
        const uint64_t q = qw + c * 64 + lane;
        const bool valid = q < nslots;
        const uint32_t t = j0 + (uint32_t)(c * 64 + lane);
        const uint32_t di = t / A;
        const uint32_t j = t - di * A;
        const uint64_t il = valid ? i0 + di : i0;
        const uint32_t Lq = valid ? args.attr_len[min(q, last_slot)] : 0u;
        const uint64_t base = args.obj_base[il];
        const uint32_t Sx = wave_scan_dpp(Lq) - Lq;
        const int head = lane - (int)j;
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
        carry = __builtin_amdgcn_readlane(off + Lq, 63);
        uint32_t code = args.uniform_code != 0xffu
                            ? args.uniform_code
                            : (__shfl(packed_codes, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
        if (!valid) code = CODE_ZERO;
        P[c] = args.blob + base + off;
        Ln[c] = Lq;
        Cd[c] = code;
        Cl[c] = valid ? work_class10(code, Lq) : 0u;
        need[c] = (code == CODE_STRING && Lq > 0) || (code >= CODE_INT64 && Lq == 8);
    }
    // byte range of this wave's slots: from its first slot's first byte to its
    // last slot's end, when every slot lies inside (packed, ascending objects);
    // otherwise the workgroup takes the fallback path
    uint32_t* my_cnt = L.cnt[w];
    if (lane < kWinClasses) my_cnt[lane] = 0;
    const uint64_t first = readfirstlane64((uint64_t)(uintptr_t)P[0]);
    // the wave's last valid slot: chunk c_last, lane l_last (wave-uniform)
    const uint64_t last_q = live ? min<uint64_t>(qw + R * 64, nslots) - 1 - qw : 0;
    const int c_last = (int)(last_q >> 6), l_last = (int)(last_q & 63);
    uint64_t last_end = 0;
#pragma unroll
    for (int c = 0; c < R; ++c) {
        if (c == c_last) {
            const uint64_t e = (uint64_t)(uintptr_t)P[c] + Ln[c];
            last_end = pack64(__builtin_amdgcn_readlane((uint32_t)e, l_last),
                              __builtin_amdgcn_readlane((uint32_t)(e >> 32), l_last));
        }
    }
    bool inside = true;
#pragma unroll
    for (int c = 0; c < R; ++c) {
        const uint64_t a = (uint64_t)(uintptr_t)P[c];
        inside &= !need[c] || (a >= first && a + Ln[c] <= last_end);
        __hip_atomic_fetch_add(&my_cnt[Cl[c]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
    if (lane == 0) {
        L.lo[w] = live ? first : ~0ull;
        L.hi[w] = live ? last_end : 0ull;
        L.ok[w] = __all(inside);
    }
    __syncthreads();  // ---- barrier 1 ----

    uint64_t wlo = ~0ull, whi = 0;
    bool ok = true;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
        wlo = min(wlo, L.lo[v]);
        whi = max(whi, L.hi[v]);
        ok = ok && L.ok[v];
    }
    const uint64_t wbase = wlo & ~15ull;
    const uint64_t t16 = whi > wlo ? ((whi + 15) & ~15ull) - wbase : 0;
    const bool staged = ok && t16 <= (uint64_t)WIN;
    bool bad = false;

    if (staged) {
        // ---- B: stage [wbase, wbase + t16) with coalesced LDS DMA ------------
        const uint32_t units = (uint32_t)(t16 >> 4);
        for (uint32_t u0 = (uint32_t)w * 64; u0 < units; u0 += 256) {
            const uint32_t u = u0 + (uint32_t)lane;
            if (u < units)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(uintptr_t)(wbase + 16ull * u),
                    (__attribute__((address_space(3))) void*)&L.win[u0 * 4], 16, 0, 0);
        }
        // slot descriptors (byte offset in the window, length) and codes
#pragma unroll
        for (int c = 0; c < R; ++c) {
            const uint32_t sl = (uint32_t)(w * R * 64 + c * 64 + lane);
            const uint32_t off = need[c] ? (uint32_t)((uint64_t)(uintptr_t)P[c] - wbase) : 0u;
            // strings here lie inside the window (< 64 KiB); numerics keep 0, 8 or "bad"
            const uint32_t n = Cd[c] == CODE_STRING ? Ln[c] : min(Ln[c], 9u);
            L.desc[sl] = off | (n << 16);
            L.code[sl] = (uint8_t)Cd[c];
        }
        // counting sort by class: lane k (k < classes) computes where this
        // wave's class-k slots start (slots of lower classes + class-k slots of
        // lower waves) into a wave-private cursor; each slot then takes its
        // position with an LDS fetch-add on its class's cursor
        uint32_t tot = 0, before = 0;
        if (lane < kWinClasses) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint32_t x = L.cnt[v][lane];
                tot += x;
                before += v < w ? x : 0u;
            }
        }
        const bool uniform = __any(tot == (uint32_t)S);
        if (!uniform) {
            const uint32_t start = wave_scan_dpp(tot) - tot + before;  // exclusive over classes
            uint32_t* cursor = L.cur[w];
            if (lane < kWinClasses) cursor[lane] = start;
#pragma unroll
            for (int c = 0; c < R; ++c) {
                const uint32_t pos = __hip_atomic_fetch_add(&cursor[Cl[c]], 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WAVEFRONT);
                L.perm[pos] = (uint16_t)(w * R * 64 + c * 64 + lane);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);  // the LDS DMA has landed
        __syncthreads();                 // ---- barrier 2 ----

        // ---- C: class-homogeneous passes read from the window --------------
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint32_t tpos = (uint32_t)((u * 4 + w) * 64 + lane);
            const uint32_t sl = uniform ? tpos : L.perm[tpos];
            const uint32_t d = L.desc[sl];
            const uint32_t code = L.code[sl];
            const uint32_t off = d & 0xffffu, n = d >> 16;
            const Blk b = lds_block_a4(L.win, code, off, n);
            const uint64_t h = NOHASH ? b.v0.x ^ b.v1.y ^ b.v2.x ^ b.v3.y : hash_blk_lds(L.win, code, off, n, b, bad);
            const uint64_t q = qwg + sl;
            if (q < nslots) __builtin_nontemporal_store(h, args.coords + q);
        }
    } else if (live) {
        // ---- fallback: this wave's slots in order, from global memory --------
#pragma unroll
        for (int c = 0; c < R; ++c) {
            const uint64_t q = qw + c * 64 + lane;
            const Raw r = issue_block_a4(Cd[c], P[c], Ln[c]);
            const uint64_t h = hash_blk<false, false, true>(Cd[c], P[c], Ln[c], funnel_raw(r), bad);
            if (q < nslots) __builtin_nontemporal_store(h, args.coords + q);
        }
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// ===========================================================================
// Pipelined form (variants 52/53): a persistent workgroup walks windows of 256
// slots (one chunk per wave) with two LDS buffers, so that window k+1's bytes
// stream into LDS (LDS DMA) and window k+2's lengths / object bases load while
// window k is hashed — one barrier per window, no exposed memory latency in
// steady state.  Per iteration, with b = k's buffer:
//   wait for every load in flight (window k's DMA, window k+1's metadata)
//   A(k+1): addresses, classes, byte range -> meta[b^1]          [barrier]
//   B(k+1): stage into win[b^1], descriptors, class sort -> perm[b^1]
//   issue window k+2's metadata loads
//   C(k):   hash window k from win[b] (or from global memory when it did not fit)
// Buffer b^1 is free at the barrier: window k-1, its last user, was hashed
// before it.
// ===========================================================================
template <int WIN>
struct PipeLds {
    uint32_t win[2][WIN / 4 + 8];
    uint32_t desc[2][256];
    uint16_t perm[2][256];
    uint8_t code[2][256];
    uint64_t lo[2][4], hi[2][4];
    uint32_t ok[2][4];
    uint32_t cnt[2][4][kWinClasses];
    uint32_t cur[4][kWinClasses];
};

// One wave's 64 slots of a window: metadata loads in flight ...
struct ChunkLoads {
    uint32_t len;
    uint64_t base;
    uint32_t carry[4];  // lengths of the wave's first object's slots before the chunk
    uint32_t j0;
    uint64_t i0;
};
// ... and what they resolve to.
struct ChunkSlots {
    const uint8_t* p;
    uint32_t n, code, cls;
    bool need;
};

__device__ __forceinline__ ChunkLoads chunk_issue(const BatchArgs& args, uint64_t q0, uint64_t nslots, int lane) {
    ChunkLoads c;
    const uint32_t A = args.A;
    split_slot(q0, A, c.i0, c.j0);
    const uint64_t q = q0 + lane;
    const bool valid = q < nslots;
    const uint32_t t = c.j0 + (uint32_t)lane;
    const uint32_t di = t / A;
    c.len = valid ? args.attr_len[q] : 0u;
    c.base = args.obj_base[valid ? c.i0 + di : c.i0];
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // j0 < A <= 256
        const uint32_t idx = (uint32_t)(r * 64 + lane);
        c.carry[r] = (uint32_t)(r * 64) < c.j0 && idx < c.j0 ? args.attr_len[q0 - c.j0 + idx] : 0u;
    }
    return c;
}

__device__ __forceinline__ ChunkSlots chunk_resolve(const BatchArgs& args, const ChunkLoads& c, uint64_t q0,
                                                    uint64_t nslots, int lane, uint32_t packed_codes) {
    const uint32_t A = args.A;
    uint32_t carry = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if ((uint32_t)(r * 64) < c.j0) carry += wave_sum_dpp(c.carry[r]);
    const bool valid = q0 + lane < nslots;
    const uint32_t t = c.j0 + (uint32_t)lane;
    const uint32_t di = t / A;
    const uint32_t j = t - di * A;
    const uint32_t L = c.len;
    const uint32_t Sx = wave_scan_dpp(L) - L;
    const int head = lane - (int)j;
    const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
    const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
    uint32_t code = args.uniform_code != 0xffu
                        ? args.uniform_code
                        : (__shfl(packed_codes, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
    if (!valid) code = CODE_ZERO;
    ChunkSlots s;
    s.p = args.blob + c.base + off;
    s.n = L;
    s.code = code;
    s.cls = valid ? work_class10(code, L) : 0u;
    s.need = (code == CODE_STRING && L > 0) || (code >= CODE_INT64 && L == 8);
    return s;
}

template <int WIN>
__global__ void __launch_bounds__(256)
hash_window_pipe_kernel(const BatchArgs args, uint64_t nwin) {
    static_assert(WIN % 16 == 0 && WIN < 65536, "window shape");
    __shared__ __attribute__((aligned(16))) PipeLds<WIN> L;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const uint64_t nslots = args.n * args.A;
    const uint64_t step = gridDim.x;
    uint64_t k = blockIdx.x;
    if (k >= nwin) return;  // whole workgroup
    uint32_t packed_codes = 0;
    if (args.uniform_code == 0xffu) packed_codes = reinterpret_cast<const uint32_t*>(args.codes)[lane];

    // A: publish a window's byte range and class counts into meta[b]
    auto publish = [&](const ChunkSlots& s, uint64_t q0, int b) {
        const bool live = q0 < nslots;
        if (lane < kWinClasses) L.cnt[b][w][lane] = 0;
        __hip_atomic_fetch_add(&L.cnt[b][w][s.cls], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        const uint64_t first = readfirstlane64((uint64_t)(uintptr_t)s.p);
        const int l_last = live ? (int)min<uint64_t>(63, nslots - 1 - q0) : 0;
        const uint64_t e = (uint64_t)(uintptr_t)s.p + s.n;
        const uint64_t last_end = pack64(__builtin_amdgcn_readlane((uint32_t)e, l_last),
                                         __builtin_amdgcn_readlane((uint32_t)(e >> 32), l_last));
        const uint64_t a = (uint64_t)(uintptr_t)s.p;
        const bool inside = !s.need || (a >= first && a + s.n <= last_end);
        const bool ok = __all(inside);
        if (lane == 0) {
            L.lo[b][w] = live ? first : ~0ull;
            L.hi[b][w] = live ? last_end : 0ull;
            L.ok[b][w] = ok;
        }
    };
    // B: stage a window into buffer b, write its descriptors, sort it;
    // returns whether it was staged (and whether it needs no permutation)
    auto stage = [&](const ChunkSlots& s, int b, bool& uniform) -> bool {
        uint64_t wlo = ~0ull, whi = 0;
        bool ok = true;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            wlo = min(wlo, L.lo[b][v]);
            whi = max(whi, L.hi[b][v]);
            ok = ok && L.ok[b][v];
        }
        const uint64_t wbase = wlo & ~15ull;
        const uint64_t t16 = whi > wlo ? ((whi + 15) & ~15ull) - wbase : 0;
        uniform = false;
        if (!(ok && t16 <= (uint64_t)WIN)) return false;
        const uint32_t units = (uint32_t)(t16 >> 4);
        for (uint32_t u0 = (uint32_t)w * 64; u0 < units; u0 += 256) {
            const uint32_t u = u0 + (uint32_t)lane;
            if (u < units)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(uintptr_t)(wbase + 16ull * u),
                    (__attribute__((address_space(3))) void*)&L.win[b][u0 * 4], 16, 0, 0);
        }
        const uint32_t sl = (uint32_t)(w * 64 + lane);
        const uint32_t off = s.need ? (uint32_t)((uint64_t)(uintptr_t)s.p - wbase) : 0u;
        const uint32_t n = s.code == CODE_STRING ? s.n : min(s.n, 9u);
        L.desc[b][sl] = off | (n << 16);
        L.code[b][sl] = (uint8_t)s.code;
        uint32_t tot = 0, before = 0;
        if (lane < kWinClasses) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint32_t x = L.cnt[b][v][lane];
                tot += x;
                before += v < w ? x : 0u;
            }
        }
        uniform = __any(tot == 256u);
        if (!uniform) {
            const uint32_t start = wave_scan_dpp(tot) - tot + before;
            if (lane < kWinClasses) L.cur[w][lane] = start;
            const uint32_t pos = __hip_atomic_fetch_add(&L.cur[w][s.cls], 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WAVEFRONT);
            L.perm[b][pos] = (uint16_t)sl;
        }
        return true;
    };

    // prologue: window k's metadata, publish, barrier, stage; window k+1's loads
    uint64_t q0 = k * 256 + (uint64_t)w * 64;
    ChunkSlots cur = chunk_resolve(args, chunk_issue(args, min(q0, nslots - 1), nslots, lane), q0, nslots, lane,
                                   packed_codes);
    publish(cur, q0, 0);
    __syncthreads();
    bool cur_uniform;
    bool cur_staged = stage(cur, 0, cur_uniform);
    uint64_t q0n = (k + step) * 256 + (uint64_t)w * 64;
    ChunkLoads nl;
    if (k + step < nwin) nl = chunk_issue(args, min(q0n, nslots - 1), nslots, lane);
    bool bad = false;
    for (int b = 0;; b ^= 1) {
        const bool has_next = k + step < nwin;
        __builtin_amdgcn_s_waitcnt(0);  // window k's DMA and window k+1's metadata
        ChunkSlots nxt;
        if (has_next) {
            nxt = chunk_resolve(args, nl, q0n, nslots, lane, packed_codes);
            publish(nxt, q0n, b ^ 1);
        }
        __syncthreads();
        bool nxt_uniform = false, nxt_staged = false;
        const uint64_t q0nn = (k + 2 * step) * 256 + (uint64_t)w * 64;
        if (has_next) {
            nxt_staged = stage(nxt, b ^ 1, nxt_uniform);
            if (k + 2 * step < nwin) nl = chunk_issue(args, min(q0nn, nslots - 1), nslots, lane);
        }
        // C: hash window k
        const uint64_t qwg = k * 256;
        if (cur_staged) {
            const uint32_t tpos = (uint32_t)(w * 64 + lane);
            const uint32_t sl = cur_uniform ? tpos : L.perm[b][tpos];
            const uint32_t d = L.desc[b][sl];
            const uint32_t code = L.code[b][sl];
            const uint32_t off = d & 0xffffu, n = d >> 16;
            const Blk blk = lds_block_a4(L.win[b], code, off, n);
            const uint64_t h = hash_blk_lds(L.win[b], code, off, n, blk, bad);
            const uint64_t q = qwg + sl;
            if (q < nslots) __builtin_nontemporal_store(h, args.coords + q);
        } else if (q0 < nslots) {
            const Raw r = issue_block_a4(cur.code, cur.p, cur.n);
            const uint64_t h = hash_blk<false, false, true>(cur.code, cur.p, cur.n, funnel_raw(r), bad);
            if (q0 + lane < nslots) __builtin_nontemporal_store(h, args.coords + q0 + lane);
        }
        if (!has_next) break;
        k += step;
        q0 = q0n;
        q0n = q0nn;
        cur = nxt;
        cur_staged = nxt_staged;
        cur_uniform = nxt_uniform;
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int WIN, int WG_PER_CU>
static hipError_t launch_window_pipe(const BatchArgs& args, hipStream_t stream) {
    static const int cus = [] {
        int dev = 0, n = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return 256;
        return n > 0 ? n : 256;
    }();
    const uint64_t nwin = (args.n * args.A + 255) / 256;
    if (nwin == 0) return hipSuccess;
    const uint64_t cap = (uint64_t)cus * WG_PER_CU;
    const uint64_t grid = nwin < cap ? nwin : cap;
    hipLaunchKernelGGL((hash_window_pipe_kernel<WIN>), dim3((uint32_t)grid), dim3(256), 0, stream, args, nwin);
    return hipGetLastError();
}

template <int S, int WIN, bool NOHASH = false>
static hipError_t launch_window(const BatchArgs& args, hipStream_t stream) {
    const uint64_t blocks = (args.n * args.A + S - 1) / S;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_window_kernel<S, WIN, NOHASH>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

hipError_t launch_hash_window(const BatchArgs& args, hipStream_t stream, int variant) {
    switch (variant) {
        case 50: return launch_window<256, 20480>(args, stream);
        case 51: return launch_window<512, 35840>(args, stream);
        case 59: return launch_window<512, 35840, true>(args, stream);
        case 52: return launch_window_pipe<17920, 4>(args, stream);
        case 53: return launch_window_pipe<24576, 3>(args, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace hdx
