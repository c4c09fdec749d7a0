// hdx_stream.hip — the streamed batch hash: one persistent workgroup per CU
// pulls consecutive batches of whole objects through LDS.
//
// hdx_hash_batch_device's contract (include/hdxhash.h): coords[i*A + j] =
// hs[j] of hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68),
// every attribute through hash(type, slice) (hash.cc:34-46): CityHash64 v1.1
// for strings (cityhash/city.cc:361-397), the ordered encodings for
// int64/float, the calendar hash for timestamps, 0 for the non-hashable types.
//
// Why this shape.  On mixed schemas (config 3b) the
// gather kernels pay twice: every lane loads its own value (one cache line per
// lane per load, the L1's miss handling is the bound), and a wave's 64..128
// slots span three to five CityHash regimes, so every pass runs the union of
// their code (variant 44: 1104 VALU per 128 slots against ~430 for the same
// slots hashed regime by regime, profiles/r3/regime_costs_v209.txt).  Here a
// workgroup of WAVES waves owns a contiguous range of objects and walks it in
// batches of up to 64*WAVES slots:
//   * the batch's bytes (one span for a packed layout) are copied into one of
//     two LDS windows by coalesced LDS DMA (global_load_lds_dwordx4, 1 KiB per
//     wave-instruction) a whole batch ahead, so the copy of batch b+1 streams
//     while batch b is hashed;
//   * the batch's slots are counting-sorted by CityHash regime over the whole
//     workgroup (ballot/popcount/mbcnt per wave, one barrier), so each of the
//     <= WAVES passes of 64 slots runs one regime, two at a class boundary;
//   * every string is hashed from LDS with two 32-byte reads (its first and
//     last 32 bytes: dword reads + v_alignbyte) that serve every regime
//     (HashLen0to16 / 17to32 / 33to64 / the > 64-byte tail block), so a
//     regime costs its arithmetic only; the > 64-byte loop reads its blocks
//     from the window (hdx_lds_hash.h);
//   * coordinates are parked in LDS and stored in slot order, one coalesced
//     512-byte non-temporal store per wave.
// Batch sizing is adaptive: batch b ends before the first object whose start
// lies more than the window's capacity past the batch's first byte (from the
// object bases, loaded a batch ahead).  A slot whose bytes are not inside its
// batch's window (gaps, shuffled objects, an object larger than the window,
// the launch's very last batch whose end is unknown) is hashed from global
// memory with the gather kernels' loads (hdx_loads.h), sorted into a class of
// its own — every layout gives the reference's coordinates.
//
// Synchronisation per batch b: three workgroup barriers — B1 (per-wave slot
// counts per class, the next batch's size), B2 (sorted descriptors written),
// B3 (coordinates parked).  The DMA of batch b+1 is
// issued after B1 of batch b and waited for with s_waitcnt vmcnt(1) at the top
// of batch b+1 (the only younger VMEM operation a wave may still have in
// flight there is its coordinate store of batch b: loads, stores and LDS DMA
// complete in issue order, MI355X_MICROARCH.md), before B1 publishes it.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>

#include "hdx_lds_hash.h"
#include "hdx_regroup.h"

namespace hdx {
namespace {

typedef __attribute__((address_space(3))) void* lds_void_t;

constexpr uint32_t kInvalid = 0xffffffffu;
constexpr uint32_t kFront = 32;   // window bytes before the span (tail reads of short strings)
constexpr uint32_t kBack = 128;   // after it (head reads of short strings, dword over-reads)
constexpr uint32_t kLenBits = 17, kLenMax = (1u << kLenBits) - 1;

// Sort classes, most expensive first: > 64-byte strings by loop blocks (4+,
// 3, 2, 1), 33..64, 17..32, 0..16, int64/float, timestamps, non-hashable, and
// last every slot hashed from global memory.
constexpr uint32_t kStreamClasses = 11;
constexpr uint32_t kClassGlobal = 10;

__device__ __forceinline__ uint32_t stream_class(uint32_t code, uint32_t n, bool staged) {
    if (!staged) return kClassGlobal;
    if (code == CODE_STRING) {
        if (n > 64) {
            const uint32_t b = (n - 1) >> 6;
            return b >= 4 ? 0u : 4u - b;
        }
        return n > 32 ? 4u : n > 16 ? 5u : 6u;
    }
    if (code == CODE_INT64 || code == CODE_FLOAT) return 7;
    if (code == CODE_ZERO) return 9;
    return 8;
}

// 32 bytes at window byte offset o (any alignment): q[k] = bytes [o+8k, o+8k+8)
struct Q32 {
    uint64_t q0, q1, q2, q3;
};
__device__ __forceinline__ Q32 lds_read32(ldsw_t w, uint32_t o) {
    const ldsw_t d = w + (o >> 2);
    const uint32_t r = o & 3;
    uint32_t x[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) x[i] = d[i];
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

// hash(type, slice) of a slot whose bytes start at window byte offset off.
__device__ __forceinline__ uint64_t hash_slot_window(ldsw_t w, uint32_t code, uint32_t off, uint32_t n, bool& bad) {
    if (code == CODE_STRING) {
        const Q32 t = lds_read32(w, off + n - 32);  // s[n-32, n): the front pad covers n < 32
        const u64x2 t01 = {t.q0, t.q1}, t23 = {t.q2, t.q3};
        if (n > 64) {
            const Q32 u = lds_read32(w, off + n - 64);
            Blk b;
            b.v0 = u64x2{u.q0, u.q1};
            b.v1 = u64x2{u.q2, u.q3};
            b.v2 = t01;
            b.v3 = t23;
            return city_gt64_lds(w, off, n, b);
        }
        const Q32 h = lds_read32(w, off);  // s[0, 32): the back pad covers n < 32
        const u64x2 h01 = {h.q0, h.q1};
        if (n > 32) return city_33to64(h01, u64x2{h.q2, h.q3}, t01, t23, n);
        if (n > 16) return city_17to32(h01, t23, n);
        return city_le16_ht(h.q0, t.q3, n);
    }
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

// The same from global memory (the gather kernels' dword-aligned loads).
__device__ __forceinline__ uint64_t hash_slot_global(const uint8_t* p, uint32_t code, uint32_t n, bool& bad) {
    return hash_blk<false, false, true>(code, p, n, consume_any<true>(issue_any<true>(code, p, n)), bad);
}

template <int WAVES, uint32_t W>
struct StreamLds {
    static constexpr uint32_t S = 64 * WAVES;            // slots per batch at most
    uint8_t win[2][kFront + W + kBack] __attribute__((aligned(16)));
    uint64_t sdesc[S];        // class-sorted {offset, slot | code | staged | len}; then the coordinate
    uint32_t bdelta[2][S];    // per batch parity: base[o0 + t] - base[o0], or kInvalid
    uint32_t wcls[WAVES][kStreamClasses];  // per wave: slots per class
    uint32_t kfirst[2];       // per batch parity: the first object that does not fit (atomic min)
    uint8_t codes[64];
};

}  // namespace

// One batch's uniform description (every wave holds a copy in SGPRs).
struct StreamBatch {
    uint64_t o0;     // first object
    uint64_t base0;  // its base
    uint32_t K;      // objects
    uint32_t span;   // base[o0 + K] - base0 (the bytes the window holds), or kInvalid
    uint32_t lead;   // (blob + base0) & 15: the span's offset in its first DMA unit
};

template <int WAVES, uint32_t W>
__global__ void __launch_bounds__(64 * WAVES)
hash_stream_kernel(const BatchArgs args) {
    typedef StreamLds<WAVES, W> L;
    constexpr uint32_t S_MAX = L::S;
    __shared__ L lds;
    const uint32_t tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t w = tid >> 6;
    const uint32_t A = args.A;  // 1..64
    const uint64_t n = args.n;
    const uint32_t kcap = std::min<uint32_t>(S_MAX / A, S_MAX - 1);  // objects per batch at most (lane kcap: its end)

    // this workgroup's objects
    const uint64_t G = gridDim.x;
    const uint64_t r0 = n * blockIdx.x / G, r1 = n * (blockIdx.x + 1) / G;
    if (r0 >= r1) return;  // (uniform: no barrier reached)

    if (tid < 64) lds.codes[tid] = tid < A ? args.codes[tid] : (uint8_t)CODE_ZERO;
    if (tid < 2) lds.kfirst[tid] = kInvalid;
    __syncthreads();

    // ---- the next batch's size from its bases (lane t: base[o1 + t]) --------
    // fit(t): object o1 + t starts inside the window when the batch starts at
    // o1, i.e. the batch may end before it; the batch is the objects before
    // the first t >= 1 that does not fit.
    auto size_next = [&](uint64_t o1, uint64_t bt, uint32_t par) {
        const uint64_t b0 = args.obj_base[o1];  // wave-uniform: a scalar load
        const uint32_t lead = (uint32_t)((uintptr_t)(args.blob + b0) & 15);
        const uint64_t kmax = std::min<uint64_t>(kcap, r1 - o1);
        const bool in = tid <= kmax;
        const bool fit = in && o1 + tid < n && bt >= b0 && bt - b0 + lead <= W;
        const uint64_t nf = __ballot(tid >= 1 && in && !fit);
        if (nf != 0 && lane == 0) atomicMin(&lds.kfirst[par], w * 64 + (uint32_t)__builtin_ctzll(nf));
        if (in) lds.bdelta[par][tid] = fit ? (uint32_t)(bt - b0) : kInvalid;
    };
    auto read_next = [&](uint64_t o1, uint32_t par) {
        StreamBatch nb;
        nb.o0 = o1;
        nb.base0 = args.obj_base[o1];
        nb.lead = (uint32_t)((uintptr_t)(args.blob + nb.base0) & 15);
        const uint64_t kmax = std::min<uint64_t>(kcap, r1 - o1);
        const uint32_t kf = std::min<uint64_t>(lds.kfirst[par], kmax + 1);
        nb.K = kf >= 2 ? kf - 1 : 1u;
        nb.span = kf >= 2 ? lds.bdelta[par][nb.K] : kInvalid;
        return nb;
    };
    // the DMA of a batch's span into window par; its lengths (lane t: slot t,
    // and slot t - 64 for the carry of an object straddling two waves) and
    // the bases after it — unconditional, clamped loads: they must be a
    // wave's youngest VMEM operations but for its coordinate store
    auto issue_next = [&](const StreamBatch& nb, uint32_t par, uint32_t& lnext, uint32_t& pnext, uint64_t& bnext) {
        if (nb.span != kInvalid) {
            const uint8_t* s16 = args.blob + nb.base0 - nb.lead;
            const uint32_t units = (nb.lead + nb.span + 15) >> 4;
            for (uint32_t k = w; k * 64 < units; k += WAVES) {
                const uint32_t u = k * 64 + lane;
                if (u < units)
                    __builtin_amdgcn_global_load_lds((const void*)(s16 + 16ull * u),
                                                     (lds_void_t)(lds.win[par] + kFront + 1024 * k), 16, 0, 0);
            }
        }
        const uint64_t q = std::min<uint64_t>(nb.o0 * A + tid, n * A - 1);
        lnext = args.attr_len[q];
        pnext = args.attr_len[q >= 64 ? q - 64 : 0];
        const uint64_t o2 = nb.o0 + nb.K;
        bnext = args.obj_base[std::min<uint64_t>(o2 + tid, n - 1)];
    };

    // ---- prologue: batch 0's size, DMA, lengths; batch 1's bases ------------
    uint64_t bn = args.obj_base[std::min<uint64_t>(r0 + tid, n - 1)];
    size_next(r0, bn, 0);
    __syncthreads();
    StreamBatch cur = read_next(r0, 0);
    uint32_t lc = 0, lp = 0;
    issue_next(cur, 0, lc, lp, bn);
    bool bad = false;

    for (uint32_t b = 0;; ++b) {
        const uint32_t par = b & 1;
        const uint32_t S = cur.K * A;
        const uint64_t o1 = cur.o0 + cur.K;
        const bool more = o1 < r1;
        // batch b's DMA, its lengths and batch b+1's bases have landed
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        // (A) batch b+1's size (lane t holds base[o1 + t])
        if (more) size_next(o1, bn, par ^ 1);

        // (B) describe batch b: slot t = tid
        const bool valid = tid < S;
        const uint32_t len = valid ? lc : 0u;
        const uint32_t orel = div_small(tid, args.a_magic);  // object within the batch
        const uint32_t j = tid - orel * A;
        const uint32_t code = valid ? (uint32_t)lds.codes[j] : (uint32_t)CODE_ZERO;
        const uint32_t xex = wave_scan_dpp(len) - len;
        // in-object offset: from this wave's head of the object, or — an
        // object straddling two waves (A <= 64) — the previous wave's slots
        // from its last head on (lp = length of slot t - 64)
        const int head = lane - (int)j;
        uint32_t inoff;
        if (w == 0) {
            inoff = xex - __shfl(xex, head, 64);
        } else {
            const uint32_t sp = tid - 64;
            const uint32_t jp = sp - div_small(sp, args.a_magic) * A;
            const uint64_t heads = __ballot(jp == 0);  // a wave always holds a head (A <= 64)
            const int lasth = 63 - __builtin_clzll(heads);
            const uint32_t pin = wave_scan_dpp(lp);
            const uint32_t carry = __builtin_amdgcn_readlane(pin, 63) -
                                   (__builtin_amdgcn_readlane(pin, lasth) - __builtin_amdgcn_readlane(lp, lasth));
            inoff = head >= 0 ? xex - __shfl(xex, head, 64) : xex + carry;
        }
        // staged: the slot's bytes lie inside the batch's window
        const uint32_t od = lds.bdelta[par][orel];
        const bool staged = valid && cur.span != kInvalid && od != kInvalid && od + inoff + len <= cur.span;
        const uint32_t cls = valid ? stream_class(code, len, staged) : kStreamClasses;
        uint32_t rank = 0, mycnt = 0;
#pragma unroll
        for (uint32_t k = 0; k < kStreamClasses; ++k) {
            const uint64_t m = __ballot(cls == k);
            if (cls == k) rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (lane == (int)k) mycnt = (uint32_t)__popcll(m);
        }
        if (lane < (int)kStreamClasses) lds.wcls[w][lane] = mycnt;
        __syncthreads();  // ---------------------------------------------- B1 (class counts, next batch's size)

        // (C) batch b+1: its size, the DMA of its span, its lengths, batch
        // b+2's bases
        StreamBatch nxt{};
        uint32_t lnext = 0, pnext = 0;
        uint64_t bnext = 0;
        if (more) {
            nxt = read_next(o1, par ^ 1);
            issue_next(nxt, par ^ 1, lnext, pnext, bnext);
        }
        if (tid == 0) lds.kfirst[par] = kInvalid;  // every wave read it before B1; next used for batch b+2

        // (D) class positions: lane k < classes: class k's start over the
        // workgroup + the slots of class k in waves before this one
        uint32_t tot = 0, before = 0;
        if (lane < (int)kStreamClasses) {
#pragma unroll
            for (int v = 0; v < WAVES; ++v) {
                const uint32_t x = lds.wcls[v][lane];
                tot += x;
                before += (uint32_t)v < w ? x : 0u;
            }
        }
        const uint32_t cstart = wave_scan_dpp(tot) - tot + before;
        const uint32_t pos = (uint32_t)__shfl((int)cstart, (int)std::min<uint32_t>(cls, kStreamClasses - 1), 64) + rank;
        if (valid) {
            const uint32_t off = staged ? kFront + cur.lead + od + inoff : inoff;
            const uint32_t hi = tid | (code << 10) | ((uint32_t)staged << 14) | (std::min(len, kLenMax) << 15);
            lds.sdesc[pos] = (uint64_t)off | ((uint64_t)hi << 32);
        }
        __syncthreads();  // ---------------------------------------------- B2 (descriptors)

        // (E) pass w: 64 class-sorted slots
        {
            const uint32_t idx = w * 64 + lane;
            if (idx < S) {
                const uint64_t e = lds.sdesc[idx];
                const uint32_t off = (uint32_t)e, hi = (uint32_t)(e >> 32);
                const uint32_t cd = (hi >> 10) & 15u;
                uint32_t ln = hi >> 15;
                uint64_t h;
                if ((hi >> 14) & 1u) {
                    h = hash_slot_window(as_ldsw(lds.win[par]), cd, off, ln, bad);
                } else {
                    const uint32_t t = hi & 1023u;
                    const uint32_t ob = div_small(t, args.a_magic);
                    if (ln == kLenMax) ln = args.attr_len[cur.o0 * A + t];
                    const uint8_t* p = args.blob + args.obj_base[cur.o0 + ob] + off;
                    h = hash_slot_global(p, cd, ln, bad);
                }
                lds.sdesc[idx] = h;
            }
        }
        __syncthreads();  // ---------------------------------------------- B3 (coordinates parked)

        // (F) coordinates in slot order
        if (valid) __builtin_nontemporal_store(lds.sdesc[pos], args.coords + cur.o0 * A + tid);
        if (!more) break;
        cur = nxt;
        lc = lnext;
        lp = pnext;
        bn = bnext;
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int WAVES, uint32_t W>
static hipError_t launch_stream_t(const BatchArgs& args, hipStream_t stream, uint32_t wgs) {
    static_assert(sizeof(StreamLds<WAVES, W>) <= 163840, "one workgroup per CU");
    if (args.A == 0 || args.A > 64) return hipErrorInvalidValue;
    const uint64_t kcap = (64ull * WAVES) / args.A;
    uint64_t g = std::min<uint64_t>(wgs, (args.n + kcap - 1) / kcap);
    if (g == 0) g = 1;
    hipLaunchKernelGGL((hash_stream_kernel<WAVES, W>), dim3((uint32_t)g), dim3(64 * WAVES), 0, stream, args);
    return hipGetLastError();
}

static uint32_t device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 256;
    return (uint32_t)cus;
}

// form 0: 16 waves, two 64 KiB windows, one workgroup per CU;
// form 1: 8 waves, two 32 KiB windows, two per CU;
// form 2: 16 waves, two 60 KiB windows.
hipError_t launch_hash_stream(const BatchArgs& args, hipStream_t stream, int form) {
    if (args.n == 0) return hipSuccess;
    const uint32_t cus = device_cus();
    switch (form) {
        case 0: return launch_stream_t<16, 65536 - 1024>(args, stream, cus);
        case 1: return launch_stream_t<8, 32768 - 1024>(args, stream, 2 * cus);
        case 2: return launch_stream_t<16, 61440>(args, stream, cus);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace hdx
