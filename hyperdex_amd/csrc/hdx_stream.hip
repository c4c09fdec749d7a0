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
// B3 (coordinates parked, the next batch's copies landed).  Everything the
// next batch needs — its span, its slot lengths, the object bases after it —
// arrives by LDS DMA issued after B1 of batch b, so no register waits on it;
// each wave drains its own copies (s_waitcnt vmcnt(0)) just before B3.
// Batch b's coordinates are stored from LDS early in batch b+1, so that drain
// never waits for a fresh store.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <algorithm>

#include "hdx_lds_hash.h"
#include "hdx_regroup.h"

namespace hdx {
namespace {

typedef __attribute__((address_space(3))) void* lds_void_t;

constexpr uint32_t kFront = 32;   // window bytes before the span (tail reads of short strings)
constexpr uint32_t kBack = 256;  // after it (head reads of short strings; the 64-lane tail copy)
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

// The same from global memory (the gather kernels' dword-aligned loads).
__device__ __forceinline__ uint64_t hash_slot_global(const uint8_t* p, uint32_t code, uint32_t n, bool& bad) {
    return hash_blk<false, false, true>(code, p, n, consume_any<true>(issue_any<true>(code, p, n)), bad);
}

// Batch x's buffers: span window, lengths and object bases x % 3 (copied two
// batches ahead); its bounds base[o0], base[o0 + K] come from the bounds
// ring, copied 256 batches at a time a block ahead.
template <int WAVES, uint32_t W>
struct StreamLds {
    static constexpr uint32_t S = 64 * WAVES;  // slots per batch at most
    uint8_t win[3][kFront + W + kBack] __attribute__((aligned(16)));
    uint32_t lens[3][S];             // slot lengths (LDS DMA; past the batch: garbage)
    uint32_t bases[3][S];            // object bases o0 .. o0 + S/2 - 1, u64 as dword pairs (LDS DMA)
    uint32_t bnd[2][576];            // per block of 256 batches: base[o0] of its batches and the end, dword pairs
    uint64_t sdesc[S];               // class-sorted {offset, slot | code | staged | len}; then the coordinate
    uint32_t cnt[2][16];             // per batch parity: slots per class (LDS atomics)
    uint32_t lastpos[2];             // per batch parity: the sorted position of the batch's last slot
    uint32_t dummy[64];              // the tail copy of waves that have no tail
    uint8_t codes[64];
};

// A workgroup barrier for LDS traffic only: this wave's LDS reads and writes
// are complete, then s_barrier.  __syncthreads()' workgroup-scope release
// fence would also wait for every LDS DMA in flight.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// s_waitcnt vmcnt(N) (expcnt / lgkmcnt untouched) as the builtin, so that the
// compiler's wait tracking sees it; N is an immediate, hence the switch.
template <int N>
__device__ __forceinline__ void vm_wait() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0x0f70 | (N & 15) | ((N >> 4) << 14));
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
__device__ __forceinline__ void vm_wait_le(uint32_t n) {
    switch (n) {
        case 0: vm_wait<0>(); break;   case 1: vm_wait<1>(); break;   case 2: vm_wait<2>(); break;
        case 3: vm_wait<3>(); break;   case 4: vm_wait<4>(); break;   case 5: vm_wait<5>(); break;
        case 6: vm_wait<6>(); break;   case 7: vm_wait<7>(); break;   case 8: vm_wait<8>(); break;
        case 9: vm_wait<9>(); break;   case 10: vm_wait<10>(); break; case 11: vm_wait<11>(); break;
        case 12: vm_wait<12>(); break; case 13: vm_wait<13>(); break; case 14: vm_wait<14>(); break;
        case 15: vm_wait<15>(); break; case 16: vm_wait<16>(); break; case 17: vm_wait<17>(); break;
        case 18: vm_wait<18>(); break; case 19: vm_wait<19>(); break; case 20: vm_wait<20>(); break;
        case 21: vm_wait<21>(); break; case 22: vm_wait<22>(); break; case 23: vm_wait<23>(); break;
        default: vm_wait<24>(); break;
    }
}
// LDS DMA (global_load_lds_dwordx4 / _dword: this lane's 16 / 4 bytes at src
// to dst + 16 * lane / 4 * lane; dst wave-uniform, through M0) issued from
// inline assembly: the compiler then neither counts it nor — unable to tell
// the buffers apart — waits for it before every later LDS read (it would
// drain the next batches' copies before hashing this one).  Every lane
// issues (sources clamped to valid bytes), so a wave's count of copies per
// batch is fixed and the kernel waits for its own with counted vm_wait_le.
__device__ __forceinline__ void dma_x4(const void* src, const void* dst) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t)dst);
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}
__device__ __forceinline__ void dma_x1(const void* src, const void* dst) {
    const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t)dst);
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}

}  // namespace

// SHAPE (debug variants only, WRONG coordinates): bit 0 = no hashing (each
// slot's descriptor is stored), bit 1 = no copy of the span (the window is
// hashed as it is).
template <int WAVES, uint32_t W, int SHAPE = 0>
__global__ void __launch_bounds__(64 * WAVES)
hash_stream_kernel(const BatchArgs args) {
    typedef StreamLds<WAVES, W> L;
    constexpr uint32_t S_MAX = L::S;
    constexpr uint32_t NI = W / 1024;  // span copy instructions per batch
    static_assert(W % 1024 == 0, "whole 1 KiB copy instructions");
    __shared__ L lds;
    const uint32_t tid = threadIdx.x;
    const int lane = tid & 63;
    const uint32_t w = tid >> 6;
    const uint32_t A = args.A;  // 1..64
    const uint64_t n = args.n;
    // this wave's copies per batch: span instructions + tail + lengths + bases
    const uint32_t per_span = (NI + WAVES - 1 - w) / WAVES + 3;

    // this workgroup's objects, in batches of K (fixed, so that every batch's
    // start is known ahead and the copies run two batches ahead)
    const uint64_t G = gridDim.x;
    const uint64_t r0 = n * blockIdx.x / G, r1 = n * (blockIdx.x + 1) / G;
    if (r0 >= r1) return;  // (uniform: no barrier reached)
    // K from the range's mean object size: ~90 % of a window per batch
    const uint32_t kcap = std::min<uint32_t>(S_MAX / A, S_MAX / 2 - 1);  // K + 1 bases per buffer
    uint32_t K = kcap;
    {
        const uint64_t re = r1 < n ? r1 : n - 1;
        const uint64_t b0 = args.obj_base[r0], b1 = args.obj_base[re];
        if (re > r0 && b1 > b0) {
            const uint64_t mean = (b1 - b0) / (re - r0);
            const uint64_t k = mean ? (uint64_t)(W * 9 / 10) / mean : kcap;
            K = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(k, kcap));
        }
    }
    const uint32_t nbatch = (uint32_t)((r1 - r0 + K - 1) / K);

    if (tid < 64) lds.codes[tid] = tid < A ? args.codes[tid] : (uint8_t)CODE_ZERO;
    if (tid < 32) (&lds.cnt[0][0])[tid] = 0;

    auto batch_o0 = [&](uint32_t x) { return r0 + (uint64_t)x * K; };
    auto batch_k = [&](uint32_t x) { return (uint32_t)std::min<uint64_t>(K, r1 - batch_o0(x)); };
    auto base_at = [&](uint32_t x, uint32_t i) { return pack64(lds.bases[x % 3][2 * i], lds.bases[x % 3][2 * i + 1]); };
    auto bound = [&](uint32_t x) {  // base[o0] of batch x (x = nbatch: the range's end)
        const uint32_t* v = lds.bnd[(x >> 8) & 1] + 2 * (x & 255);
        return pack64(v[0], v[1]);
    };
    // the span of batch x held in its window: bytes from its first 16-byte
    // unit (0 for the launch's last batch, whose end is unknown: hashed from
    // global memory)
    auto held_bytes = [&](uint32_t x, uint64_t& b0, uint32_t& lead) {
        const uint64_t o0 = batch_o0(x);
        const uint32_t k = batch_k(x);
        b0 = bound(x);
        lead = (uint32_t)((uintptr_t)(args.blob + b0) & 15);
        if (o0 + k >= n) return 0u;
        const uint64_t be = (x & 255) == 255 ? pack64(lds.bnd[(x >> 8) & 1][512], lds.bnd[(x >> 8) & 1][513]) : bound(x + 1);
        return be > b0 ? (uint32_t)std::min<uint64_t>(lead + (be - b0), W) : 0u;
    };
    // the bounds of block q's batches 256q .. 256q + 255 and the end of the
    // last: one copy per wave (a lane a dword of base[o0 of batch 256q + v])
    auto issue_bounds = [&](uint32_t q) {
        const uint32_t v = tid >> 1;
        const uint64_t o = std::min<uint64_t>(batch_o0(256 * q + std::min(v, 256u)), n - 1);
        dma_x1((const uint32_t*)args.obj_base + 2 * o + (tid & 1), w < 9 ? lds.bnd[q & 1] + 64 * w : lds.dummy);
    };
    // batch x's span, lengths and bases: per_span copies per wave (every lane
    // issues, sources clamped)
    auto issue_span = [&](uint32_t x) {
        const uint32_t buf = x % 3;
        uint64_t b0;
        uint32_t lead;
        const uint32_t bytes = held_bytes(x, b0, lead);
        const uint8_t* s16 = args.blob + b0 - lead;
        const uint32_t units = SHAPE & 2 ? 1u : bytes >> 4;
        for (uint32_t i = w; i < NI; i += WAVES) {
            const uint32_t u = std::min<uint32_t>(i * 64 + lane, units ? units - 1 : 0);
            dma_x4(s16 + 16ull * u, lds.win[buf] + kFront + 1024 * i);
        }
        // the last partial unit as dwords (a dword never crosses a page), by
        // the wave whose 16-byte copy wrote a clamped lane's bytes there just
        // before (a wave's LDS DMA lands in issue order)
        const uint32_t tdw = ((bytes & 15) + 3) >> 2;
        const bool tail = w == (units >> 6) % WAVES && tdw != 0 && !(SHAPE & 2);
        dma_x1(tail ? (const void*)(s16 + 16ull * units + 4 * std::min<uint32_t>(lane, tdw - 1)) : (const void*)args.attr_len,
               tail ? (const void*)(lds.win[buf] + kFront + 16 * units) : (const void*)lds.dummy);
        dma_x1(args.attr_len + std::min<uint64_t>(batch_o0(x) * A + tid, n * A - 1), lds.lens[buf] + 64 * w);
        dma_x1((const uint32_t*)args.obj_base + std::min<uint64_t>(2 * batch_o0(x) + tid, 2 * n - 1),
               lds.bases[buf] + 64 * w);
    };

    // prologue: the bounds of blocks 0 and 1; spans 0 and 1
    issue_bounds(0);
    issue_bounds(1);
    vm_wait<0>();
    lds_barrier();
    issue_span(0);
    if (1 < nbatch) issue_span(1);
    vm_wait_le(1 < nbatch ? per_span : 0u);
    lds_barrier();

    bool bad = false;
    uint64_t prev_o0 = 0;
    uint32_t prev_S = 0, prev_pos = 0;
    uint64_t tph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // SHAPE & 4: shader cycles per phase (wave 0 of workgroup 0)
    uint64_t tlast = 0;
    auto stamp = [&](int ph) {
        if constexpr ((SHAPE & 4) != 0) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            tph[ph] += t - tlast;
            tlast = t;
        }
    };
    for (uint32_t b = 0; b < nbatch; ++b) {
        stamp(0);
        // here: batch b's span and lengths, and the bases of batches <= b + 2, are in LDS
        const uint32_t buf = b % 3, par = b & 1;
        const uint64_t o0 = batch_o0(b);
        const uint32_t k = batch_k(b);
        const uint32_t S = k * A;
        // copies: at a block's start, the bounds of the block after the next;
        // then batch b+2's span, lengths and bases
        if ((b & 255) == 0 && b > 0 && b + 256 < nbatch) issue_bounds((b >> 8) + 1);
        const bool span2 = b + 2 < nbatch;
        if (span2) issue_span(b + 2);
        stamp(1);
        // batch b-1's coordinates, parked in sdesc, in slot order (every lane
        // stores — slot min(t, S - 1) — so that the store is always issued)
        if (prev_S) {
            const uint32_t t = std::min<uint32_t>(tid, prev_S - 1);
            const uint32_t pp = tid < prev_S ? prev_pos : lds.lastpos[par ^ 1];
            __builtin_nontemporal_store(lds.sdesc[pp], args.coords + prev_o0 * A + t);
        }
        const uint32_t stores = prev_S ? 1u : 0u;
        stamp(2);

        // describe batch b: slot t = tid
        const bool valid = tid < S;
        uint64_t base0;
        uint32_t lead;
        const uint32_t held = SHAPE & 2 ? W : held_bytes(b, base0, lead);
        if (SHAPE & 2) {
            base0 = base_at(b, 0);
            lead = (uint32_t)((uintptr_t)(args.blob + base0) & 15);
        }
        const uint32_t len = valid ? lds.lens[buf][tid] : 0u;
        const uint32_t orel = div_small(tid, args.a_magic);  // object within the batch
        const uint32_t j = tid - orel * A;
        const uint32_t code = valid ? (uint32_t)lds.codes[j] : (uint32_t)CODE_ZERO;
        const uint32_t xex = wave_scan_dpp(len) - len;
        // in-object offset: from this wave's head of the object, or — an
        // object straddling two waves (A <= 64) — the previous wave's slots
        // from its last head on
        const int head = lane - (int)j;
        uint32_t inoff;
        if (w == 0) {
            inoff = xex - __shfl(xex, head, 64);
        } else {
            const uint32_t sp = tid - 64;
            const uint32_t lp = sp < S ? lds.lens[buf][sp] : 0u;
            const uint32_t jp = sp - div_small(sp, args.a_magic) * A;
            const uint64_t heads = __ballot(jp == 0);  // a wave always holds a head (A <= 64)
            const int lasth = 63 - __builtin_clzll(heads);
            const uint32_t pin = wave_scan_dpp(lp);
            const uint32_t carry = __builtin_amdgcn_readlane(pin, 63) -
                                   (__builtin_amdgcn_readlane(pin, lasth) - __builtin_amdgcn_readlane(lp, lasth));
            inoff = head >= 0 ? xex - __shfl(xex, head, 64) : xex + carry;
        }
        // staged: the slot's bytes lie inside the held part of the window
        const uint64_t ob = base_at(b, orel < k ? orel : 0);
        const uint64_t wo = ob - base0 + lead;  // the object's offset in the window (when ob >= base0)
        const bool staged = valid && ob >= base0 && wo + inoff + len <= held;
        const uint32_t cls = valid ? stream_class(code, len, staged) : kStreamClasses;
        uint32_t rank = 0, mycnt = 0;
#pragma unroll
        for (uint32_t c = 0; c < kStreamClasses; ++c) {
            const uint64_t m = __ballot(cls == c);
            if (cls == c) rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (lane == (int)c) mycnt = (uint32_t)__popcll(m);
        }
        // this wave's slots of class c go after those of the waves that got there first
        uint32_t before = 0;
        if (lane < (int)kStreamClasses && mycnt) before = atomicAdd(&lds.cnt[par][lane], mycnt);
        stamp(3);
        lds_barrier();  // ------------------------------------------------- B1 (class counts)
        stamp(4);

        // class positions: class c's start over the workgroup + this wave's
        // offset in it + the slot's rank in this wave
        const uint32_t tot = lane < (int)kStreamClasses ? lds.cnt[par][lane] : 0u;
        const uint32_t cstart = wave_scan_dpp(tot) - tot + before;
        const uint32_t pos = (uint32_t)__shfl((int)cstart, (int)std::min<uint32_t>(cls, kStreamClasses - 1), 64) + rank;
        if (valid) {
            const uint32_t off = staged ? kFront + (uint32_t)wo + inoff : inoff;
            const uint32_t hi = tid | (code << 10) | ((uint32_t)staged << 14) | (std::min(len, kLenMax) << 15);
            lds.sdesc[pos] = (uint64_t)off | ((uint64_t)hi << 32);
        }
        if (tid == S - 1) lds.lastpos[par] = pos;
        stamp(5);
        lds_barrier();  // ------------------------------------------------- B2 (descriptors)
        stamp(6);
        if (tid < 16) lds.cnt[par][tid] = 0;  // read by every wave before B2; next used by batch b + 2

        // pass w: 64 class-sorted slots
        {
            const uint32_t idx = w * 64 + lane;
            if (idx < S && !(SHAPE & 1)) {
                const uint64_t e = lds.sdesc[idx];
                const uint32_t off = (uint32_t)e, hi = (uint32_t)(e >> 32);
                const uint32_t cd = (hi >> 10) & 15u;
                uint32_t ln = hi >> 15;
                uint64_t h;
                if ((hi >> 14) & 1u) {
                    h = hash_slot_window(as_ldsw(lds.win[buf]), cd, off, ln, bad);
                } else {
                    const uint32_t t = hi & 1023u;
                    const uint32_t ot = div_small(t, args.a_magic);
                    if (ln == kLenMax) ln = args.attr_len[o0 * A + t];
                    const uint8_t* p = args.blob + args.obj_base[o0 + ot] + off;
                    h = hash_slot_global(p, cd, ln, bad);
                }
                lds.sdesc[idx] = h;
            }
        }
        // batch b+1's copies (and a new block's bounds) have landed (this
        // wave's; every wave's after B3): younger are batch b+2's copies and
        // the store
        stamp(7);
        vm_wait_le((span2 ? per_span : 0u) + stores);
        stamp(8);
        lds_barrier();  // ------------------------------------------------- B3 (coordinates parked)
        stamp(9);
        prev_o0 = o0;
        prev_S = S;
        prev_pos = pos;
    }
    if (tid < prev_S) __builtin_nontemporal_store(lds.sdesc[prev_pos], args.coords + prev_o0 * A + tid);
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
    if constexpr ((SHAPE & 4) != 0) {
        if (blockIdx.x == 0 && tid == 0) {
            tph[0] = nbatch;  // (phase 0 is the loop's own overhead: report the batch count instead)
            for (int i = 0; i < 10; ++i) args.coords[i] = tph[i];
        }
    }
}

template <int WAVES, uint32_t W, int SHAPE = 0>
static hipError_t launch_stream_t(const BatchArgs& args, hipStream_t stream, uint32_t wgs) {
    static_assert(sizeof(StreamLds<WAVES, W>) <= 163840, "one workgroup per CU");
    if (args.A == 0 || args.A > 64) return hipErrorInvalidValue;
    const uint64_t kcap = (64ull * WAVES) / args.A;
    uint64_t g = std::min<uint64_t>(wgs, (args.n + kcap - 1) / kcap);
    if (g == 0) g = 1;
    hipLaunchKernelGGL((hash_stream_kernel<WAVES, W, SHAPE>), dim3((uint32_t)g), dim3(64 * WAVES), 0, stream, args);
    return hipGetLastError();
}

static uint32_t device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 256;
    return (uint32_t)cus;
}

// form 0: 16 waves, 40 KiB windows; form 1: 16 waves, 32 KiB windows;
// form 2: 8 waves, 16 KiB windows (two workgroups per CU).
hipError_t launch_hash_stream(const BatchArgs& args, hipStream_t stream, int form) {
    if (args.n == 0) return hipSuccess;
    const uint32_t cus = device_cus();
    switch (form) {
        case 0: return launch_stream_t<16, 40960>(args, stream, cus);
        case 1: return launch_stream_t<16, 32768>(args, stream, cus);
        case 2: return launch_stream_t<8, 16384>(args, stream, 2 * cus);
        // debug shapes of form 0 (WRONG coordinates): no hashing / no span copy / neither
        case 3: return launch_stream_t<16, 40960, 1>(args, stream, cus);
        case 4: return launch_stream_t<16, 40960, 2>(args, stream, cus);
        case 5: return launch_stream_t<16, 40960, 3>(args, stream, cus);
        // form 0 with per-phase shader-cycle counters of workgroup 0, wave 0, in coords[0..9]
        case 6: return launch_stream_t<16, 40960, 4>(args, stream, cus);
        case 7: return launch_stream_t<16, 40960, 7>(args, stream, cus);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace hdx
