// tools/lwbench.hip — loading > 64-byte strings, one string per lane: the
// question behind config 3b's long-string cost.
//
// Every wave takes 64 consecutive strings of a packed buffer (offsets u64,
// lengths u32, as the batch layout) and reads, per string, the 64-byte windows
// CityHash64's > 64-byte path reads (the tail window at p + len - 64, then the
// loop blocks at p + 64 b, b < (len - 1) / 64), XOR-folding them (no hash
// arithmetic), and stores 8 bytes per string.  Modes:
//   lane   the product's A4 form: per window 4 dwordx4 + 1 dword from the
//          window's dword floor, one window per lane (each instruction touches
//          ~64 distinct lines);
//   dma    per window set, the 64 windows copied slot-major into LDS by
//          global_load_lds_dwordx4 — unit u = 64 i + lane is piece u % 5 of
//          window u / 5, so one instruction covers ~13 windows (~20 lines) —
//          then s_waitcnt vmcnt(0) and 5 ds_read_b128 per lane at an 80-byte
//          window stride (conflict-free: 5 is odd);
//   dma2   dma double-buffered: window set t + 1's DMA is issued before set t
//          is read (vmcnt(5));
//   stage  the wave's 64 strings (one contiguous span) copied to LDS by
//          coalesced DMA, windows read back with ds_read_b32 + v_alignbyte;
//   stage2 stage over four groups per wave, group g + 1's DMA under group g's
//          LDS reads (two buffers).
// Prints one JSON line per (mode, data): GB/s of string bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(4))) u32x4_a4;
typedef const __attribute__((address_space(1))) u32x4_a4* gptr4;
typedef const __attribute__((address_space(1))) uint32_t* gptr1;
typedef __attribute__((address_space(3))) void* lptr;

struct Args {
    const uint8_t* buf;
    const uint64_t* off;
    const uint32_t* len;
    uint64_t n;
    uint64_t* out;
};

__device__ __forceinline__ uint32_t fold_window(const uint8_t* p) {
    // A4: pieces from the dword floor + the dword after (funnel omitted: XOR only)
    const uint8_t* a = (const uint8_t*)((uintptr_t)p & ~(uintptr_t)3);
    const u32x4 x0 = *(gptr4)(a), x1 = *(gptr4)(a + 16), x2 = *(gptr4)(a + 32), x3 = *(gptr4)(a + 48);
    const uint32_t e = *(gptr1)(a + 64);
    const u32x4 x = x0 ^ x1 ^ x2 ^ x3;
    return __builtin_amdgcn_alignbyte(x.x ^ x.y, x.z ^ x.w ^ e, (uint32_t)(uintptr_t)p & 3);
}

__global__ void __launch_bounds__(256) k_lane(Args a) {
    const int lane = threadIdx.x & 63;
    const uint64_t s = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 + lane;
    if (s >= a.n) return;
    const uint8_t* p = a.buf + a.off[s];
    const uint32_t L = a.len[s];
    uint32_t acc = fold_window(p + L - 64);
    const uint32_t nb = (L - 1) >> 6;
    for (uint32_t b = 0; b < nb; ++b) acc += fold_window(p + 64 * b);
    a.out[s] = acc;
}

// window w of the set: its dword-aligned start relative to the wave's base
template <bool DOUBLE>
__global__ void __launch_bounds__(256) k_dma(Args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    uint8_t* win = lds + w * (DOUBLE ? 2 : 1) * 5120;
    const uint64_t s0 = ((uint64_t)blockIdx.x * 4 + w) * 64;
    if (s0 >= a.n) return;
    const uint64_t s = s0 + lane;
    const bool valid = s < a.n;
    const uint64_t o = valid ? a.off[s] : a.off[s0];
    const uint32_t L = valid ? a.len[s] : 65u;
    // (readfirstlane returns int: widen through uint32_t, or offsets >= 2 GiB sign-extend)
    const uint64_t wbase = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a.off[s0]) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a.off[s0] >> 32)) << 32);
    const uint8_t* gb = a.buf + (wbase & ~3ull);
    const uint32_t rel = (uint32_t)(o - (wbase & ~3ull));  // this lane's string, from the wave's dword floor
    const uint32_t nb = (L - 1) >> 6;
    const uint32_t nbmax = __builtin_amdgcn_readfirstlane(
        (uint32_t)__reduce_max_sync(~0ull, (int)nb));
    // per unit instruction i: the window (source lane) and piece it copies
    uint32_t srcl[5], piece[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t u = 64 * i + lane;
        srcl[i] = u / 5;
        piece[i] = u - 5 * srcl[i];
    }
    auto start = [&](uint32_t t) -> uint32_t {  // window set t: 0 = tail, 1 + b = loop block b
        const uint32_t bb = t == 0 ? 0u : min(t - 1, nb ? nb - 1 : 0u);
        return t == 0 ? rel + L - 64 : rel + 64 * bb;
    };
    auto issue = [&](uint32_t t, uint8_t* dst) {
        const uint32_t st = start(t) & ~3u;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const uint32_t sw = __shfl(st, srcl[i] < 64 ? (int)srcl[i] : 63, 64);
            if (srcl[i] < 64)
                __builtin_amdgcn_global_load_lds((const void*)(gb + sw + 16 * piece[i]), (lptr)(dst + 1024 * i), 16, 0, 0);
        }
    };
    auto consume = [&](uint32_t t, const uint8_t* src) -> uint32_t {
        const uint32_t sh = start(t) & 3u;
        const __attribute__((address_space(3))) u32x4* q =
            (const __attribute__((address_space(3))) u32x4*)(src + 80 * lane);
        const u32x4 x = q[0] ^ q[1] ^ q[2] ^ q[3];
        const uint32_t e = q[4].x;
        return __builtin_amdgcn_alignbyte(x.x ^ x.y, x.z ^ x.w ^ e, sh);
    };
    uint32_t acc = 0;
    const uint32_t sets = 1 + nbmax;
    if (!DOUBLE) {
        for (uint32_t t = 0; t < sets; ++t) {
            issue(t, win);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t v = consume(t, win);
            if (t == 0 || t - 1 < nb) acc += v;
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        issue(0, win);
        for (uint32_t t = 0; t < sets; ++t) {
            uint8_t* cur = win + (t & 1) * 5120;
            if (t + 1 < sets) {
                issue(t + 1, win + ((t + 1) & 1) * 5120);
                asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const uint32_t v = consume(t, cur);
            if (t == 0 || t - 1 < nb) acc += v;
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (valid) a.out[s] = acc;
}


// stage: the wave's 64 consecutive strings are one contiguous span; it is
// copied into wave-private LDS with coalesced global_load_lds_dwordx4 (1 KiB
// per instruction, ~8 lines), then each lane reads its windows from LDS with
// ds_read_b32 + v_alignbyte (17 dwords per window).  GROUPS > 1: the wave
// takes GROUPS consecutive groups, the next group's DMA in flight while the
// current one is read (two LDS buffers).
template <int GROUPS>
__global__ void __launch_bounds__(256) k_stage(Args a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr uint32_t WB = 13312;  // per buffer: 64 strings of <= 195 B + alignment (832 units)
    constexpr uint32_t KI = WB / 1024;  // DMA instructions per group, always all issued
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    uint8_t* win0 = lds + w * (GROUPS > 1 ? 2 : 1) * WB;
    const uint64_t ngroups = (a.n + 63) / 64;
    uint64_t g = ((uint64_t)blockIdx.x * 4 + w) * GROUPS;
    if (g >= ngroups) return;
    auto span = [&](uint64_t gg, uint64_t& b16, uint32_t& units) {
        const uint64_t s0 = gg * 64, s1 = min(s0 + 64, a.n) - 1;
        const uint64_t lo = a.off[s0], hi = a.off[s1] + a.len[s1];
        b16 = lo & ~15ull;
        units = (uint32_t)((hi - b16 + 15) >> 4);
    };
    auto issue = [&](uint64_t b16, uint32_t units, uint8_t* dst) {
        const uint8_t* src = a.buf + b16;
#pragma unroll
        for (uint32_t i = 0; i < KI; ++i) {  // every lane, every instruction: vmcnt stays countable
            const uint32_t u = min(i * 64 + (uint32_t)lane, units - 1);
            __builtin_amdgcn_global_load_lds((const void*)(src + 16ull * u), (lptr)(dst + 1024 * i), 16, 0, 0);
        }
    };
    auto fold = [&](const uint8_t* win, uint32_t o) -> uint32_t {
        uint32_t x = 0;
        const __attribute__((address_space(3))) uint32_t* d = (const __attribute__((address_space(3))) uint32_t*)(win + (o & ~3u));
        uint32_t prev = d[0];
#pragma unroll
        for (int k = 1; k <= 16; ++k) {
            const uint32_t cur = d[k];
            x ^= __builtin_amdgcn_alignbyte(cur, prev, o & 3);
            prev = cur;
        }
        return x;
    };
    uint64_t b16, nb16 = 0;
    uint32_t units, nunits = 0;
    span(g, b16, units);
    issue(b16, units, win0);
    for (int t = 0; t < GROUPS && g < ngroups; ++t, ++g) {
        uint8_t* cur = win0 + (t & 1) * WB;
        const uint64_t s = g * 64 + lane;
        const bool valid = s < a.n;
        const uint64_t so = valid ? a.off[s] : 0;
        const uint32_t L = valid ? a.len[s] : 65u;
        const bool more = GROUPS > 1 && t + 1 < GROUPS && g + 1 < ngroups;
        if (more) span(g + 1, nb16, nunits);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this group's DMA (issued a group ago) + metadata
        if (more) issue(nb16, nunits, win0 + ((t + 1) & 1) * WB);
        if (valid) {
            const uint32_t o = (uint32_t)(so - b16);
            uint32_t acc = fold(cur, o + L - 64);
            const uint32_t nb = (L - 1) >> 6;
            for (uint32_t bb = 0; bb < nb; ++bb) acc += fold(cur, o + 64 * bb);
            a.out[s] = acc;
        }
        __builtin_amdgcn_wave_barrier();
        b16 = nb16;
        units = nunits;
    }
}

static double time_kernel(void (*launch)(const Args&), const Args& a, int reps = 5) {
    launch(a);
    CK(hipDeviceSynchronize());
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    CK(hipEventRecord(s));
    for (int r = 0; r < reps; ++r) launch(a);
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, s, e));
    return ms / reps;
}

static uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + 255) / 256); }
static void launch_lane(const Args& a) { hipLaunchKernelGGL(k_lane, dim3(blocks_for(a.n)), dim3(256), 0, 0, a); }
static void launch_dma(const Args& a) { hipLaunchKernelGGL(k_dma<false>, dim3(blocks_for(a.n)), dim3(256), 4 * 5120, 0, a); }
static void launch_stage(const Args& a) { hipLaunchKernelGGL(k_stage<1>, dim3(blocks_for(a.n)), dim3(256), 4 * 13312 + 64, 0, a); }
static void launch_stage2(const Args& a) {
    hipLaunchKernelGGL(k_stage<4>, dim3((uint32_t)(((a.n + 63) / 64 + 15) / 16)), dim3(256), 8 * 13312 + 64, 0, a);
}
static void launch_dma2(const Args& a) { hipLaunchKernelGGL(k_dma<true>, dim3(blocks_for(a.n)), dim3(256), 8 * 5120, 0, a); }

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
    struct Data { const char* name; uint32_t lo, hi; };
    const Data data[] = {{"u150", 150, 150}, {"u100", 100, 100}, {"u65_195", 65, 195}};
    uint64_t* out;
    CK(hipMalloc(&out, n * 8));
    for (const Data& d : data) {
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> len(n);
        uint64_t x = 0x9e3779b97f4a7c15ull, tot = 0;
        for (uint64_t i = 0; i < n; ++i) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            len[i] = d.lo + (uint32_t)(x % (d.hi - d.lo + 1));
            off[i] = tot;
            tot += len[i];
        }
        uint8_t* buf;
        uint64_t* doff;
        uint32_t* dlen;
        CK(hipMalloc(&buf, tot + 64));
        CK(hipMemset(buf, 7, tot + 64));
        CK(hipMalloc(&doff, n * 8));
        CK(hipMalloc(&dlen, n * 4));
        CK(hipMemcpy(doff, off.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dlen, len.data(), n * 4, hipMemcpyHostToDevice));
        Args a{buf, doff, dlen, n, out};
        struct M { const char* name; void (*fn)(const Args&); };
        for (M m : {M{"lane", launch_lane}, M{"dma", launch_dma}, M{"dma2", launch_dma2}, M{"stage", launch_stage},
                    M{"stage2", launch_stage2}, M{"lane", launch_lane}}) {
            const double ms = time_kernel(m.fn, a);
            printf("{\"tool\": \"lwbench\", \"mode\": \"%s\", \"data\": \"%s\", \"strings\": %llu, \"bytes\": %llu, "
                   "\"ms\": %.4f, \"GBps\": %.1f, \"GBps_incl_meta\": %.1f}\n",
                   m.name, d.name, (unsigned long long)n, (unsigned long long)tot, ms, tot / (ms / 1e3) / 1e9,
                   (tot + n * 20) / (ms / 1e3) / 1e9);
            fflush(stdout);
        }
        CK(hipFree(buf));
        CK(hipFree(doff));
        CK(hipFree(dlen));
    }
    return 0;
}
