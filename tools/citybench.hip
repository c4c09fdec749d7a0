// tools/citybench.hip — what one CityHash64 > 64-byte loop block costs on
// gfx950, apart from memory: blocks per second over the whole chip and shader
// cycles per wave-block, for the loop body the kernels run
// (hdx_lds_hash.h city_gt64_lds: city.cc:374-396), with its 64 bytes
//   reg      generated in registers (arithmetic only);
//   lds      read from a wave-private LDS window at a per-lane byte offset
//            (17 dwords + v_alignbyte, as the staged kernels do);
//   lds16    read from the window at 16-byte-aligned per-lane offsets
//            (ds_read_b128, no funnel);
// at 2 / 4 / 8 waves per SIMD, and with 1 or 2 independent strings per lane
// (x2: two chains interleaved, for instruction-level parallelism).
// Prints one JSON line per case.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../hyperdex_amd/csrc/hdx_lds_hash.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

using namespace hdx;

constexpr int kBlocks = 512;  // loop blocks per string
constexpr uint32_t kWin = 8192;

struct State {
    uint64_t x, y, z, v0, v1, w0, w1;
};

__device__ __forceinline__ void city_step(State& s, const Blk& b) {
    uint64_t x = s.x, y = s.y, z = s.z, v0 = s.v0, v1 = s.v1, w0 = s.w0, w1 = s.w1;
    x = ror(x + y + v0 + b.v0.y, 37) * K1;
    y = ror(y + v1 + b.v3.x, 42) * K1;
    x ^= w1;
    y += v0 + b.v2.y;
    z = ror(z + w0, 33) * K1;
    uint64_t nv0, nv1, nw0, nw1;
    weak32(b.v0.x, b.v0.y, b.v1.x, b.v1.y, v1 * K1, x + w0, nv0, nv1);
    weak32(b.v2.x, b.v2.y, b.v3.x, b.v3.y, z + w1, y + b.v1.x, nw0, nw1);
    s.v0 = nv0; s.v1 = nv1; s.w0 = nw0; s.w1 = nw1;
    s.z = x; s.x = z; s.y = y;
}

__device__ __forceinline__ Blk reg_block(uint32_t seed, uint32_t k) {
    Blk b;
    const uint64_t a = pack64(seed ^ k, seed + k);
    b.v0 = u64x2{a, a ^ 1};
    b.v1 = u64x2{a ^ 2, a ^ 3};
    b.v2 = u64x2{a ^ 4, a ^ 5};
    b.v3 = u64x2{a ^ 6, a ^ 7};
    return b;
}

__device__ __forceinline__ Blk lds16_block(ldsw_t w, uint32_t s) {  // s 16-byte aligned
    typedef const __attribute__((address_space(3))) u64x2* l128_t;
    const l128_t q = (l128_t)(w + (s >> 2));
    Blk b;
    b.v0 = q[0];
    b.v1 = q[1];
    b.v2 = q[2];
    b.v3 = q[3];
    return b;
}

template <int MODE, int NS>
__global__ void __launch_bounds__(256) k_city(uint64_t* out, uint32_t seed, unsigned long long* clk) {
    __shared__ __attribute__((aligned(16))) uint8_t win_all[4][kWin + 128];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t* win = win_all[w];
    for (uint32_t i = lane * 4; i < kWin + 128; i += 256) *(uint32_t*)(win + i) = seed * (i + 1);
    __syncthreads();
    const ldsw_t lw = as_ldsw(win);
    State s[NS];
    uint32_t off[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        s[j] = State{seed + lane, seed ^ lane, (uint64_t)j, 1, 2, 3, 4};
        // per-lane windows 108 / 112 bytes apart (the staged kernels' spread)
        off[j] = MODE == 2 ? ((lane * 7 + j * 3) % 64) * 112 % (kWin - 64) & ~15u
                           : ((lane * 37 + j * 11) % 64) * 109 % (kWin - 64);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < kBlocks; ++k) {
#pragma unroll
        for (int j = 0; j < NS; ++j) {
            Blk b;
            if (MODE == 0) b = reg_block(seed + j, (uint32_t)k);
            else if (MODE == 1) b = lds_block64(lw, (off[j] + 64u * (k & 1)) );
            else b = lds16_block(lw, off[j] + 64u * (k & 1));
            city_step(s[j], b);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t w1 = __builtin_amdgcn_s_memrealtime();
    uint64_t r = 0;
#pragma unroll
    for (int j = 0; j < NS; ++j) r ^= s[j].x ^ s[j].y ^ s[j].z ^ s[j].v0 ^ s[j].v1 ^ s[j].w0 ^ s[j].w1;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = w1 - w0;
    }
}

template <int MODE, int NS>
static void bench(uint64_t* out, unsigned long long* clk, int cus, int waves_per_simd) {
    const int blocks = cus * waves_per_simd;  // 4 waves per block = one per SIMD
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_city<MODE, NS>), dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_city<MODE, NS>), dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long h[2];
    CK(hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;
    const double lane_blocks = (double)blocks * 256 * kBlocks * NS;
    const double wave_blocks_per_simd = (double)waves_per_simd * kBlocks * NS;
    static const char* names[] = {"reg", "lds", "lds16"};
    printf("{\"mode\": \"%s\", \"strings_per_lane\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
           "\"Gblocks_per_s\": %.1f, \"TBps_equiv\": %.2f, \"simd_cycles_per_wave_block\": %.1f, "
           "\"in_kernel_cycles_per_wave_block\": %.1f}\n",
           names[MODE], NS, waves_per_simd, ms, ghz, lane_blocks / (ms * 1e-3) / 1e9,
           lane_blocks * 64 / (ms * 1e-3) / 1e12, ms * 1e-3 * ghz * 1e9 / wave_blocks_per_simd,
           (double)h[0] / ((double)kBlocks * NS) / waves_per_simd);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint64_t* out;
    unsigned long long* clk;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 8));
    CK(hipMalloc(&clk, 16));
    fprintf(stderr, "%s: %d CUs\n", p.gcnArchName, cus);
    for (int wps : {2, 4}) {  // LDS: 4 x 8.3 KiB per block -> at most 4 blocks per CU
        bench<0, 1>(out, clk, cus, wps);
        bench<0, 2>(out, clk, cus, wps);
        bench<1, 1>(out, clk, cus, wps);
        bench<1, 2>(out, clk, cus, wps);
        bench<2, 1>(out, clk, cus, wps);
        bench<2, 2>(out, clk, cus, wps);
    }
    return 0;
}
