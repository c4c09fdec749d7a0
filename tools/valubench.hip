// tools/valubench.hip — issue cost of the VALU instructions the CityHash
// kernels are made of, on gfx950: how many shader cycles one SIMD spends per
// wave64 instruction (v_mul_lo_u32 / v_mad_u64_u32 are the 64-bit constant
// multiply's pieces; v_alignbit_b32 the rotates; v_lshl_add_u64 the 64-bit
// adds).  Every lane runs 8 independent chains (no dependency stalls), 8 waves
// per SIMD; the shader clock comes from s_memtime against s_memrealtime
// (100 MHz) inside the kernel.  Prints one JSON line per instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kIters = 4096;

#define OP32(name, text)                                                                     \
    struct name {                                                                            \
        static constexpr const char* s = text;                                               \
        __device__ static void run(uint32_t (&r)[8], uint32_t k) {                           \
            _Pragma("unroll") for (int i = 0; i < 8; ++i)                                    \
                asm volatile(text " %0, %0, %1" : "+v"(r[i]) : "v"(k));                      \
        }                                                                                    \
    };
OP32(Add, "v_add_u32")
OP32(Xor, "v_xor_b32")
OP32(MulLo, "v_mul_lo_u32")
OP32(MulHi, "v_mul_hi_u32")
OP32(MulU24, "v_mul_u32_u24")

struct AlignBit {
    static constexpr const char* s = "v_alignbit_b32";
    __device__ static void run(uint32_t (&r)[8], uint32_t k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(r[i]) : "v"(k));
    }
};
struct MadU64 {
    static constexpr const char* s = "v_mad_u64_u32";
    __device__ static void run(uint32_t (&r)[8], uint32_t k) {
        // pairs of registers as the 64-bit accumulator
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            uint64_t acc = ((uint64_t)r[i + 1] << 32) | r[i];
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(k), "v"(r[i]));
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(k), "v"(r[i]));
            r[i] = (uint32_t)acc;
            r[i + 1] = (uint32_t)(acc >> 32);
        }
    }
};
struct LshlAdd64 {
    static constexpr const char* s = "v_lshl_add_u64";
    __device__ static void run(uint32_t (&r)[8], uint32_t k) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            uint64_t acc = ((uint64_t)r[i + 1] << 32) | r[i];
            const uint64_t kk = ((uint64_t)k << 32) | k;
            asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc) : "v"(kk));
            asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc) : "v"(kk));
            r[i] = (uint32_t)acc;
            r[i + 1] = (uint32_t)(acc >> 32);
        }
    }
};
struct Fma64 {
    static constexpr const char* s = "v_fma_f64";
    __device__ static void run(uint32_t (&r)[8], uint32_t k) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            double acc = __builtin_bit_cast(double, ((uint64_t)r[i + 1] << 32) | r[i]);
            const double kk = (double)k;
            asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc) : "v"(kk));
            asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc) : "v"(kk));
            const uint64_t u = __builtin_bit_cast(uint64_t, acc);
            r[i] = (uint32_t)u;
            r[i + 1] = (uint32_t)(u >> 32);
        }
    }
};

// LANES: how many lanes of each wave run the loop (64 = all; 32 = the
// lower half only; 8; 1) — does a wave64 instruction cost less on the
// SIMD-32 when one half of its exec mask is empty?
template <class Op, int LANES = 64>
__global__ void __launch_bounds__(256) k_valu(uint32_t* out, uint32_t seed, unsigned long long* clk) {
    uint32_t r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = seed * (threadIdx.x + 1) + i;
    const uint32_t k = seed | 1u;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    if (LANES == 64 || (int)(threadIdx.x & 63) < LANES)
        for (int it = 0; it < kIters; ++it) Op::run(r, k);
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t w1 = __builtin_amdgcn_s_memrealtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = w1 - w0;
    }
}

template <class Op, int LANES = 64>
static void bench(uint32_t* out, unsigned long long* clk, int cus) {
    const int waves_per_simd = 8;
    const int blocks = cus * waves_per_simd;  // 4 waves per block = one per SIMD
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_valu<Op, LANES>), dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_valu<Op, LANES>), dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long h[2];
    CK(hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost));
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;  // shader clock of block 0's run
    const double wave_instr_per_simd = (double)waves_per_simd * kIters * 8;
    const double cycles_per_instr = (ms * 1e-3 * ghz * 1e9) / wave_instr_per_simd;
    // in-kernel: block 0's wave 0 cycles over its own instructions (it shares the SIMD with 7 others)
    const double incl = (double)h[0] / ((double)kIters * 8) / waves_per_simd;
    printf("{\"op\": \"%s\", \"lanes\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, \"cycles_per_wave_instr\": %.2f, "
           "\"in_kernel_cycles_per_wave_instr\": %.2f}\n", Op::s, LANES, ms, ghz, cycles_per_instr, incl);
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    unsigned long long* clk;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    CK(hipMalloc(&clk, 16));
    fprintf(stderr, "%s: %d CUs\n", p.gcnArchName, cus);
    bench<Add>(out, clk, cus);
    bench<Xor>(out, clk, cus);
    bench<AlignBit>(out, clk, cus);
    bench<MulU24>(out, clk, cus);
    bench<MulLo>(out, clk, cus);
    bench<MulHi>(out, clk, cus);
    bench<MadU64>(out, clk, cus);
    bench<LshlAdd64>(out, clk, cus);
    bench<Fma64>(out, clk, cus);
    // half-empty exec masks
    bench<Add, 32>(out, clk, cus);
    bench<Add, 8>(out, clk, cus);
    bench<AlignBit, 32>(out, clk, cus);
    bench<MulLo, 32>(out, clk, cus);
    bench<MadU64, 32>(out, clk, cus);
    bench<MadU64, 8>(out, clk, cus);
    bench<LshlAdd64, 32>(out, clk, cus);
    return 0;
}
