// tools/mulbench.hip — issue cost of the VALU instructions CityHash's 64-bit
// arithmetic compiles to on gfx950 (v_mad_u64_u32 / v_mul_lo_u32 for a
// 64 x 64 -> 64 multiply, v_alignbit / v_alignbyte for rotates and funnels,
// the 24-bit multiplies, FP64 FMA), as SIMD cycles per wave64 instruction with
// 8 independent chains per wave and 8 waves per SIMD (throughput, not latency).
// Prints one JSON line per instruction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kIters = 4096;

#define REP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

template <int OP>
__global__ void __launch_bounds__(256) k_op(uint32_t* out, uint32_t seed, unsigned long long* clk) {
    uint32_t a[8], b[8];
    uint64_t q[8], cy = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = seed * (threadIdx.x + i + 1);
        b[i] = seed ^ (threadIdx.x * 7 + i);
        q[i] = ((uint64_t)a[i] << 32) | b[i];
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < kIters; ++k) {
#define STEP(i)                                                                                                  \
        if constexpr (OP == 0) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));              \
        if constexpr (OP == 1) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));              \
        if constexpr (OP == 2) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(q[i]), "=s"(cy) : "v"(a[i]), "v"(b[i])); \
        if constexpr (OP == 3) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));                 \
        if constexpr (OP == 4) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a[i]) : "v"(b[i]));        \
        if constexpr (OP == 5) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b[i]));         \
        if constexpr (OP == 6) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));          \
        if constexpr (OP == 7) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(q[i]) : "v"(q[(i + 1) & 7])); \
        if constexpr (OP == 8) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(q[i]) : "v"(q[(i + 1) & 7]));   \
        if constexpr (OP == 9) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(a[i]) : "v"(b[i]));            \
        if constexpr (OP == 10) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
        REP8(STEP)
#undef STEP
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r ^= a[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32);
    r ^= (uint32_t)cy;
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
}

template <int OP>
static void bench(const char* name, uint32_t* out, unsigned long long* clk, int cus) {
    const int wps = 8;  // waves per SIMD: 4 waves per block, one per SIMD
    const int blocks = cus * wps;
    hipLaunchKernelGGL((k_op<OP>), dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_op<OP>), dim3(blocks), dim3(256), 0, 0, out, 7u, clk);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long h;
    CK(hipMemcpy(&h, clk, sizeof h, hipMemcpyDeviceToHost));
    const double insts_per_simd = (double)wps * kIters * 8;
    printf("{\"inst\": \"%s\", \"ms\": %.4f, \"in_kernel_cycles_per_wave_inst_per_simd\": %.2f}\n", name, ms,
           (double)h / insts_per_simd);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* out;
    unsigned long long* clk;
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
    CK(hipMalloc(&clk, 16));
    bench<3>("v_add_u32", out, clk, cus);
    bench<10>("v_xor_b32", out, clk, cus);
    bench<9>("v_add3_u32", out, clk, cus);
    bench<4>("v_alignbit_b32", out, clk, cus);
    bench<0>("v_mul_lo_u32", out, clk, cus);
    bench<1>("v_mul_hi_u32", out, clk, cus);
    bench<2>("v_mad_u64_u32", out, clk, cus);
    bench<5>("v_mad_u32_u24", out, clk, cus);
    bench<6>("v_mul_hi_u32_u24", out, clk, cus);
    bench<7>("v_lshl_add_u64", out, clk, cus);
    bench<8>("v_fma_f64", out, clk, cus);
    return 0;
}
