// tools/tabench.hip — issue cost of global_load_dwordx4 by lane layout, with
// the data in L1/L2 so HBM is not the limit (the question behind config 3b's
// address-unit bound: is a scattered 16-byte-per-lane load dearer per byte
// than a coalesced one, i.e. would lanes cooperating on a value's bytes
// relieve the texture-address unit?).
//
// Every wave loops over 4 independent dwordx4 loads per iteration from a
// 32 KiB (L1-sized) or 1 MiB (L2-resident) region, lane addresses per mode:
//   coalesced     lane * 16            (1 KiB contiguous per instruction)
//   stride64      lane * 64            (64 lanes in 64 different 64-byte lines)
//   stride64_o4   lane * 64 + 4        (dword-aligned, as the A4 pieces)
//   stride64_o52  lane * 64 + 52       (each 16-byte piece straddles a 64-byte line)
//   stride128     lane * 128           (64 different 128-byte lines)
//   quad          (lane / 4) * 64 + (lane % 4) * 16 + 4
//                                      (4 lanes cooperate on one 64-byte span)
// Prints one JSON line per (mode, region): ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(4))) u32x4_a4;
typedef const __attribute__((address_space(1))) u32x4_a4* gptr;

template <int MODE>
__device__ __forceinline__ uint32_t lane_off(uint32_t lane) {
    switch (MODE) {
        case 0: return lane * 16;
        case 1: return lane * 64;
        case 2: return lane * 64 + 4;
        case 3: return lane * 64 + 52;
        case 4: return lane * 128;
        default: return (lane >> 2) * 64 + (lane & 3) * 16 + 4;
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) k_ta(const uint8_t* buf, uint32_t mask, uint32_t iters, uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lo = lane_off<MODE>(lane);
    uint32_t base = (wave * 8192u) & mask;
    u32x4 acc = {0, 0, 0, 0};
    for (uint32_t i = 0; i < iters; ++i) {
        const u32x4 a = *(gptr)(buf + ((base + lo) & mask));
        const u32x4 b = *(gptr)(buf + ((base + 8192 + lo) & mask));
        const u32x4 c = *(gptr)(buf + ((base + 16384 + lo) & mask));
        const u32x4 d = *(gptr)(buf + ((base + 24576 + lo) & mask));
        acc ^= a ^ b ^ c ^ d;
        base = (base + 32768) & mask;
        asm volatile("" : "+v"(base));  // opaque to the optimiser: the loads stay in the loop
    }
    const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (r == 0x12345678u) out[wave] = r;
}

template <int MODE>
static void run(const char* name, const uint8_t* buf, uint32_t region, uint32_t* out, int cus) {
    const uint32_t iters = 2048, blocks = cus * 8;
    hipLaunchKernelGGL(k_ta<MODE>, dim3(blocks), dim3(256), 0, 0, buf, region - 1, iters, out);
    CK(hipDeviceSynchronize());
    hipEvent_t s, e;
    CK(hipEventCreate(&s));
    CK(hipEventCreate(&e));
    CK(hipEventRecord(s));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_ta<MODE>, dim3(blocks), dim3(256), 0, 0, buf, region - 1, iters, out);
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, s, e));
    ms /= 5;
    const double instr_per_cu = (double)blocks * 4 * iters * 4 / cus;
    printf("{\"tool\": \"tabench\", \"mode\": \"%s\", \"region_bytes\": %u, \"ms\": %.4f, "
           "\"ns_per_wave_instr_per_cu\": %.3f, \"GBps_requested\": %.1f}\n",
           name, region, ms, ms * 1e6 / instr_per_cu, (double)blocks * 4 * iters * 4 * 1024 / (ms / 1e3) / 1e9);
    fflush(stdout);
}

int main() {
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, 1 << 20));
    CK(hipMemset(buf, 1, 1 << 20));
    CK(hipMalloc(&out, cus * 32 * sizeof(uint32_t)));
    for (uint32_t region : {16384u << 1, 1u << 20}) {
        run<0>("coalesced", buf, region, out, cus);
        run<1>("stride64", buf, region, out, cus);
        run<2>("stride64_o4", buf, region, out, cus);
        run<3>("stride64_o52", buf, region, out, cus);
        run<4>("stride128", buf, region, out, cus);
        run<5>("quad_o4", buf, region, out, cus);
    }
    return 0;
}
