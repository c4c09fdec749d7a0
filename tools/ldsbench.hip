// tools/ldsbench.hip — cost of reading 16-byte pieces from LDS at arbitrary
// byte addresses on gfx950 (the question behind a staged hash kernel: can
// lanes read their variable-length values out of an LDS window as cheaply as
// global_load_dwordx4 reads them from L2/HBM?).
//
// Every lane reads 4 x 16 B per step at its own byte offset into a 16 KiB LDS
// window (offsets spread ~67 B apart across lanes, like packed 64-byte values)
// and folds them by XOR.  Variants:
//   b128u  ds_read_b128 at the unaligned address
//   b32u   4 x ds_read_b32 at unaligned addresses (per 16 B)
//   r2b32u 2 x ds_read2_b32 at unaligned addresses (per 16 B)
//   b128a  ds_read_b128 at the 16-aligned address below (baseline; wrong bytes)
//   b32a   5 x ds_read_b32 aligned + 4 v_alignbyte (the bytes, aligned reads)
//   b64u   2 x ds_read_b64 at unaligned addresses
// Prints one JSON line per variant: ms and LDS bytes read per clock per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kWin = 16384;
constexpr int kSteps = 256;

template <int V>
__global__ void __launch_bounds__(256) k_lds(uint32_t* out, uint32_t seed) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kWin + 256];
    for (int i = threadIdx.x; i < (kWin + 256) / 4; i += blockDim.x)
        reinterpret_cast<uint32_t*>(win)[i] = i * 2654435761u ^ seed;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t off = (lane * 67 + w * 1031 + seed) & (kWin - 1);
    const uint32_t base = (uint32_t)(uintptr_t)win;
    uint32_t acc = 0;
    for (int s = 0; s < kSteps; ++s) {
        const uint32_t a = base + off;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t ak = a + 16 * k;
            uint32_t x0, x1, x2, x3;
            if constexpr (V == 0) {
                uint4 v;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ak));
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            } else if constexpr (V == 1) {
                asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %4 offset:4\n\t"
                             "ds_read_b32 %2, %4 offset:8\n\tds_read_b32 %3, %4 offset:12\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3) : "v"(ak));
                acc ^= x0 ^ x1 ^ x2 ^ x3;
            } else if constexpr (V == 2) {
                uint2 p, q;
                asm volatile("ds_read2_b32 %0, %2 offset1:1\n\tds_read2_b32 %1, %2 offset0:2 offset1:3\n\t"
                             "s_waitcnt lgkmcnt(0)" : "=v"(p), "=v"(q) : "v"(ak));
                acc ^= p.x ^ p.y ^ q.x ^ q.y;
            } else if constexpr (V == 3) {
                uint4 v;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ak & ~15u));
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            } else if constexpr (V == 4) {
                const uint32_t al = ak & ~3u, r = ak & 3u;
                uint32_t d0, d1, d2, d3, d4;
                asm volatile("ds_read_b32 %0, %5\n\tds_read_b32 %1, %5 offset:4\n\t"
                             "ds_read_b32 %2, %5 offset:8\n\tds_read_b32 %3, %5 offset:12\n\t"
                             "ds_read_b32 %4, %5 offset:16\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(d0), "=v"(d1), "=v"(d2), "=v"(d3), "=v"(d4) : "v"(al));
                acc ^= __builtin_amdgcn_alignbyte(d1, d0, r) ^ __builtin_amdgcn_alignbyte(d2, d1, r) ^
                       __builtin_amdgcn_alignbyte(d3, d2, r) ^ __builtin_amdgcn_alignbyte(d4, d3, r);
            } else if constexpr (V == 5) {
                uint2 p, q;
                asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(p), "=v"(q) : "v"(ak));
                acc ^= p.x ^ p.y ^ q.x ^ q.y;
            } else if constexpr (V == 6) {  // b128 at the dword floor (4-byte aligned, not 16)
                uint4 v;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ak & ~3u));
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            } else if constexpr (V == 7) {  // 2 x b64 at the dword floor
                uint2 p, q;
                asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(p), "=v"(q) : "v"(ak & ~3u));
                acc ^= p.x ^ p.y ^ q.x ^ q.y;
            } else if constexpr (V == 8) {  // b64 at the 8-byte floor
                uint2 p, q;
                asm volatile("ds_read_b64 %0, %2\n\tds_read_b64 %1, %2 offset:8\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(p), "=v"(q) : "v"(ak & ~7u));
                acc ^= p.x ^ p.y ^ q.x ^ q.y;
            }
        }
        off = (off + 61 * (acc & 7) + 64) & (kWin - 1);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int V>
static void run(const char* name, uint32_t* out, int blocks, int cus) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_lds<V>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_lds<V>, dim3(blocks), dim3(256), 0, 0, out, (uint32_t)r);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        if (t < best) best = t;
    }
    const double bytes = (double)blocks * 256 * kSteps * 64;
    const double clk = 2.1e9;
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"B_per_clk_per_CU\": %.1f}\n", name, best,
           bytes / (best * 1e-3) / clk / cus);
    fflush(stdout);
}

int main() {
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = cus * 8;  // 8 workgroups (32 waves) per CU
    uint32_t* out;
    CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
    run<3>("b128a", out, blocks, cus);
    run<0>("b128u", out, blocks, cus);
    run<1>("b32u", out, blocks, cus);
    run<2>("r2b32u", out, blocks, cus);
    run<4>("b32a+alignbyte", out, blocks, cus);
    run<5>("b64u", out, blocks, cus);
    run<6>("b128 dword-aligned", out, blocks, cus);
    run<7>("2 x b64 dword-aligned", out, blocks, cus);
    run<8>("2 x b64 8-byte-aligned", out, blocks, cus);
    CK(hipFree(out));
    return 0;
}
