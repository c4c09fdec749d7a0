// tools/gldbench.hip — cost of global_load_dwordx4 by address alignment on
// gfx950 (the question behind the hash kernels' per-lane value loads: does a
// 16-byte load at a byte / dword / 16-byte misaligned address cost the
// texture-address unit more than an aligned one?).
//
// Every lane reads a 64-byte span as 4 x global_load_dwordx4 at
//   buf + chunk * 4096 + lane * 64 + off
// (lanes 64 B apart, the shape of 64-byte packed values), folds it by XOR and
// stores one dword.  One pass over 4 GiB per launch; prints GB/s per offset.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 __attribute__((aligned(1))) u32x4_u;
typedef const __attribute__((address_space(1))) u32x4_u* gptr;

// MODE 0: 4 x dwordx4 at span + off (span = 64 B per lane)
// MODE 1: 5 x dwordx4 at the 16-aligned span start (the aligned cover of a
//         misaligned 64-byte span), no funnel shift
// MODE 2: 4 x dwordx4 + 1 dword at the 4-aligned span start
template <int MODE>
__global__ void __launch_bounds__(256) k_span(const uint8_t* buf, size_t chunks, uint32_t off, uint32_t* out) {
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (wave >= chunks) return;
    const uint8_t* p = buf + wave * 4096 + lane * 64 + off;
    u32x4 acc = {0, 0, 0, 0};
    if (MODE == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= *(gptr)(p + 16 * k);
    } else if (MODE == 1) {
        const uint8_t* a = p - ((uintptr_t)p & 15);
#pragma unroll
        for (int k = 0; k < 5; ++k) acc ^= *(gptr)(a + 16 * k);
    } else {
        const uint8_t* a = p - ((uintptr_t)p & 3);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc ^= *(gptr)(a + 16 * k);
        acc.x ^= *(const __attribute__((address_space(1))) uint32_t*)(a + 64);
    }
    out[wave * 64 + lane] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}

template <int MODE>
static void run(const char* name, const uint8_t* buf, size_t chunks, uint32_t off, uint32_t* out) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint32_t blocks = (uint32_t)((chunks + 3) / 4);
    hipLaunchKernelGGL(k_span<MODE>, dim3(blocks), dim3(256), 0, 0, buf, chunks, off, out);
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_span<MODE>, dim3(blocks), dim3(256), 0, 0, buf, chunks, off, out);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        if (t < best) best = t;
    }
    const double bytes = (double)chunks * 4096;
    printf("{\"mode\": \"%s\", \"off\": %u, \"ms\": %.4f, \"GBps\": %.1f}\n", name, off, best,
           bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
}

int main() {
    const size_t chunks = (size_t)1 << 20;  // 4 GiB
    uint8_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, chunks * 4096 + 256));
    CK(hipMemset(buf, 0x5a, chunks * 4096 + 256));
    CK(hipMalloc(&out, chunks * 64 * 4));
    const uint32_t offs[] = {0, 1, 3, 4, 8, 12, 16, 32, 48};
    for (uint32_t off : offs) run<0>("x4", buf, chunks, off, out);
    for (uint32_t off : {1u, 4u, 8u}) run<1>("x4_aligned16_cover", buf, chunks, off, out);
    for (uint32_t off : {1u, 5u}) run<2>("x4_aligned4_cover", buf, chunks, off, out);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
