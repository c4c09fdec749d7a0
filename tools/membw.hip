// tools/membw.hip — HBM access-pattern calibration for the hash kernel (gfx950).
//
// Measures, on a buffer the size of the config-3a blob (10.88 GB), the
// bandwidth of the read patterns the hashing kernel can use:
//   coalesced    : lane l reads 16 B at 16*l of each 1 KiB wave chunk
//   stride64     : lane l reads its own 64 B (4 x 16 B), lanes 64 B apart
//                  (the direct per-lane string load of hash_batch_kernel)
//   stride64_lds : wave loads its 4 KiB coalesced, stages it through LDS,
//                  each lane reads its 64 B back from LDS (padded rows)
//   copy / write : reference points
// Prints one JSON line per pattern.  Usage: membw [GB] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_fill(u32x4* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = u32x4{(uint32_t)i, (uint32_t)(i * 3), (uint32_t)(i * 7), (uint32_t)(i >> 3)};
}

// one wave per 4 KiB chunk (like one hash round of 64 x 64 B strings)
__global__ void __launch_bounds__(256) k_coalesced(const u32x4* p, size_t chunks, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    size_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
    if (w >= chunks) return;
    const u32x4* c = p + w * 256;
    u32x4 a = c[lane] ^ c[64 + lane] ^ c[128 + lane] ^ c[192 + lane];
    uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
    if (x == 0x12345678u) out[0] = x;
}

__global__ void __launch_bounds__(256) k_stride64(const u32x4* p, size_t chunks, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    size_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
    if (w >= chunks) return;
    const u32x4* c = p + w * 256 + lane * 4;
    u32x4 a = c[0] ^ c[1] ^ c[2] ^ c[3];
    uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
    if (x == 0x12345678u) out[0] = x;
}

// stride64 + one 8-byte store per 64 B read (the coords write)
__global__ void __launch_bounds__(256) k_stride64_w8(const u32x4* p, size_t chunks, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    size_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
    if (w >= chunks) return;
    const u32x4* c = p + w * 256 + lane * 4;
    u32x4 a = c[0] ^ c[1] ^ c[2] ^ c[3];
    out[w * 64 + lane] = ((uint64_t)(a.x ^ a.y) << 32) | (a.z ^ a.w);
}

__global__ void __launch_bounds__(256) k_stride64_lds(const u32x4* p, size_t chunks, uint32_t* out) {
    __shared__ u32x4 lds[4][64 * 5];  // 80 B rows: conflict-free ds_read_b128
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    size_t w = blockIdx.x * 4ull + wv;
    if (w >= chunks) return;
    const u32x4* c = p + w * 256;
    u32x4 v0 = c[lane], v1 = c[64 + lane], v2 = c[128 + lane], v3 = c[192 + lane];
    // element e = 64*k + lane belongs to string e/4, quarter e%4
    int e0 = lane, e1 = 64 + lane, e2 = 128 + lane, e3 = 192 + lane;
    lds[wv][(e0 >> 2) * 5 + (e0 & 3)] = v0;
    lds[wv][(e1 >> 2) * 5 + (e1 & 3)] = v1;
    lds[wv][(e2 >> 2) * 5 + (e2 & 3)] = v2;
    lds[wv][(e3 >> 2) * 5 + (e3 & 3)] = v3;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    u32x4 a = lds[wv][lane * 5] ^ lds[wv][lane * 5 + 1] ^ lds[wv][lane * 5 + 2] ^ lds[wv][lane * 5 + 3];
    uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
    if (x == 0x12345678u) out[0] = x;
}


// read 64 B/lane + 8 B coordinate per lane, stored non-temporally
__global__ void __launch_bounds__(256) k_stride64_w8nt(const u32x4* p, size_t chunks, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    size_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
    if (w >= chunks) return;
    const u32x4* c = p + w * 256 + lane * 4;
    u32x4 a = c[0] ^ c[1] ^ c[2] ^ c[3];
    __builtin_nontemporal_store(((uint64_t)(a.x ^ a.y) << 32) | (a.z ^ a.w), out + w * 64 + lane);
}

// each wave walks R consecutive 4 KiB chunks (like A rounds of one hash wave),
// keeping its R coordinate vectors in registers and storing them at the end
template <int R, bool NT>
__global__ void __launch_bounds__(256) k_rounds_w8(const u32x4* p, size_t chunks, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    size_t w0 = (blockIdx.x * 4ull + (threadIdx.x >> 6)) * R;
    if (w0 >= chunks) return;
    uint64_t acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const u32x4* c = p + (w0 + r) * 256 + lane * 4;
        u32x4 a = (w0 + r < chunks) ? (c[0] ^ c[1] ^ c[2] ^ c[3]) : u32x4{0, 0, 0, 0};
        acc[r] = ((uint64_t)(a.x ^ a.y) << 32) | (a.z ^ a.w);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (w0 + r < chunks) {
            if (NT) __builtin_nontemporal_store(acc[r], out + (w0 + r) * 64 + lane);
            else out[(w0 + r) * 64 + lane] = acc[r];
        }
}

// the hash kernel's exact traffic without the hash: per round a coalesced u32
// length load, then 64 B per lane, then an 8 B store; R rounds per wave
template <int R, bool NT>
__global__ void __launch_bounds__(256) k_hashshape(const u32x4* p, const uint32_t* lens, size_t chunks, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    size_t w0 = (blockIdx.x * 4ull + (threadIdx.x >> 6)) * R;
    for (int r = 0; r < R; ++r) {
        size_t w = w0 + r;
        if (w >= chunks) return;
        uint32_t L = lens[w * 64 + lane];
        const u32x4* c = p + w * 256 + lane * 4 + (L >> 31);
        u32x4 a = c[0] ^ c[1] ^ c[2] ^ c[3];
        uint64_t h = ((uint64_t)(a.x ^ a.y) << 32) | (a.z ^ a.w) ^ L;
        if (NT) __builtin_nontemporal_store(h, out + w * 64 + lane);
        else out[w * 64 + lane] = h;
    }
}


// one 4 KiB chunk per wave with the hash kernel's dependency chain: previous
// chunk's lengths (carry) + this chunk's lengths -> dependent 64 B/lane loads
// -> 8 B store.  Consecutive waves take consecutive chunks (linear front).
template <bool NT>
__global__ void __launch_bounds__(256) k_hashshape1(const u32x4* p, const uint32_t* lens, size_t chunks, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    size_t w = blockIdx.x * 4ull + (threadIdx.x >> 6);
    if (w >= chunks) return;
    uint32_t Lp = w ? lens[(w - 1) * 64 + lane] : 0;
    uint32_t L = lens[w * 64 + lane];
    const u32x4* c = p + w * 256 + lane * 4 + ((L + Lp) >> 31);
    u32x4 a = c[0] ^ c[1] ^ c[2] ^ c[3];
    uint64_t h = ((uint64_t)(a.x ^ a.y) << 32) | (a.z ^ a.w) ^ L;
    if (NT) __builtin_nontemporal_store(h, out + w * 64 + lane);
    else out[w * 64 + lane] = h;
}

// 17 dependent rounds per wave but rounds strided by the whole grid
// (round r of wave w = chunk r * W + w): same per-wave chain as hashshape17,
// linear chip-wide front.
template <int R>
__global__ void __launch_bounds__(256) k_hashshape_strided(const u32x4* p, const uint32_t* lens, size_t chunks, uint64_t* out) {
    const int lane = threadIdx.x & 63;
    const size_t W = (size_t)gridDim.x * 4;
    size_t w0 = blockIdx.x * 4ull + (threadIdx.x >> 6);
    for (int r = 0; r < R; ++r) {
        size_t w = w0 + r * W;
        if (w >= chunks) return;
        uint32_t L = lens[w * 64 + lane];
        const u32x4* c = p + w * 256 + lane * 4 + (L >> 31);
        u32x4 a = c[0] ^ c[1] ^ c[2] ^ c[3];
        out[w * 64 + lane] = ((uint64_t)(a.x ^ a.y) << 32) | (a.z ^ a.w) ^ L;
    }
}

// grid-stride streaming read, 2048 blocks, 4 x 16 B in flight per lane
__global__ void __launch_bounds__(256) k_stream(const u32x4* p, size_t n16, uint32_t* out) {
    u32x4 a = {0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) a ^= p[i] ^ p[i + stride] ^ p[i + 2 * stride] ^ p[i + 3 * stride];
    for (; i < n16; i += stride) a ^= p[i];
    uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
    if (x == 0x12345678u) out[0] = x;
}

__global__ void __launch_bounds__(256) k_copy(const u32x4* p, u32x4* q, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += stride) q[i] = p[i];
}

__global__ void __launch_bounds__(256) k_write(u32x4* q, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += stride)
        q[i] = u32x4{(uint32_t)i, 1, 2, 3};
}

template <typename F>
static void timeit(const char* name, double bytes, int reps, F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a, 0));
        launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    float med = ms[ms.size() / 2];
    printf("{\"pattern\": \"%s\", \"GB\": %.3f, \"ms_median\": %.4f, \"ms_min\": %.4f, \"GBps\": %.1f}\n", name,
           bytes / 1e9, med, ms[0], bytes / (med / 1e3) / 1e9);
    fflush(stdout);
}

int main(int argc, char** argv) {
    double gb = argc > 1 ? atof(argv[1]) : 10.88;
    int reps = argc > 2 ? atoi(argv[2]) : 10;
    size_t chunks = (size_t)(gb * 1e9 / 4096);
    size_t bytes = chunks * 4096, n16 = bytes / 16;
    u32x4 *p, *q;
    uint32_t* out;
    uint64_t* coords;
    CK(hipMalloc(&p, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&coords, chunks * 64 * 8));
    k_fill<<<4096, 256>>>(p, n16);
    CK(hipDeviceSynchronize());
    const unsigned blocks = (unsigned)((chunks + 3) / 4);
    timeit("coalesced_wave4k", bytes, reps, [&] { k_coalesced<<<blocks, 256>>>(p, chunks, out); });
    timeit("stride64_wave4k", bytes, reps, [&] { k_stride64<<<blocks, 256>>>(p, chunks, out); });
    timeit("stride64_lds_wave4k", bytes, reps, [&] { k_stride64_lds<<<blocks, 256>>>(p, chunks, out); });
    timeit("stride64_w8_wave4k", bytes + chunks * 64 * 8.0, reps,
           [&] { k_stride64_w8<<<blocks, 256>>>(p, chunks, coords); });

    timeit("stride64_w8nt_wave4k", bytes + chunks * 64 * 8.0, reps,
           [&] { k_stride64_w8nt<<<blocks, 256>>>(p, chunks, coords); });
    {
        const unsigned b17 = (unsigned)((chunks + 4 * 17 - 1) / (4 * 17));
        timeit("rounds17_w8_deferred", bytes + chunks * 64 * 8.0, reps,
               [&] { k_rounds_w8<17, false><<<b17, 256>>>(p, chunks, coords); });
        timeit("rounds17_w8nt_deferred", bytes + chunks * 64 * 8.0, reps,
               [&] { k_rounds_w8<17, true><<<b17, 256>>>(p, chunks, coords); });
        uint32_t* lens;
        CK(hipMalloc(&lens, chunks * 64 * 4));
        CK(hipMemset(lens, 0, chunks * 64 * 4));
        timeit("hashshape17_plain", bytes + chunks * 64 * 12.0, reps,
               [&] { k_hashshape<17, false><<<b17, 256>>>(p, lens, chunks, coords); });
        timeit("hashshape17_nt", bytes + chunks * 64 * 12.0, reps,
               [&] { k_hashshape<17, true><<<b17, 256>>>(p, lens, chunks, coords); });
        timeit("hashshape1_plain", bytes + chunks * 64 * 12.0, reps,
               [&] { k_hashshape1<false><<<blocks, 256>>>(p, lens, chunks, coords); });
        timeit("hashshape1_nt", bytes + chunks * 64 * 12.0, reps,
               [&] { k_hashshape1<true><<<blocks, 256>>>(p, lens, chunks, coords); });
        timeit("hashshape17_strided", bytes + chunks * 64 * 12.0, reps,
               [&] { k_hashshape_strided<17><<<b17, 256>>>(p, lens, chunks, coords); });
        CK(hipFree(lens));
    }
    for (unsigned g : {1024u, 2048u, 4096u, 8192u})
        timeit(g == 1024 ? "stream_gs1024" : g == 2048 ? "stream_gs2048" : g == 4096 ? "stream_gs4096" : "stream_gs8192",
               bytes, reps, [&] { k_stream<<<g, 256>>>(p, n16, out); });
    CK(hipFree(coords));
    size_t half = bytes / 2;
    q = (u32x4*)((char*)p + half);
    timeit("copy_half", 2.0 * half, reps, [&] { k_copy<<<8192, 256>>>(p, q, half / 16); });
    timeit("write", bytes, reps, [&] { k_write<<<8192, 256>>>(p, n16); });
    return 0;
}
