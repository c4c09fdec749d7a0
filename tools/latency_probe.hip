// Where a lone batcher caller's round trip goes: the pieces
// of one small batch, each timed 3000 times on one stream (p50 / p99 us).
//
//   latency_probe            (links ../hyperdex_amd/libhdxhash.so)
//
//   launch_sync        empty kernel + hipStreamSynchronize
//   launch_event_spin  empty kernel + event, host spins on hipEventQuery
//   launch_flag_spin   empty kernel + hipStreamWriteValue32 on a pinned word,
//                      host spins on the word
//   fused_1 / fused_64 hdx_hash_batch_regions_device (3 tables) over 1 / 64
//                      config-3b objects in pinned mapped staging + sync
//   fused_1_flag       the same, completion seen through the pinned word
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <vector>

#include "hdxhash.h"

using Clock = std::chrono::steady_clock;

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            exit(2);                                                       \
        }                                                                  \
    } while (0)

__global__ void empty_kernel(int* p) {
    if (p && threadIdx.x == 1024) *p = 0;  // never true: keeps the argument live
}

static void report(const char* name, std::vector<double>& us) {
    std::sort(us.begin(), us.end());
    printf("{\"tool\": \"latency_probe\", \"step\": \"%s\", \"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, "
           "\"n\": %zu}\n",
           name, us[us.size() / 2], us[us.size() * 9 / 10], us[us.size() * 99 / 100], us.size());
    fflush(stdout);
}

template <class F>
static void timeit(const char* name, F f, int reps = 3000) {
    for (int i = 0; i < 200; ++i) f();
    std::vector<double> us;
    us.reserve(reps);
    for (int i = 0; i < reps; ++i) {
        const auto t0 = Clock::now();
        f();
        us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    report(name, us);
}

static hdx_region_table grid(std::vector<uint16_t> attrs, uint32_t cells, uint64_t first_id) {
    const uint32_t D = (uint32_t)attrs.size();
    uint32_t R = 1;
    for (uint32_t d = 0; d < D; ++d) R *= cells;
    std::vector<uint64_t> lo((size_t)R * D), up((size_t)R * D), ids(R);
    const uint64_t step = UINT64_MAX / cells;
    for (uint32_t r = 0; r < R; ++r) {
        uint32_t x = r;
        for (uint32_t d = 0; d < D; ++d) {
            const uint32_t c = x % cells;
            x /= cells;
            lo[(size_t)r * D + d] = c * step + (c ? 1 : 0);
            up[(size_t)r * D + d] = c + 1 == cells ? UINT64_MAX : (c + 1) * step;
        }
        ids[r] = first_id + r;
    }
    hdx_region_table t = nullptr;
    if (hdx_region_table_create(D, R, attrs.data(), lo.data(), up.data(), ids.data(), &t) != HDX_OK) exit(2);
    return t;
}

template <class T>
static T* mapped(size_t n, T** dev) {
    T* h = nullptr;
    CK(hipHostMalloc((void**)&h, n * sizeof(T) + 64, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)dev, h, 0));
    return h;
}

int main() {
    if (hdx_init(0) != HDX_OK) return 2;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint32_t* dflag = nullptr;
    volatile uint32_t* flag = mapped<uint32_t>(1, &dflag);
    *flag = 0;
    uint32_t seq = 0;

    timeit("launch_sync", [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
        CK(hipStreamSynchronize(s));
    });
    timeit("launch_event_spin", [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
        CK(hipEventRecord(ev, s));
        while (hipEventQuery(ev) == hipErrorNotReady) {
        }
    });
    timeit("launch_flag_spin", [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, nullptr);
        CK(hipStreamWriteValue32(s, dflag, ++seq, 0));
        while (*flag != seq) __builtin_ia32_pause();
    });

    // config 3b objects (key 64 B; 10 STRING U{0..195}; 3 INT64; 3 FLOAT)
    const uint32_t A = 17;
    uint32_t types[A];
    for (uint32_t j = 0; j <= 10; ++j) types[j] = 9217;
    for (uint32_t j = 11; j <= 13; ++j) types[j] = 9218;
    for (uint32_t j = 14; j <= 16; ++j) types[j] = 9219;
    hdx_region_table tables[3] = {grid({0}, 64, 1), grid({1, 11, 14}, 4, 100), grid({2, 12, 15}, 4, 200)};
    const uint32_t nmax = 64;
    uint8_t* dblob;
    uint64_t* dbase;
    uint32_t* dlen;
    uint64_t *dids, *dcoords;
    uint8_t* blob = mapped<uint8_t>(nmax * 2048, &dblob);
    uint64_t* base = mapped<uint64_t>(nmax, &dbase);
    uint32_t* len = mapped<uint32_t>(nmax * A, &dlen);
    mapped<uint64_t>(3 * nmax, &dids);
    mapped<uint64_t>(nmax * A, &dcoords);
    std::mt19937_64 rng(7);
    uint64_t off = 0;
    for (uint32_t i = 0; i < nmax; ++i) {
        base[i] = off;
        for (uint32_t j = 0; j < A; ++j) {
            len[i * A + j] = j == 0 ? 64 : j <= 10 ? (uint32_t)(rng() % 196) : 8;
            off += len[i * A + j];
        }
    }
    for (uint64_t k = 0; k < off; ++k) blob[k] = (uint8_t)rng();
    for (uint32_t n : {1u, 64u}) {
        char name[32];
        snprintf(name, sizeof name, "fused_%u", n);
        timeit(name, [&] {
            if (hdx_hash_batch_regions_device(types, A, dblob, dbase, dlen, n, tables, 3, dids, dcoords, nullptr,
                                              (hdx_stream)s) != HDX_OK)
                exit(3);
            CK(hipStreamSynchronize(s));
        });
    }
    timeit("fused_1_flag", [&] {
        if (hdx_hash_batch_regions_device(types, A, dblob, dbase, dlen, 1, tables, 3, dids, dcoords, nullptr,
                                          (hdx_stream)s) != HDX_OK)
            exit(3);
        CK(hipStreamWriteValue32(s, dflag, ++seq, 0));
        while (*flag != seq) __builtin_ia32_pause();
    });
    CK(hipStreamSynchronize(s));
    for (auto t : tables) hdx_region_table_destroy(t);
    return 0;
}
