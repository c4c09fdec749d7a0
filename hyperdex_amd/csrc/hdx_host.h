// hdx_host.h — host-side helpers shared by the C-ABI translation units
// (argument checking, error text, device binding, staging growth).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <vector>

#include "hdx_internal.h"

namespace hdx {

hdx_status hip_fail(hipError_t e, const char* what);

#define HIP_TRY(expr)                                     \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

// Validates a schema and fills codes_out[A] (may be NULL).
hdx_status check_schema(const uint32_t* types, uint32_t A, uint8_t* codes_out);
// Device scratch owned by the library (per-thread staging and streams),
// registered so hdx_shutdown can free every thread's (track_scratch /
// untrack_scratch; release() must leave the object reusable).
struct Scratch {
    virtual void release() = 0;
    virtual ~Scratch() = default;
};
void track_scratch(Scratch* s);
void untrack_scratch(Scratch* s);
// Binds the calling thread to `want` (-1: its current device) after checking it is gfx950.
hdx_status bind_device(int want);
// Frees the calling thread's library scratch now (streams, staging) and
// unregisters it: a thread the library owns calls it as its last job, so no
// HIP call runs in its thread-local destructors at exit (rocprofv3, among
// others, has torn down its per-thread state by then).
void release_thread_scratch();
// The calling thread's library stream (created on first use).
hdx_status thread_stream(hipStream_t* out);
// The single-device host-resident pipeline (hdx_capi.cpp) on the calling
// thread's device: codes validated, n > 0.
hdx_status hash_host(const uint8_t* codes, uint32_t A, const uint8_t* blob, uint64_t blob_bytes,
                     const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords);
// The device set of hdx_init_mask (hdx_multi.cpp): create (replacing a set
// of another mask), tear down (joins its workers), and the host-resident
// batch split over it.
hdx_status device_set_create(uint64_t mask, const std::vector<int>& devs);
void device_set_teardown();
bool host_batch_uses_set();
hdx_status hash_host_set(const uint8_t* codes, uint32_t A, const uint8_t* blob, uint64_t blob_bytes,
                         const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords);

template <typename T>
inline hdx_status grow_dev(T** p, size_t* cap, size_t need) {
    if (need <= *cap) return HDX_OK;
    size_t n = std::max(need, *cap * 3 / 2);
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipMalloc((void**)p, n * sizeof(T)) != hipSuccess) {
        (void)hipGetLastError();
        return fail(HDX_E_NOMEM, "hipMalloc(%zu) failed", n * sizeof(T));
    }
    *cap = n;
    return HDX_OK;
}

template <typename T>
inline hdx_status grow_pinned(T** p, size_t* cap, size_t need) {
    if (need <= *cap) return HDX_OK;
    size_t n = std::max(need, *cap * 3 / 2);
    (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipHostMalloc((void**)p, n * sizeof(T), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return fail(HDX_E_NOMEM, "hipHostMalloc(%zu) failed", n * sizeof(T));
    }
    *cap = n;
    return HDX_OK;
}

}  // namespace hdx

// Device copy of one subspace's region table (include/hdxhash.h).
struct hdx_region_table_s {
    int device;
    uint32_t D, R;
    uint16_t attrs[16];
    uint64_t* d_lower;
    uint64_t* d_upper;
    uint64_t* d_ids;
    uint64_t* d_index;  // interval index (NULL: lookups scan the boxes)
    uint32_t W, index_words;
    // host copies (the batcher's calling-thread lookups)
    std::vector<uint64_t> h_lower, h_upper, h_ids, h_index;
};

// configuration::lookup_region (common/configuration.cc:698-735) on the host
// (hdx_region_index.h): through the table's interval index when it has one,
// else the reference's scan.
inline uint64_t region_lookup_host(const hdx_region_table_s* t, const uint64_t* hs) {
    return hdx::region_lookup_arrays(t->D, t->R, t->W, t->attrs, t->h_lower.data(), t->h_upper.data(), t->h_ids.data(),
                                     t->h_index.empty() ? nullptr : t->h_index.data(), hs);
}

