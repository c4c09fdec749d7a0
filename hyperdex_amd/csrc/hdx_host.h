// hdx_host.h — host-side helpers shared by the C-ABI translation units
// (argument checking, error text, device binding, staging growth).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <functional>
#include <mutex>
#include <vector>

#include "hdx_internal.h"

namespace hdx {

hdx_status hip_fail(hipError_t e, const char* what);

#define HIP_TRY(expr)                                     \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

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

// Validates a schema and fills codes_out[A] (may be NULL).
hdx_status check_schema(const uint32_t* types, uint32_t A, uint8_t* codes_out);
// The kernels' code table from codes[0..A): the kernarg copy, and for wide
// schemas (the wide kernels, hdx_wide.hip) a device copy on the calling
// thread's current device.
hdx_status set_codes(BatchArgs& args, const uint8_t* codes, uint32_t A);
hdx_status set_codes(EncodedArgs& a, const uint8_t* codes, uint32_t A);
// Region tables of a call: at most kMaxSweepTables, none NULL, every
// subspace attribute < A; region_ids non-NULL when there are tables.
hdx_status check_tables(const hdx_region_table* tables, uint32_t ntables, uint32_t A, const uint64_t* region_ids);
// the table list alone (count, NULLs, subspace attributes < A): no output pointer
hdx_status check_table_list(const hdx_region_table* tables, uint32_t ntables, uint32_t A);
// A packed batch's kernel arguments on device `dev` (the calling thread's
// current device): codes, arrays, and T tables whose ids go to ids + t *
// ids_stride.
hdx_status batch_args(BatchArgs& args, const uint8_t* codes, uint32_t A, const uint8_t* blob,
                      const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords,
                      uint32_t* status, const hdx_region_table* tables, uint32_t T, uint64_t* ids,
                      uint64_t ids_stride, int dev);
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
// Hands the frees of an exiting thread's scratch to the library: a
// thread-local destructor makes no HIP call itself (the runtime or a
// profiler's per-thread state may be gone at thread exit); hdx_shutdown or
// the next thread binding a device runs them.
void park_orphan(std::function<void()> free_fn);
// The calling thread's library stream (created on first use).
hdx_status thread_stream(hipStream_t* out);
// The device the calling thread is bound to (-1: none yet).
int thread_device();
// True for page-locked host memory (hipHostMalloc / registered).
bool is_pinned(const void* p);

// One of a thread's two host-pipeline slots (hdx_hostpath.cpp): a stream,
// device staging and pinned staging, grown on demand, freed with the thread's
// scratch (hdx_capi.cpp).
template <typename T>
struct DevBuf {  // hipMalloc'd
    T* p = nullptr;
    size_t cap = 0;
    hdx_status need(size_t n) { return grow_dev(&p, &cap, n); }
};
template <typename T>
struct PinBuf {  // hipHostMalloc'd
    T* p = nullptr;
    size_t cap = 0;
    hdx_status need(size_t n) { return grow_pinned(&p, &cap, n); }
};
struct HostSlot {
    hipStream_t s = nullptr;
    DevBuf<uint8_t> d_blob, d_keys;       // packed blob or stored values (records: keys too); keys
    DevBuf<uint64_t> d_base, d_coords, d_ids, d_koff, d_voff, d_ver;
    DevBuf<uint32_t> d_len, d_klen, d_vlen, d_status;
    PinBuf<uint8_t> h_blob, h_keys;       // only for pageable inputs
    PinBuf<uint64_t> h_base, h_coords, h_ids, h_koff, h_voff, h_ver;
    PinBuf<uint32_t> h_len, h_klen, h_vlen, h_status;
    // packed chunks (objects out of address order): the extents' source
    // offsets and lengths for the gather kernel (hdx_gather.hip)
    DevBuf<uint64_t> d_src, d_src2;
    DevBuf<uint32_t> d_sz, d_sz2;
    PinBuf<uint64_t> h_src, h_src2;
    PinBuf<uint32_t> h_sz, h_sz2;
};
// The device view of pinned host memory p (for a kernel to read it), or NULL
// when p is not pinned.
const uint8_t* device_view(const uint8_t* p);
// Waits for the slot's stream, frees everything, destroys the stream (on the
// current device, which must be the slot's).
void free_host_slot(HostSlot& s);
// The calling thread's two slots (binds the thread; streams created).
hdx_status thread_slots(HostSlot** out);

// Region outputs of a host-resident call: table t's id of the call's object
// i goes to ids[t * stride + i].
struct HostRegions {
    const hdx_region_table* tables;
    uint32_t T;
    uint64_t* ids;
    uint64_t stride;
};

// The single-device host-resident pipelines (hdx_hostpath.cpp) on the calling
// thread's device; codes validated, n > 0.  coords may be NULL when R has
// tables; R may be NULL.
hdx_status hash_host(const uint8_t* codes, uint32_t A, const uint8_t* blob, uint64_t blob_bytes,
                     const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords,
                     const HostRegions* R);
// Stored objects: *status_bits receives the OR of the device status words
// (1 << HDX_E_BADENC, 1 << HDX_E_BADSIZE); versions may be NULL.
hdx_status hash_encoded_host(const uint8_t* codes, uint32_t A, const uint8_t* keys, uint64_t keys_bytes,
                             const uint64_t* key_off, const uint32_t* key_len, const uint8_t* vals,
                             uint64_t vals_bytes, const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                             uint64_t* coords, uint64_t* versions, const HostRegions* R, uint32_t* status_bits);

// The device set of hdx_init_mask (hdx_multi.cpp): create (replacing a set
// of another mask), tear down (waits for calls in progress, joins its
// workers), and the host-resident calls split over it (the calling thread's
// device alone without a set).
hdx_status device_set_create(uint64_t mask, const std::vector<int>& devs);
void device_set_teardown();
hdx_status hash_host_any(const uint8_t* codes, uint32_t A, const uint8_t* blob, uint64_t blob_bytes,
                         const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords,
                         const HostRegions* R);
hdx_status hash_encoded_host_any(const uint8_t* codes, uint32_t A, const uint8_t* keys, uint64_t keys_bytes,
                                 const uint64_t* key_off, const uint32_t* key_len, const uint8_t* vals,
                                 uint64_t vals_bytes, const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                                 uint64_t* coords, uint64_t* versions, const HostRegions* R);

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
    // host copies (the batcher's calling-thread lookups, the replicas below)
    std::vector<uint64_t> h_lower, h_upper, h_ids, h_index;
    // copies on the other devices a call has used the table on (the device
    // set's entry points), made on first use and freed with the table
    struct Replica {
        int device;
        uint64_t *lower, *upper, *ids, *index;
    };
    std::mutex rep_mu;
    std::vector<Replica> replicas;
};

namespace hdx {
// Table t's fields for a launch on the calling thread's current device
// (`dev`), its id output at `out`: the table's own device arrays on the device
// it was created on, else a replica there (uploaded on first use).
hdx_status fill_sweep_table(SweepTable& st, hdx_region_table_s* t, int dev, uint64_t* out);
}  // namespace hdx

// configuration::lookup_region (common/configuration.cc:698-735) on the host
// (hdx_region_index.h): through the table's interval index when it has one,
// else the reference's scan.
inline uint64_t region_lookup_host(const hdx_region_table_s* t, const uint64_t* hs) {
    return hdx::region_lookup_arrays(t->D, t->R, t->W, t->attrs, t->h_lower.data(), t->h_upper.data(), t->h_ids.data(),
                                     t->h_index.empty() ? nullptr : t->h_index.data(), hs);
}

