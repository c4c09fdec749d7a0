// hdx_capi.cpp — C-ABI of libhdxhash.so (include/hdxhash.h).
//
// Host side of the engine: argument validation, the hyperdatatype -> dispatch
// code table, per-thread streams and the pipelined host-resident batch path.
// Every batch entry point runs the gfx950 kernels, with no CPU substitute; the
// per-object entry points that mirror common/hash.h are hdx_cpu.cpp's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "hdx_host.h"
#include "../../include/hdxhash_debug.h"

#ifndef HDX_DEBUG_BUILD
#define HDX_DEBUG_BUILD 0
#endif


namespace hdx {

// ---- errors -------------------------------------------------------------

static thread_local std::string t_err;

hdx_status fail(hdx_status s, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return s;
}

hdx_status hip_fail(hipError_t e, const char* what) {
    return fail(e == hipErrorOutOfMemory ? HDX_E_NOMEM : HDX_E_DEVICE, "%s: %s", what, hipGetErrorString(e));
}


// ---- types (include/hyperdex.h:53-102; datatype_info.cc:72-141) ----------

hdx_status check_schema(const uint32_t* types, uint32_t A, uint8_t* codes_out) {
    if (!types) return fail(HDX_E_INVALID, "types is NULL");
    if (A == 0 || A > HDX_MAX_ATTRS)
        return fail(HDX_E_INVALID, "attrs_sz=%u outside [1, %d]", A, HDX_MAX_ATTRS);
    for (uint32_t j = 0; j < A; ++j) {
        const int c = type_code(types[j]);
        if (c < 0) return fail(HDX_E_BADTYPE, "attribute %u: unknown hyperdatatype %u", j, types[j]);
        if (codes_out) codes_out[j] = (uint8_t)c;
    }
    return HDX_OK;
}

// Attribute classes in device memory for the wide kernels (packed A > 256,
// stored A > 128, hdx_wide.hip): one copy per (device, schema), cached until
// hdx_shutdown (free_device_codes, after a device synchronisation, so no
// launch still reads one).  On the calling thread's current device.
static std::mutex g_codes_mu;
static std::map<std::pair<int, std::string>, uint8_t*>* g_codes = new std::map<std::pair<int, std::string>, uint8_t*>();

static hdx_status device_codes(const uint8_t* codes, uint32_t A, const uint8_t** out) {
    std::map<std::pair<int, std::string>, uint8_t*>* cache = g_codes;
    int dev = -1;
    HIP_TRY(hipGetDevice(&dev));
    std::pair<int, std::string> key(dev, std::string((const char*)codes, A));
    std::lock_guard<std::mutex> lk(g_codes_mu);
    auto it = cache->find(key);
    if (it != cache->end()) {
        *out = it->second;
        return HDX_OK;
    }
    uint8_t* d = nullptr;
    if (hipMalloc((void**)&d, A) != hipSuccess) {
        (void)hipGetLastError();
        return fail(HDX_E_NOMEM, "hipMalloc(%u) for the attribute classes", A);
    }
    HIP_TRY(hipMemcpy(d, codes, A, hipMemcpyHostToDevice));
    (*cache)[key] = d;
    *out = d;
    return HDX_OK;
}

static void free_device_codes() {
    std::lock_guard<std::mutex> lk(g_codes_mu);
    for (auto& kv : *g_codes) {
        if (hipSetDevice(kv.first.first) == hipSuccess && hipDeviceSynchronize() == hipSuccess) (void)hipFree(kv.second);
        (void)hipGetLastError();
    }
    g_codes->clear();
}

// (debug library: variants 300 / 301 force the wide kernels at any A)
hdx_status set_codes(BatchArgs& args, const uint8_t* codes, uint32_t A) {
    std::memcpy(args.codes, codes, std::min(A, kKernargCodes));
    args.codes_dev = nullptr;
    // only hash_wide_kernel (A > kKernargCodes) reads the device copy
    return A > kKernargCodes || hash_variant() == 300 ? device_codes(codes, A, &args.codes_dev) : HDX_OK;
}

hdx_status set_codes(EncodedArgs& a, const uint8_t* codes, uint32_t A) {
    std::memcpy(a.codes, codes, std::min(A, kKernargCodes));
    a.codes_dev = nullptr;
    return A > kWsweepMaxAttrs || hash_variant() == 301 ? device_codes(codes, A, &a.codes_dev) : HDX_OK;
}

// ---- device binding -------------------------------------------------------

static std::once_flag g_probe_once;
static int g_ndev = -1;
static std::vector<int> g_is_gfx950;

static void probe() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    g_ndev = n;
    g_is_gfx950.assign(n, 0);
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, d) == hipSuccess)
            g_is_gfx950[d] = std::strncmp(p.gcnArchName, "gfx950", 6) == 0;
    }
}

// Per-thread device scratch (streams, host-path staging) and the search
// staging of hdx_capi_index.cpp register here, so hdx_shutdown can free every
// thread's scratch, not only the caller's.
static std::mutex g_scratch_mu;
static std::vector<Scratch*> g_scratch;

void track_scratch(Scratch* s) {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    g_scratch.push_back(s);
}
void untrack_scratch(Scratch* s) {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    g_scratch.erase(std::remove(g_scratch.begin(), g_scratch.end(), s), g_scratch.end());
}

// Scratch of threads that exited.  A thread-local destructor makes no HIP
// call: at thread (or process) exit the runtime, or a profiler's per-thread
// state (rocprofv3), may already be gone, and a HIP call there aborted the
// process (round 4).  The destructor parks the frees here instead; the next
// hdx_shutdown, or the next thread that binds a device, runs them.  Whatever
// is still parked when the process exits is released with the process.
// Leaked on purpose: thread-local destructors may run after static ones.
struct Orphans {
    std::mutex mu;
    std::vector<std::function<void()>> frees;
    std::atomic<size_t> count{0};
};
static Orphans& orphans() {
    static Orphans* o = new Orphans();
    return *o;
}

void park_orphan(std::function<void()> free_fn) {
    Orphans& o = orphans();
    std::lock_guard<std::mutex> lk(o.mu);
    o.frees.push_back(std::move(free_fn));
    o.count.store(o.frees.size(), std::memory_order_release);
}

// Runs the parked frees on the calling thread; restores its HIP device.
static void reap_orphans() {
    Orphans& o = orphans();
    if (o.count.load(std::memory_order_acquire) == 0) return;
    std::vector<std::function<void()>> todo;
    {
        std::lock_guard<std::mutex> lk(o.mu);
        todo.swap(o.frees);
        o.count.store(0, std::memory_order_release);
    }
    int dev = -1;
    const bool had = hipGetDevice(&dev) == hipSuccess;
    for (auto& f : todo) f();
    if (had && dev >= 0) (void)hipSetDevice(dev);
    (void)hipGetLastError();
}

struct ThreadState : Scratch {
    int device = -1;
    bool tracked = false;
    hipStream_t stream = nullptr;
    HostSlot slot[2];  // the host-resident pipelines (hdx_hostpath.cpp)
    // The frees of everything held, as one job (empty when nothing is held);
    // leaves the state unbound (the thread rebinds lazily on its next call).
    std::function<void()> detach() {
        if (device < 0) return {};
        const int dev = device;
        HostSlot held[2] = {slot[0], slot[1]};
        hipStream_t st = stream;
        for (auto& s : slot) s = HostSlot{};
        stream = nullptr;
        device = -1;
        return [dev, held, st]() mutable {
            (void)hipSetDevice(dev);
            for (auto& s : held) free_host_slot(s);
            if (st) {
                (void)hipStreamSynchronize(st);
                (void)hipStreamDestroy(st);
            }
        };
    }
    void release() override {
        if (auto f = detach()) f();
    }
    ~ThreadState() {  // no HIP call here: park the frees (reap_orphans)
        if (tracked) untrack_scratch(this);
        if (auto f = detach()) park_orphan(std::move(f));
    }
};
static thread_local ThreadState t_state;

hdx_status bind_device(int want /* -1: current */) {
    std::call_once(g_probe_once, probe);
    if (g_ndev <= 0) return fail(HDX_E_DEVICE, "no HIP device visible (this library has no CPU path)");
    int dev = want;
    if (dev < 0) {
        if (t_state.device >= 0) return HDX_OK;
        HIP_TRY(hipGetDevice(&dev));
    }
    if (dev >= g_ndev) return fail(HDX_E_INVALID, "device %d >= device count %d", dev, g_ndev);
    if (!g_is_gfx950[dev]) return fail(HDX_E_DEVICE, "device %d is not gfx950 (MI355X)", dev);
    HIP_TRY(hipSetDevice(dev));
    if (t_state.device != dev) {
        if (t_state.device >= 0)
            return fail(HDX_E_INVALID, "thread already bound to device %d", t_state.device);
        reap_orphans();  // exited threads' scratch (restores the current device)
        t_state.device = dev;
        if (!t_state.tracked) {
            track_scratch(&t_state);
            t_state.tracked = true;
        }
    }
    return HDX_OK;
}

void release_thread_scratch() {
    t_state.release();
    if (t_state.tracked) {
        untrack_scratch(&t_state);
        t_state.tracked = false;
    }
}

hdx_status thread_stream(hipStream_t* out) {
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    if (!t_state.stream) HIP_TRY(hipStreamCreateWithFlags(&t_state.stream, hipStreamNonBlocking));
    *out = t_state.stream;
    return HDX_OK;
}

int thread_device() { return t_state.device; }

hdx_status thread_slots(HostSlot** out) {
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    for (auto& s : t_state.slot)
        if (!s.s) HIP_TRY(hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking));
    *out = t_state.slot;
    return HDX_OK;
}

bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

}  // namespace hdx

using namespace hdx;

// ---- exported C-ABI --------------------------------------------------------

HDX_EXPORT int hdx_abi_version(void) { return HDX_ABI_VERSION; }

HDX_EXPORT const char* hdx_version(void) {
    return "hdxhash " "1.0" " (gfx950; CityHash64 v1.1 / ordered encodings / timestamp)";
}

HDX_EXPORT const char* hdx_last_error(void) { return t_err.c_str(); }

HDX_EXPORT int hdx_device_count(void) {
    std::call_once(g_probe_once, probe);
    return g_ndev < 0 ? 0 : g_ndev;
}

HDX_EXPORT hdx_status hdx_init(int device) {
    if (device < 0) return fail(HDX_E_INVALID, "device %d", device);
    return bind_device(device);
}

HDX_EXPORT hdx_status hdx_init_mask(uint64_t device_mask) {
    std::call_once(g_probe_once, probe);
    if (device_mask == 0) return fail(HDX_E_INVALID, "empty device mask");
    if (g_ndev <= 0) return fail(HDX_E_DEVICE, "no HIP device visible");
    std::vector<int> devs;
    for (int d = 0; d < 64; ++d) {
        if (!(device_mask >> d & 1)) continue;
        if (d >= g_ndev) return fail(HDX_E_INVALID, "device %d in the mask >= device count %d", d, g_ndev);
        if (!g_is_gfx950[d]) return fail(HDX_E_DEVICE, "device %d is not gfx950 (MI355X)", d);
        devs.push_back(d);
    }
    hdx_status st = bind_device(devs[0]);
    if (st != HDX_OK) return st;
    hipStream_t s;
    if ((st = thread_stream(&s)) != HDX_OK) return st;
    // one worker, stream set and staging per device (hdx_multi.cpp)
    return device_set_create(device_mask, devs);
}

HDX_EXPORT hdx_status hdx_shutdown(void) {
    // the device set's workers exit first (their scratch is released as they
    // do); then each remaining release() binds its scratch's device and the
    // caller's current device is restored, so its lazy rebind returns to it
    device_set_teardown();
    reap_orphans();
    int dev = -1;
    const bool had = hipGetDevice(&dev) == hipSuccess;
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        for (Scratch* s : g_scratch) s->release();
    }
    trim_region_pools();
    free_device_codes();
    if (had && dev >= 0) (void)hipSetDevice(dev);
    (void)hipGetLastError();
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_sync(hdx_stream stream) {
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(hipStreamSynchronize(s));
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_schema_check(const uint32_t* types, uint32_t attrs_sz) {
    return check_schema(types, attrs_sz, nullptr);
}

HDX_EXPORT int hdx_type_hashable(uint32_t type) { return type_code(type) > 0 ? 1 : 0; }

HDX_EXPORT hdx_status hdx_hash_batch_device(const uint32_t* types, uint32_t attrs_sz,
                                            const uint8_t* blob, const uint64_t* obj_base,
                                            const uint32_t* attr_len, uint64_t n,
                                            uint64_t* coords, uint32_t* status_dev,
                                            hdx_stream stream) {
    BatchArgs args{};
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    hdx_status st = check_schema(types, attrs_sz, codes.data());
    if (st != HDX_OK) return st;
    if (n == 0) return HDX_OK;
    if (!blob || !obj_base || !attr_len || !coords)
        return fail(HDX_E_INVALID, "NULL device pointer");
    if ((st = bind_device(-1)) != HDX_OK) return st;
    if ((st = set_codes(args, codes.data(), attrs_sz)) != HDX_OK) return st;
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream
    args.blob = blob;
    args.obj_base = obj_base;
    args.attr_len = attr_len;
    args.coords = coords;
    args.status = status_dev;
    args.n = n;
    args.A = attrs_sz;
    finalize_args(args);
    HIP_TRY(launch_hash_batch(args, s));
    return HDX_OK;
}

namespace hdx {
hdx_status fill_sweep_table(SweepTable& st, hdx_region_table_s* t, int dev, uint64_t* out) {
    st = SweepTable{};
    st.lower = t->d_lower;
    st.upper = t->d_upper;
    st.ids = t->d_ids;
    st.index = t->d_index;
    if (dev != t->device) {
        std::lock_guard<std::mutex> lk(t->rep_mu);
        const hdx_region_table_s::Replica* r = nullptr;
        for (const auto& x : t->replicas)
            if (x.device == dev) r = &x;
        if (!r) {
            hdx_region_table_s::Replica c{dev, nullptr, nullptr, nullptr, nullptr};
            const size_t box = t->h_lower.size() * 8;
            auto up = [](uint64_t** d, const std::vector<uint64_t>& h, size_t extra) {
                if (hipMalloc((void**)d, h.size() * 8 + extra) != hipSuccess) return false;
                return h.empty() || hipMemcpy(*d, h.data(), h.size() * 8, hipMemcpyHostToDevice) == hipSuccess;
            };
            const bool ok = up(&c.lower, t->h_lower, 8) && up(&c.upper, t->h_upper, 8) && up(&c.ids, t->h_ids, 8) &&
                            (t->h_index.empty() || !t->d_index || up(&c.index, t->h_index, 0));
            (void)box;
            if (!ok) {
                (void)hipGetLastError();
                (void)hipFree(c.lower); (void)hipFree(c.upper); (void)hipFree(c.ids); (void)hipFree(c.index);
                return fail(HDX_E_NOMEM, "region table replica on device %d", dev);
            }
            t->replicas.push_back(c);
            r = &t->replicas.back();
        }
        st.lower = r->lower;
        st.upper = r->upper;
        st.ids = r->ids;
        st.index = r->index;
    }
    st.out = out;
    st.W = t->W;
    st.D = t->D;
    st.R = t->R;
    st.index_words = t->index_words;
    std::memcpy(st.attrs, t->attrs, sizeof st.attrs);
    return HDX_OK;
}
}  // namespace hdx

static hdx_status hash_encoded(const uint32_t* types, uint32_t attrs_sz, const uint8_t* keys,
                               const uint64_t* key_off, const uint32_t* key_len, const uint8_t* vals,
                               const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                               const hdx_region_table* tables, uint32_t ntables, uint64_t* region_ids,
                               uint64_t* coords, uint64_t* versions, uint32_t* status_dev, hdx_stream stream) {
    EncodedArgs a{};
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    hdx_status st = check_schema(types, attrs_sz, codes.data());
    if (st != HDX_OK) return st;
    if ((st = check_tables(tables, ntables, attrs_sz, region_ids)) != HDX_OK) return st;
    if (n == 0) return HDX_OK;
    if (!keys || !key_off || !key_len || !vals || !val_off || !val_len || (!coords && !ntables))
        return fail(HDX_E_INVALID, "NULL device pointer");
    if ((st = bind_device(-1)) != HDX_OK) return st;
    if ((st = set_codes(a, codes.data(), attrs_sz)) != HDX_OK) return st;
    a.T = ntables;
    for (uint32_t t = 0; t < ntables; ++t)
        if ((st = fill_sweep_table(a.t[t], tables[t], t_state.device, region_ids + (size_t)t * n)) != HDX_OK) return st;
    a.keys = keys;
    a.key_off = key_off;
    a.key_len = key_len;
    a.vals = vals;
    a.val_off = val_off;
    a.val_len = val_len;
    a.coords = coords;
    a.versions = versions;
    a.status = status_dev;
    a.n = n;
    a.A = attrs_sz;
    HIP_TRY(launch_hash_encoded(a, (hipStream_t)stream));
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_hash_encoded_device(const uint32_t* types, uint32_t attrs_sz,
                                              const uint8_t* keys, const uint64_t* key_off,
                                              const uint32_t* key_len, const uint8_t* vals,
                                              const uint64_t* val_off, const uint32_t* val_len,
                                              uint64_t n, uint64_t* coords, uint64_t* versions,
                                              uint32_t* status_dev, hdx_stream stream) {
    return hash_encoded(types, attrs_sz, keys, key_off, key_len, vals, val_off, val_len, n, nullptr, 0, nullptr,
                        coords, versions, status_dev, stream);
}

HDX_EXPORT hdx_status hdx_hash_encoded_regions_device(const uint32_t* types, uint32_t attrs_sz,
                                                      const uint8_t* keys, const uint64_t* key_off,
                                                      const uint32_t* key_len, const uint8_t* vals,
                                                      const uint64_t* val_off, const uint32_t* val_len,
                                                      uint64_t n, const hdx_region_table* tables,
                                                      uint32_t ntables, uint64_t* region_ids, uint64_t* coords,
                                                      uint64_t* versions, uint32_t* status_dev,
                                                      hdx_stream stream) {
    if (ntables == 0) return fail(HDX_E_INVALID, "no region tables");
    return hash_encoded(types, attrs_sz, keys, key_off, key_len, vals, val_off, val_len, n, tables, ntables,
                        region_ids, coords, versions, status_dev, stream);
}

namespace hdx {
hdx_status check_table_list(const hdx_region_table* tables, uint32_t ntables, uint32_t A) {
    if (ntables > kMaxSweepTables)
        return fail(HDX_E_INVALID, "%u region tables (at most %u)", ntables, kMaxSweepTables);
    if (ntables && !tables) return fail(HDX_E_INVALID, "NULL tables / region_ids");
    for (uint32_t t = 0; t < ntables; ++t) {
        if (!tables[t]) return fail(HDX_E_INVALID, "NULL table %u", t);
        for (uint32_t d = 0; d < tables[t]->D; ++d)
            if (tables[t]->attrs[d] >= A)
                return fail(HDX_E_INVALID, "table %u: subspace attribute %u >= attrs_sz %u", t, tables[t]->attrs[d], A);
    }
    return HDX_OK;
}

hdx_status check_tables(const hdx_region_table* tables, uint32_t ntables, uint32_t A, const uint64_t* region_ids) {
    if (ntables && !region_ids) return fail(HDX_E_INVALID, "NULL tables / region_ids");
    return check_table_list(tables, ntables, A);
}

hdx_status batch_args(BatchArgs& args, const uint8_t* codes, uint32_t A, const uint8_t* blob,
                      const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords,
                      uint32_t* status, const hdx_region_table* tables, uint32_t T, uint64_t* ids,
                      uint64_t ids_stride, int dev) {
    args = BatchArgs{};
    hdx_status st = set_codes(args, codes, A);
    if (st != HDX_OK) return st;
    args.blob = blob;
    args.obj_base = obj_base;
    args.attr_len = attr_len;
    args.coords = coords;
    args.status = status;
    args.n = n;
    args.A = A;
    finalize_args(args);
    args.T = T;
    for (uint32_t t = 0; t < T; ++t)
        if ((st = fill_sweep_table(args.t[t], tables[t], dev, ids + t * ids_stride)) != HDX_OK) return st;
    return HDX_OK;
}
}  // namespace hdx

HDX_EXPORT hdx_status hdx_hash_batch_regions_device(const uint32_t* types, uint32_t attrs_sz, const uint8_t* blob,
                                                    const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n,
                                                    const hdx_region_table* tables, uint32_t ntables,
                                                    uint64_t* region_ids, uint64_t* coords, uint32_t* status_dev,
                                                    hdx_stream stream) {
    if (ntables == 0) return fail(HDX_E_INVALID, "no region tables");
    if (n && !attr_len) return fail(HDX_E_INVALID, "NULL device pointer");
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    hdx_status st = check_schema(types, attrs_sz, codes.data());
    if (st != HDX_OK) return st;
    if ((st = check_tables(tables, ntables, attrs_sz, region_ids)) != HDX_OK) return st;
    if (n == 0) return HDX_OK;
    if (!blob || !obj_base) return fail(HDX_E_INVALID, "NULL device pointer");
    if ((st = bind_device(-1)) != HDX_OK) return st;
    BatchArgs args;
    if ((st = batch_args(args, codes.data(), attrs_sz, blob, obj_base, attr_len, n, coords, status_dev, tables,
                         ntables, region_ids, n, t_state.device)) != HDX_OK)
        return st;
    HIP_TRY(launch_hash_batch_regions(args, (hipStream_t)stream));
    return HDX_OK;
}


// hdx_hash_value / hdx_hash_key / hdx_hash_object: the per-object entry points
// run on the host CPU (hdx_cpu.cpp).

HDX_EXPORT hdx_status hdx_alloc_pinned(size_t bytes, void** out) {
    if (!out) return fail(HDX_E_INVALID, "out is NULL");
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    if (hipHostMalloc(out, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return fail(HDX_E_NOMEM, "hipHostMalloc(%zu) failed", bytes);
    }
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_free_pinned(void* p) {
    HIP_TRY(hipHostFree(p));
    return HDX_OK;
}

static hdx_status synth_args(const hdx_synth_rule* rules, uint32_t A, uint64_t seed, uint64_t first,
                             uint64_t n, SynthArgs* a) {
    if (!rules || A == 0 || A > 64) return fail(HDX_E_INVALID, "synth: 1 <= attrs_sz <= 64");
    *a = SynthArgs{};
    a->seed = seed;
    a->first = first;
    a->n = n;
    a->A = A;
    for (uint32_t j = 0; j < A; ++j) {
        if (type_code(rules[j].type) < 0) return fail(HDX_E_BADTYPE, "synth: type %u", rules[j].type);
        if (rules[j].kind > 2 || (rules[j].kind == 1 && rules[j].hi < rules[j].lo))
            return fail(HDX_E_INVALID, "synth: bad rule at %u", j);
        a->rules[j] = rules[j];
    }
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_synth_encode_values(const uint8_t* blob_dev, const uint64_t* obj_base_dev,
                                              const uint32_t* attr_len_dev, uint32_t attrs_sz, uint64_t n,
                                              uint64_t first_version, const uint64_t* val_off_dev,
                                              uint8_t* vals_dev, hdx_stream stream) {
    if (attrs_sz == 0 || attrs_sz > 65535) return fail(HDX_E_INVALID, "attrs_sz=%u", attrs_sz);
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    HIP_TRY(launch_synth_encode(blob_dev, obj_base_dev, attr_len_dev, attrs_sz, n, first_version,
                                val_off_dev, vals_dev, (hipStream_t)stream));
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_synth_encode_store(const uint8_t* blob_dev, const uint64_t* obj_base_dev,
                                             const uint32_t* attr_len_dev, uint32_t attrs_sz, uint64_t n,
                                             uint64_t first_version, const uint64_t* val_off_dev, uint8_t* vals_dev,
                                             const uint64_t* key_off_dev, uint8_t* keys_dev, hdx_stream stream) {
    if (attrs_sz == 0 || attrs_sz > 65535) return fail(HDX_E_INVALID, "attrs_sz=%u", attrs_sz);
    if (n && (!key_off_dev || !keys_dev)) return fail(HDX_E_INVALID, "NULL key column");
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    HIP_TRY(launch_synth_encode(blob_dev, obj_base_dev, attr_len_dev, attrs_sz, n, first_version, val_off_dev,
                                vals_dev, (hipStream_t)stream, key_off_dev, keys_dev));
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_synth_lengths(const hdx_synth_rule* rules, uint32_t attrs_sz, uint64_t seed,
                                        uint64_t first, uint64_t n, uint32_t* attr_len_dev,
                                        hdx_stream stream) {
    SynthArgs a;
    hdx_status st = synth_args(rules, attrs_sz, seed, first, n, &a);
    if (st != HDX_OK) return st;
    if ((st = bind_device(-1)) != HDX_OK) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(launch_synth_lengths(a, attr_len_dev, s));
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_synth_fill(const hdx_synth_rule* rules, uint32_t attrs_sz, uint64_t seed,
                                     uint64_t first, uint64_t n, const uint64_t* obj_base_dev,
                                     const uint32_t* attr_len_dev, uint8_t* blob_dev, uint64_t bytes,
                                     hdx_stream stream) {
    SynthArgs a;
    hdx_status st = synth_args(rules, attrs_sz, seed, first, n, &a);
    if (st != HDX_OK) return st;
    if ((st = bind_device(-1)) != HDX_OK) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(launch_synth_fill(a, obj_base_dev, attr_len_dev, blob_dev, bytes, s));
    return HDX_OK;
}

// ---- region tables (hdx_regions.hip) ----------------------------------------

// Debug library only: HDX_REGION_SCAN=1 (A/B runs) — tables created afterwards
// keep no interval index, so lookups scan the boxes as the reference does.
static bool region_index_disabled() {
#if HDX_DEBUG_BUILD
    const char* e = getenv("HDX_REGION_SCAN");
    return e && *e == '1';
#else
    return false;
#endif
}


HDX_EXPORT hdx_status hdx_region_table_create(uint32_t dims, uint32_t regions, const uint16_t* attrs,
                                              const uint64_t* lower, const uint64_t* upper,
                                              const uint64_t* ids, hdx_region_table* out) {
    if (!out || !attrs || (regions && (!lower || !upper || !ids)))
        return fail(HDX_E_INVALID, "NULL pointer");
    if (dims == 0 || dims > 16) return fail(HDX_E_INVALID, "dims=%u outside [1, 16]", dims);
    *out = nullptr;
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    hdx_region_table t = new hdx_region_table_s();
    t->device = t_state.device;
    t->D = dims;
    t->R = regions;
    std::memcpy(t->attrs, attrs, dims * sizeof(uint16_t));
    t->h_lower.assign(lower, lower + (size_t)regions * dims);
    t->h_upper.assign(upper, upper + (size_t)regions * dims);
    t->h_ids.assign(ids, ids + regions);
    const size_t box = (size_t)regions * dims * 8;
    if (hipMalloc((void**)&t->d_lower, box + 8) != hipSuccess ||
        hipMalloc((void**)&t->d_upper, box + 8) != hipSuccess ||
        hipMalloc((void**)&t->d_ids, (size_t)regions * 8 + 8) != hipSuccess) {
        (void)hipGetLastError();
        hdx_region_table_destroy(t);
        return fail(HDX_E_NOMEM, "region table of %u regions", regions);
    }
    if (regions &&
        (hipMemcpy(t->d_lower, lower, box, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(t->d_upper, upper, box, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(t->d_ids, ids, (size_t)regions * 8, hipMemcpyHostToDevice) != hipSuccess)) {
        hdx_region_table_destroy(t);
        return fail(HDX_E_DEVICE, "region table upload failed");
    }
    // the interval index (hdx_regions.hip) for tables of up to 256 regions
    std::vector<uint64_t> index;
    region_index_build(dims, regions, lower, upper, index, t->W);
    if (!index.empty() && !region_index_disabled()) {
        t->h_index = index;
        t->index_words = (uint32_t)index.size();
        if (hipMalloc((void**)&t->d_index, index.size() * 8) != hipSuccess ||
            hipMemcpy(t->d_index, index.data(), index.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipGetLastError();
            hdx_region_table_destroy(t);
            return fail(HDX_E_DEVICE, "region index upload failed");
        }
    }
    *out = t;
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_region_table_destroy(hdx_region_table t) {
    if (!t) return HDX_OK;
    (void)hipFree(t->d_lower);
    (void)hipFree(t->d_upper);
    (void)hipFree(t->d_ids);
    (void)hipFree(t->d_index);
    for (const auto& r : t->replicas) {
        (void)hipFree(r.lower);
        (void)hipFree(r.upper);
        (void)hipFree(r.ids);
        (void)hipFree(r.index);
    }
    delete t;
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_lookup_region_device(hdx_region_table t, const uint64_t* coords,
                                               uint32_t attrs_sz, uint64_t n, uint64_t* region_ids,
                                               hdx_stream stream) {
    if (!t) return fail(HDX_E_INVALID, "NULL table");
    if (n == 0) return HDX_OK;
    if (!coords || !region_ids) return fail(HDX_E_INVALID, "NULL device pointer");
    for (uint32_t d = 0; d < t->D; ++d)
        if (t->attrs[d] >= attrs_sz)
            return fail(HDX_E_INVALID, "subspace attribute %u >= attrs_sz %u", t->attrs[d], attrs_sz);
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    SweepTable tb;
    if ((st = fill_sweep_table(tb, t, t_state.device, region_ids)) != HDX_OK) return st;
    RegionArgs a{};
    a.lower = tb.lower;
    a.upper = tb.upper;
    a.ids = tb.ids;
    a.index = tb.index;
    a.W = t->W;
    a.index_words = t->index_words;
    a.coords = coords;
    a.out = region_ids;
    a.n = n;
    a.A = attrs_sz;
    a.D = t->D;
    a.R = t->R;
    std::memcpy(a.attrs, t->attrs, sizeof a.attrs);
    HIP_TRY(launch_lookup_region(a, (hipStream_t)stream));
    return HDX_OK;
}

// ---- tuning hooks (include/hdxhash_debug.h) --------------------------------

#if HDX_DEBUG_BUILD
HDX_EXPORT int hdxdbg_set_kernel_variant(int variant) { return set_hash_variant(variant); }
HDX_EXPORT int hdxdbg_kernel_variant(void) { return hash_variant(); }
#endif

HDX_EXPORT int hdxdbg_stream_probe(const void* src, uint64_t bytes, uint64_t* sink, int write, void* stream) {
    if (!src || (write && !sink) || write < 0 || write > 4 || bytes % 4096) return HDX_E_INVALID;
    HIP_TRY(launch_stream_probe((const uint8_t*)src, bytes, sink, write, (hipStream_t)stream));
    return HDX_OK;
}

HDX_EXPORT uint64_t hdxdbg_region_chunk_objects(uint64_t n, uint32_t attrs_sz) {
    return attrs_sz ? regions_chunk_objects(n, attrs_sz) : 0;
}

HDX_EXPORT int hdxdbg_kernel_for(const uint32_t* types, uint32_t attrs_sz, uint64_t n, const char** name) {
    BatchArgs a{};
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    if (check_schema(types, attrs_sz, codes.data()) != HDX_OK) return -2;
    std::memcpy(a.codes, codes.data(), std::min(attrs_sz, kKernargCodes));
    a.A = attrs_sz;
    a.n = n;
    finalize_args(a);
    const int v = chosen_variant(a);
    if (name) *name = variant_kernel_name(v);
    return v;
}
