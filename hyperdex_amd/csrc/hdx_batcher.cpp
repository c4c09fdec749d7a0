// hdx_batcher.cpp — the daemon batching shim (include/hdxhash.h).
//
// key_state::hash_objects (daemon/key_state.cc:1455-1543) is called per
// replicated op from every daemon::loop thread (daemon.cc:345-351) and hashes
// one or two whole objects, then looks them up in up to three subspaces
// (configuration::lookup_region, configuration.cc:698-735).  One object is far
// too little work for a launch, so callers meet here:
//
//   caller threads    reserve (object index, byte offset) in the FILLING slot
//                     under the lock, copy key + values into its pinned staging
//                     outside the lock, then sleep on the slot's generation;
//   flush thread      seals the FILLING slot as soon as no batch is in flight,
//                     when it is full, or max_delay after its first object;
//                     waits for the slot's writers to finish, then launches,
//                     on the slot's own stream, ONE kernel that hashes the
//                     batch and looks every object up in the space's tables
//                     (hash_regroup_regions_kernel, <= 4 tables; more tables:
//                     the hash kernel + one lookup kernel for all of them).
//                     By default the kernel reads the pinned staging and
//                     writes coordinates / region ids into pinned memory in
//                     place (no copies); HDX_BATCHER_STAGE_DEVICE stages
//                     through HBM (H2D, kernel, D2H) instead;
//   completion thread waits for each shipped slot's stream in order, publishes
//                     the status and wakes the slot's callers, who copy their
//                     rows out; the last reader frees the slot.
//
// By default no object reaches any of that: the calling thread hashes it with
// the per-object CPU path (hdx_cpu.cpp) and looks it up in host copies of the
// tables.  One core does a config-3b object in ~0.27 us with three lookups,
// a lone caller's device round trip costs ~36 us, and at no object size does
// the device win one synchronous object: CityHash is serial within a string,
// so a 1 MB object takes 42 us on a core and 2.9 ms as a one-object device
// batch.  host_max_bytes sends larger objects to the device;
// HDX_BATCHER_DEVICE_ONLY ships everything, for hosts whose cores are needed
// elsewhere (the device then does the work while the callers sleep).
//
// Shipping as soon as the pipeline is idle keeps a lone caller's latency at
// one round trip, while concurrent callers pile into the next batch during
// the current one (batch size adapts to load).  With `slots` >= 2 buffers in
// rotation, filling, transfer and kernels of consecutive batches overlap.
// Objects above max_bytes go through a private slot of their own size on the
// caller's thread.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "hdx_host.h"

using namespace hdx;
using Clock = std::chrono::steady_clock;

namespace {

enum SlotState { FREE, FILLING, SEALED, INFLIGHT, DONE };

struct Slot {
    // pinned staging + device twins
    uint8_t* h_blob = nullptr;
    uint64_t* h_base = nullptr;
    uint32_t* h_len = nullptr;
    uint64_t* h_out = nullptr;  // coords [max_obj*A] then regions [T][max_obj]
    uint32_t* h_status = nullptr;
    // device buffers (HDX_BATCHER_STAGE_DEVICE) or device views of the pinned ones
    uint8_t* d_blob = nullptr;
    uint64_t* d_base = nullptr;
    uint32_t* d_len = nullptr;
    uint64_t* d_out = nullptr;
    uint32_t* d_status = nullptr;
    bool owns_device = false;
    hipStream_t stream = nullptr;
    uint32_t cap_obj = 0;
    uint64_t cap_bytes = 0;
    // fill state, under the batcher's mutex (writers is also read by the flusher)
    SlotState st = FREE;
    uint32_t nobj = 0;
    uint64_t nbytes = 0;
    uint32_t writers = 0;
    uint64_t gen = 0;       // bumped each time the slot starts filling
    hdx_status result = HDX_OK;
    // completion, published without the batcher's mutex: callers spin briefly
    // on done_gen, then sleep on the slot's own condition variable, and copy
    // their rows out lock-free; the last reader frees the slot
    std::atomic<uint64_t> done_gen{0};  // == gen once the slot's batch has completed
    std::atomic<uint32_t> readers{0};
    std::mutex done_mu;
    std::condition_variable done_cv;
    Clock::time_point first;
    bool full = false;
};

}  // namespace

struct hdx_batcher_s {
    ~hdx_batcher_s() {
        if (codes_dev) {  // after hdx_batcher_destroy's slot frees, or a failed create
            (void)hipSetDevice(device);
            (void)hipFree((void*)codes_dev);
            (void)hipGetLastError();
        }
    }
    int device = -1;
    uint32_t A = 0;
    std::vector<uint8_t> codes;
    std::vector<uint32_t> types;
    const uint8_t* codes_dev = nullptr;  // A > 256: the wide kernel's classes, owned (freed with the batcher)
    uint64_t host_max_bytes = 0;  // 0 with HDX_BATCHER_DEVICE_ONLY
    uint32_t max_obj = 0;
    uint64_t max_bytes = 0;
    bool stage_device = false;
    std::chrono::microseconds delay{50};
    std::vector<hdx_region_table> tables;
    std::unique_ptr<Slot[]> slots;  // fixed at creation (Slot holds atomics and a mutex)
    uint32_t nslots = 0;
    Slot direct;  // oversized objects, under direct_mu
    std::mutex direct_mu;

    std::mutex mu;
    std::condition_variable cv_flush;  // flusher: new object, seal, last writer done, stop
    std::condition_variable cv_free;   // callers: a slot became FILLING
    std::condition_variable cv_ship;   // completer: a slot was shipped
    int cur = -1;                      // FILLING slot, or -1 when none is free
    std::deque<int> sealed, inflight;
    uint32_t pending = 0;              // sealed or shipped, not yet completed
    bool stop = false, flusher_done = false;
    std::thread flusher, completer;

    std::atomic<uint64_t> n_objects{0}, n_batches{0}, n_full{0}, n_direct{0};
    // calling-thread objects, counted per thread shard: one shared counter
    // bounced between 16 callers' cores cost more than the hash itself
    struct alignas(64) Shard {
        std::atomic<uint64_t> v{0};
    };
    Shard n_host[32];
    uint64_t host_total() const {
        uint64_t s = 0;
        for (const Shard& c : n_host) s += c.v.load(std::memory_order_relaxed);
        return s;
    }
    std::atomic<int> spinners{0};
};

static constexpr int kMaxSpinners = 2;

namespace {

size_t out_words(const hdx_batcher_s* b, uint32_t cap_obj) {
    return (size_t)cap_obj * b->A + (size_t)b->tables.size() * cap_obj;
}

void free_slot(Slot& s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    (void)hipHostFree(s.h_blob); (void)hipHostFree(s.h_base); (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_out); (void)hipHostFree(s.h_status);
    if (s.owns_device) {
        (void)hipFree(s.d_blob); (void)hipFree(s.d_base); (void)hipFree(s.d_len);
        (void)hipFree(s.d_out); (void)hipFree(s.d_status);
    }
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s.h_blob = nullptr; s.h_base = nullptr; s.h_len = nullptr; s.h_out = nullptr; s.h_status = nullptr;
    s.d_blob = nullptr; s.d_base = nullptr; s.d_len = nullptr; s.d_out = nullptr; s.d_status = nullptr;
    s.owns_device = false;
    s.stream = nullptr;
    s.cap_obj = 0;
    s.cap_bytes = 0;
}

template <typename T>
bool device_view(T* host, T** dev) {
    void* p = nullptr;
    if (hipHostGetDevicePointer(&p, host, 0) != hipSuccess) return false;
    *dev = static_cast<T*>(p);
    return true;
}

hdx_status alloc_slot(hdx_batcher_s* b, Slot& s, uint32_t cap_obj, uint64_t cap_bytes) {
    free_slot(s);
    const size_t words = out_words(b, cap_obj);
    const size_t blob = cap_bytes + 64;  // the kernel's aligned 16-byte reads may touch the tail
    const unsigned fl = hipHostMallocMapped;
    bool ok = hipHostMalloc((void**)&s.h_blob, blob, fl) == hipSuccess &&
              hipHostMalloc((void**)&s.h_base, (size_t)cap_obj * 8, fl) == hipSuccess &&
              hipHostMalloc((void**)&s.h_len, (size_t)cap_obj * b->A * 4, fl) == hipSuccess &&
              hipHostMalloc((void**)&s.h_out, words * 8, fl) == hipSuccess &&
              hipHostMalloc((void**)&s.h_status, 64, fl) == hipSuccess &&
              hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) == hipSuccess;
    if (ok && b->stage_device) {
        s.owns_device = true;
        ok = hipMalloc((void**)&s.d_blob, blob) == hipSuccess &&
             hipMalloc((void**)&s.d_base, (size_t)cap_obj * 8) == hipSuccess &&
             hipMalloc((void**)&s.d_len, (size_t)cap_obj * b->A * 4) == hipSuccess &&
             hipMalloc((void**)&s.d_out, words * 8) == hipSuccess &&
             hipMalloc((void**)&s.d_status, 64) == hipSuccess;
    } else if (ok) {
        ok = device_view(s.h_blob, &s.d_blob) && device_view(s.h_base, &s.d_base) &&
             device_view(s.h_len, &s.d_len) && device_view(s.h_out, &s.d_out);
        s.d_status = nullptr;  // sizes are validated on the host before staging
    }
    if (!ok) {
        (void)hipGetLastError();
        free_slot(s);
        return fail(HDX_E_NOMEM, "batcher staging (%u objects, %llu bytes)", cap_obj,
                    (unsigned long long)cap_bytes);
    }
    if (s.h_status) *s.h_status = 0;
    s.cap_obj = cap_obj;
    s.cap_bytes = cap_bytes;
    return HDX_OK;
}

// One fused hash + lookup launch on the slot's stream (asynchronous; two
// launches beyond 4 tables), with H2D / D2H around it when staging through HBM.
hipError_t ship(hdx_batcher_s* b, Slot& s) {
    hipError_t e;
    const uint32_t n = s.nobj;
    const bool dev = s.owns_device;
#define SHIP_TRY(x) if ((e = (x)) != hipSuccess) return e
    if (dev) {
        SHIP_TRY(hipMemcpyAsync(s.d_blob, s.h_blob, s.nbytes, hipMemcpyHostToDevice, s.stream));
        SHIP_TRY(hipMemcpyAsync(s.d_base, s.h_base, (size_t)n * 8, hipMemcpyHostToDevice, s.stream));
        SHIP_TRY(hipMemcpyAsync(s.d_len, s.h_len, (size_t)n * b->A * 4, hipMemcpyHostToDevice, s.stream));
        SHIP_TRY(hipMemsetAsync(s.d_status, 0, 4, s.stream));
    }
    BatchArgs a{};
    a.blob = s.d_blob;
    a.obj_base = s.d_base;
    a.attr_len = s.d_len;
    a.coords = s.d_out;
    a.status = s.d_status;
    a.n = n;
    a.A = b->A;
    std::memcpy(a.codes, b->codes.data(), std::min(b->A, kKernargCodes));
    a.codes_dev = b->codes_dev;
    finalize_args(a);
    const size_t region_base = (size_t)s.cap_obj * b->A;
    if (!b->tables.empty() && b->tables.size() <= kMaxSweepTables && b->A <= 128) {
        // one launch: hash + every table's lookup_region (hash_regroup_regions_kernel)
        a.T = (uint32_t)b->tables.size();
        for (uint32_t t = 0; t < a.T; ++t) {
            const hdx_region_table tb = b->tables[t];
            a.t[t].index = tb->d_index;
            a.t[t].lower = tb->d_lower;
            a.t[t].upper = tb->d_upper;
            a.t[t].ids = tb->d_ids;
            a.t[t].out = s.d_out + region_base + (size_t)t * s.cap_obj;
            a.t[t].W = tb->W;
            a.t[t].D = tb->D;
            a.t[t].R = tb->R;
            a.t[t].index_words = tb->index_words;
            std::memcpy(a.t[t].attrs, tb->attrs, sizeof a.t[t].attrs);
        }
        SHIP_TRY(launch_hash_batch_regions(a, s.stream));
    } else {
        SHIP_TRY(launch_hash_batch(a, s.stream));
    }
    if (b->tables.size() > kMaxSweepTables || (!b->tables.empty() && b->A > 128)) {
        // more tables than the fused kernel takes: one lookup kernel for all of them
        MultiRegionArgs r{};
        r.coords = s.d_out;
        r.out = s.d_out + region_base;
        r.n = n;
        r.out_stride = s.cap_obj;
        r.A = b->A;
        r.T = (uint32_t)b->tables.size();
        for (uint32_t t = 0; t < r.T; ++t) {
            const hdx_region_table tb = b->tables[t];
            r.t[t].lower = tb->d_lower;
            r.t[t].upper = tb->d_upper;
            r.t[t].ids = tb->d_ids;
            r.t[t].index = tb->d_index;
            r.t[t].W = tb->W;
            r.t[t].index_words = tb->index_words;
            r.t[t].D = tb->D;
            r.t[t].R = tb->R;
            std::memcpy(r.t[t].attrs, tb->attrs, sizeof r.t[t].attrs);
        }
        SHIP_TRY(launch_lookup_regions_multi(r, s.stream));
    }
    if (dev) {
        SHIP_TRY(hipMemcpyAsync(s.h_out, s.d_out, (size_t)n * b->A * 8, hipMemcpyDeviceToHost, s.stream));
        if (!b->tables.empty())
            SHIP_TRY(hipMemcpyAsync(s.h_out + region_base, s.d_out + region_base,
                                    ((b->tables.size() - 1) * s.cap_obj + n) * 8, hipMemcpyDeviceToHost,
                                    s.stream));
        SHIP_TRY(hipMemcpyAsync(s.h_status, s.d_status, 4, hipMemcpyDeviceToHost, s.stream));
    }
#undef SHIP_TRY
    return hipSuccess;
}

hdx_status finish(Slot& s, hipError_t launched) {
    hipError_t e = launched == hipSuccess ? hipStreamSynchronize(s.stream) : launched;
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return HDX_E_DEVICE;
    }
    return *s.h_status ? HDX_E_BADSIZE : HDX_OK;
}

// Writes object (key, values) at staging index idx / byte offset off.
void stage(const hdx_batcher_s* b, Slot& s, uint32_t idx, uint64_t off, const uint8_t* key, size_t key_len,
           const uint8_t* const* values, const size_t* value_lens) {
    s.h_base[idx] = off;
    uint32_t* len = s.h_len + (size_t)idx * b->A;
    uint8_t* p = s.h_blob + off;
    len[0] = (uint32_t)key_len;
    if (key_len) std::memcpy(p, key, key_len);
    p += key_len;
    for (uint32_t j = 1; j < b->A; ++j) {
        const size_t L = value_lens[j - 1];
        len[j] = (uint32_t)L;
        if (L) std::memcpy(p, values[j - 1], L);
        p += L;
    }
}

void copy_out(const hdx_batcher_s* b, const Slot& s, uint32_t idx, uint64_t* hs, uint64_t* region_ids) {
    std::memcpy(hs, s.h_out + (size_t)idx * b->A, (size_t)b->A * 8);
    if (region_ids)
        for (size_t t = 0; t < b->tables.size(); ++t)
            region_ids[t] = s.h_out[(size_t)s.cap_obj * b->A + t * s.cap_obj + idx];
}

// Under mu: the FILLING slot stops taking objects; a FREE slot (if any) takes over.
void seal_locked(hdx_batcher_s* b) {
    Slot& s = b->slots[b->cur];
    s.st = SEALED;
    ++b->pending;
    b->sealed.push_back(b->cur);
    b->cur = -1;
    for (uint32_t i = 0; i < b->nslots; ++i)
        if (b->slots[i].st == FREE) {
            Slot& f = b->slots[i];
            f.st = FILLING;
            f.nobj = 0;
            f.nbytes = 0;
            f.full = false;
            ++f.gen;
            b->cur = (int)i;
            break;
        }
    b->cv_flush.notify_one();
}

void flusher_main(hdx_batcher_s* b) {
    (void)hipSetDevice(b->device);
    std::unique_lock<std::mutex> lk(b->mu);
    for (;;) {
        // ship every sealed slot whose writers are done, in order
        if (!b->sealed.empty() && b->slots[b->sealed.front()].writers == 0) {
            const int i = b->sealed.front();
            b->sealed.pop_front();
            Slot& s = b->slots[i];
            s.st = INFLIGHT;
            b->n_batches.fetch_add(1, std::memory_order_relaxed);
            if (s.full) b->n_full.fetch_add(1, std::memory_order_relaxed);
            lk.unlock();
            const hipError_t e = ship(b, s);
            lk.lock();
            s.result = e == hipSuccess ? HDX_OK : HDX_E_DEVICE;
            b->inflight.push_back(i);
            b->cv_ship.notify_one();
            continue;
        }
        if (b->cur >= 0 && b->slots[b->cur].nobj > 0) {
            const Clock::time_point deadline = b->slots[b->cur].first + b->delay;
            if (b->stop || b->pending == 0 || Clock::now() >= deadline) {
                seal_locked(b);
                continue;
            }
            // woken early by a seal, a finished writer or stop; else at the deadline
            b->cv_flush.wait_until(lk, deadline);
            continue;
        }
        if (b->stop && b->sealed.empty()) break;
        b->cv_flush.wait(lk);
    }
    b->flusher_done = true;
    b->cv_ship.notify_one();
}

void completer_main(hdx_batcher_s* b) {
    (void)hipSetDevice(b->device);
    std::unique_lock<std::mutex> lk(b->mu);
    for (;;) {
        b->cv_ship.wait(lk, [b] { return !b->inflight.empty() || b->flusher_done; });
        if (b->inflight.empty()) break;
        const int i = b->inflight.front();
        b->inflight.pop_front();
        Slot& s = b->slots[i];
        const hdx_status shipped = s.result;
        lk.unlock();
        hdx_status st = finish(s, shipped == HDX_OK ? hipSuccess : hipErrorUnknown);
        lk.lock();
        s.result = st;
        s.st = DONE;
        s.readers.store(s.nobj, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> dl(s.done_mu);
            s.done_gen.store(s.gen, std::memory_order_release);
        }
        s.done_cv.notify_all();
        if (--b->pending == 0) b->cv_flush.notify_one();  // the pipeline is idle: ship the next batch now
    }
}

}  // namespace

HDX_EXPORT hdx_status hdx_batcher_create(const uint32_t* types, uint32_t attrs_sz,
                                         const hdx_batcher_config* cfg, hdx_batcher* out) {
    if (!out) return fail(HDX_E_INVALID, "out is NULL");
    *out = nullptr;
    hdx_batcher_config c{};
    if (cfg) c = *cfg;
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    hdx_status st = check_schema(types, attrs_sz, codes.data());
    if (st != HDX_OK) return st;
    if (c.ntables > 16) return fail(HDX_E_INVALID, "ntables=%u > 16", c.ntables);
    if (c.ntables && !c.tables) return fail(HDX_E_INVALID, "tables is NULL");
    if ((st = bind_device(c.device)) != HDX_OK) return st;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    auto* b = new hdx_batcher_s();
    b->device = dev;
    b->A = attrs_sz;
    b->codes.assign(codes.begin(), codes.begin() + attrs_sz);
    {
        BatchArgs tmp{};
        if ((st = set_codes(tmp, codes.data(), attrs_sz)) != HDX_OK) {
            delete b;
            return st;
        }
        if (tmp.codes_dev) {
            // its own copy: the library's cache is freed at hdx_shutdown, a
            // batcher may outlive that
            uint8_t* own = nullptr;
            if (hipMalloc((void**)&own, attrs_sz) != hipSuccess ||
                hipMemcpy(own, codes.data(), attrs_sz, hipMemcpyHostToDevice) != hipSuccess) {
                (void)hipGetLastError();
                (void)hipFree(own);
                delete b;
                return fail(HDX_E_NOMEM, "batcher: device copy of %u attribute classes", attrs_sz);
            }
            b->codes_dev = own;
        }
    }
    b->max_obj = c.max_objects ? c.max_objects : 4096;
    b->max_bytes = c.max_bytes ? c.max_bytes : (8ull << 20);
    b->delay = std::chrono::microseconds(c.max_delay_us ? c.max_delay_us : 50);
    b->stage_device = (c.flags & HDX_BATCHER_STAGE_DEVICE) != 0;
    b->types.assign(types, types + attrs_sz);
    b->host_max_bytes = (c.flags & HDX_BATCHER_DEVICE_ONLY) ? 0 : c.host_max_bytes ? c.host_max_bytes : UINT64_MAX;
    const uint32_t nslots = c.slots ? std::max(c.slots, 2u) : 4;
    for (uint32_t t = 0; t < c.ntables; ++t) {
        if (!c.tables[t]) {
            delete b;
            return fail(HDX_E_INVALID, "tables[%u] is NULL", t);
        }
        if (c.tables[t]->device != dev) {
            delete b;
            return fail(HDX_E_INVALID, "tables[%u] lives on device %d, batcher on %d", t,
                        c.tables[t]->device, dev);
        }
        for (uint32_t d = 0; d < c.tables[t]->D; ++d)
            if (c.tables[t]->attrs[d] >= attrs_sz) {
                delete b;
                return fail(HDX_E_INVALID, "tables[%u]: attribute %u >= attrs_sz %u", t,
                            c.tables[t]->attrs[d], attrs_sz);
            }
        b->tables.push_back(c.tables[t]);
    }
    b->slots.reset(new Slot[nslots]);
    b->nslots = nslots;
    for (uint32_t i = 0; i < nslots; ++i)
        if ((st = alloc_slot(b, b->slots[i], b->max_obj, b->max_bytes)) != HDX_OK) {
            for (uint32_t f = 0; f < nslots; ++f) free_slot(b->slots[f]);
            delete b;
            return st;
        }
    b->cur = 0;
    b->slots[0].st = FILLING;
    b->slots[0].gen = 1;
    b->flusher = std::thread(flusher_main, b);
    b->completer = std::thread(completer_main, b);
    *out = b;
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_batcher_destroy(hdx_batcher b) {
    if (!b) return HDX_OK;
    {
        std::lock_guard<std::mutex> lk(b->mu);
        b->stop = true;
        b->cv_flush.notify_all();
    }
    b->flusher.join();
    b->completer.join();
    (void)hipSetDevice(b->device);
    for (uint32_t i = 0; i < b->nslots; ++i) free_slot(b->slots[i]);
    free_slot(b->direct);
    delete b;
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_batcher_get_stats(hdx_batcher b, hdx_batcher_stats* out) {
    if (!b || !out) return fail(HDX_E_INVALID, "NULL pointer");
    const uint64_t host = b->host_total();
    out->objects = b->n_objects.load() + host;
    out->batches = b->n_batches.load();
    out->full_batches = b->n_full.load();
    out->direct = b->n_direct.load();
    out->host = host;
    return HDX_OK;
}

static hdx_status hash_direct(hdx_batcher b, uint64_t total, const uint8_t* key, size_t key_len,
                              const uint8_t* const* values, const size_t* value_lens, uint64_t* hs,
                              uint64_t* region_ids) {
    std::lock_guard<std::mutex> lk(b->direct_mu);
    int prev = -1;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(b->device));
    hdx_status st = HDX_OK;
    Slot& s = b->direct;
    if (s.cap_bytes < total) st = alloc_slot(b, s, 1, total);
    if (st == HDX_OK) {
        s.nobj = 1;
        s.nbytes = total;
        stage(b, s, 0, 0, key, key_len, values, value_lens);
        st = finish(s, ship(b, s));
        if (st == HDX_OK) copy_out(b, s, 0, hs, region_ids);
        else if (st == HDX_E_DEVICE) fail(st, "batcher: device error on a direct batch");
    }
    (void)hipSetDevice(prev);
    b->n_direct.fetch_add(1, std::memory_order_relaxed);
    b->n_objects.fetch_add(1, std::memory_order_relaxed);
    return st;
}

HDX_EXPORT hdx_status hdx_batcher_hash_object(hdx_batcher b, const uint8_t* key, size_t key_len,
                                              const uint8_t* const* values, const size_t* value_lens,
                                              uint64_t* hs, uint64_t* region_ids) {
    if (!b || !hs || (!key && key_len) || (b->A > 1 && (!values || !value_lens)))
        return fail(HDX_E_INVALID, "NULL pointer");
    // host-side checks the kernel would otherwise report per batch
    uint64_t total = key_len;
    if (key_len >= (1ull << 32)) return fail(HDX_E_INVALID, "key of %zu bytes", key_len);
    if (b->codes[0] >= CODE_INT64 && key_len != 0 && key_len != 8)
        return fail(HDX_E_BADSIZE, "key: numeric value of %zu bytes", key_len);
    for (uint32_t j = 1; j < b->A; ++j) {
        const size_t L = value_lens[j - 1];
        if (L && !values[j - 1]) return fail(HDX_E_INVALID, "value %u is NULL", j - 1);
        if (L >= (1ull << 32)) return fail(HDX_E_INVALID, "value of %zu bytes", L);
        if (b->codes[j] >= CODE_INT64 && L != 0 && L != 8)
            return fail(HDX_E_BADSIZE, "attribute %u: numeric value of %zu bytes", j, L);
        total += L;
    }
    if (b->host_max_bytes && total <= b->host_max_bytes) {
        // the calling thread: the per-object CPU path and host lookups
        hdx_status st = hdx_hash_object(b->types.data(), b->A, key, key_len, values, value_lens, hs);
        if (st != HDX_OK) return st;
        if (region_ids)
            for (size_t t = 0; t < b->tables.size(); ++t) region_ids[t] = region_lookup_host(b->tables[t], hs);
        static std::atomic<uint32_t> next_shard{0};
        thread_local const uint32_t shard = next_shard.fetch_add(1, std::memory_order_relaxed) % 32;
        b->n_host[shard].v.fetch_add(1, std::memory_order_relaxed);
        return HDX_OK;
    }
    if (total > b->max_bytes) return hash_direct(b, total, key, key_len, values, value_lens, hs, region_ids);

    std::unique_lock<std::mutex> lk(b->mu);
    int si;
    for (;;) {
        if (b->stop) return fail(HDX_E_INVALID, "batcher is being destroyed");
        if (b->cur >= 0) {
            Slot& s = b->slots[b->cur];
            if (s.nobj < b->max_obj && s.nbytes + total <= b->max_bytes) break;
            s.full = true;
            seal_locked(b);
            continue;
        }
        b->cv_free.wait(lk);
    }
    si = b->cur;
    Slot& s = b->slots[si];
    const uint32_t idx = s.nobj++;
    const uint64_t off = s.nbytes;
    s.nbytes += total;
    ++s.writers;
    const uint64_t gen = s.gen;
    if (idx == 0) {
        s.first = Clock::now();
        b->cv_flush.notify_one();
    }
    if (s.nobj == b->max_obj) {
        s.full = true;
        seal_locked(b);
    }
    lk.unlock();

    stage(b, s, idx, off, key, key_len, values, value_lens);

    lk.lock();
    if (--s.writers == 0 && s.st == SEALED) b->cv_flush.notify_one();
    lk.unlock();

    // wait for the batch: a few callers spin for about one round trip (the
    // rest sleep at once, so spinners never starve the flush and completion
    // threads of CPU), then sleep
    if (b->spinners.fetch_add(1, std::memory_order_relaxed) < kMaxSpinners) {
        const Clock::time_point spin_until = Clock::now() + std::chrono::microseconds(100);
        while (s.done_gen.load(std::memory_order_acquire) != gen && Clock::now() < spin_until)
            __builtin_ia32_pause();
    }
    b->spinners.fetch_sub(1, std::memory_order_relaxed);
    if (s.done_gen.load(std::memory_order_acquire) != gen) {
        std::unique_lock<std::mutex> dl(s.done_mu);
        s.done_cv.wait(dl, [&] { return s.done_gen.load(std::memory_order_acquire) == gen; });
    }
    const hdx_status st = s.result;
    if (st == HDX_OK) copy_out(b, s, idx, hs, region_ids);
    if (s.readers.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        lk.lock();
        s.st = FREE;
        if (b->cur < 0) {
            s.st = FILLING;
            s.nobj = 0;
            s.nbytes = 0;
            s.full = false;
            ++s.gen;
            b->cur = si;
        }
        b->cv_free.notify_all();
        lk.unlock();
    }
    b->n_objects.fetch_add(1, std::memory_order_relaxed);
    if (st == HDX_E_DEVICE) return fail(st, "batcher: device error");
    if (st == HDX_E_BADSIZE) return fail(st, "batcher: numeric value of bad size");
    return st;
}
