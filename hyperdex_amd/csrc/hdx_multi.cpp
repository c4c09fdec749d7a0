// hdx_multi.cpp — the device set of hdx_init_mask and the entry points that
// span it (include/hdxhash.h, "multi-device").
//
// HyperDex hashes objects from N daemon::loop threads of one process
// (daemon/daemon.cc:345-351 -> key_state::hash_objects, daemon/key_state.cc:
// 1455-1543 -> hyperdex::hash, common/hash.cc:56-68).  Objects are
// independent, so a batch splits into contiguous object ranges, one per
// device, balanced by payload bytes — the rule of
// hyperdex_amd/dist.py:shard_ranges, restated here so a C++ daemon gets it
// without Python or torch:
//   * the host-resident batch (hdx_hash_batch_host): one worker thread per
//     device pipelines its range's H2D -> kernel -> D2H straight into the
//     caller's coordinate rows (the single-device pipeline of hdx_capi.cpp,
//     run on each worker's own streams and staging);
//   * device-resident shards (hdx_hash_batch_device_multi): each device
//     hashes its shard into its rows of its own full coordinate matrix, then
//     one in-process RCCL all-gather over xGMI (ncclCommInitAll over the
//     mask) fills the rest in place.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hdx_cuts.h"
#include "hdx_host.h"

namespace hdx {

// ---- byte-balanced cuts: hdx_cuts.h ------------------------------------------

// ---- worker threads ---------------------------------------------------------

class Worker {
public:
    Worker() : th_([this] { run(); }) {}
    void post(std::function<void()> job) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(std::move(job));
        }
        cv_.notify_one();
    }
    void join() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_one();
        th_.join();
    }

private:
    void run() {
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                job = std::move(q_.front());
                q_.pop_front();
            }
            job();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
    std::thread th_;  // last: started once the queue exists
};

// Waits for `count` posted jobs.
class Latch {
public:
    explicit Latch(size_t count) : left_(count) {}
    void done() {
        std::lock_guard<std::mutex> lk(mu_);
        if (--left_ == 0) cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return left_ == 0; });
    }

private:
    std::mutex mu_;
    std::condition_variable cv_;
    size_t left_;
};

// ---- the device set -----------------------------------------------------------

struct DeviceSet {
    uint64_t mask = 0;
    std::vector<int> devs;                        // ascending HIP ordinals
    std::vector<std::unique_ptr<Worker>> workers;  // one per device: the host path
    std::vector<hipStream_t> streams;             // one per device: device-resident shards
    std::vector<ncclComm_t> comms;                // created on the first gather
    std::mutex call_mu;                           // one device-resident multi call at a time
};

static std::mutex g_set_mu;
static DeviceSet* g_set = nullptr;

static void destroy_set(DeviceSet* ds) {
    if (!ds) return;
    // workers first: each frees its thread's scratch as its last job (not in
    // a thread-local destructor at exit) before hdx_shutdown walks the
    // scratch registry
    for (auto& w : ds->workers) {
        w->post([] { release_thread_scratch(); });
        w->join();
    }
    ds->workers.clear();
    for (size_t k = 0; k < ds->comms.size(); ++k) {
        (void)hipSetDevice(ds->devs[k]);
        (void)ncclCommDestroy(ds->comms[k]);
    }
    for (size_t k = 0; k < ds->streams.size(); ++k) {
        if (!ds->streams[k]) continue;
        (void)hipSetDevice(ds->devs[k]);
        (void)hipStreamSynchronize(ds->streams[k]);
        (void)hipStreamDestroy(ds->streams[k]);
    }
    delete ds;
}

void device_set_teardown() {
    DeviceSet* ds;
    {
        std::lock_guard<std::mutex> lk(g_set_mu);
        ds = g_set;
        g_set = nullptr;
    }
    destroy_set(ds);
}

hdx_status device_set_create(uint64_t mask, const std::vector<int>& devs) {
    {
        std::lock_guard<std::mutex> lk(g_set_mu);
        if (g_set && g_set->mask == mask && g_set->devs == devs) return HDX_OK;
    }
    device_set_teardown();  // a different mask replaces the set (no call may be in progress)
    int cur = -1;
    const bool had = hipGetDevice(&cur) == hipSuccess;
    auto* ds = new DeviceSet();
    ds->mask = mask;
    ds->devs = devs;
    ds->streams.assign(devs.size(), nullptr);
    for (size_t k = 0; k < devs.size(); ++k) {
        if (hipSetDevice(devs[k]) != hipSuccess ||
            hipStreamCreateWithFlags(&ds->streams[k], hipStreamNonBlocking) != hipSuccess) {
            const hipError_t e = hipGetLastError();
            destroy_set(ds);
            if (had) (void)hipSetDevice(cur);
            return fail(HDX_E_DEVICE, "device %d: stream creation failed: %s", devs[k], hipGetErrorString(e));
        }
    }
    for (size_t k = 0; k < devs.size(); ++k) ds->workers.emplace_back(new Worker());
    if (had) (void)hipSetDevice(cur);
    std::lock_guard<std::mutex> lk(g_set_mu);
    g_set = ds;
    return HDX_OK;
}

static DeviceSet* current_set() {
    std::lock_guard<std::mutex> lk(g_set_mu);
    return g_set;
}

// Restores the caller's HIP device on scope exit.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

// ---- host-resident batch over the set ------------------------------------------

// Runs one job per device on the workers; returns the first failing device's
// status (in device order) with that worker's message.
static hdx_status run_on_workers(DeviceSet* ds, const std::function<hdx_status(size_t k)>& job) {
    const size_t nd = ds->devs.size();
    std::vector<hdx_status> st(nd, HDX_OK);
    std::vector<std::string> msg(nd);
    Latch latch(nd);
    for (size_t k = 0; k < nd; ++k) {
        ds->workers[k]->post([&, k] {
            st[k] = job(k);
            if (st[k] != HDX_OK) msg[k] = hdx_last_error();
            latch.done();
        });
    }
    latch.wait();
    for (size_t k = 0; k < nd; ++k)
        if (st[k] != HDX_OK) return fail(st[k], "device %d: %s", ds->devs[k], msg[k].c_str());
    return HDX_OK;
}

bool host_batch_uses_set() { return current_set() != nullptr; }

hdx_status hash_host_set(const uint8_t* codes, uint32_t A, const uint8_t* blob, uint64_t blob_bytes,
                         const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords) {
    DeviceSet* ds = current_set();
    if (!ds) return fail(HDX_E_INVALID, "no device set (hdx_init_mask)");
    const uint32_t world = (uint32_t)ds->devs.size();
    std::vector<uint64_t> first(world + 1);
    if (world == 1) {
        first[0] = 0;
        first[1] = n;
    } else {
        Prefix p{attr_len, A, n, {}};
        const uint64_t blocks = (n + kCutBlock - 1) / kCutBlock;
        std::vector<uint64_t> bsum(blocks);
        hdx_status st = run_on_workers(ds, [&](size_t k) {
            for (uint64_t b = blocks * k / world; b < blocks * (k + 1) / world; ++b)
                bsum[b] = block_bytes(attr_len, A, n, b);
            return HDX_OK;
        });
        if (st != HDX_OK) return st;
        p.bprefix.assign(blocks + 1, 0);
        for (uint64_t b = 0; b < blocks; ++b) p.bprefix[b + 1] = p.bprefix[b] + bsum[b];
        cuts_from_prefix(p, world, 0.0, first.data());
    }
    return run_on_workers(ds, [&](size_t k) -> hdx_status {
        const uint64_t f = first[k], cnt = first[k + 1] - first[k];
        if (cnt == 0) return HDX_OK;
        hdx_status s = bind_device(ds->devs[k]);
        if (s != HDX_OK) return s;
        return hash_host(codes, A, blob, blob_bytes, obj_base + f, attr_len + f * A, cnt, coords + f * A);
    });
}

}  // namespace hdx

using namespace hdx;

// ---- exported -------------------------------------------------------------------

HDX_EXPORT hdx_status hdx_shard_ranges(const uint32_t* attr_len, uint32_t attrs_sz, uint64_t n, uint32_t world,
                                       double equal_count_tol, uint64_t* first) {
    if (!first || world == 0) return fail(HDX_E_INVALID, "first is NULL or world == 0");
    if (attr_len && (attrs_sz == 0 || attrs_sz > HDX_MAX_ATTRS))
        return fail(HDX_E_INVALID, "attrs_sz=%u outside [1, %d]", attrs_sz, HDX_MAX_ATTRS);
    shard_cuts(attr_len, attrs_sz, n, world, equal_count_tol, first);  // no sizes: counts differ by at most one
    return HDX_OK;
}

HDX_EXPORT int hdx_device_set(int* devices, int max_devices) {
    DeviceSet* ds = current_set();
    if (!ds) return 0;
    const int nd = (int)ds->devs.size();
    for (int k = 0; k < nd && k < max_devices && devices; ++k) devices[k] = ds->devs[k];
    return nd;
}

static const char* nccl_text(ncclResult_t r) { return ncclGetErrorString(r); }

#define NCCL_TRY(expr)                                                             \
    do {                                                                           \
        ncclResult_t r_ = (expr);                                                  \
        if (r_ != ncclSuccess) return fail(HDX_E_DEVICE, "%s: %s", #expr, nccl_text(r_)); \
    } while (0)

// A device pointer must live on the device its shard runs on (a kernel on
// another device would read through the fabric or fault).  Host (pinned)
// pointers are accepted.
static hdx_status check_on_device(const void* p, int dev, uint32_t k, const char* what) {
    if (!p) return HDX_OK;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return HDX_OK;  // unregistered host memory: the kernel would fault, but the caller may map it
    }
    if (a.type == hipMemoryTypeDevice && a.device != dev)
        return fail(HDX_E_INVALID, "shard %u: %s is memory of device %d, the shard runs on device %d", k, what,
                    a.device, dev);
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_hash_batch_device_multi(const uint32_t* types, uint32_t attrs_sz, const hdx_shard* shards,
                                                  uint32_t nshards, int gather) {
    uint8_t codes[HDX_MAX_ATTRS];
    hdx_status st = check_schema(types, attrs_sz, codes);
    if (st != HDX_OK) return st;
    DeviceSet* ds = current_set();
    if (!ds) return fail(HDX_E_INVALID, "no device set: call hdx_init_mask first");
    if (!shards || nshards != ds->devs.size())
        return fail(HDX_E_INVALID, "%u shards for a device set of %zu devices", nshards, ds->devs.size());
    uint64_t total = 0;
    for (uint32_t k = 0; k < nshards; ++k) total += shards[k].n;
    if (total == 0) return HDX_OK;
    for (uint32_t k = 0; k < nshards; ++k) {
        const hdx_shard& s = shards[k];
        if (s.n && (!s.blob || !s.obj_base || !s.attr_len || !s.coords))
            return fail(HDX_E_INVALID, "shard %u: NULL device pointer", k);
        if (gather && !s.coords) return fail(HDX_E_INVALID, "shard %u: NULL coords", k);
        const int dev = ds->devs[k];
        if ((st = check_on_device(s.blob, dev, k, "blob")) != HDX_OK ||
            (st = check_on_device(s.obj_base, dev, k, "obj_base")) != HDX_OK ||
            (st = check_on_device(s.attr_len, dev, k, "attr_len")) != HDX_OK ||
            (st = check_on_device(s.coords, dev, k, "coords")) != HDX_OK ||
            (st = check_on_device(s.status_dev, dev, k, "status_dev")) != HDX_OK)
            return st;
    }
    DeviceGuard guard;
    std::lock_guard<std::mutex> call(ds->call_mu);
    // hash: each shard into its rows of its device's matrix (gather) or into
    // its own coords (no gather)
    uint64_t row = 0;
    for (uint32_t k = 0; k < nshards; ++k) {
        const hdx_shard& s = shards[k];
        if (s.n) {
            HIP_TRY(hipSetDevice(ds->devs[k]));
            BatchArgs args{};
            std::memcpy(args.codes, codes, attrs_sz);
            args.blob = s.blob;
            args.obj_base = s.obj_base;
            args.attr_len = s.attr_len;
            args.coords = s.coords + (gather ? row * attrs_sz : 0);
            args.status = s.status_dev;
            args.n = s.n;
            args.A = attrs_sz;
            finalize_args(args);
            HIP_TRY(launch_hash_batch(args, ds->streams[k]));
        }
        row += s.n;
    }
    if (gather) {
        for (uint32_t k = 1; k < nshards; ++k)
            for (uint32_t j = 0; j < k; ++j)
                if (ds->devs[j] == ds->devs[k])  // hdxdbg_init_devices: no communicator over one GPU twice
                    return fail(HDX_E_INVALID, "device %d twice in the set: no RCCL gather", ds->devs[k]);
        if (ds->comms.empty()) {
            ds->comms.resize(nshards);
            ncclResult_t r = ncclCommInitAll(ds->comms.data(), (int)nshards, ds->devs.data());
            if (r != ncclSuccess) {
                ds->comms.clear();
                return fail(HDX_E_DEVICE, "ncclCommInitAll over %u devices: %s", nshards, nccl_text(r));
            }
        }
        bool equal = true;
        for (uint32_t k = 1; k < nshards; ++k) equal = equal && shards[k].n == shards[0].n;
        // one RCCL group: an in-place all-gather for equal counts, else one
        // in-place broadcast per shard (no staging matrix; hyperdex_amd/dist.py
        // pads instead because torch has no grouped broadcast over unequal rows)
        NCCL_TRY(ncclGroupStart());
        ncclResult_t r = ncclSuccess;  // the group is closed whatever happens inside it
        if (equal) {
            const size_t cnt = (size_t)shards[0].n * attrs_sz;
            for (uint32_t k = 0; k < nshards && r == ncclSuccess; ++k)
                r = ncclAllGather(shards[k].coords + (size_t)k * cnt, shards[k].coords, cnt, ncclUint64,
                                  ds->comms[k], ds->streams[k]);
        } else {
            uint64_t first = 0;
            for (uint32_t src = 0; src < nshards && r == ncclSuccess; ++src) {
                const size_t cnt = (size_t)shards[src].n * attrs_sz;
                for (uint32_t k = 0; cnt && k < nshards && r == ncclSuccess; ++k) {
                    uint64_t* rows = shards[k].coords + first * attrs_sz;
                    r = ncclBroadcast(rows, rows, cnt, ncclUint64, (int)src, ds->comms[k], ds->streams[k]);
                }
                first += shards[src].n;
            }
        }
        const ncclResult_t e = ncclGroupEnd();
        if (r != ncclSuccess) return fail(HDX_E_DEVICE, "RCCL gather: %s", nccl_text(r));
        if (e != ncclSuccess) return fail(HDX_E_DEVICE, "ncclGroupEnd: %s", nccl_text(e));
    }
    for (uint32_t k = 0; k < nshards; ++k) {
        HIP_TRY(hipSetDevice(ds->devs[k]));
        HIP_TRY(hipStreamSynchronize(ds->streams[k]));
    }
    return HDX_OK;
}

#if HDX_DEBUG_BUILD
// Debug library only (include/hdxhash_debug.h): a device set of explicit
// ordinals, repeats allowed, so the multi-device host path and ungathered
// shards run at world 2, 3, ... on a one-GPU box (tests/test_multi.py).
HDX_EXPORT hdx_status hdxdbg_init_devices(const int* devices, int n) {
    if (!devices || n <= 0 || n > 64) return fail(HDX_E_INVALID, "1 <= n <= 64 devices");
    const int nd = hdx_device_count();
    std::vector<int> devs(devices, devices + n);
    for (int d : devs)
        if (d < 0 || d >= nd) return fail(HDX_E_INVALID, "device %d (count %d)", d, nd);
    hdx_status st = bind_device(devs[0]);
    if (st != HDX_OK) return st;
    return device_set_create(1ull << 63, devs);  // mask bit 63: an explicit list
}
#endif
