// cpu_per_object.cc — times the product's per-object CPU path (hdx_hash_object
// / hdx_hash_key of libhdxhash.so, i.e. what the C++ drop-in
// include/hyperdex_amd/hash.h runs for common/hash.cc:48-68) the way daemon
// threads call it: one synchronous call per object, the value slices built
// from the caller's buffers, N threads each walking its own range of objects.
// bench.py loads this as tools/libhdxcpubench.so and reports the rate as
// `cpu_per_object` next to the oracle's `cpu_baseline`.
#include <hdxhash.h>

#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

// One pass over objects [lo, hi).  Returns the first non-OK status.
int pass(const uint32_t* types, uint32_t A, const uint8_t* blob, const uint64_t* obj_base,
         const uint32_t* attr_len, uint64_t lo, uint64_t hi, uint64_t* coords, int key_only) {
    std::vector<const uint8_t*> vals(A > 1 ? A - 1 : 1);
    std::vector<size_t> lens(A > 1 ? A - 1 : 1);
    for (uint64_t i = lo; i < hi; ++i) {
        const uint32_t* L = attr_len + i * A;
        const uint8_t* p = blob + obj_base[i];
        const uint8_t* key = p;
        size_t key_len = L[0];
        int rc;
        if (key_only) {
            rc = hdx_hash_key(types, A, key, key_len, coords + i * A);
        } else {
            p += key_len;
            for (uint32_t j = 1; j < A; ++j) {
                vals[j - 1] = p;
                lens[j - 1] = L[j];
                p += L[j];
            }
            rc = hdx_hash_object(types, A, key, key_len, vals.data(), lens.data(), coords + i * A);
        }
        if (rc != HDX_OK) return rc;
    }
    return HDX_OK;
}

}  // namespace

extern "C" __attribute__((visibility("default")))
int hdxcpu_time_objects(const uint32_t* types, uint32_t A, const uint8_t* blob, const uint64_t* obj_base,
                        const uint32_t* attr_len, uint64_t n, uint64_t* coords, int nthreads,
                        int key_only, double min_seconds, uint64_t* passes_out, double* seconds_out) {
    if (nthreads < 1) nthreads = 1;
    using clk = std::chrono::steady_clock;
    uint64_t passes = 0;
    int status = HDX_OK;
    auto t0 = clk::now();
    double dt = 0;
    do {
        std::vector<std::thread> th;
        std::vector<int> rc(nthreads, HDX_OK);
        for (int t = 0; t < nthreads; ++t) {
            uint64_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
            th.emplace_back([&, t, lo, hi] {
                rc[t] = pass(types, A, blob, obj_base, attr_len, lo, hi, coords, key_only);
            });
        }
        for (auto& x : th) x.join();
        for (int r : rc)
            if (r != HDX_OK) status = r;
        ++passes;
        dt = std::chrono::duration<double>(clk::now() - t0).count();
    } while (status == HDX_OK && dt < min_seconds);
    *passes_out = passes;
    *seconds_out = dt;
    return status;
}
