// multi_test.cc — a C++ caller of the multi-device C-ABI, the way a HyperDex
// daemon would use it (one process, N daemon::loop threads,
// daemon/daemon.cc:345-351): no Python, no torch.
//
//   multi_test [n]
//
// 1. hdx_init_mask over every visible device;
// 2. one host-resident batch hashed by 4 threads at once through
//    hdx_hash_batch_host (split over the set by the library);
// 3. the same batch sharded over the set by hdx_shard_ranges, each shard
//    uploaded to its device, hashed by hdx_hash_batch_device_multi with the
//    RCCL gather, and every device's full matrix read back;
// 4. the region-id forms: hdx_hash_batch_regions_host (split over the set)
//    and hdx_hash_batch_regions_device_multi with the gather of region ids
//    only (16 bytes per object for two tables instead of 104 of coordinates);
// all coordinates checked against the product's per-object CPU path
// (hdx_hash_object, common/hash.cc:56-68's signature), region ids against a
// first-match scan of the boxes (configuration::lookup_region,
// common/configuration.cc:698-735).  Prints "multi ok".
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "hdxhash.h"

#define CHECK(x)                                                                      \
    do {                                                                              \
        hdx_status s_ = (x);                                                          \
        if (s_ != HDX_OK) {                                                           \
            std::printf("FAIL %s: %d %s\n", #x, (int)s_, hdx_last_error());           \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)
#define HCHECK(x)                                                                     \
    do {                                                                              \
        if ((x) != hipSuccess) {                                                      \
            std::printf("FAIL %s\n", #x);                                             \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

// configuration::lookup_region: the first region whose box holds the
// subspace's coordinates (inclusive), else 0
struct Table {
    std::vector<uint16_t> attrs;
    std::vector<uint64_t> lower, upper, ids;
    uint64_t lookup(const uint64_t* hs) const {
        const size_t D = attrs.size();
        for (size_t r = 0; r < ids.size(); ++r) {
            bool in = true;
            for (size_t d = 0; d < D && in; ++d) {
                const uint64_t h = hs[attrs[d]];
                in = lower[r * D + d] <= h && h <= upper[r * D + d];
            }
            if (in) return ids[r];
        }
        return 0;
    }
};

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000;
    // key STRING + 6 strings of 0..150 bytes + 3 INT64 + 3 FLOAT (a config-3b-like mix)
    std::vector<uint32_t> types = {9217, 9217, 9217, 9217, 9217, 9217, 9217, 9218, 9218, 9218, 9219, 9219, 9219};
    const uint32_t A = (uint32_t)types.size();
    std::vector<uint32_t> len(n * A);
    std::vector<uint64_t> base(n);
    uint64_t rng = 0x4859504552444558ull, total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        base[i] = total;
        for (uint32_t j = 0; j < A; ++j) {
            const uint32_t L = j == 0 ? 64 : types[j] == 9217 ? (uint32_t)(splitmix(rng) % 151) : 8;
            len[i * A + j] = L;
            total += L;
        }
    }
    std::vector<uint8_t> blob(total + 1);
    for (uint64_t b = 0; b < total; b += 8) {
        const uint64_t r = splitmix(rng);
        std::memcpy(&blob[b], &r, std::min<uint64_t>(8, total - b));
    }

    // the product's per-object CPU path
    std::vector<uint64_t> want(n * A);
    for (uint64_t i = 0; i < n; ++i) {
        const uint8_t* vals[16];
        size_t lens[16];
        uint64_t off = base[i] + len[i * A];
        for (uint32_t j = 1; j < A; ++j) {
            vals[j - 1] = &blob[off];
            lens[j - 1] = len[i * A + j];
            off += len[i * A + j];
        }
        CHECK(hdx_hash_object(types.data(), A, &blob[base[i]], len[i * A], vals, lens, &want[i * A]));
    }

    const int ndev = hdx_device_count();
    if (ndev <= 0) {
        std::printf("FAIL no device\n");
        return 1;
    }
    const uint64_t mask = ndev >= 64 ? ~0ull : (1ull << ndev) - 1;
    CHECK(hdx_init_mask(mask));
    int devs[64];
    const int nd = hdx_device_set(devs, 64);
    if (nd != ndev) {
        std::printf("FAIL device set has %d of %d devices\n", nd, ndev);
        return 1;
    }

    // 2. host-resident, 4 caller threads at once
    std::vector<std::vector<uint64_t>> got(4, std::vector<uint64_t>(n * A));
    std::vector<hdx_status> st(4);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
        th.emplace_back([&, t] {
            st[t] = hdx_hash_batch_host(types.data(), A, blob.data(), total, base.data(), len.data(), n,
                                        got[t].data());
        });
    for (auto& x : th) x.join();
    for (int t = 0; t < 4; ++t) {
        if (st[t] != HDX_OK || got[t] != want) {
            std::printf("FAIL host batch, thread %d: status %d\n", t, (int)st[t]);
            return 1;
        }
    }

    // 3. device-resident shards + RCCL gather
    std::vector<uint64_t> first(nd + 1);
    CHECK(hdx_shard_ranges(len.data(), A, n, (uint32_t)nd, 1e-3, first.data()));
    std::vector<hdx_shard> shards(nd);
    std::vector<void*> allocs;
    for (int k = 0; k < nd; ++k) {
        const uint64_t f = first[k], c = first[k + 1] - first[k];
        const uint64_t lo = c ? base[f] : 0, hi = c ? base[f + c - 1] + [&] {
            uint64_t s = 0;
            for (uint32_t j = 0; j < A; ++j) s += len[(f + c - 1) * A + j];
            return s;
        }() : 0;
        std::vector<uint64_t> rb(c ? c : 1);
        for (uint64_t i = 0; i < c; ++i) rb[i] = base[f + i] - lo;
        HCHECK(hipSetDevice(devs[k]));
        void *d_blob, *d_base, *d_len, *d_coords;
        HCHECK(hipMalloc(&d_blob, hi - lo + 1));
        HCHECK(hipMalloc(&d_base, rb.size() * 8));
        HCHECK(hipMalloc(&d_len, (c ? c : 1) * A * 4));
        HCHECK(hipMalloc(&d_coords, n * A * 8));
        HCHECK(hipMemcpy(d_blob, &blob[lo], hi - lo, hipMemcpyHostToDevice));
        HCHECK(hipMemcpy(d_base, rb.data(), c * 8, hipMemcpyHostToDevice));
        HCHECK(hipMemcpy(d_len, &len[f * A], c * A * 4, hipMemcpyHostToDevice));
        HCHECK(hipMemset(d_coords, 0, n * A * 8));
        allocs.insert(allocs.end(), {d_blob, d_base, d_len, d_coords});
        shards[k] = hdx_shard{(const uint8_t*)d_blob, (const uint64_t*)d_base, (const uint32_t*)d_len, c,
                              (uint64_t*)d_coords, nullptr};
    }
    CHECK(hdx_hash_batch_device_multi(types.data(), A, shards.data(), (uint32_t)nd, 1));
    std::vector<uint64_t> back(n * A);
    for (int k = 0; k < nd; ++k) {
        HCHECK(hipSetDevice(devs[k]));
        HCHECK(hipMemcpy(back.data(), shards[k].coords, n * A * 8, hipMemcpyDeviceToHost));
        if (back != want) {
            std::printf("FAIL gathered matrix on device %d differs\n", devs[k]);
            return 1;
        }
    }

    // 4. region ids: a key grid of 64 equal ranges and a 2-attribute table of
    // random (overlapping) boxes
    std::vector<Table> tabs(2);
    tabs[0].attrs = {0};
    for (uint64_t r = 0; r < 64; ++r) {
        tabs[0].lower.push_back(r << 58);
        tabs[0].upper.push_back(r == 63 ? ~0ull : ((r + 1) << 58) - 1);
        tabs[0].ids.push_back(100 + r);
    }
    tabs[1].attrs = {3, 8};
    for (uint64_t r = 0; r < 40; ++r) {
        for (int d = 0; d < 2; ++d) {
            uint64_t a = splitmix(rng), b = splitmix(rng);
            tabs[1].lower.push_back(std::min(a, b));
            tabs[1].upper.push_back(std::max(a, b));
        }
        tabs[1].ids.push_back(500 + r);
    }
    std::vector<hdx_region_table> handles(2);
    for (int t = 0; t < 2; ++t)
        CHECK(hdx_region_table_create((uint32_t)tabs[t].attrs.size(), (uint32_t)tabs[t].ids.size(),
                                      tabs[t].attrs.data(), tabs[t].lower.data(), tabs[t].upper.data(),
                                      tabs[t].ids.data(), &handles[t]));
    std::vector<uint64_t> want_ids(2 * n);
    for (int t = 0; t < 2; ++t)
        for (uint64_t i = 0; i < n; ++i) want_ids[t * n + i] = tabs[t].lookup(&want[i * A]);
    std::vector<uint64_t> host_ids(2 * n), host_coords(n * A);
    CHECK(hdx_hash_batch_regions_host(types.data(), A, blob.data(), total, base.data(), len.data(), n,
                                      handles.data(), 2, host_ids.data(), host_coords.data()));
    if (host_ids != want_ids || host_coords != want) {
        std::printf("FAIL hdx_hash_batch_regions_host\n");
        return 1;
    }
    std::vector<hdx_region_shard> rshards(nd);
    std::vector<void*> id_allocs(nd);
    for (int k = 0; k < nd; ++k) {
        HCHECK(hipSetDevice(devs[k]));
        HCHECK(hipMalloc(&id_allocs[k], 2 * n * 8));
        HCHECK(hipMemset(id_allocs[k], 0, 2 * n * 8));
        rshards[k] = hdx_region_shard{shards[k].blob, shards[k].obj_base, shards[k].attr_len, shards[k].n,
                                      (uint64_t*)id_allocs[k], nullptr, nullptr};
    }
    CHECK(hdx_hash_batch_regions_device_multi(types.data(), A, rshards.data(), (uint32_t)nd, handles.data(), 2, 1));
    std::vector<uint64_t> ids_back(2 * n);
    for (int k = 0; k < nd; ++k) {
        HCHECK(hipSetDevice(devs[k]));
        HCHECK(hipMemcpy(ids_back.data(), id_allocs[k], 2 * n * 8, hipMemcpyDeviceToHost));
        if (ids_back != want_ids) {
            std::printf("FAIL gathered region ids on device %d differ\n", devs[k]);
            return 1;
        }
        HCHECK(hipFree(id_allocs[k]));
    }
    for (auto h : handles) CHECK(hdx_region_table_destroy(h));

    for (size_t a = 0; a < allocs.size(); ++a) {
        HCHECK(hipSetDevice(devs[a / 4]));
        HCHECK(hipFree(allocs[a]));
    }
    CHECK(hdx_shutdown());
    std::printf("multi ok devices=%d objects=%llu shards=", nd, (unsigned long long)n);
    for (int k = 0; k < nd; ++k) std::printf("%llu%s", (unsigned long long)(first[k + 1] - first[k]), k + 1 < nd ? "," : "\n");
    return 0;
}
