// Throughput and latency of the daemon batching shim.
//
//   batcher_bench [threads] [seconds] [max_objects] [delay_us] [tables] [flags] [host_max_bytes] [scale]
//
// `threads` callers (daemon::loop threads) each hash config-3b objects (key
// STRING 64 B; 10 STRING U{0..195}; 3 INT64; 3 FLOAT) through
// hdx_batcher_hash_object back to back for `seconds`, with `tables` region
// tables attached (0-3: the key subspace and two 3-attribute subspaces, the
// prev/this/next lookups of key_state::hash_objects).  Objects are
// pre-generated so the timed loop is staging + waiting only.  Prints one JSON
// line: objects/s, batches, mean batch size and caller latency percentiles.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <random>
#include <thread>
#include <vector>

#include "hdxhash.h"

using Clock = std::chrono::steady_clock;

static const uint32_t A = 17;

static hdx_region_table grid(std::vector<uint16_t> attrs, uint32_t cells_per_dim, uint64_t first_id) {
    // a regular grid over the attrs (the partition() shape for these sizes)
    const uint32_t D = (uint32_t)attrs.size();
    uint32_t R = 1;
    for (uint32_t d = 0; d < D; ++d) R *= cells_per_dim;
    std::vector<uint64_t> lo((size_t)R * D), up((size_t)R * D), ids(R);
    const uint64_t step = UINT64_MAX / cells_per_dim;
    for (uint32_t r = 0; r < R; ++r) {
        uint32_t x = r;
        for (uint32_t d = 0; d < D; ++d) {
            const uint32_t c = x % cells_per_dim;
            x /= cells_per_dim;
            lo[(size_t)r * D + d] = c * step + (c ? 1 : 0);
            up[(size_t)r * D + d] = c + 1 == cells_per_dim ? UINT64_MAX : (c + 1) * step;
        }
        ids[r] = first_id + r;
    }
    hdx_region_table t = nullptr;
    if (hdx_region_table_create(D, R, attrs.data(), lo.data(), up.data(), ids.data(), &t) != HDX_OK) {
        fprintf(stderr, "table: %s\n", hdx_last_error());
        exit(2);
    }
    return t;
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 16;
    const double seconds = argc > 2 ? atof(argv[2]) : 3.0;
    hdx_batcher_config cfg = {};
    cfg.max_objects = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
    cfg.max_delay_us = argc > 4 ? (uint32_t)atoi(argv[4]) : 0;
    const uint32_t ntables = argc > 5 ? (uint32_t)atoi(argv[5]) : 3;
    cfg.flags = argc > 6 ? (uint32_t)atoi(argv[6]) : 0;
    cfg.host_max_bytes = argc > 7 ? (uint64_t)atoll(argv[7]) : 0;
    // scale > 1 multiplies every string length (object-size sweeps for the crossover)
    const uint32_t scale = argc > 8 ? (uint32_t)atoi(argv[8]) : 1;
    cfg.device = -1;
    if (hdx_init(0) != HDX_OK) {
        fprintf(stderr, "init: %s\n", hdx_last_error());
        return 2;
    }
    uint32_t types[A];
    types[0] = 9217;
    for (int j = 1; j <= 10; ++j) types[j] = 9217;
    for (int j = 11; j <= 13; ++j) types[j] = 9218;
    for (int j = 14; j <= 16; ++j) types[j] = 9219;
    hdx_region_table tables[3] = {grid({0}, 64, 1), grid({1, 11, 14}, 4, 100), grid({2, 12, 15}, 4, 200)};
    cfg.tables = tables;
    cfg.ntables = std::min(ntables, 3u);
    hdx_batcher b = nullptr;
    if (hdx_batcher_create(types, A, &cfg, &b) != HDX_OK) {
        fprintf(stderr, "create: %s\n", hdx_last_error());
        return 2;
    }
    // pre-generated objects, 1024 per thread, reused round robin
    const int kObj = scale > 16 ? 64 : 1024;
    struct Obj {
        std::vector<uint8_t> bytes;
        size_t len[A];
    };
    std::vector<std::vector<Obj>> objs(threads);
    for (int t = 0; t < threads; ++t) {
        std::mt19937_64 rng(77 + t);
        objs[t].resize(kObj);
        for (auto& o : objs[t]) {
            size_t total = 0;
            for (uint32_t j = 0; j < A; ++j) {
                o.len[j] = j == 0 ? 64 : j <= 10 ? (rng() % 196) * scale : (rng() % 100 == 0 ? 0 : 8);
                total += o.len[j];
            }
            o.bytes.resize(total);
            for (auto& c : o.bytes) c = (uint8_t)rng();
        }
    }
    std::atomic<bool> go(false), stop(false);
    std::atomic<long> errors(0);
    std::vector<std::vector<float>> lat(threads);
    std::vector<long> done(threads, 0);
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            lat[t].reserve(1 << 20);
            while (!go.load()) std::this_thread::yield();
            uint64_t hs[A], rid[3];
            const uint8_t* vp[A];
            size_t vl[A];
            long k = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                const Obj& o = objs[t][k % kObj];
                size_t off = o.len[0];
                for (uint32_t j = 1; j < A; ++j) {
                    vp[j - 1] = o.bytes.data() + off;
                    vl[j - 1] = o.len[j];
                    off += o.len[j];
                }
                const auto t0 = Clock::now();
                if (hdx_batcher_hash_object(b, o.bytes.data(), o.len[0], vp, vl, hs, rid) != HDX_OK) ++errors;
                const auto t1 = Clock::now();
                if (lat[t].size() < lat[t].capacity())
                    lat[t].push_back(std::chrono::duration<float, std::micro>(t1 - t0).count());
                ++k;
            }
            done[t] = k;
        });
    // warm up 0.3 s, then measure
    go = true;
    std::this_thread::sleep_for(std::chrono::milliseconds(300));
    hdx_batcher_stats s0;
    hdx_batcher_get_stats(b, &s0);
    const auto t0 = Clock::now();
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    hdx_batcher_stats s1;
    hdx_batcher_get_stats(b, &s1);
    const double el = std::chrono::duration<double>(Clock::now() - t0).count();
    stop = true;
    for (auto& th : pool) th.join();
    std::vector<float> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : (double)all[(size_t)(p * (all.size() - 1))]; };
    const double objs_s = (double)(s1.objects - s0.objects) / el;
    const double batches = (double)(s1.batches - s0.batches);
    printf("{\"tool\": \"batcher_bench\", \"threads\": %d, \"tables\": %u, \"max_objects\": %u, "
           "\"max_delay_us\": %u, \"flags\": %u, \"objects_per_s\": %.0f, \"batches_per_s\": %.0f, "
           "\"mean_batch\": %.1f, \"full_batches\": %llu, \"lat_us_p50\": %.1f, \"lat_us_p90\": %.1f, "
           "\"lat_us_p99\": %.1f, \"lat_us_max\": %.1f, \"errors\": %ld, \"host_objects_per_s\": %.0f, "
           "\"host_max_bytes\": %llu, \"scale\": %u}\n",
           threads, cfg.ntables, cfg.max_objects ? cfg.max_objects : 4096,
           cfg.max_delay_us ? cfg.max_delay_us : 50, cfg.flags, objs_s, batches / el,
           batches > 0 ? (double)(s1.objects - s0.objects) / batches : 0.0,
           (unsigned long long)(s1.full_batches - s0.full_batches), pct(0.5), pct(0.9), pct(0.99),
           pct(1.0), errors.load(), (double)(s1.host - s0.host) / el, (unsigned long long)cfg.host_max_bytes,
           scale);
    hdx_batcher_destroy(b);
    for (auto t : tables) hdx_region_table_destroy(t);
    return errors.load() ? 1 : 0;
}
