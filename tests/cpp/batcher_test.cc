// Daemon batching shim under concurrent callers, checked
// against the oracle (test infrastructure: oracle/hdx_oracle.c).
//
//   batcher_test <threads> <objects per thread> <max_objects> <slots> <delay_us> [flags]
//
// Every thread hashes random objects of a mixed schema (every CityHash regime,
// int64/float with special values, timestamps, a non-hashable attribute)
// through hdx_batcher_hash_object with two region tables attached, and checks
// every coordinate and region id; some objects exceed max_bytes (direct path)
// and some carry a mis-sized numeric value (HDX_E_BADSIZE, nothing queued).
// Exit 0 and "batcher ok" on success.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "hdxhash.h"
#include "hdx_oracle.h"

static const uint32_t kTypes[] = {9217, 9217, 9217, 9218, 9219, 9473, 9478, 9281, 9217};
static const uint32_t A = sizeof(kTypes) / sizeof(kTypes[0]);

struct Table {
    std::vector<uint16_t> attrs;
    std::vector<uint64_t> lower, upper, ids;
    uint32_t R = 0;
    hdx_region_table h = nullptr;
};

static Table make_table(std::vector<uint16_t> attrs, uint32_t servers, uint64_t first_id) {
    Table t;
    t.attrs = attrs;
    const uint32_t D = (uint32_t)attrs.size();
    t.R = (uint32_t)hdxo_partition(D, servers, nullptr, nullptr, 0);
    t.lower.resize((size_t)t.R * D);
    t.upper.resize((size_t)t.R * D);
    hdxo_partition(D, servers, t.lower.data(), t.upper.data(), t.R);
    for (uint32_t r = 0; r < t.R; ++r) t.ids.push_back(first_id + r);
    if (hdx_region_table_create(D, t.R, t.attrs.data(), t.lower.data(), t.upper.data(), t.ids.data(), &t.h) !=
        HDX_OK) {
        fprintf(stderr, "region table: %s\n", hdx_last_error());
        exit(2);
    }
    return t;
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 16;
    const int per_thread = argc > 2 ? atoi(argv[2]) : 2000;
    hdx_batcher_config cfg = {};
    cfg.max_objects = argc > 3 ? (uint32_t)atoi(argv[3]) : 0;
    cfg.slots = argc > 4 ? (uint32_t)atoi(argv[4]) : 0;
    cfg.max_delay_us = argc > 5 ? (uint32_t)atoi(argv[5]) : 0;
    cfg.flags = argc > 6 ? (uint32_t)atoi(argv[6]) : 0;
    cfg.host_max_bytes = argc > 7 ? (uint64_t)atoll(argv[7]) : 0;
    cfg.max_bytes = 64 << 10;  // objects above 64 KiB take the direct path
    cfg.device = -1;
    if (hdx_init(0) != HDX_OK) {
        fprintf(stderr, "init: %s\n", hdx_last_error());
        return 2;
    }
    Table key_space = make_table({0}, 64, 1);       // point_leader's subspace
    Table sub = make_table({1, 3, 4}, 64, 1000);    // a 3-attribute subspace
    hdx_region_table tables[2] = {key_space.h, sub.h};
    cfg.tables = tables;
    cfg.ntables = 2;
    hdx_batcher b = nullptr;
    if (hdx_batcher_create(kTypes, A, &cfg, &b) != HDX_OK) {
        fprintf(stderr, "create: %s\n", hdx_last_error());
        return 2;
    }
    std::atomic<long> failures(0), checked(0), badsize(0);
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            std::mt19937_64 rng(1234 + t);
            std::vector<std::vector<uint8_t>> vals(A);
            for (int k = 0; k < per_thread; ++k) {
                const bool huge = rng() % 997 == 0;
                const bool mis = rng() % 499 == 0;
                for (uint32_t j = 0; j < A; ++j) {
                    size_t L;
                    if (kTypes[j] == 9217 || kTypes[j] == 9281)
                        L = huge && j == 1 ? 70000 + rng() % 5000 : rng() % 200;
                    else
                        L = rng() % 50 == 0 ? 0 : 8;
                    if (mis && j == 3) L = 5;
                    vals[j].resize(L);
                    for (auto& c : vals[j]) c = (uint8_t)rng();
                    if (kTypes[j] == 9219 && L == 8 && rng() % 10 == 0) {
                        static const uint64_t sp[] = {0, 0x8000000000000000ull, 0x7ff0000000000000ull,
                                                      0xfff0000000000000ull, 0x7ff8000000000001ull, 1};
                        memcpy(vals[j].data(), &sp[rng() % 6], 8);
                    }
                }
                const uint8_t* vp[A];
                size_t vl[A];
                for (uint32_t j = 1; j < A; ++j) {
                    vp[j - 1] = vals[j].data();
                    vl[j - 1] = vals[j].size();
                }
                uint64_t hs[A], rid[2];
                const hdx_status st =
                    hdx_batcher_hash_object(b, vals[0].data(), vals[0].size(), vp, vl, hs, rid);
                if (mis) {
                    if (st != HDX_E_BADSIZE) {
                        fprintf(stderr, "thread %d obj %d: mis-sized value gave status %d\n", t, k, (int)st);
                        ++failures;
                    }
                    ++badsize;
                    continue;
                }
                if (st != HDX_OK) {
                    fprintf(stderr, "thread %d obj %d: status %d %s\n", t, k, (int)st, hdx_last_error());
                    ++failures;
                    continue;
                }
                uint64_t want[A];
                for (uint32_t j = 0; j < A; ++j) {
                    int err = 0;
                    want[j] = hdxo_hash_value(kTypes[j], vals[j].data(), vals[j].size(), &err);
                    if (hs[j] != want[j]) {
                        if (failures < 20)
                            fprintf(stderr, "thread %d obj %d attr %u: %016llx want %016llx\n", t, k, j,
                                    (unsigned long long)hs[j], (unsigned long long)want[j]);
                        ++failures;
                    }
                }
                uint64_t wr[2];
                hdxo_lookup_region(1, key_space.R, key_space.attrs.data(), key_space.lower.data(),
                                   key_space.upper.data(), key_space.ids.data(), want, A, 1, &wr[0]);
                hdxo_lookup_region(3, sub.R, sub.attrs.data(), sub.lower.data(), sub.upper.data(),
                                   sub.ids.data(), want, A, 1, &wr[1]);
                if (rid[0] != wr[0] || rid[1] != wr[1]) {
                    fprintf(stderr, "thread %d obj %d: regions %llu %llu want %llu %llu\n", t, k,
                            (unsigned long long)rid[0], (unsigned long long)rid[1],
                            (unsigned long long)wr[0], (unsigned long long)wr[1]);
                    ++failures;
                }
                ++checked;
            }
        });
    for (auto& th : pool) th.join();
    hdx_batcher_stats s;
    hdx_batcher_get_stats(b, &s);
    hdx_batcher_destroy(b);
    hdx_region_table_destroy(key_space.h);
    hdx_region_table_destroy(sub.h);
    printf("objects %llu batches %llu full %llu direct %llu host %llu checked %ld badsize %ld failures %ld\n",
           (unsigned long long)s.objects, (unsigned long long)s.batches, (unsigned long long)s.full_batches,
           (unsigned long long)s.direct, (unsigned long long)s.host, checked.load(), badsize.load(),
           failures.load());
    if (failures == 0 && checked + badsize == (long)threads * per_thread && s.objects == (uint64_t)checked) {
        printf("batcher ok\n");
        return 0;
    }
    return 1;
}
