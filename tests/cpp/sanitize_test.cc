// sanitize_test.cc — the product's host-only code under AddressSanitizer and
// UndefinedBehaviorSanitizer ("run the CPU path's unit tests under
// -fsanitize=address,undefined"), built and run by tests/test_sanitize.py:
//   * the per-object C-ABI (hdx_cpu.cpp: hdx_hash_value / hdx_hash_key /
//     hdx_hash_object) on values held in buffers of exactly their length, so
//     a read past a value's end is a reported error, against the oracle
//     (oracle/hdx_oracle.c, test infrastructure);
//   * the device set's byte-balanced cuts (hdx_cuts.h) against a direct
//     restatement of dist.shard_ranges' rule;
//   * the region tables' interval index and host lookup (hdx_region_index.h,
//     the batcher's calling-thread path) against the oracle's lookup_region,
//     index and scan, with every table array in an exact-size buffer;
//   * the device set's exchange plan (hdx_exchange.h: which collective moves
//     which rows) applied to per-device matrices holding only their own
//     rows, for equal, unequal and empty shards at world 1..8, coordinates
//     and region-id sections: every device must end with the full matrix;
//   * the cut rule over stored objects (key + value bytes, the host sweep).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cmath>
#include <memory>
#include <random>
#include <vector>

#include "hdx_cuts.h"
#include "hdx_exchange.h"
#include "hdx_host_common.h"
#include "hdx_region_index.h"

extern "C" {
#include "hdx_oracle.h"
}

namespace hdx {
// hdx_capi.cpp's error text is not linked here: keep the status.
hdx_status fail(hdx_status s, const char*, ...) { return s; }
}  // namespace hdx

static int failures = 0;
#define CHECK(c, ...)                                     \
    do {                                                  \
        if (!(c)) {                                       \
            if (failures++ < 20) {                        \
                fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
                fprintf(stderr, __VA_ARGS__);             \
                fputc('\n', stderr);                      \
            }                                             \
        }                                                 \
    } while (0)

// a value in a heap buffer of exactly n bytes (n == 0: a 1-byte buffer, unread)
struct Exact {
    std::unique_ptr<uint8_t[]> p;
    size_t n;
    Exact(std::mt19937_64& g, size_t len) : p(new uint8_t[len ? len : 1]), n(len) {
        for (size_t i = 0; i < len; ++i) p[i] = (uint8_t)g();
    }
};

static const uint32_t kTypes[] = {9217, 9218, 9219, 9473, 9474, 9475, 9476, 9477, 9478, 9223, 9281, 9417};

int main() {
    std::mt19937_64 g(0x4859504552444558ull);
    // every string length 0..600, each in its own exact buffer
    for (size_t n = 0; n <= 600; ++n) {
        Exact v(g, n);
        uint64_t h = 0;
        CHECK(hdx_hash_value(9217, v.p.get(), n, &h) == HDX_OK, "string %zu", n);
        CHECK(h == hdxo_cityhash64(v.p.get(), n), "string %zu: %llx vs %llx", n, (unsigned long long)h,
              (unsigned long long)hdxo_cityhash64(v.p.get(), n));
    }
    // numerics and timestamps: 0 and 8 bytes hash, other sizes are rejected
    for (uint32_t t : kTypes) {
        for (int rep = 0; rep < 2000; ++rep) {
            const size_t n = t == 9217 || t == 9223 || t == 9281 || t == 9417 ? g() % 80 : (rep % 5 == 0 ? 0 : 8);
            Exact v(g, n);
            uint64_t h = 0;
            int err = 0;
            const uint64_t want = hdxo_hash_value(t, v.p.get(), n, &err);
            CHECK(hdx_hash_value(t, v.p.get(), n, &h) == HDX_OK && err == 0 && h == want, "type %u len %zu", t, n);
        }
        if (t != 9217 && t != 9223 && t != 9281 && t != 9417) {
            Exact v(g, 7);
            uint64_t h = 0;
            CHECK(hdx_hash_value(t, v.p.get(), 7, &h) == HDX_E_BADSIZE, "type %u: 7 bytes accepted", t);
        }
    }
    uint64_t h = 0;
    CHECK(hdx_hash_value(12345, nullptr, 0, &h) == HDX_E_BADTYPE, "unknown type accepted");
    // whole objects: key + values of mixed types, every value its own buffer
    for (int rep = 0; rep < 3000; ++rep) {
        const uint32_t A = 1 + (uint32_t)(g() % 24);
        std::vector<uint32_t> types(A);
        std::vector<Exact> vals;
        vals.reserve(A);
        for (uint32_t j = 0; j < A; ++j) {
            types[j] = j == 0 ? 9217 : kTypes[g() % (sizeof(kTypes) / sizeof(kTypes[0]))];
            const bool num = types[j] == 9218 || types[j] == 9219 || (types[j] >= 9473 && types[j] <= 9478);
            vals.emplace_back(g, num ? (g() % 4 ? 8 : 0) : (size_t)(g() % 300));
        }
        std::vector<const uint8_t*> vp(A > 1 ? A - 1 : 1);
        std::vector<size_t> vl(A > 1 ? A - 1 : 1);
        for (uint32_t j = 1; j < A; ++j) {
            vp[j - 1] = vals[j].p.get();
            vl[j - 1] = vals[j].n;
        }
        std::vector<uint64_t> got(A);
        CHECK(hdx_hash_object(types.data(), A, vals[0].p.get(), vals[0].n, vp.data(), vl.data(), got.data()) == HDX_OK,
              "object %d", rep);
        for (uint32_t j = 0; j < A; ++j) {
            int err = 0;
            const uint64_t want = hdxo_hash_value(types[j], vals[j].p.get(), vals[j].n, &err);
            CHECK(err == 0 && got[j] == want, "object %d attr %u", rep, j);
        }
        uint64_t k = 0;
        CHECK(hdx_hash_key(types.data(), A, vals[0].p.get(), vals[0].n, &k) == HDX_OK && k == got[0], "key %d", rep);
    }
    // cuts: against a direct restatement of dist.shard_ranges (prefix sums as
    // float64, searchsorted side="left", equal counts within tol)
    for (int rep = 0; rep < 400; ++rep) {
        const uint64_t n = rep < 8 ? (uint64_t)rep : g() % 300000;
        const uint32_t A = 1 + (uint32_t)(g() % 17), world = 1 + (uint32_t)(g() % 9);
        const double tol = rep % 3 == 0 ? 0.0 : 1e-3;
        std::vector<uint32_t> len(n * A);
        const uint32_t spread = rep % 4 == 0 ? 1u : 1u + (uint32_t)(g() % 2000);
        for (auto& x : len) x = (uint32_t)(g() % spread);
        std::vector<uint64_t> first(world + 1);
        hdx::shard_cuts(len.data(), A, n, world, tol, first.data());
        std::vector<uint64_t> pre(n + 1, 0);
        for (uint64_t i = 0; i < n; ++i) {
            uint64_t s = 0;
            for (uint32_t j = 0; j < A; ++j) s += len[i * A + j];
            pre[i + 1] = pre[i] + s;
        }
        const uint64_t total = pre[n];
        std::vector<uint64_t> want(world + 1);
        bool even = tol > 0;
        for (uint32_t k = 0; k <= world; ++k) want[k] = (uint64_t)((unsigned __int128)n * k / world);
        if (even && total > 0) {
            const double share = (double)total / world;
            for (uint32_t k = 1; k <= world; ++k)
                if (std::abs((double)(pre[want[k]] - pre[want[k - 1]]) - share) > tol * share) even = false;
        }
        if (!even) {
            for (uint32_t k = 1; k < world; ++k) {
                const double target = (double)total * k / world;
                uint64_t i = 0;
                while (i <= n && (double)pre[i] < target) ++i;  // searchsorted(pre[1:], target): first i with pre >= target
                uint64_t c = i;  // cut before object c
                if (c > n) c = n;
                want[k] = std::min(std::max(c, want[k - 1]), n);
            }
            want[0] = 0;
            want[world] = n;
        }
        for (uint32_t k = 0; k <= world; ++k)
            CHECK(first[k] == want[k], "cuts rep %d (n %llu A %u world %u tol %g) k %u: %llu vs %llu", rep,
                  (unsigned long long)n, A, world, tol, k, (unsigned long long)first[k], (unsigned long long)want[k]);
    }
    // region tables: equal partitions (the reference's), random overlapping
    // and empty boxes, full-range bounds; coordinates at and beside every edge
    for (int rep = 0; rep < 300; ++rep) {
        const uint32_t D = 1 + (uint32_t)(g() % 4), A = D + (uint32_t)(g() % 5);
        const uint32_t R = rep % 10 == 0 ? 300 + (uint32_t)(g() % 40) : 1 + (uint32_t)(g() % 256);
        std::unique_ptr<uint64_t[]> lower(new uint64_t[(size_t)R * D]), upper(new uint64_t[(size_t)R * D]),
            ids(new uint64_t[R]);
        std::unique_ptr<uint16_t[]> attrs(new uint16_t[D]);
        for (uint32_t d = 0; d < D; ++d) attrs[d] = (uint16_t)((d * 7 + rep) % A);
        const int kind = rep % 3;
        for (uint32_t r = 0; r < R; ++r) {
            ids[r] = 1000 + r;
            for (uint32_t d = 0; d < D; ++d) {
                uint64_t lo, up;
                if (kind == 0) {  // equal partitions of the first dimension, others full
                    lo = d == 0 ? (uint64_t)(((unsigned __int128)r << 64) / R) : 0;
                    up = d == 0 ? (r + 1 == R ? UINT64_MAX : (uint64_t)(((unsigned __int128)(r + 1) << 64) / R) - 1)
                                : UINT64_MAX;
                } else {
                    uint64_t a = g(), b = g();
                    if (kind == 2) { a >>= 56; b >>= 56; a <<= 56; b <<= 56; }  // edges on bucket boundaries
                    lo = std::min(a, b);
                    up = std::max(a, b);
                    if (g() % 16 == 0) std::swap(lo, up);  // an empty box
                    if (g() % 16 == 0) up = UINT64_MAX;
                }
                lower[(size_t)r * D + d] = lo;
                upper[(size_t)r * D + d] = up;
            }
        }
        std::vector<uint64_t> index;
        uint32_t W = 0;
        hdx::region_index_build(D, R, lower.get(), upper.get(), index, W);
        CHECK((R <= hdx::kIndexMaxRegions) == !index.empty(), "index presence R %u", R);
        std::unique_ptr<uint64_t[]> idx(new uint64_t[index.size() ? index.size() : 1]);
        if (!index.empty()) std::memcpy(idx.get(), index.data(), index.size() * 8);
        const uint64_t n = 2000;
        std::unique_ptr<uint64_t[]> hs(new uint64_t[n * A]), want(new uint64_t[n]);
        for (uint64_t i = 0; i < n * A; ++i) {
            const uint64_t e = lower[(g() % R) * D + g() % D];
            switch (g() % 4) {
                case 0: hs[i] = g(); break;
                case 1: hs[i] = e; break;
                case 2: hs[i] = e - 1; break;
                default: hs[i] = upper[(g() % R) * D + g() % D] + (g() % 2); break;
            }
        }
        hdxo_lookup_region(D, R, attrs.get(), lower.get(), upper.get(), ids.get(), hs.get(), A, n, want.get());
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t* row = hs.get() + i * A;
            const uint64_t a = hdx::region_lookup_arrays(D, R, W, attrs.get(), lower.get(), upper.get(), ids.get(),
                                                         index.empty() ? nullptr : idx.get(), row);
            const uint64_t b = hdx::region_lookup_arrays(D, R, W, attrs.get(), lower.get(), upper.get(), ids.get(),
                                                         nullptr, row);
            CHECK(a == want[i] && b == want[i], "regions rep %d (D %u R %u kind %d) object %llu: %llu / %llu vs %llu",
                  rep, D, R, kind, (unsigned long long)i, (unsigned long long)a, (unsigned long long)b,
                  (unsigned long long)want[i]);
        }
    }
    // exchange plans: equal / unequal / empty shards, world 1..8, coordinate
    // rows (one section of N * A) and region-id sections (T sections of N)
    for (int rep = 0; rep < 600; ++rep) {
        const uint32_t world = 1 + (uint32_t)(g() % 8);
        std::vector<uint64_t> counts(world);
        const int kind = rep % 4;
        for (auto& c : counts) c = kind == 0 ? 37 : (uint64_t)(g() % (kind == 3 ? 3 : 200));  // kind 3: many empty
        if (kind == 1 && world > 1) counts[g() % world] = 0;
        const bool ids = rep % 2 == 1;
        const uint32_t A = 1 + (uint32_t)(g() % 20), T = 1 + (uint32_t)(g() % 4);
        uint64_t N = 0;
        for (auto c : counts) N += c;
        const uint64_t row = ids ? 1 : A, sections = ids ? T : 1, stride = ids ? N : N * A;
        const std::vector<hdx::ExchangeOp> plan = hdx::exchange_plan(counts.data(), world, row, (uint32_t)sections, stride);
        bool equal = true;
        for (auto c : counts) equal = equal && c == counts[0];
        uint64_t nonempty = 0;
        for (auto c : counts) nonempty += c != 0;
        const size_t want_ops = N == 0 ? 0 : equal ? sections : sections * nonempty;
        CHECK(plan.size() == want_ops, "plan rep %d: %zu ops, want %zu", rep, plan.size(), want_ops);
        // the full matrix, and each device holding only its own rows (others poisoned)
        std::vector<uint64_t> full(sections * stride);
        for (auto& x : full) x = g();
        std::vector<std::vector<uint64_t>> mats(world, std::vector<uint64_t>(full.size(), 0xdeadbeefdeadbeefull));
        uint64_t first = 0;
        for (uint32_t k = 0; k < world; ++k) {
            for (uint64_t s2 = 0; s2 < sections; ++s2)
                for (uint64_t e = first * row; e < (first + counts[k]) * row; ++e)
                    mats[k][s2 * stride + e] = full[s2 * stride + e];
            first += counts[k];
        }
        hdx::exchange_apply(plan, mats);
        for (uint32_t k = 0; k < world; ++k)
            CHECK(mats[k] == full, "plan rep %d (world %u, %s): device %u's matrix differs", rep, world,
                  ids ? "ids" : "coords", k);
        // bytes a device receives: every row but its own, once per section
        for (uint32_t k = 0; k < world && N; ++k)
            CHECK(hdx::exchange_bytes_in(plan, world, k) == (N - counts[k]) * row * sections * 8,
                  "plan rep %d: device %u receives %llu bytes", rep, k,
                  (unsigned long long)hdx::exchange_bytes_in(plan, world, k));
    }
    // cuts over stored objects (key + value bytes) against a direct prefix search
    for (int rep = 0; rep < 200; ++rep) {
        const uint64_t n = rep < 5 ? (uint64_t)rep : g() % 200000;
        const uint32_t world = 1 + (uint32_t)(g() % 8);
        std::vector<uint32_t> kl(n), vl(n);
        for (uint64_t i = 0; i < n; ++i) {
            kl[i] = (uint32_t)(g() % 100);
            vl[i] = rep % 3 == 0 && i < n / 2 ? 0u : (uint32_t)(g() % 3000);
        }
        std::vector<uint64_t> first(world + 1);
        hdx::shard_cuts_of(hdx::StoredSizes{kl.data(), vl.data()}, n, world, 0.0, first.data());
        std::vector<uint64_t> pre(n + 1, 0);
        for (uint64_t i = 0; i < n; ++i) pre[i + 1] = pre[i] + kl[i] + vl[i];
        std::vector<uint64_t> want(world + 1);
        want[0] = 0;
        want[world] = n;
        for (uint32_t k = 1; k < world; ++k) {
            const double target = (double)pre[n] * k / world;
            uint64_t i = 0;
            while (i <= n && (double)pre[i] < target) ++i;
            want[k] = std::min(std::max(std::min(i, n), want[k - 1]), n);
        }
        for (uint32_t k = 0; k <= world; ++k)
            CHECK(first[k] == want[k], "stored cuts rep %d k %u: %llu vs %llu", rep, k, (unsigned long long)first[k],
                  (unsigned long long)want[k]);
    }
    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("sanitize_test ok\n");
    return 0;
}
