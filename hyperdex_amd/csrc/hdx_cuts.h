// hdx_cuts.h — byte-balanced contiguous object ranges for the device set
// (hdx_multi.cpp: hdx_shard_ranges, hdx_hash_batch_host over the set), the
// rule of hyperdex_amd/dist.py:shard_ranges restated in C++, over a packed
// batch's attribute lengths or stored objects' key + value lengths.  Host-only, no
// HIP: tests/cpp/sanitize_test.cc builds it under ASan/UBSan.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace hdx {

// Object sizes are the sums of their attribute lengths.  Every prefix is an
// exact integer (< 2^53), so comparing it as a double against
// total * k / world reproduces numpy's float64 searchsorted(side="left")
// bit for bit.  The prefix at any object is a block prefix plus a scan of
// at most one block, so the lengths are read once (in parallel by the
// device workers when there are any) plus one block per cut.
constexpr uint64_t kCutBlock = 1ull << 16;  // objects per prefix block

inline uint64_t object_bytes(const uint32_t* attr_len, uint32_t A, uint64_t i) {
    uint64_t s = 0;
    const uint32_t* l = attr_len + i * A;
    for (uint32_t j = 0; j < A; ++j) s += l[j];
    return s;
}

// Object sizes of a packed batch: the sums of its attribute lengths.
struct PackedSizes {
    const uint32_t* attr_len;
    uint32_t A;
    uint64_t operator()(uint64_t i) const { return object_bytes(attr_len, A, i); }
};
// Object sizes of stored objects (hdx_hash_encoded_host): key + value bytes.
struct StoredSizes {
    const uint32_t* key_len;
    const uint32_t* val_len;
    uint64_t operator()(uint64_t i) const { return (uint64_t)key_len[i] + val_len[i]; }
};

template <typename Sizes>
inline uint64_t block_bytes(const Sizes& size, uint64_t n, uint64_t b) {
    const uint64_t lo = b * kCutBlock, hi = std::min(n, lo + kCutBlock);
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += size(i);
    return s;
}
inline uint64_t block_bytes(const uint32_t* attr_len, uint32_t A, uint64_t n, uint64_t b) {
    return block_bytes(PackedSizes{attr_len, A}, n, b);
}

// bprefix[b] = bytes of objects [0, b * kCutBlock), b in [0, blocks]
template <typename Sizes>
struct PrefixOf {
    Sizes size;
    uint64_t n;
    std::vector<uint64_t> bprefix;
    uint64_t at(uint64_t i) const {  // bytes of objects [0, i)
        const uint64_t b = i / kCutBlock;
        uint64_t s = bprefix[b];
        for (uint64_t k = b * kCutBlock; k < i; ++k) s += size(k);
        return s;
    }
    // first i in [0, n] with prefix(i) >= target (numpy searchsorted, side="left")
    uint64_t search(double target) const {
        const uint64_t blocks = bprefix.size() - 1;
        uint64_t lo = 0, hi = blocks;  // last block b with (double)bprefix[b] < target
        if (!((double)bprefix[0] < target)) return 0;
        while (lo < hi) {
            const uint64_t mid = (lo + hi + 1) / 2;
            if ((double)bprefix[mid] < target) lo = mid; else hi = mid - 1;
        }
        uint64_t i = lo * kCutBlock, s = bprefix[lo];
        while (i < n && (double)s < target) s += size(i++);
        return (double)s < target ? n : i;
    }
};
using Prefix = PrefixOf<PackedSizes>;

template <typename Sizes>
inline void cuts_from_prefix(const PrefixOf<Sizes>& p, uint32_t world, double tol, uint64_t* first) {
    const uint64_t n = p.n;
    std::vector<uint64_t> even(world + 1);
    for (uint32_t k = 0; k <= world; ++k) even[k] = (uint64_t)((unsigned __int128)n * k / world);
    const uint64_t total = p.bprefix.back();
    if (tol > 0) {  // dist._within: every equal-count shard within tol of the mean share
        bool ok = true;
        if (total > 0) {
            const double share = (double)total / world;
            uint64_t a = 0;
            for (uint32_t k = 1; k <= world && ok; ++k) {
                const uint64_t b = p.at(even[k]);
                ok = std::abs((double)(b - a) - share) <= tol * share;
                a = b;
            }
        }
        if (ok) {
            std::memcpy(first, even.data(), (world + 1) * sizeof(uint64_t));
            return;
        }
    }
    first[0] = 0;
    for (uint32_t k = 1; k < world; ++k) {
        const uint64_t c = p.search((double)total * k / world);
        first[k] = std::min(std::max(c, first[k - 1]), n);
    }
    first[world] = n;
}

// The cuts of n objects of sizes size(i) over world ranges: first[k] = range
// k's first object, first[world] = n.
template <typename Sizes>
inline void shard_cuts_of(const Sizes& size, uint64_t n, uint32_t world, double tol, uint64_t* first) {
    PrefixOf<Sizes> p{size, n, {}};
    const uint64_t blocks = (n + kCutBlock - 1) / kCutBlock;
    p.bprefix.assign(blocks + 1, 0);
    for (uint64_t b = 0; b < blocks; ++b) p.bprefix[b + 1] = p.bprefix[b] + block_bytes(size, n, b);
    cuts_from_prefix(p, world, tol, first);
}

// The same over a packed batch's attribute lengths; attr_len NULL: counts
// that differ by at most one.
inline void shard_cuts(const uint32_t* attr_len, uint32_t A, uint64_t n, uint32_t world, double tol, uint64_t* first) {
    if (!attr_len) {
        for (uint32_t k = 0; k <= world; ++k) first[k] = (uint64_t)((unsigned __int128)n * k / world);
        return;
    }
    shard_cuts_of(PackedSizes{attr_len, A}, n, world, tol, first);
}

}  // namespace hdx
