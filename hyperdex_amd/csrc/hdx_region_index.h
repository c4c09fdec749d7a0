// hdx_region_index.h — the host side of configuration::lookup_region
// (common/configuration.cc:698-735): the interval index of a region table
// (built once at hdx_region_table_create, read by the region kernels,
// hdx_region_lookup.h) and the host lookup the batcher's calling-thread path
// uses.  Host-only, no HIP: tests/cpp/sanitize_test.cc builds it under
// ASan/UBSan.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <vector>

namespace hdx {

constexpr uint32_t kMaxLookupDims = 16;
// u64 words of a dimension's 257 u16 bucket starts (region_index_build),
// stored just below its boundaries
constexpr uint32_t kIndexBucketWords = 65;
// tables of more regions keep no index (lookups scan the boxes)
constexpr uint32_t kIndexMaxRegions = 256;

// ---------------------------------------------------------------------------
// Interval index.  For every subspace dimension d the table's box edges
// (lower[r][d] and upper[r][d] + 1) cut the u64 line into at most 2R+1
// intervals, and every point of one interval lies in the same set of the
// table's boxes on that dimension — a bit mask over the regions.  The first
// region (in table order) whose box holds the coordinates is then the lowest
// set bit of the AND of the D masks of the coordinates' intervals: exactly the
// reference's first-match scan (configuration.cc:698-735), overlapping or
// empty boxes included, at D binary searches instead of up to R*D compares.
// Layout, u64 words: D headers (m | boundaries offset << 16 | masks offset
// << 40), then per dimension: kIndexBucketWords words of u16 bucket starts
// (start[b] = boundaries <= b << 56, b = 0..256, so a coordinate whose top
// byte is b has its interval in [start[b], start[b + 1]]: the search is over
// that range only — zero or one step for the reference's equal partitions),
// its m sorted boundaries, and (m + 1) * W mask words.
// ---------------------------------------------------------------------------
inline void region_index_build(uint32_t D, uint32_t R, const uint64_t* lower, const uint64_t* upper,
                               std::vector<uint64_t>& index, uint32_t& W) {
    index.clear();
    W = 0;
    if (R == 0 || R > kIndexMaxRegions || D == 0 || D > kMaxLookupDims) return;
    W = (R + 63) / 64;
    index.assign(D, 0);
    std::vector<uint64_t> pts;
    for (uint32_t d = 0; d < D; ++d) {
        pts.clear();
        for (uint32_t r = 0; r < R; ++r) {
            pts.push_back(lower[(size_t)r * D + d]);
            if (upper[(size_t)r * D + d] != UINT64_MAX) pts.push_back(upper[(size_t)r * D + d] + 1);
        }
        std::sort(pts.begin(), pts.end());
        pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
        const uint64_t m = pts.size();
        uint16_t start[kIndexBucketWords * 4] = {};
        for (uint32_t b = 0; b <= 256; ++b)
            start[b] = (uint16_t)(b == 256 ? m
                                           : std::upper_bound(pts.begin(), pts.end(), (uint64_t)b << 56) - pts.begin());
        const size_t soff = index.size();
        index.resize(soff + kIndexBucketWords);
        std::memcpy(&index[soff], start, sizeof start);
        const uint64_t boff = index.size();
        index.insert(index.end(), pts.begin(), pts.end());
        const uint64_t moff = index.size();
        for (uint64_t i = 0; i <= m; ++i) {
            const uint64_t x = i == 0 ? 0 : pts[i - 1];  // a point of interval i (interval 0 may be empty)
            uint64_t mask[kIndexMaxRegions / 64] = {0, 0, 0, 0};
            for (uint32_t r = 0; r < R; ++r)
                if (lower[(size_t)r * D + d] <= x && x <= upper[(size_t)r * D + d]) mask[r >> 6] |= 1ull << (r & 63);
            index.insert(index.end(), mask, mask + W);
        }
        index[d] = m | (boff << 16) | (moff << 40);
    }
}

// The first region (table order) whose box holds hs[attrs[d]] on every
// dimension d (bounds inclusive), else 0 (region_id()): through the interval
// index when the table has one (per dimension the top byte's bucket, a binary
// search, the interval's mask; the lowest bit of the masks' AND — the device
// form is hdx_region_lookup.h's lookup_indexed_fn), else the reference's scan.
inline uint64_t region_lookup_arrays(uint32_t D, uint32_t R, uint32_t W, const uint16_t* attrs, const uint64_t* lower,
                                     const uint64_t* upper, const uint64_t* ids, const uint64_t* idx,
                                     const uint64_t* hs) {
    if (idx) {
        uint64_t acc[kIndexMaxRegions / 64] = {~0ull, ~0ull, ~0ull, ~0ull};
        for (uint32_t d = 0; d < D; ++d) {
            const uint64_t hdr = idx[d];
            const uint64_t* B = idx + ((hdr >> 16) & 0xffffff);
            const uint64_t hv = hs[attrs[d]];
            uint16_t start[2];
            std::memcpy(start, reinterpret_cast<const uint16_t*>(B - kIndexBucketWords) + (hv >> 56), sizeof start);
            uint32_t pos = start[0], cnt = start[1] - pos;
            while (cnt) {
                const uint32_t half = cnt >> 1;
                if (B[pos + half] <= hv) {
                    pos += half + 1;
                    cnt -= half + 1;
                } else {
                    cnt = half;
                }
            }
            const uint64_t* mask = idx + (hdr >> 40) + (size_t)pos * W;
            for (uint32_t w = 0; w < W; ++w) acc[w] &= mask[w];
        }
        for (uint32_t w = 0; w < W; ++w)
            if (acc[w]) return ids[64 * w + __builtin_ctzll(acc[w])];
        return 0;
    }
    for (uint32_t r = 0; r < R; ++r) {
        const uint64_t* lo = lower + (size_t)r * D;
        const uint64_t* up = upper + (size_t)r * D;
        bool in = true;
        for (uint32_t d = 0; in && d < D; ++d) {
            const uint64_t h = hs[attrs[d]];
            in = lo[d] <= h && h <= up[d];
        }
        if (in) return ids[r];
    }
    return 0;
}

}  // namespace hdx
