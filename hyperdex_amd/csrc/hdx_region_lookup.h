// hdx_region_lookup.h — configuration::lookup_region's first-match test
// (common/configuration.cc:698-735) as device functions, shared by the region
// kernels (hdx_regions.hip) and the fused reindex sweep (hdx_encoded.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hdx {

constexpr uint32_t kMaxLookupDims = 16;
// u64 words of a dimension's 257 u16 bucket starts (region_index_build),
// stored just below its boundaries
constexpr uint32_t kIndexBucketWords = 65;

// Region id of coordinates hd(0..D) through the interval index idx (hd reads
// one coordinate, so a caller holding them in LDS need not copy them out).
template <class HD>
__device__ __forceinline__ uint64_t lookup_indexed_fn(const uint64_t* idx, uint32_t W, uint32_t D, HD hd,
                                                      const uint64_t* ids) {
    uint64_t acc[4] = {~0ull, ~0ull, ~0ull, ~0ull};
#pragma unroll
    for (uint32_t d = 0; d < kMaxLookupDims; ++d) {
        if (d >= D) break;
        const uint64_t hdr = idx[d];
        const uint64_t* B = idx + ((hdr >> 16) & 0xffffff);
        // number of boundaries <= h[d]: the top byte's bucket bounds it to
        // [start[b], start[b + 1]], then a binary search over that range
        const uint64_t hv = hd(d);
        const uint16_t* start = reinterpret_cast<const uint16_t*>(B - kIndexBucketWords);
        const uint32_t b = (uint32_t)(hv >> 56);
        uint32_t pos = start[b], cnt = start[b + 1] - pos;
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
#pragma unroll
        for (uint32_t w = 0; w < 4; ++w)
            if (w < W) acc[w] &= mask[w];
    }
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w)
        if (w < W && acc[w]) return ids[64 * w + __builtin_ctzll(acc[w])];
    return 0;  // region_id()
}

__device__ __forceinline__ uint64_t lookup_indexed(const uint64_t* idx, uint32_t W, uint32_t D, const uint64_t* h,
                                                   const uint64_t* ids) {
    return lookup_indexed_fn(idx, W, D, [h](uint32_t d) { return h[d]; }, ids);
}

// The reference's scan: the first region whose box holds h on every dimension.
__device__ __forceinline__ uint64_t lookup_scan(const uint64_t* lower, const uint64_t* upper, const uint64_t* ids,
                                                uint32_t R, uint32_t D, const uint64_t* h) {
    for (uint32_t r = 0; r < R; ++r) {
        bool match = true;
#pragma unroll
        for (uint32_t d = 0; d < kMaxLookupDims; ++d)
            if (d < D) match &= lower[r * D + d] <= h[d] && h[d] <= upper[r * D + d];
        if (match) return ids[r];
    }
    return 0;  // region_id()
}

}  // namespace hdx
