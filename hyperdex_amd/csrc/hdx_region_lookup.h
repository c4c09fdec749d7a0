// hdx_region_lookup.h — configuration::lookup_region's first-match test
// (common/configuration.cc:698-735) as device functions, shared by the region
// kernels (hdx_regions.hip) and the fused reindex sweep (hdx_encoded.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_internal.h"
#include "hdx_region_index.h"

namespace hdx {

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

// configuration::lookup_region for a wave's nobj objects whose coordinates are
// parked in LDS (coords[o * A + j]), every table of tabs[0..T): indexed tables
// with one lane per (object, table dimension) — each searches its interval
// and parks the mask words in the scratch (LDS, nobj * sum(D) * 32 bytes) —
// then one lane per (object, table) ANDs them: a few dependent round trips
// for all the tables instead of ~3 per dimension one after another.  Scanned
// tables, or more than 64 searches: lane = object, table by table.  Region
// ids go to tabs[t].out[o0 + o].  The whole wave calls it.
template <class FENCE>
__device__ __forceinline__ void lookup_tables_wave(const SweepTable* tabs, uint32_t T, const uint64_t* coords,
                                                   uint32_t A, uint32_t nobj, uint64_t o0, uint64_t* scratch,
                                                   FENCE fence) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t P = 0;
    bool all_indexed = true;
    for (uint32_t t = 0; t < T; ++t) {
        P += tabs[t].D;
        all_indexed &= tabs[t].index != nullptr;
    }
    if (all_indexed && nobj * P <= 64) {
        if (lane < nobj * P) {
            const uint32_t o = lane / P, p = lane - o * P;
            uint32_t t = 0, d = p;
            while (d >= tabs[t].D) d -= tabs[t++].D;
            const SweepTable& tb = tabs[t];
            const uint64_t hv = coords[o * A + tb.attrs[d]];
            const uint64_t hdr = tb.index[d];
            const uint64_t* B = tb.index + ((hdr >> 16) & 0xffffff);
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
            const uint64_t* mask = tb.index + (hdr >> 40) + (size_t)pos * tb.W;
#pragma unroll
            for (uint32_t w = 0; w < 4; ++w) scratch[(o * P + p) * 4 + w] = w < tb.W ? mask[w] : 0;
        }
        fence();
        if (lane < nobj * T) {
            const uint32_t o = lane / T, t = lane - o * T;
            uint32_t p0 = 0;
            for (uint32_t u = 0; u < t; ++u) p0 += tabs[u].D;
            const SweepTable& tb = tabs[t];
            uint64_t acc[4] = {~0ull, ~0ull, ~0ull, ~0ull};
            for (uint32_t d = 0; d < tb.D; ++d)
#pragma unroll
                for (uint32_t w = 0; w < 4; ++w) acc[w] &= scratch[(o * P + p0 + d) * 4 + w];
            uint64_t r = 0;
#pragma unroll
            for (int w = 3; w >= 0; --w)
                if ((uint32_t)w < tb.W && acc[w]) r = tb.ids[64 * w + __builtin_ctzll(acc[w])];
            tb.out[o0 + o] = r;
        }
    } else if (lane < nobj) {
        const uint64_t* po = coords + lane * A;
        for (uint32_t t = 0; t < T; ++t) {
            const SweepTable& tb = tabs[t];
            uint64_t r;
            if (tb.index) {
                r = lookup_indexed_fn(tb.index, tb.W, tb.D, [&](uint32_t d) { return po[tb.attrs[d]]; }, tb.ids);
            } else {
                uint64_t h[kMaxLookupDims];
#pragma unroll
                for (uint32_t d = 0; d < kMaxLookupDims; ++d)
                    if (d < tb.D) h[d] = po[tb.attrs[d]];
                r = lookup_scan(tb.lower, tb.upper, tb.ids, tb.R, tb.D, h);
            }
            tb.out[o0 + lane] = r;
        }
    }
}

}  // namespace hdx
