// hdx_regions.hip — coordinates -> region ids on gfx950.
//
// configuration::lookup_region (common/configuration.cc:698-735): the first
// region r of a subspace whose box holds the object's coordinates,
//   lower[r][a] <= hs[attrs[a]] <= upper[r][a]   for every subspace dimension a,
// else region_id() (0).  point_leader (:427-497) is the same lookup on subspace
// 0 (attrs = {0}).  One lane per object; the region table is staged in LDS
// once per workgroup and every lane walks it in the reference's order, so the
// table reads are LDS broadcasts.  The region boxes come from
// admin/partition.cc and are taken as input (coordinator-assigned ids,
// coordinator/coordinator.cc:586-596), never recomputed here.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <mutex>

#include "hdx_internal.h"
#include "hdx_region_lookup.h"

#ifndef HDX_DEBUG_BUILD
#define HDX_DEBUG_BUILD 0
#endif

namespace hdx {

// The interval index (region_index_build) is built on the host: hdx_region_index.h.

template <bool IN_LDS, bool INDEX = false>
__global__ void __launch_bounds__(256)
lookup_region_kernel(const RegionArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const uint64_t* lower = a.lower;
    const uint64_t* upper = a.upper;
    const uint64_t* ids = a.ids;
    const uint64_t* index = a.index;
    if (INDEX) {
        if (IN_LDS) {
            for (uint32_t k = threadIdx.x; k < a.index_words; k += blockDim.x) smem[k] = a.index[k];
            for (uint32_t k = threadIdx.x; k < a.R; k += blockDim.x) smem[a.index_words + k] = a.ids[k];
            __syncthreads();
            index = smem;
            ids = smem + a.index_words;
        }
        const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= a.n) return;
        uint64_t h[kMaxLookupDims];
        const uint64_t* row = a.coords + i * a.A;
#pragma unroll
        for (uint32_t d = 0; d < kMaxLookupDims; ++d)
            if (d < a.D) h[d] = row[a.attrs[d]];
        a.out[i] = lookup_indexed(index, a.W, a.D, h, ids);
        return;
    }
    if (IN_LDS) {
        const uint32_t box = a.R * a.D;
        for (uint32_t k = threadIdx.x; k < box; k += blockDim.x) {
            smem[k] = a.lower[k];
            smem[box + k] = a.upper[k];
        }
        for (uint32_t k = threadIdx.x; k < a.R; k += blockDim.x) smem[2 * box + k] = a.ids[k];
        __syncthreads();
        lower = smem;
        upper = smem + box;
        ids = smem + 2 * box;
    }
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint64_t h[kMaxLookupDims];
    const uint64_t* row = a.coords + i * a.A;
#pragma unroll
    for (uint32_t d = 0; d < kMaxLookupDims; ++d)
        if (d < a.D) h[d] = row[a.attrs[d]];
    uint64_t rid = 0;  // region_id()
    for (uint32_t r = 0; r < a.R; ++r) {
        bool match = true;
#pragma unroll
        for (uint32_t d = 0; d < kMaxLookupDims; ++d)
            if (d < a.D) match &= lower[r * a.D + d] <= h[d] && h[d] <= upper[r * a.D + d];
        if (match) {
            rid = ids[r];
            break;
        }
    }
    a.out[i] = rid;
}

hipError_t launch_lookup_region(const RegionArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    const uint64_t blocks = (a.n + 255) / 256;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    if (a.index) {
        const size_t lds = ((size_t)a.index_words + a.R) * 8;
        if (lds <= 48 * 1024)
            hipLaunchKernelGGL((lookup_region_kernel<true, true>), dim3((uint32_t)blocks), dim3(256), lds, stream, a);
        else
            hipLaunchKernelGGL((lookup_region_kernel<false, true>), dim3((uint32_t)blocks), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    const size_t lds = (size_t)a.R * a.D * 16 + (size_t)a.R * 8;
    if (lds <= 48 * 1024) {
        hipLaunchKernelGGL(lookup_region_kernel<true>, dim3((uint32_t)blocks), dim3(256), lds, stream, a);
    } else {
        hipLaunchKernelGGL(lookup_region_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
    }
    return hipGetLastError();
}

bool regions_by_lookup_pays(uint64_t n) {
#if HDX_DEBUG_BUILD
    if (hash_variant() == 235 || hash_variant() == 247) return true;
#endif
    return n >= kRegionLookupMinObjects;
}

uint64_t regions_chunk_objects(uint64_t n, uint32_t A) {
    uint64_t bytes = kRegionChunkBytes;
#if HDX_DEBUG_BUILD
    if (hash_variant() == 235 || hash_variant() == 247) bytes = 64ull << 20;  // tests: several chunks at small n
#endif
    return std::min<uint64_t>(n, std::max<uint64_t>(1, bytes / (8ull * A)));
}

// The regions scratch comes from a memory pool of the library's own per
// device that keeps up to one chunk cached between calls (the device's default
// pool returns freed memory at every synchronisation, so each call would map
// its chunk afresh); the pool is trimmed at hdx_shutdown.
static std::mutex g_pool_mu;
static hipMemPool_t g_pool[64];

static hipError_t region_pool(hipStream_t stream, hipMemPool_t* out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool[dev]) {
        hipMemPoolProps props{};
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        if ((e = hipMemPoolCreate(&g_pool[dev], &props)) != hipSuccess) {
            g_pool[dev] = nullptr;
            return e;
        }
        uint64_t keep = kRegionChunkBytes;
        (void)hipMemPoolSetAttribute(g_pool[dev], hipMemPoolAttrReleaseThreshold, &keep);
    }
    (void)stream;
    *out = g_pool[dev];
    return hipSuccess;
}

void trim_region_pools() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (hipMemPool_t p : g_pool)
        if (p) (void)hipMemPoolTrimTo(p, 0);
}

hipError_t regions_by_lookup(uint64_t n, uint32_t A, const SweepTable* t, uint32_t T, uint64_t* coords,
                             const RegionHashFn& hash, hipStream_t stream, bool* no_scratch) {
    *no_scratch = false;
    if (n == 0) return hipSuccess;
    const uint64_t chunk = coords ? n : regions_chunk_objects(n, A);
    uint64_t* scratch = nullptr;
    hipError_t e = hipSuccess;
    if (!coords) {
        hipMemPool_t pool = nullptr;
        e = region_pool(stream, &pool);
        if (e == hipSuccess) e = hipMallocFromPoolAsync((void**)&scratch, chunk * A * 8, pool, stream);
#if HDX_DEBUG_BUILD
        if (e == hipSuccess && hash_variant() == 247) {  // tests: the allocation "fails"
            (void)hipFreeAsync(scratch, stream);
            scratch = nullptr;
            e = hipErrorOutOfMemory;
        }
#endif
        if (e != hipSuccess) {
            // nothing launched yet: the caller runs its fused form, which
            // needs no scratch (no new out-of-memory failure)
            (void)hipGetLastError();
            *no_scratch = true;
            return hipSuccess;
        }
    }
    for (uint64_t first = 0; first < n && e == hipSuccess; first += chunk) {
        const uint64_t count = std::min(chunk, n - first);
        uint64_t* c = coords ? coords + first * A : scratch;
        if ((e = hash(first, count, c)) != hipSuccess) break;
        for (uint32_t k = 0; k < T && e == hipSuccess; ++k) {
            RegionArgs r{};
            r.lower = t[k].lower;
            r.upper = t[k].upper;
            r.ids = t[k].ids;
            r.index = t[k].index;
            r.W = t[k].W;
            r.index_words = t[k].index_words;
            r.coords = c;
            r.out = t[k].out + first;
            r.n = count;
            r.A = A;
            r.D = t[k].D;
            r.R = t[k].R;
            std::memcpy(r.attrs, t[k].attrs, sizeof r.attrs);
            e = launch_lookup_region(r, stream);
        }
    }
    if (scratch) {
        const hipError_t f = hipFreeAsync(scratch, stream);
        if (e == hipSuccess) e = f;
    }
    return e;
}

// One lane per (table, object): small batches from the daemon shim, where a
// launch per table would cost more than the lookups.  Every table's boxes
// and ids are staged in LDS per workgroup (the walk is then LDS broadcasts,
// as in lookup_region_kernel); tables too large for that are walked in global
// memory.
// A table with an interval index stages the index (in the lower slot) and its
// ids; one without stages its boxes and ids.
struct MultiLayout {
    uint32_t lower[kMaxMultiTables], upper[kMaxMultiTables], ids[kMaxMultiTables];  // u64 offsets
    uint32_t words;
};

__host__ __device__ inline MultiLayout multi_layout(const MultiRegionArgs& a) {
    MultiLayout l{};
    uint32_t w = 0;
    for (uint32_t t = 0; t < a.T; ++t) {
        const uint32_t box = a.t[t].index ? a.t[t].index_words : a.t[t].R * a.t[t].D;
        l.lower[t] = w;
        l.upper[t] = w + box;
        l.ids[t] = a.t[t].index ? w + box : w + 2 * box;
        w = l.ids[t] + a.t[t].R;
    }
    l.words = w;
    return l;
}

template <bool IN_LDS>
__global__ void __launch_bounds__(256) lookup_regions_multi_kernel(const MultiRegionArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    const MultiLayout l = multi_layout(a);
    if (IN_LDS) {
        for (uint32_t t = 0; t < a.T; ++t) {
            if (a.t[t].index) {
                for (uint32_t k = threadIdx.x; k < a.t[t].index_words; k += blockDim.x)
                    smem[l.lower[t] + k] = a.t[t].index[k];
            } else {
                const uint32_t box = a.t[t].R * a.t[t].D;
                for (uint32_t k = threadIdx.x; k < box; k += blockDim.x) {
                    smem[l.lower[t] + k] = a.t[t].lower[k];
                    smem[l.upper[t] + k] = a.t[t].upper[k];
                }
            }
            for (uint32_t k = threadIdx.x; k < a.t[t].R; k += blockDim.x) smem[l.ids[t] + k] = a.t[t].ids[k];
        }
        __syncthreads();
    }
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t t = g / a.n, i = g - t * a.n;
    if (t >= a.T) return;
    const MultiRegionArgs::Table& tb = a.t[t];
    const uint64_t* lower = IN_LDS ? smem + l.lower[t] : tb.lower;
    const uint64_t* upper = IN_LDS ? smem + l.upper[t] : tb.upper;
    const uint64_t* ids = IN_LDS ? smem + l.ids[t] : tb.ids;
    const uint64_t* row = a.coords + i * a.A;
    uint64_t h[kMaxLookupDims];
#pragma unroll
    for (uint32_t d = 0; d < kMaxLookupDims; ++d)
        if (d < tb.D) h[d] = row[tb.attrs[d]];
    if (tb.index) {
        a.out[t * a.out_stride + i] = lookup_indexed(IN_LDS ? smem + l.lower[t] : tb.index, tb.W, tb.D, h, ids);
        return;
    }
    uint64_t rid = 0;
    for (uint32_t r = 0; r < tb.R; ++r) {
        bool match = true;
#pragma unroll
        for (uint32_t d = 0; d < kMaxLookupDims; ++d)
            if (d < tb.D) match &= lower[r * tb.D + d] <= h[d] && h[d] <= upper[r * tb.D + d];
        if (match) {
            rid = ids[r];
            break;
        }
    }
    a.out[t * a.out_stride + i] = rid;
}

hipError_t launch_lookup_regions_multi(const MultiRegionArgs& a, hipStream_t stream) {
    const uint64_t work = a.n * a.T;
    if (work == 0) return hipSuccess;
    const uint64_t blocks = (work + 255) / 256;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    const size_t lds = (size_t)multi_layout(a).words * 8;
    if (lds <= 48 * 1024)
        hipLaunchKernelGGL(lookup_regions_multi_kernel<true>, dim3((uint32_t)blocks), dim3(256), lds, stream, a);
    else
        hipLaunchKernelGGL(lookup_regions_multi_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
