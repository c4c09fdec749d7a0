// hdx_gather.hip — packing scattered extents into device staging (the
// host-resident pipelines, hdx_hostpath.cpp).
//
// A host batch whose objects do not lie in index order (DESIGN §2 allows any
// order and gaps) cannot be moved as one span per chunk without dragging every
// gap byte across PCIe.  Instead the pipeline uploads the chunk's extents
// (source offset, length, packed destination offset) and this kernel reads
// the caller's pinned memory through its device mapping and writes the
// extents back to back into the slot's device staging — in index order, so
// the hash kernels see a packed batch (the wave-staged kernels' span DMA
// needs objects back to back).
//
// One wave per extent: lane l reads the 16-byte-aligned source chunk l of the
// extent (aligned chunks never cross a page, so nothing outside the pages the
// extent lives in is read), takes lane l+1's chunk by shuffle, funnel-shifts
// the pair to the destination's alignment and stores one aligned 16-byte
// chunk; the two chunks at the extent's ends, shared with the neighbouring
// extents, are written byte by byte.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "hdx_internal.h"

namespace hdx {

namespace {
struct GatherArgs {
    const uint8_t* src;      // device view of the source (pinned host memory)
    const uint64_t* src_off; // [n]
    const uint32_t* len;     // [n]
    const uint64_t* dst_off; // [n]
    uint8_t* dst;
    uint64_t n;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pick(const uint32_t (&w)[8], uint32_t k, uint32_t i, uint32_t b) {
    return __builtin_amdgcn_alignbyte(w[k + i + 1], w[k + i], b);
}
}  // namespace

__global__ void __launch_bounds__(256) gather_extents_kernel(const GatherArgs g) {
    const int lane = threadIdx.x & 63;
    for (uint64_t e = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); e < g.n; e += (uint64_t)gridDim.x * 4) {
        const uint32_t L = g.len[e];
        if (L == 0) continue;
        const uint8_t* s = g.src + g.src_off[e];
        uint8_t* d = g.dst + g.dst_off[e];
        const uint32_t lead = (uint32_t)((uintptr_t)s & 15), dlead = (uint32_t)((uintptr_t)d & 15);
        const u32x4* sa = (const u32x4*)(s - lead);
        u32x4* da = (u32x4*)(d - dlead);
        // 64-bit chunk and byte positions: an extent may reach 4 GiB
        const int64_t nsc = (int64_t)(((uint64_t)lead + L + 15) >> 4), ndc = (int64_t)(((uint64_t)dlead + L + 15) >> 4);
        const int sh = (int)lead - (int)dlead;     // -15 .. 15
        const int bofs = sh < 0 ? -1 : 0;
        const uint32_t r = (uint32_t)(sh - 16 * bofs);  // 0 .. 15: the pair's byte offset
        const uint32_t k = r >> 2, b = r & 3;           // wave-uniform
        for (int64_t q0 = 0; q0 < ndc; q0 += 64) {
            const int64_t q = q0 + lane, c = q + bofs;
            const u32x4 zero = {0u, 0u, 0u, 0u};
            const u32x4 x = c >= 0 && c < nsc ? __builtin_nontemporal_load(sa + c) : zero;
            u32x4 y;
            y.x = (uint32_t)__shfl((int)x.x, (lane + 1) & 63, 64);
            y.y = (uint32_t)__shfl((int)x.y, (lane + 1) & 63, 64);
            y.z = (uint32_t)__shfl((int)x.z, (lane + 1) & 63, 64);
            y.w = (uint32_t)__shfl((int)x.w, (lane + 1) & 63, 64);
            if (lane == 63) y = c + 1 >= 0 && c + 1 < nsc ? __builtin_nontemporal_load(sa + c + 1) : zero;
            if (q >= ndc) continue;
            const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
            u32x4 o;
            switch (k) {  // wave-uniform
                case 0: o = {pick(w, 0, 0, b), pick(w, 0, 1, b), pick(w, 0, 2, b), pick(w, 0, 3, b)}; break;
                case 1: o = {pick(w, 1, 0, b), pick(w, 1, 1, b), pick(w, 1, 2, b), pick(w, 1, 3, b)}; break;
                case 2: o = {pick(w, 2, 0, b), pick(w, 2, 1, b), pick(w, 2, 2, b), pick(w, 2, 3, b)}; break;
                default: o = {pick(w, 3, 0, b), pick(w, 3, 1, b), pick(w, 3, 2, b), pick(w, 3, 3, b)}; break;
            }
            // dst chunk q holds object bytes [16q - dlead, 16q - dlead + 16)
            const int64_t j0 = 16 * q - (int64_t)dlead;
            if (j0 >= 0 && j0 + 16 <= (int64_t)L) {
                da[q] = o;
            } else {
                const uint32_t ob[4] = {o.x, o.y, o.z, o.w};
                uint8_t* dq = (uint8_t*)(da + q);
                for (int t = 0; t < 16; ++t)
                    if (j0 + t >= 0 && j0 + t < (int64_t)L) dq[t] = (uint8_t)(ob[t >> 2] >> (8 * (t & 3)));
            }
        }
    }
}

// Up to eight contiguous arrays copied by the compute queue (dwords; the
// sources device views of pinned host memory): the chunk's offsets, sizes and
// lengths reach the device without an SDMA copy that the gather would wait on
// (the pipeline's two slots share one hardware queue).
namespace {
struct LinearCopies {
    const uint32_t* src[8];
    uint32_t* dst[8];
    uint64_t dwords[8];
    uint32_t count;
};
}  // namespace

__global__ void __launch_bounds__(256) copy_linear_kernel(const LinearCopies c) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint32_t r = 0; r < c.count; ++r)
        for (uint64_t d = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; d < c.dwords[r]; d += stride)
            c.dst[r][d] = __builtin_nontemporal_load(c.src[r] + d);
}

hipError_t launch_copy_linear(const void* const* src, void* const* dst, const uint64_t* bytes, uint32_t count,
                              hipStream_t stream) {
    LinearCopies c{};
    uint64_t most = 0;
    if (count > 8) return hipErrorInvalidValue;
    for (uint32_t r = 0; r < count; ++r) {
        if (bytes[r] & 3) return hipErrorInvalidValue;
        c.src[c.count] = (const uint32_t*)src[r];
        c.dst[c.count] = (uint32_t*)dst[r];
        c.dwords[c.count] = bytes[r] / 4;
        most = std::max<uint64_t>(most, bytes[r] / 4);
        ++c.count;
    }
    if (most == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((most + 255) / 256, 512);
    hipLaunchKernelGGL(copy_linear_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, c);
    return hipGetLastError();
}

hipError_t launch_gather_extents(const uint8_t* src, const uint64_t* src_off, const uint32_t* len,
                                 const uint64_t* dst_off, uint8_t* dst, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    // a bounded grid (grid-stride over the extents): 2048 waves keep ~2 MiB of reads
    // in flight, and leave the CUs to the other slot's hash kernel
    const uint64_t blocks = std::min<uint64_t>((n + 3) / 4, 512);
    hipLaunchKernelGGL(gather_extents_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream,
                       GatherArgs{src, src_off, len, dst_off, dst, n});
    return hipGetLastError();
}

}  // namespace hdx
