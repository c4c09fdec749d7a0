// hdx_index.hip — secondary-index keys and search pruning on gfx950.
//
// (1) Index-key encoders.  The daemon's secondary indices key every entry by
//     the attribute's hash in big-endian byte order, so the index's byte
//     order is the value order:
//       index_encoding_int64::encode      daemon/index_int64.cc:76-79
//           pack64be(hash(INT64, v))                              -> 8 B
//       index_encoding_timestamp::encode  daemon/index_timestamp.cc:79-82
//           = the int64 encoding (ordered int64, NOT the calendar hash) -> 8 B
//       index_encoding_float::encode      daemon/index_float.cc:75-90
//           pack64be(hash(FLOAT, v)) ++ packdoublele(v or 0.0)    -> 16 B
//     One lane per value, 8-byte loads at any alignment, 8/16-byte stores.
// (2) Search endpoints.  configuration::lookup_search
//     (common/configuration.cc:775-858) drops a region of a subspace when a
//     range's hashed endpoint falls outside the region's box.  One lane per
//     region over the ranges that name a subspace attribute; the endpoint
//     hashes come from the batch hash kernel launched just before.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"

namespace hdx {

typedef uint64_t __attribute__((aligned(1))) u64_u;
typedef const __attribute__((address_space(1))) u64_u* gu64_ptr;

__global__ void __launch_bounds__(256) index_encode_kernel(const IndexArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.len[i];
    uint64_t bits = 0;
    bool bad = false;
    if (n == 8)
        bits = *(gu64_ptr)(a.blob + a.off[i]);
    else if (n != 0)
        bad = true;
    if (a.code == CODE_FLOAT) {
        const uint64_t h = bad ? 0 : encode_double(bits);
        u64x2 e;
        e.x = __builtin_bswap64(h);
        e.y = bits;  // packdoublele(number): the value's own bytes, 0.0 when empty
        reinterpret_cast<u64x2*>(a.out)[i] = e;
    } else {
        reinterpret_cast<uint64_t*>(a.out)[i] = bad ? 0 : __builtin_bswap64(encode_int64(bits));
    }
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

hipError_t launch_index_encode(const IndexArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    const uint64_t blocks = (a.n + 255) / 256;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(index_encode_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

// configuration.cc:789-853 for region r, restricted to the ranges whose
// attribute the subspace holds (the others `continue` there).  A box with
// lower > upper on a ranged dimension clears the whole server list
// (:810-815); ranges are visited in order and stop at the first exclusion,
// exactly like the reference's `!exclude` loop.
__global__ void __launch_bounds__(256) search_regions_kernel(const SearchArgs a) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.R) return;
    if (a.replicas && !a.replicas[r]) {  // configuration.cc:782-785, before any range test
        a.include[r] = 0;
        return;
    }
    bool exclude = false, cleared = false;
    for (uint32_t k = 0; k < a.m && !exclude; ++k) {
        const uint32_t l = a.dim[k];
        const uint64_t lo = a.lower[(uint64_t)r * a.D + l], hi = a.upper[(uint64_t)r * a.D + l];
        if (lo > hi) {
            cleared = true;
            break;
        }
        const uint64_t hs = a.hashes[2 * k], he = a.hashes[2 * k + 1];
        if (a.kind[k] == SEARCH_STRING_EQ) {
            exclude = lo > hs || hi < hs;
        } else if (a.kind[k] == SEARCH_ORDERED) {
            if ((a.flags[k] & 1) && hi < hs) exclude = true;
            if ((a.flags[k] & 2) && lo > he) exclude = true;
        }
    }
    a.include[r] = exclude ? 0 : 1;
    if (cleared) atomicOr(a.cleared, 1u);
}

hipError_t launch_search_regions(const SearchArgs& a, hipStream_t stream) {
    if (a.R == 0) return hipSuccess;
    hipLaunchKernelGGL(search_regions_kernel, dim3((a.R + 255) / 256), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
