// hdx_kernels.hip — batched hyperspace attribute hashing for gfx950.
//
// One launch hashes every attribute of n objects in the packed layout of
// include/hdxhash.h and writes coords[i*A + j] — the reference's
// hs[j] of hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68) for
// object i.
//
// Work decomposition:
//   * one wave64 owns 64 consecutive objects and walks their 64*A attributes
//     in A rounds of 64 consecutive (object, attr) slots, so every attr_len
//     load and every coords store is one coalesced 256 B / 512 B access;
//   * a lane's byte offset inside its object is a wave-wide segmented prefix
//     sum of the round's lengths (DPP scan) plus a carry from the previous round;
//   * each lane hashes one attribute: type dispatch through an LDS code table,
//     strings read as 16 B vectors straight from HBM.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"

namespace hdx {

// Inclusive wave64 prefix sum (u32, modular).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t hash_attr(uint32_t code, const uint8_t* p, uint32_t len,
                                              bool& bad) {
    if (code == CODE_STRING) return cityhash64(p, len);
    if (code == CODE_ZERO) return 0;
    // int64 / float / timestamp: 0 or 8 bytes (datatype_*::unpack)
    uint64_t bits = 0;
    if (len == 8) {
        bits = ld8(p);
    } else if (len != 0) {
        bad = true;
        return 0;
    }
    if (code == CODE_INT64) return encode_int64(bits);
    if (code == CODE_FLOAT) return encode_double(bits);
    return hash_timestamp(code - CODE_TS_SECOND, bits);
}

__global__ void __launch_bounds__(256)
hash_batch_kernel(const BatchArgs args) {
    __shared__ uint8_t codes[HDX_MAX_ATTRS];
    for (uint32_t j = threadIdx.x; j < args.A; j += blockDim.x) codes[j] = args.codes[j];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t o0 = wave * 64;
    if (o0 >= args.n) return;
    const uint32_t nobj = (uint32_t)min<uint64_t>(64, args.n - o0);
    const uint32_t A = args.A;
    const uint32_t rounds = A;  // 64*A slots, 64 per round

    // slot q = 64*r + lane  ->  (object il = q / A, attribute j = q % A)
    uint32_t il = (uint32_t)lane / A;
    uint32_t j = (uint32_t)lane % A;
    const uint32_t qA = 64 / A, rA = 64 % A;

    const uint32_t* lens = args.attr_len + o0 * A;
    uint64_t* out = args.coords + o0 * A;
    uint32_t carry = 0;
    bool bad = false;

    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t q = r * 64 + lane;
        const bool valid = il < nobj;
        const uint32_t L = valid ? lens[q] : 0;
        const uint32_t S = wave_inclusive_scan(L, lane);
        const uint32_t Sx = S - L;
        const int head = lane - (int)j;  // lane holding this object's attr 0, if in this round
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        const uint32_t off = head >= 0 ? Sx - head_sx : carry + Sx;
        carry = __shfl(off + L, 63, 64);
        if (valid) {
            const uint8_t* p = args.blob + args.obj_base[o0 + il] + off;
            out[q] = hash_attr(codes[j], p, L, bad);
        }
        j += rA;
        il += qA;
        if (j >= A) {
            j -= A;
            ++il;
        }
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

hipError_t launch_hash_batch(const BatchArgs& args, hipStream_t stream) {
    const uint64_t waves = (args.n + 63) / 64;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(hash_batch_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}

}  // namespace hdx
