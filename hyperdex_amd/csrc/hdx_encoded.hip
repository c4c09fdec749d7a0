// hdx_encoded.hip — reindex sweep over stored objects.
//
// The daemon stores an object as a LevelDB value
//   [u64 BE version][u16 BE count]{[u32 BE len][bytes]}*count
// (daemon/datalayer_encodings.cc:139-166, decoded by decode_value :168-217)
// with the key kept in the LevelDB key.  The datalayer_indexer_thread sweep
// (daemon/datalayer_indexer_thread.cc:161-176) iterates resident objects,
// decodes each value and works per attribute; here every object is decoded
// and re-hashed (common/hash.cc:56-68) in one fused launch.
//
// One wave = 64 objects.  Phase 0: each lane touches its value's cache lines
// (one dword per 128 B, up to 4 KiB) so the parse that follows walks L2-hot
// lines.  Phase 1: each lane walks its value's length prefixes (a sequential
// chain, as in the reference) and writes one 8-byte {offset, length} slot
// descriptor per attribute into the wave's LDS, key first.  Phase 2: A passes
// of 64 slots in object-major order — adjacent lanes hash adjacent attributes
// of the same values — with the next pass's bytes in flight and one coalesced
// coordinate store per pass.  (A lane-per-object variant that overlaps the
// prefix chain with hashing and needs no LDS ran 1.35-1.5x slower.)  A value that does not decode into A-1 attributes lying
// inside its bytes yields zero coordinates and sets HDX_E_BADENC in status.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_loads.h"

namespace hdx {

typedef uint32_t __attribute__((aligned(1))) u32_u;
typedef uint64_t __attribute__((aligned(1))) u64_u;
typedef uint16_t __attribute__((aligned(1))) u16_u;

__device__ __forceinline__ uint32_t load_be32(const uint8_t* p) {
    return __builtin_bswap32(*(const __attribute__((address_space(1))) u32_u*)p);
}
__device__ __forceinline__ uint64_t load_be64(const uint8_t* p) {
    return __builtin_bswap64(*(const __attribute__((address_space(1))) u64_u*)p);
}
__device__ __forceinline__ uint32_t load_be16(const uint8_t* p) {
    const uint16_t v = *(const __attribute__((address_space(1))) u16_u*)p;
    return (uint32_t)(uint16_t)((v >> 8) | (v << 8));
}

// Compact slot descriptor: byte offset inside the object's value (or key, for
// attribute 0) and length; kZeroSlot marks a slot hashed as 0.
struct alignas(8) EncDesc {
    uint32_t off;
    uint32_t len;
};
constexpr uint32_t kZeroSlot = 0xffffffffu;

template <bool TOUCH>
__global__ void __launch_bounds__(256)
hash_encoded_kernel(const EncodedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const uint32_t A = a.A;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    EncDesc* desc = reinterpret_cast<EncDesc*>(smem_raw) + (size_t)w * 64 * A;
    const uint64_t o0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + w) * 64;
    if (o0 >= a.n) return;  // no workgroup barrier: waves are independent
    const uint32_t nobj = (uint32_t)min<uint64_t>(64, a.n - o0);
    const bool valid = (uint32_t)lane < nobj;
    const uint64_t i = o0 + (valid ? lane : 0);

    const uint64_t voff = a.val_off[i], koff = a.key_off[i];
    const uint32_t vlen = valid ? a.val_len[i] : 0u, klen = valid ? a.key_len[i] : 0u;
    const uint8_t* v = a.vals + voff;

    // phase 0: pull the value's lines toward L2 (independent loads, consumed late)
    uint32_t sink = 0;
    if (TOUCH) {
        const uint32_t touch = vlen >= 4 ? min(vlen - 3, 4096u) : 0u;
        for (uint32_t off = 0; off < touch; off += 128)
            sink ^= *(const __attribute__((address_space(1))) u32_u*)(v + off);
    }

    // phase 1: decode_value (datalayer_encodings.cc:168-217) into descriptors
    bool ok = valid && vlen >= 10;
    const uint64_t version = ok ? load_be64(v) : 0;
    ok = ok && load_be16(v + 8) == A - 1;
    desc[lane * A] = EncDesc{0u, klen};
    uint32_t pos = 10;
    for (uint32_t k = 0; k + 1 < A; ++k) {
        uint32_t len = 0;
        if (ok) {
            if (vlen - pos < 4) {
                ok = false;
            } else {
                len = load_be32(v + pos);
                pos += 4;
                if (len > vlen - pos) ok = false;  // the reference does not check this (:201-213)
            }
        }
        desc[lane * A + 1 + k] = EncDesc{ok ? pos : kZeroSlot, ok ? len : 0u};
        if (ok) pos += len;
    }
    if (!ok)  // undecodable (or past the batch end): every coordinate of the object is 0
        for (uint32_t j = 0; j < A; ++j) desc[lane * A + j] = EncDesc{kZeroSlot, 0u};
    if (valid && a.versions) a.versions[i] = ok ? version : 0;
    const bool any_bad = __any(valid && !ok);
    if (TOUCH) asm volatile("; touch sink %0" ::"v"(sink));  // keeps the phase-0 loads live
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // phase 2: A passes of 64 slots, slot s = object * A + attribute; the
    // object's key/value bases come from its owner lane by ds_bpermute
    const uint32_t nslots = nobj * A;
    uint64_t* out = a.coords + o0 * A;
    const uint32_t packed_codes = reinterpret_cast<const uint32_t*>(a.codes)[lane];
    struct Pass {
        const uint8_t* p;
        uint32_t n, code;
        Blk blk;
    };
    auto load_pass = [&](uint32_t t, Pass& P) {
        const uint32_t s = min(t * 64 + (uint32_t)lane, nslots - 1);
        const uint32_t obj = s / A, j = s - obj * A;
        const EncDesc d = desc[s];
        const uint32_t vlo = __shfl((uint32_t)voff, (int)obj, 64), vhi = __shfl((uint32_t)(voff >> 32), (int)obj, 64);
        const uint32_t klo = __shfl((uint32_t)koff, (int)obj, 64), khi = __shfl((uint32_t)(koff >> 32), (int)obj, 64);
        const uint64_t base = j == 0 ? (((uint64_t)khi << 32) | klo) : (((uint64_t)vhi << 32) | vlo);
        const bool zero = d.off == kZeroSlot || t * 64 + (uint32_t)lane >= nslots;
        P.code = zero ? (uint32_t)CODE_ZERO : (__shfl(packed_codes, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
        P.n = zero ? 0u : d.len;
        P.p = zero ? g_zero_pad : (j == 0 ? a.keys : a.vals) + base + d.off;
        P.blk = issue_block(P.code, P.p, P.n);
    };
    bool bad = false;
    Pass P0, P1;
    load_pass(0, P0);
    for (uint32_t t = 0;; t += 2) {
        if (t + 1 < A) load_pass(t + 1, P1);
        {
            const uint64_t h = hash_blk(P0.code, P0.p, P0.n, P0.blk, bad);
            const uint32_t s = t * 64 + lane;
            if (s < nslots) __builtin_nontemporal_store(h, out + s);
        }
        if (t + 1 >= A) break;
        if (t + 2 < A) load_pass(t + 2, P0);
        {
            const uint64_t h = hash_blk(P1.code, P1.p, P1.n, P1.blk, bad);
            const uint32_t s = (t + 1) * 64 + lane;
            if (s < nslots) __builtin_nontemporal_store(h, out + s);
        }
        if (t + 2 >= A) break;
    }
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

hipError_t launch_hash_encoded(const EncodedArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    // 4 waves per workgroup while the descriptors fit (A <= 64: 32 KiB), else 1
    const uint32_t waves_per_block = a.A <= 64 ? 4 : 1;
    const uint64_t waves = (a.n + 63) / 64;
    const uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    const size_t lds = (size_t)waves_per_block * 64 * a.A * sizeof(EncDesc);
    if (hash_variant() == 33)
        hipLaunchKernelGGL((hash_encoded_kernel<false>), dim3((uint32_t)blocks), dim3(64 * waves_per_block),
                           lds, stream, a);
    else
        hipLaunchKernelGGL((hash_encoded_kernel<true>), dim3((uint32_t)blocks), dim3(64 * waves_per_block),
                           lds, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
