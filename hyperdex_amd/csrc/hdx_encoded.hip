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
// chain, as in the reference) and writes one 16-byte slot descriptor per
// attribute into the wave's LDS, key first.  Phase 2: A passes of 64 slots in
// object-major order — adjacent lanes hash adjacent attributes of the same
// values — with the next pass's bytes in flight and one coalesced coordinate
// store per pass.  A value that does not decode into A-1 attributes lying
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

template <bool NT_STORE>
__global__ void __launch_bounds__(128)
hash_encoded_kernel(const EncodedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const uint32_t A = a.A;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    SlotDesc* desc = reinterpret_cast<SlotDesc*>(smem_raw) + (size_t)w * 64 * A;
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
    const uint32_t touch = vlen >= 4 ? min(vlen - 3, 4096u) : 0u;
    for (uint32_t off = 0; off < touch; off += 128)
        sink ^= *(const __attribute__((address_space(1))) u32_u*)(v + off);

    // phase 1: decode_value (datalayer_encodings.cc:168-217) into descriptors
    bool ok = valid && vlen >= 10;
    const uint64_t version = ok ? load_be64(v) : 0;
    const uint32_t count = ok ? load_be16(v + 8) : 0;
    ok = ok && count == A - 1;
    SlotDesc d;
    d.p = a.keys + koff;
    d.n = klen;
    d.code_slot = valid ? a.codes[0] : (uint32_t)CODE_ZERO;
    desc[lane * A] = d;
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
        d.p = ok ? v + pos : g_zero_pad;
        d.n = ok ? len : 0u;
        d.code_slot = ok ? a.codes[k + 1] : (uint32_t)CODE_ZERO;
        desc[lane * A + 1 + k] = d;
        if (ok) pos += len;
    }
    if (valid && !ok) {  // undecodable: every coordinate of the object is 0
        d.p = g_zero_pad;
        d.n = 0;
        d.code_slot = CODE_ZERO;
        for (uint32_t j = 0; j < A; ++j) desc[lane * A + j] = d;
    }
    if (valid && a.versions) a.versions[i] = ok ? version : 0;
    const bool any_bad = __any(valid && !ok);
    asm volatile("; touch sink %0" ::"v"(sink));  // keeps the phase-0 loads live
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // phase 2: A passes of 64 slots, slot s = object * A + attribute
    const uint32_t nslots = nobj * A;
    uint64_t* out = a.coords + o0 * A;
    struct Pass {
        SlotDesc d;
        Blk blk;
    };
    auto load_pass = [&](uint32_t t, Pass& P) {
        const uint32_t s = t * 64 + lane;
        P.d = desc[min(s, nslots - 1)];
        if (s >= nslots) P.d.code_slot = CODE_ZERO, P.d.n = 0, P.d.p = g_zero_pad;
        P.blk = issue_block(P.d.code_slot, P.d.p, P.d.n);
    };
    bool bad = false;
    Pass P0, P1;
    load_pass(0, P0);
    for (uint32_t t = 0;; t += 2) {
        if (t + 1 < A) load_pass(t + 1, P1);
        {
            const uint64_t h = hash_blk(P0.d.code_slot, P0.d.p, P0.d.n, P0.blk, bad);
            const uint32_t s = t * 64 + lane;
            if (s < nslots) {
                if (NT_STORE) __builtin_nontemporal_store(h, out + s);
                else out[s] = h;
            }
        }
        if (t + 1 >= A) break;
        if (t + 2 < A) load_pass(t + 2, P0);
        {
            const uint64_t h = hash_blk(P1.d.code_slot, P1.d.p, P1.d.n, P1.blk, bad);
            const uint32_t s = (t + 1) * 64 + lane;
            if (s < nslots) {
                if (NT_STORE) __builtin_nontemporal_store(h, out + s);
                else out[s] = h;
            }
        }
        if (t + 2 >= A) break;
    }
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// Lane-per-object variant: lane l owns object o0+l and walks its value once,
// hashing attribute t while the length prefix of attribute t+2 is in flight
// (the prefix of t+1 arrived during t-1).  Attribute positions share one
// type, so every pass is type-uniform; no LDS.  Coordinates are stored as they
// are produced; an object found undecodable later is zeroed afterwards.
template <bool TOUCH>
__global__ void __launch_bounds__(256)
hash_encoded_lane_kernel(const EncodedArgs a) {
    const uint32_t A = a.A;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint64_t voff = a.val_off[i], koff = a.key_off[i];
    const uint32_t vlen = a.val_len[i], klen = a.key_len[i];
    const uint8_t* v = a.vals + voff;
    uint32_t sink = 0;
    if (TOUCH) {
        const uint32_t touch = vlen >= 4 ? min(vlen - 3, 4096u) : 0u;
        for (uint32_t off = 0; off < touch; off += 128)
            sink ^= *(const __attribute__((address_space(1))) u32_u*)(v + off);
    }
    bool ok = vlen >= 10;
    const uint64_t version = ok ? load_be64(v) : 0;
    ok = ok && load_be16(v + 8) == A - 1;
    uint64_t* out = a.coords + i * A;
    bool bad = false;

    // attribute t = 0 is the key; the value's attributes follow their prefixes
    const uint8_t* p = a.keys + koff;
    uint32_t L = klen, pos = 10;
    uint32_t next_len = 0;  // prefix of attribute t+1, loaded one step ahead
    auto read_prefix = [&](uint32_t at) -> uint32_t {
        return (ok && vlen >= 4 && at <= vlen - 4) ? load_be32(v + at) : 0u;
    };
    if (A > 1) next_len = read_prefix(pos);
    for (uint32_t t = 0; t < A; ++t) {
        const uint32_t code = a.codes[t];
        const Blk blk = issue_block(ok ? code : (uint32_t)CODE_ZERO, ok ? p : g_zero_pad, ok ? L : 0u);
        // locate attribute t+1 and put the prefix of t+2 in flight
        const uint8_t* pn = g_zero_pad;
        uint32_t Ln = 0;
        if (t + 1 < A) {
            if (ok && vlen >= 4 && pos <= vlen - 4 && next_len <= vlen - pos - 4) {
                pn = v + pos + 4;
                Ln = next_len;
                pos += 4 + next_len;
                next_len = t + 2 < A ? read_prefix(pos) : 0u;
            } else {
                ok = false;
            }
        }
        const uint64_t h = hash_blk(ok ? code : (uint32_t)CODE_ZERO, p, ok ? L : 0u, blk, bad);
        __builtin_nontemporal_store(h, out + t);
        p = pn;
        L = Ln;
    }
    if (!ok) {
        for (uint32_t t = 0; t < A; ++t) out[t] = 0;
        if (a.status) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    }
    if (a.versions) a.versions[i] = ok ? version : 0;
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
    if (TOUCH) asm volatile("; touch sink %0" ::"v"(sink));
}

hipError_t launch_hash_encoded(const EncodedArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    const int v = hash_variant();
    if (v == 31 || v == 32 || v == -1) {
        const uint64_t blocks = (a.n + 255) / 256;
        if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
        if (v == 32)
            hipLaunchKernelGGL(hash_encoded_lane_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
        else
            hipLaunchKernelGGL(hash_encoded_lane_kernel<true>, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
        return hipGetLastError();
    }
    const uint32_t waves_per_block = a.A <= 32 ? 2 : 1;
    const uint64_t waves = (a.n + 63) / 64;
    const uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    const size_t lds = (size_t)waves_per_block * 64 * a.A * sizeof(SlotDesc);
    hipLaunchKernelGGL((hash_encoded_kernel<true>), dim3((uint32_t)blocks), dim3(64 * waves_per_block),
                       lds, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
