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

__host__ __device__ constexpr size_t encoded_lds_per_wave(uint32_t A) {
    return 64 * 16 + 256 + (size_t)64 * A * sizeof(EncDesc);
}

template <bool TOUCH>
__global__ void __launch_bounds__(256)
hash_encoded_kernel(const EncodedArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const uint32_t A = a.A;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    // wave-private LDS: 64 object bases {value, key}, the code table, descriptors
    uint8_t* wsmem = smem_raw + (size_t)w * encoded_lds_per_wave(A);
    uint64_t* bases = reinterpret_cast<uint64_t*>(wsmem);           // [64][2]
    uint8_t* codes = wsmem + 64 * 16;                                // [256]
    EncDesc* desc = reinterpret_cast<EncDesc*>(wsmem + 64 * 16 + 256);
    const uint64_t o0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + w) * 64;
    if (o0 >= a.n) return;  // no workgroup barrier: waves are independent
    const uint32_t nobj = (uint32_t)min<uint64_t>(64, a.n - o0);
    const bool valid = (uint32_t)lane < nobj;
    const uint64_t i = o0 + (valid ? lane : 0);

    const uint64_t voff = a.val_off[i], koff = a.key_off[i];
    const uint32_t vlen = valid ? a.val_len[i] : 0u, klen = valid ? a.key_len[i] : 0u;
    const uint8_t* v = a.vals + voff;
    bases[2 * lane] = voff;
    bases[2 * lane + 1] = koff;
    for (uint32_t j = lane; j < A; j += 64) codes[j] = a.codes[j];

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

    // phase 2: A passes of 64 slots, slot s = object * A + attribute.  The
    // object's bases and the attribute's code are read from LDS, not from other
    // lanes: in a partial pass the lanes past the batch end are inactive, and a
    // ds_bpermute from an inactive lane returns 0.
    const uint32_t nslots = nobj * A;
    uint64_t* out = a.coords + o0 * A;
    struct Pass {
        const uint8_t* p;
        uint32_t n, code;
        Blk blk;
    };
    auto load_pass = [&](uint32_t t, Pass& P) {
        const uint32_t s = min(t * 64 + (uint32_t)lane, nslots - 1);
        const uint32_t obj = s / A, j = s - obj * A;
        const EncDesc d = desc[s];
        const uint64_t base = bases[2 * obj + (j == 0)];
        const bool zero = d.off == kZeroSlot || t * 64 + (uint32_t)lane >= nslots;
        P.code = zero ? (uint32_t)CODE_ZERO : (uint32_t)codes[j];
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

// ===========================================================================
// Staged sweep: one wave = G objects.  (1) The wave's 2G segments (each
// object's value and key) are copied into its LDS with streaming, aligned
// 16-byte loads — every byte read from HBM once, in address order within a
// segment.  (2) Lane j walks object j's length prefixes in LDS.  (3)
// ceil(G*A / 64) passes hash the slots straight out of LDS; coordinates leave
// in one coalesced store per pass.  Segments that do not fit in the stage
// buffer (W bytes) are decoded and hashed from global memory instead.
// G is chosen so that G*A fills whole passes (G = 15 for A = 17: 255 of 256
// lanes busy).
// ===========================================================================
constexpr uint32_t kNotStaged = 0xffffffffu;

typedef const __attribute__((address_space(3))) uint32_t* lds_u32_ptr;

// Bytes [off, off+4) of the stage as a little-endian u32 (two aligned reads).
__device__ __forceinline__ uint32_t lds_u32(lds_cptr base, uint32_t off) {
    const uint32_t a = off & ~3u;
    const uint32_t d0 = *(lds_u32_ptr)(base + a), d1 = *(lds_u32_ptr)(base + a + 4);
    return __builtin_amdgcn_alignbyte(d1, d0, off & 3u);
}

template <int G>
__host__ __device__ constexpr size_t staged_meta_bytes(uint32_t A) {
    // sstart/slds [2G] u32, ssrc [2G] u64, sskew [2G] u32, codes [256], desc [G*A]
    return (size_t)2 * G * (4 + 4 + 8 + 4) + 256 + (size_t)G * A * sizeof(EncDesc);
}

template <int G>
__global__ void __launch_bounds__(64)
hash_encoded_staged_kernel(const EncodedArgs a, uint32_t W) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_raw[];
    const uint32_t A = a.A;
    const int lane = threadIdx.x;
    uint8_t* stage = smem_raw;                                        // [W] + 16 slack
    uint32_t* sstart = reinterpret_cast<uint32_t*>(smem_raw + W + 16);  // [2G] stage offset (prefix)
    uint32_t* slds = sstart + 2 * G;                                  // [2G] stage offset or kNotStaged
    uint64_t* ssrc = reinterpret_cast<uint64_t*>(slds + 2 * G);       // [2G] 16-aligned global start
    uint32_t* sskew = reinterpret_cast<uint32_t*>(ssrc + 2 * G);      // [2G] segment start & 15
    uint8_t* codes = reinterpret_cast<uint8_t*>(sskew + 2 * G);       // [256]
    EncDesc* desc = reinterpret_cast<EncDesc*>(codes + 256);          // [G*A]
    const lds_cptr lstage = (lds_cptr)stage;

    const uint64_t o0 = (uint64_t)blockIdx.x * G;
    if (o0 >= a.n) return;
    const uint32_t nobj = (uint32_t)min<uint64_t>(G, a.n - o0);
    for (uint32_t j = lane; j < A; j += 64) codes[j] = a.codes[j];

    // (1) segment table: lanes [0, G) values, [G, 2G) keys
    const bool isval = lane < G;
    const uint32_t jo = isval ? (uint32_t)lane : (uint32_t)lane - G;
    const bool segv = lane < 2 * G && jo < nobj;
    const uint64_t io = o0 + (segv ? jo : 0);
    const uint8_t* sp = isval ? a.vals + a.val_off[io] : a.keys + a.key_off[io];
    const uint32_t slen = segv ? (isval ? a.val_len[io] : a.key_len[io]) : 0u;
    const uint32_t skew = addr_lo(sp) & 15;
    const uint32_t bytes = slen ? (skew + slen + 15) & ~15u : 0u;
    const uint32_t end = wave_scan_dpp(bytes);
    const uint32_t start = end - bytes;
    const bool staged = segv && end <= W;
    uint32_t total = staged ? end : 0u;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) total = max(total, (uint32_t)__shfl_xor((int)total, m, 64));
    if (lane < 2 * G) {
        sstart[lane] = start;
        slds[lane] = staged ? start : kNotStaged;
        ssrc[lane] = (uint64_t)(uintptr_t)(sp - skew);
        sskew[lane] = skew;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // (2) copy the staged byte range [0, total) chunk by chunk, 4 chunks per
    // lane in flight; each chunk's segment by binary search over the starts
    const uint32_t nch = total >> 4;
    for (uint32_t q0 = 0; q0 < nch; q0 += 256) {
        u64x2 v[4];
        uint32_t dst[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t q = min(q0 + u * 64 + (uint32_t)lane, nch - 1);
            const uint32_t byte = q << 4;
            uint32_t lo = 0, hi = 2 * G;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (sstart[mid] <= byte) lo = mid;
                else hi = mid;
            }
            const uint8_t* src = reinterpret_cast<const uint8_t*>(ssrc[lo]) + (byte - sstart[lo]);
            v[u] = gld16(src);
            dst[u] = byte;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (q0 + u * 64 + (uint32_t)lane < nch) *reinterpret_cast<u64x2*>(stage + dst[u]) = v[u];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // (3) decode_value (datalayer_encodings.cc:168-217), lane = object
    bool any_bad = false;
    if ((uint32_t)lane < nobj) {
        const uint32_t vl = slds[lane];
        const uint32_t vpos = vl + sskew[lane];  // stage offset of value byte 0 (if staged)
        const uint8_t* v = reinterpret_cast<const uint8_t*>(ssrc[lane]) + sskew[lane];
        const uint32_t vlen = a.val_len[o0 + lane], klen = a.key_len[o0 + lane];
        auto be32 = [&](uint32_t pos) -> uint32_t {
            return vl != kNotStaged ? __builtin_bswap32(lds_u32(lstage, vpos + pos)) : load_be32(v + pos);
        };
        bool ok = vlen >= 10;
        uint64_t version = 0;
        if (ok) {
            version = ((uint64_t)be32(0) << 32) | be32(4);
            ok = (be32(6) & 0xffffu) == A - 1;  // u16 BE count at byte 8
        }
        desc[lane * A] = EncDesc{0u, klen};
        uint32_t pos = 10;
        for (uint32_t k = 0; k + 1 < A; ++k) {
            uint32_t len = 0;
            if (ok) {
                if (vlen - pos < 4) {
                    ok = false;
                } else {
                    len = be32(pos);
                    pos += 4;
                    if (len > vlen - pos) ok = false;
                }
            }
            desc[lane * A + 1 + k] = EncDesc{ok ? pos : kZeroSlot, ok ? len : 0u};
            if (ok) pos += len;
        }
        if (!ok)
            for (uint32_t j = 0; j < A; ++j) desc[lane * A + j] = EncDesc{kZeroSlot, 0u};
        if (a.versions) a.versions[o0 + lane] = ok ? version : 0;
        any_bad = !ok;
    }
    any_bad = __any(any_bad);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // (4) hash G*A slots (object-major) out of the stage
    const uint32_t nslots = nobj * A;
    uint64_t* out = a.coords + o0 * A;
    bool bad = false;
    for (uint32_t t = 0; t * 64 < nslots; ++t) {
        const uint32_t s = t * 64 + (uint32_t)lane;
        const uint32_t sc = min(s, nslots - 1);
        const uint32_t obj = sc / A, j = sc - obj * A;
        const EncDesc d = desc[sc];
        const bool zero = d.off == kZeroSlot || s >= nslots;
        const uint32_t code = zero ? (uint32_t)CODE_ZERO : (uint32_t)codes[j];
        const uint32_t n = zero ? 0u : d.len;
        const uint32_t k = j == 0 ? G + obj : obj;  // key or value segment
        const uint32_t l = slds[k];
        const uint32_t rel = sskew[k] + (zero ? 0u : d.off);
        uint64_t h;
        if (zero || l != kNotStaged) {
            const lds_cptr p = lstage + (zero ? 0u : l + rel);
            const Blk blk = issue_block_t<lds_cptr>(code, p, n, lstage);
            h = hash_blk<false, lds_cptr>(code, p, n, blk, bad);
        } else {
            const uint8_t* p = reinterpret_cast<const uint8_t*>(ssrc[k]) + rel;
            const Blk blk = issue_block(code, p, n);
            h = hash_blk(code, p, n, blk, bad);
        }
        if (s < nslots) __builtin_nontemporal_store(h, out + s);
    }
    if (a.status && lane == 0 && any_bad) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

template <int G>
static hipError_t launch_staged(const EncodedArgs& a, uint32_t W, hipStream_t stream) {
    const uint64_t blocks = (a.n + G - 1) / G;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    const size_t lds = W + 16 + staged_meta_bytes<G>(a.A);
    hipLaunchKernelGGL((hash_encoded_staged_kernel<G>), dim3((uint32_t)blocks), dim3(64), lds, stream, a, W);
    return hipGetLastError();
}

hipError_t launch_hash_encoded(const EncodedArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    switch (hash_variant()) {
        case 34: return launch_staged<15>(a, 24576, stream);
        case 35: return launch_staged<11>(a, 18432, stream);
        case 36: return launch_staged<7>(a, 12288, stream);
        case 37: return launch_staged<15>(a, 20480, stream);
        default: break;
    }
    // 4 waves per workgroup while they fit in 64 KiB of LDS (A <= 28), else 1
    const uint32_t waves_per_block = 4 * encoded_lds_per_wave(a.A) <= 65536 ? 4 : 1;
    const uint64_t waves = (a.n + 63) / 64;
    const uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    const size_t lds = (size_t)waves_per_block * encoded_lds_per_wave(a.A);
    // variant 33 adds the phase-0 line touch (measured 11% slower, r1u)
    if (hash_variant() == 33)
        hipLaunchKernelGGL((hash_encoded_kernel<true>), dim3((uint32_t)blocks), dim3(64 * waves_per_block),
                           lds, stream, a);
    else
        hipLaunchKernelGGL((hash_encoded_kernel<false>), dim3((uint32_t)blocks), dim3(64 * waves_per_block),
                           lds, stream, a);
    return hipGetLastError();
}

}  // namespace hdx
