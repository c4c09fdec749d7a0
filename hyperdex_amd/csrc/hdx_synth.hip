// hdx_synth.hip — synthetic object batches generated in HBM (benchmark tooling).
//
// Counter-based, so any object range can be produced independently on any
// device and re-produced on the host by hyperdex_amd/synth.py (same rules,
// numpy).  RNG: splitmix64 finaliser over
//   R(stream, k) = mix64(seed + stream * 0xd1b54a32d192ed03 + (k + 1) * 0x9e3779b97f4a7c15)
// with seed 0x4859504552444558 ("HYPERDEX") by default.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_internal.h"

namespace hdx {

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t rnd(uint64_t seed, uint64_t stream, uint64_t k) {
    return mix64(seed + stream * 0xd1b54a32d192ed03ULL + (k + 1) * 0x9e3779b97f4a7c15ULL);
}

enum : uint32_t { KIND_FIXED = 0, KIND_UNIFORM = 1, KIND_NUMERIC = 2 };

__device__ __forceinline__ uint32_t synth_len(const hdx_synth_rule& r, uint64_t seed, uint64_t f) {
    switch (r.kind) {
        case KIND_FIXED: return r.lo;
        case KIND_UNIFORM: return r.lo + (uint32_t)(rnd(seed, 1, f) % (uint64_t)(r.hi - r.lo + 1));
        default: return rnd(seed, 4, f) % 100 == 0 ? 0u : 8u;
    }
}

__device__ __forceinline__ uint64_t synth_numeric(uint32_t type, uint64_t seed, uint64_t f) {
    const uint64_t sel = rnd(seed, 4, f) % 100;
    const uint64_t v = rnd(seed, 3, f);
    const uint64_t FRAC = 0x000fffffffffffffULL, SIGN = 0x8000000000000000ULL;
    if (type == 9218) {  // INT64: 1% INT64_MIN/MAX, rest uniform
        if (sel == 1) return (v & 1) ? 0x7fffffffffffffffULL : SIGN;
        return v;
    }
    if (type == 9219) {  // FLOAT: 1% each of +0, -0, +inf, -inf, NaN, +sub, -sub
        switch (sel) {
            case 1: return 0;
            case 2: return SIGN;
            case 3: return 0x7ff0000000000000ULL;
            case 4: return 0xfff0000000000000ULL;
            case 5: return 0x7ff8000000000000ULL | (v & 0x8007ffffffffffffULL);
            case 6: return (v & FRAC) | 1;
            case 7: return SIGN | (v & FRAC) | 1;
            default: {
                const uint64_t e = 963 + ((v >> 52) & 0x7f) % 121;
                return (v & SIGN) | (e << 52) | (v & FRAC);
            }
        }
    }
    // timestamps: half realistic microsecond clocks, half the full 64-bit range
    return sel < 50 ? (v & ((1ULL << 51) - 1)) : v;
}

__global__ void synth_lengths_kernel(const SynthArgs a, uint32_t* attr_len) {
    const uint64_t total = a.n * a.A;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t j = (uint32_t)(t % a.A);
        attr_len[t] = synth_len(a.rules[j], a.seed, a.first * a.A + t);
    }
}

__global__ void synth_bytes_kernel(uint64_t seed, uint64_t stream, uint8_t* blob, uint64_t bytes) {
    const uint64_t words = bytes >> 3;
    uint64_t* w = reinterpret_cast<uint64_t*>(blob);
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < words;
         t += (uint64_t)gridDim.x * blockDim.x)
        w[t] = rnd(seed, stream, t);
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < (bytes & 7)) {
        const uint64_t b = (words << 3) + t;
        blob[b] = (uint8_t)(rnd(seed, stream, b >> 3) >> (8 * (b & 7)));
    }
}

__global__ void synth_numeric_kernel(const SynthArgs a, const uint64_t* obj_base,
                                     const uint32_t* attr_len, uint8_t* blob) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint64_t off = obj_base[i];
    for (uint32_t j = 0; j < a.A; ++j) {
        const uint32_t L = attr_len[i * a.A + j];
        if (a.rules[j].kind == KIND_NUMERIC && L == 8) {
            const uint64_t v = synth_numeric(a.rules[j].type, a.seed, (a.first + i) * a.A + j);
            __builtin_memcpy(blob + off, &v, 8);
        }
        off += L;
    }
}

// daemon/datalayer_encodings.cc:139-166 (encode_value) for object i of a
// packed batch: attributes 1..A-1 become the value (attribute 0 is the key).
// keys (may be NULL): key i (attribute 0) is also copied to keys + key_off[i]
// (a key column, or records [key][value] when keys == vals)
__global__ void synth_encode_kernel(const uint8_t* blob, const uint64_t* obj_base, const uint32_t* attr_len,
                                    uint32_t A, uint64_t n, uint64_t first_version, const uint64_t* val_off,
                                    uint8_t* vals, const uint64_t* key_off, uint8_t* keys) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t* o = vals + val_off[i];
    if (keys) {
        const uint32_t kl = attr_len[i * A];
        const uint8_t* k = blob + obj_base[i];
        uint8_t* kd = keys + key_off[i];
        for (uint32_t b = 0; b < kl; ++b) kd[b] = k[b];
    }
    const uint64_t ver = first_version + i;
    for (int b = 0; b < 8; ++b) o[b] = (uint8_t)(ver >> (56 - 8 * b));
    o[8] = (uint8_t)((A - 1) >> 8);
    o[9] = (uint8_t)(A - 1);
    o += 10;
    const uint8_t* src = blob + obj_base[i] + attr_len[i * A];
    for (uint32_t j = 1; j < A; ++j) {
        const uint32_t L = attr_len[i * A + j];
        o[0] = (uint8_t)(L >> 24);
        o[1] = (uint8_t)(L >> 16);
        o[2] = (uint8_t)(L >> 8);
        o[3] = (uint8_t)L;
        o += 4;
        uint32_t k = 0;
        for (; k + 8 <= L; k += 8) {
            uint64_t w;
            __builtin_memcpy(&w, src + k, 8);
            __builtin_memcpy(o + k, &w, 8);
        }
        for (; k < L; ++k) o[k] = src[k];
        o += L;
        src += L;
    }
}

hipError_t launch_synth_encode(const uint8_t* blob, const uint64_t* obj_base, const uint32_t* attr_len,
                               uint32_t A, uint64_t n, uint64_t first_version, const uint64_t* val_off,
                               uint8_t* vals, hipStream_t s, const uint64_t* key_off, uint8_t* keys) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_encode_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, blob, obj_base,
                       attr_len, A, n, first_version, val_off, vals, key_off, keys);
    return hipGetLastError();
}

static uint32_t grid_for(uint64_t work, uint32_t block) {
    uint64_t g = (work + block - 1) / block;
    if (g > 65536) g = 65536;
    return g ? (uint32_t)g : 1;
}

hipError_t launch_synth_lengths(const SynthArgs& a, uint32_t* attr_len, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(synth_lengths_kernel, dim3(grid_for(a.n * a.A, 256)), dim3(256), 0, s, a,
                       attr_len);
    return hipGetLastError();
}

hipError_t launch_synth_fill(const SynthArgs& a, const uint64_t* obj_base, const uint32_t* attr_len,
                             uint8_t* blob, uint64_t bytes, hipStream_t s) {
    if (bytes) {
        hipLaunchKernelGGL(synth_bytes_kernel, dim3(grid_for(bytes >> 3, 256)), dim3(256), 0, s,
                           a.seed, 2 + (a.first << 8), blob, bytes);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (a.n) {
        hipLaunchKernelGGL(synth_numeric_kernel, dim3((uint32_t)((a.n + 255) / 256)), dim3(256), 0, s,
                           a, obj_base, attr_len, blob);
        return hipGetLastError();
    }
    return hipSuccess;
}

// ---------------------------------------------------------------------------
// Streaming probe (hdxdbg_stream_probe): the HBM rate of a plain read of
// `bytes` in the hash kernels' access shape (one wave per 4 KiB chunk, each
// lane 4 x 16 B of a 64-byte span — tools/membw.hip's fastest read shape),
// optionally with `write` (1..4) 8-byte non-temporal stores per 64 bytes read
// (1: the 1:8 write mix of the 64-byte-attribute configs; 3: config 2's
// ≈ 1:3), so the bench can quote the kernel against a measured ceiling of its
// own read/write mix beside the HBM3E spec.  bytes is a multiple of 4096.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) stream_probe_kernel(const uint8_t* src, uint64_t chunks, uint64_t* sink,
                                                         int write) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t c = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= chunks) return;
    typedef uint64_t u64x2v __attribute__((ext_vector_type(2)));
    const u64x2v* p = reinterpret_cast<const u64x2v*>(src + c * 4096 + lane * 64);
    const u64x2v v = p[0] ^ p[1] ^ p[2] ^ p[3];
    if (write) {
        for (int k = 0; k < write; ++k)  // lane-contiguous: each pass one coalesced 512-byte row
            __builtin_nontemporal_store(v.x ^ v.y ^ (uint64_t)k, sink + (c * write + k) * 64 + lane);
    } else if (sink && (v.x ^ v.y) == 0x9e3779b97f4a7c15ull) sink[0] = v.x;  // keeps the loads live
}

hipError_t launch_stream_probe(const uint8_t* src, uint64_t bytes, uint64_t* sink, int write, hipStream_t s) {
    const uint64_t chunks = bytes / 4096;
    if (chunks == 0) return hipSuccess;
    const uint64_t blocks = (chunks + 3) / 4;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(stream_probe_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, src, chunks, sink, write);
    return hipGetLastError();
}

}  // namespace hdx
