// hdx_wide_dbg.hip — debug forms of the wide sweep (libhdxhash_dbg.so only;
// hdxdbg_set_kernel_variant 304-308, 312): measured against the product's two
// launches (hdx_wide.hip) and kept for the A/B record (DESIGN §4.7,
// profiles/r6/ab_wide_stream.jsonl, ab_wide_fused.jsonl).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "hdx_wide.h"

namespace hdx {

// A streaming form (round 6, late; debug variants 304-308, not the product):
// a wave per object streams
// its value through a two-chunk LDS ring by LDS DMA — chunk c + 1 in flight
// while the walk reads chunk c — and walks the prefix chain from LDS, the
// whole wave on the same (broadcast) address, the chain's position in scalar
// registers.  Every 64 attributes the wave hashes the batch it has walked,
// a lane per attribute from global memory (the lines the DMA has just brought
// through L2), and stores 64 coordinates.  Each value byte crosses HBM once
// and the walk pays LDS latency per attribute instead of an HBM round trip
// under the load of 200 k chains.  A jump past the prefetched chunk (an
// attribute longer than a chunk) loads the chunk the next prefix is in.
// Ring: chunk c (stream bytes [c CH, (c + 1) CH) of the value from its
// 16-byte floor) in half c & 1; the first dword of an even chunk also in the
// 16-byte pad after the ring, so a prefix read across the ring's end is one
// unaligned ds_read_b32.  An undecodable object (the checks of §4.4): the
// batches already stored are overwritten with zero coordinates, version 0,
// HDX_E_BADENC.
// Measured slower than the two launches above (w200: 3.35-3.55 vs 2.50 ms;
// its walk alone, debug shape 307, 3.39 ms): one chain per wave issues ~30
// scalar instructions per prefix, and a CU's scalar unit serves all of its
// waves — the walk is scalar-issue-bound where the lane-per-object walk puts
// 64 chains in each instruction (profiles/r6/ab_wide_stream.jsonl).
// SHAPE (debug forms, WRONG coordinates): 1 = no hash (a coordinate is its
// descriptor), 2 = no walk (made-up descriptors inside the value).
template <uint32_t CH, int SHAPE = 0>
__global__ void __launch_bounds__(64) sweep_wide_stream_kernel(const EncodedArgs a) {
    static_assert(CH >= 1024 && (CH & (CH - 1)) == 0, "CH: a power of two, at least 1 KiB");
    __shared__ __attribute__((aligned(16))) uint8_t ring[2 * CH + 16];
    const uint32_t lane = threadIdx.x;
    const uint64_t i = blockIdx.x;
    const uint32_t A = a.A;
    const uint8_t* v = a.vals + a.val_off[i];
    const uint32_t vlen = a.val_len[i];
    uint64_t* out = a.coords + i * A;
    const uint8_t* sb = (const uint8_t*)((uintptr_t)v & ~(uintptr_t)15);
    const uint32_t lead = (uint32_t)((uintptr_t)v & 15);
    const uint64_t S = (uint64_t)lead + vlen;  // stream bytes
    const uint64_t nch = (S + CH - 1) / CH;

    // chunk c into half c & 1: whole 16-byte units, the last partial unit as
    // dwords (never past the dword holding the value's last byte)
    uint64_t hold[2] = {~0ull, ~0ull};
    auto load = [&](uint64_t c) {
        uint8_t* dst = ring + (c & 1) * CH;
        const uint64_t u0 = c * (CH / 16), U = S >> 4;
        if (u0 < U) dma_units16<false>(sb + 16 * u0, dst, (uint32_t)std::min<uint64_t>(CH / 16, U - u0));
        const uint64_t tb = U * 16;
        const uint32_t td = ((uint32_t)(S & 15) + 3) >> 2;
        if (td && tb >= c * CH && tb < (c + 1) * CH && lane < td)
            __builtin_amdgcn_global_load_lds(sb + tb + 4 * lane, (lds_void_t)(dst + (tb - c * CH)), 4, 0, 0);
        if (!(c & 1) && lane == 0)  // the ring's wrap: an even chunk's first dword again after the ring
            __builtin_amdgcn_global_load_lds(sb + c * CH, (lds_void_t)(ring + 2 * CH), 4, 0, 0);
        hold[c & 1] = c;
    };
    // Stream bytes below `ready` have landed in the ring (and nothing the walk
    // still reads has been overwritten): the walk's steps check only that.  At
    // the edge: the chunks [t, t + 4) lies in are loaded if not held, waited
    // for, and the next chunk prefetched into the other half when it is dead.
    uint64_t ready = 0;
    auto advance = [&](uint64_t t) {
        const uint64_t c0 = t / CH, c1 = (t + 3) / CH;
        if (hold[c0 & 1] != c0 || hold[c1 & 1] != c1) {  // a jump: no DMA still in flight into a half reloaded
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (hold[c0 & 1] != c0) load(c0);
            if (hold[c1 & 1] != c1) load(c1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // LDS DMA is not ordered before ds_read
        ready = std::min<uint64_t>(S, (c1 + 1) * CH);
        if (c1 == c0 && c0 + 1 < nch) load(c0 + 1);  // the other half is dead
    };
    auto ring_be32 = [&](uint64_t t) {
        const uint32_t r = (uint32_t)(t & (2 * CH - 1));
        return __builtin_amdgcn_readfirstlane(
            __builtin_bswap32(*(const __attribute__((address_space(3))) u32_unaligned*)(
                (const __attribute__((address_space(3))) uint8_t*)(lds_void_t)ring + r)));
    };
    if (nch) load(0);

    // :174-192 version and count
    bool ok = vlen >= 10;
    uint64_t version = 0;
    if (ok) {
        advance(lead);  // the header lies in chunk 0
        version = ((uint64_t)ring_be32(lead) << 32) | ring_be32(lead + 4);
        ok = (ring_be32(lead + 6) & 0xffffu) == A - 1;
    }
    uint32_t pos = 10;  // pos <= vlen throughout
    bool bad = false;
    for (uint32_t j0 = 0; j0 < A; j0 += 64) {
        const uint32_t jend = std::min(j0 + 64, A);
        uint32_t dpos = 0, dlen = 0;
        // :198-213, and every attribute inside the value
        for (uint32_t j = std::max(j0, 1u); ok && j < jend; ++j) {
            const uint64_t t = (uint64_t)lead + pos;
            if (vlen - pos < 4) {
                ok = false;
                break;
            }
            if (SHAPE != 2 && t + 4 > ready) advance(t);
            const uint32_t L = SHAPE == 2 ? std::min<uint32_t>(64, vlen - pos - 4) : ring_be32(t);
            pos += 4;
            if (L > vlen - pos) {
                ok = false;
                break;
            }
            if (lane == j - j0) {
                dpos = pos;
                dlen = L;
            }
            pos += L;
        }
        if (!ok) break;
        const uint32_t j = j0 + lane;
        const bool in = j < jend;
        const uint8_t* p = j == 0 ? a.keys + a.key_off[i] : v + dpos;
        const uint32_t L = j == 0 ? a.key_len[i] : dlen;
        const uint32_t code = in ? (uint32_t)a.codes_dev[j] : (uint32_t)CODE_ZERO;
        const uint64_t h = SHAPE == 1 ? (uint64_t)(uintptr_t)p ^ L : hash_one(code, p, L, bad);
        if (in) out[j] = h;
    }
    if (!ok) {
        for (uint32_t j = lane; j < A; j += 64) out[j] = 0;
        version = 0;
    }
    if (a.versions && lane == 0) a.versions[i] = version;
    if (a.status && lane == 0 && !ok) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS DMA outlives the wave
}

// One launch, a lane per object (debug 312): each step reads the attribute's
// pieces and the next prefix together (one memory latency a step), hashes the
// attribute — every lane holds attribute j of its own object, so the code is
// wave-uniform and only the string lengths diverge — and buffers 16
// coordinates per store group.  Each value byte is read once; the cost is the
// chains in flight: n objects make n / 64 waves.
__global__ void __launch_bounds__(256) sweep_wide_fused_kernel(const EncodedArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < a.n;
    const uint32_t A = a.A;
    const uint64_t ii = live ? i : 0;
    const uint8_t* v = a.vals + a.val_off[ii];
    const uint32_t vlen = live ? a.val_len[ii] : 0u;
    uint64_t* out = a.coords + ii * A;
    bool bad = false;
    // :174-192 version and count
    bool ok = live && vlen >= 10;
    uint64_t version = 0;
    if (ok) {
        version = be64_at(v);
        ok = (be32_at(v + 6) & 0xffffu) == A - 1;
    }
    uint32_t pos = 10;  // the next prefix's offset; pos <= vlen while ok
    uint32_t Lnext = ok && A > 1 && vlen - pos >= 4
                         ? __builtin_bswap32(*(const __attribute__((address_space(1))) u32_unaligned*)(v + pos))
                         : 0u;
    uint64_t buf[16];
    for (uint32_t j0 = 0; j0 < A; j0 += 16) {
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t j = j0 + k;
            uint64_t h = 0;
            if (j == 0) {
                h = hash_one(live ? (uint32_t)a.codes_dev[0] : (uint32_t)CODE_ZERO, a.keys + a.key_off[ii],
                             live ? a.key_len[ii] : 0u, bad);
            } else if (j < A) {
                // :198-213, and every attribute inside the value
                const uint32_t L = Lnext;
                if (ok && vlen - pos < 4) ok = false;
                const uint32_t at = pos + 4;
                if (ok && L > vlen - at) ok = false;
                const uint32_t np = ok ? at + L : pos;
                Lnext = ok && j + 1 < A && vlen - np >= 4
                            ? __builtin_bswap32(*(const __attribute__((address_space(1))) u32_unaligned*)(v + np))
                            : 0u;
                h = hash_one(ok ? (uint32_t)a.codes_dev[j] : (uint32_t)CODE_ZERO, v + at, ok ? L : 0u, bad);
                pos = np;
            }
            buf[k] = h;
        }
        if (live && ok) {
#pragma unroll
            for (uint32_t k = 0; k < 16; ++k)
                if (j0 + k < A) out[j0 + k] = buf[k];
        }
    }
    if (live && !ok) {
        for (uint32_t j = 0; j < A; ++j) out[j] = 0;
        version = 0;
    }
    if (live && a.versions) a.versions[i] = version;
    if (a.status && __any(live && !ok) && (threadIdx.x & 63) == 0) atomicOr(a.status, 1u << 6 /* HDX_E_BADENC */);
    if (bad && a.status) atomicOr(a.status, 1u << 2 /* HDX_E_BADSIZE */);
}

static hipError_t launch_sweep_wide_fused(const EncodedArgs& a, hipStream_t stream) {
    const uint64_t blocks = (a.n + 255) / 256;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(sweep_wide_fused_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, a);
    return hipGetLastError();
}

template <uint32_t CH, int SHAPE = 0>
static hipError_t launch_sweep_wide_stream(const EncodedArgs& a, hipStream_t stream) {
    if (a.n > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((sweep_wide_stream_kernel<CH, SHAPE>), dim3((uint32_t)a.n), dim3(64), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_sweep_wide_debug(const EncodedArgs& a, hipStream_t stream, int variant) {
    switch (variant) {
        case 304: return launch_sweep_wide_stream<4096>(a, stream);
        case 305: return launch_sweep_wide_stream<2048>(a, stream);
        case 306: return launch_sweep_wide_stream<8192>(a, stream);
        case 307: return launch_sweep_wide_stream<4096, 1>(a, stream);  // debug shape: no hash
        case 308: return launch_sweep_wide_stream<4096, 2>(a, stream);  // debug shape: no walk
        case 312: return launch_sweep_wide_fused(a, stream);              // one launch, a lane per object
        default: return hipErrorInvalidValue;
    }
}

}  // namespace hdx
