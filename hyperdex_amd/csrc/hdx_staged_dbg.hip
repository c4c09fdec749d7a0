// hdx_staged_dbg.hip — (debug library only: an A/B experiment)
// LDS-staged hashing of packed batches (variants 80-83).
//
// hdx_hash_batch_device's contract (include/hdxhash.h): coords[i*A + j] =
// hs[j] of hyperdex::hash(schema, key, value, hs) (common/hash.cc:56-68).
//
// Why this shape.  The gather kernels (hdx_kernels.hip)
// load every slot's bytes with per-lane 16-byte loads: each load instruction
// touches ~64 cache lines, and on config 3b the texture-address unit is ~78 %
// busy beside ~80 % VALU.  Here one wave owns K whole objects:
//   1. lengths (coalesced), per-object sizes and offsets (DPP scans), a
//      contiguity check;
//   2. the group's bytes -> a wave-private LDS window with global_load_lds
//      (1 KiB per instruction: 8 lines instead of 64) — one HBM round trip;
//   3. descriptors {window offset, length} + a counting sort by work class;
//   4. the non-string slots in a lean loop, then the strings in class-sorted
//      passes of 64, every byte read from LDS with dword reads + v_alignbyte;
//   5. coordinates parked over their descriptors, one coalesced store.
// A group whose objects are not back to back in the blob, or whose bytes do
// not fit the window, is hashed the same way from global memory (the A4
// loads of hdx_loads.h), so every layout gives identical coordinates.
// One wave per workgroup (each wave's LDS is released when it finishes); no
// barrier; the LDS-DMA is waited for once (vmcnt), before any window read.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hdx_device_hash.h"
#include "hdx_internal.h"
#include "hdx_lds_hash.h"
#include "hdx_loads.h"

namespace hdx {

namespace {

constexpr uint32_t kStagedSlotsMax = 256;  // K * A <= this (descriptor / perm arrays)
constexpr int kStagedClasses = 8;

// work classes in ORDER 1 (hdx_kernels.hip work_class): 0 = every non-string,
// 1 = 33..64 B, 2 = <= 16 B, 3 = 17..32 B, 4.. = > 64 B by loop blocks
__device__ __forceinline__ uint32_t staged_class(uint32_t code, uint32_t n) {
    if (code != CODE_STRING) return 0;
    if (n > 64) {
        const uint32_t b = (n - 1) >> 6;
        return b >= 4 ? 7u : 3u + b;
    }
    return n > 32 ? 1u : n <= 16 ? 2u : 3u;
}

struct alignas(8) StDesc {
    uint32_t off;  // staged: byte offset in the window; else offset inside the object
    uint32_t len;
};

// Per-wave LDS: the window (dynamic shared memory, win_bytes + 64 bytes of
// slack for the A4 over-reads) and the metadata below (static: a separate
// object, so the compiler sees that descriptor work does not touch the bytes
// the LDS-DMA is still writing, and does not wait for the DMA before it).
struct StagedMeta {
    StDesc desc[kStagedSlotsMax];  // slot descriptors, then the parked coordinates
    uint64_t obase[64];            // object bases (global form)
    uint16_t perm[kStagedSlotsMax];
    uint32_t cnt[kStagedClasses];
    uint8_t codes[256];
};
__host__ __device__ constexpr uint32_t staged_lds_bytes(uint32_t win) { return win + 64; }

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
    return pack64(__builtin_amdgcn_readlane((uint32_t)v, l), __builtin_amdgcn_readlane((uint32_t)(v >> 32), l));
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

template <int NCH /* ceil(K*A/64), compile-time upper bound */>
__global__ void __launch_bounds__(64)
hash_staged_kernel(const BatchArgs args) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ StagedMeta meta;
    const uint32_t WB = args.win_bytes;
    uint8_t* win = smem;
    StDesc* desc = meta.desc;
    uint64_t* obase = meta.obase;
    uint16_t* perm = meta.perm;
    uint32_t* cnt = meta.cnt;
    uint8_t* codes = meta.codes;
    const ldsw_t w = as_ldsw(win);

    const int lane = threadIdx.x;
    const uint32_t A = args.A, K = args.K;
    const uint64_t o0 = (uint64_t)blockIdx.x * K;
    if (o0 >= args.n) return;
    const uint32_t nobj = (uint32_t)min<uint64_t>(K, args.n - o0);
    const uint32_t ns = nobj * A;  // slots of the group (<= 256)
    const uint64_t q0 = o0 * A;

    // ---- 1. the group's byte range; its bytes -> LDS as early as possible -----
    // With a next group and back-to-back objects the range is [obj_base[o0],
    // obj_base[o0 + K]): the DMA goes out before the lengths are back (checked
    // below; a group that turns out not to be contiguous is hashed from global
    // memory instead).  The last group waits for its lengths.
    const uint8_t* blob = args.blob;
    const uint64_t b0 = args.obj_base[o0];
    const bool has_next = o0 + K < args.n;
    const uint64_t b_next = has_next ? args.obj_base[o0 + K] : 0;
    const uint32_t lead = (uint32_t)((uintptr_t)(blob + b0) & 15);
    const uint8_t* s16 = blob + b0 - lead;
    bool early = has_next && b_next > b0 && ((lead + (b_next - b0) + 15) & ~15ull) <= WB;
    uint32_t early_units = early ? (uint32_t)((lead + (b_next - b0) + 15) >> 4) : 0u;
    for (uint32_t u0 = 0; u0 < early_units; u0 += 64) {
        const uint32_t u = u0 + (uint32_t)lane;
        if (u < early_units)
            __builtin_amdgcn_global_load_lds((const void*)(s16 + 16ull * u),
                                             (__attribute__((address_space(3))) void*)(win + 16 * u0), 16, 0, 0);
    }

    // ---- 2. lengths, in-object offsets, object sizes --------------------------
    uint32_t L[NCH], off[NCH], code[NCH];
    const uint32_t packed_codes = reinterpret_cast<const uint32_t*>(args.codes)[lane];
    reinterpret_cast<uint32_t*>(codes)[lane] = packed_codes;  // the code table, for per-lane lookups
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        L[c] = s < ns ? args.attr_len[q0 + s] : 0u;
    }
    const uint64_t mybase = (uint32_t)lane < nobj ? args.obj_base[o0 + lane] : 0;
    uint32_t carry = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        const uint32_t o = div_small(s, args.a_magic);
        const uint32_t j = s - o * A;
        const uint32_t Sx = wave_scan_dpp(L[c]) - L[c];
        const int head = lane - (int)j;
        const uint32_t head_sx = __shfl(Sx, head < 0 ? 0 : head, 64);
        off[c] = head >= 0 ? Sx - head_sx : carry + Sx;
        carry = __builtin_amdgcn_readlane(off[c] + L[c], 63);
        const uint32_t cd = args.uniform_code != 0xffu
                                ? args.uniform_code
                                : (__shfl(packed_codes, (int)(j >> 2), 64) >> (8 * (j & 3))) & 0xffu;
        code[c] = s < ns ? cd : (uint32_t)CODE_ZERO;
        // object o's size: the end of its last attribute
        if (s < ns && j == A - 1) obase[o] = off[c] + L[c];  // object sizes, parked in obase for a moment
    }
    wave_lds_sync();
    const uint64_t mysize = (uint32_t)lane < nobj ? obase[lane] : 0;
    wave_lds_sync();
    if ((uint32_t)lane < nobj) obase[lane] = mybase;
    // back to back in the blob (and, with a next group, ending where it starts)
    const uint64_t nextb = pack64((uint32_t)__shfl_down((int)(uint32_t)mybase, 1, 64),
                                  (uint32_t)__shfl_down((int)(uint32_t)(mybase >> 32), 1, 64));
    const bool runs = __all((uint32_t)lane + 1 >= nobj || nextb == mybase + mysize);
    const uint64_t bend = readlane64(mybase + mysize, (int)nobj - 1);
    const uint64_t cover = (lead + (bend - b0) + 15) & ~15ull;
    const bool staged = runs && cover <= WB && (!early || bend == b_next);
    if (staged && !early) {  // the last group: its bytes now
        const uint32_t units = (uint32_t)(cover >> 4);
        for (uint32_t u0 = 0; u0 < units; u0 += 64) {
            const uint32_t u = u0 + (uint32_t)lane;
            if (u < units)
                __builtin_amdgcn_global_load_lds((const void*)(s16 + 16ull * u),
                                                 (__attribute__((address_space(3))) void*)(win + 16 * u0), 16, 0, 0);
        }
    }
    // the window is read below: every LDS-DMA of this wave must have landed
    // (the compiler does not order ds_read after global_load_lds by itself)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- 3. descriptors + counting sort by class ------------------------------
    uint32_t cls[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        const uint32_t o = div_small(s, args.a_magic);
        uint32_t dof = off[c];
        if (staged) dof += lead + (uint32_t)(obase[o < nobj ? o : 0] - b0);
        if (s < ns) desc[s] = StDesc{dof, L[c]};
        cls[c] = s < ns ? staged_class(code[c], L[c]) : 0u;
    }
    if (lane < kStagedClasses) cnt[lane] = 0;
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < NCH; ++c)
        if ((uint32_t)(c * 64 + lane) < ns)
            __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    wave_lds_sync();
    const uint32_t k = lane < kStagedClasses ? cnt[lane] : 0u;
    const uint32_t start = wave_scan_dpp(k) - k;
    const uint32_t n0 = __builtin_amdgcn_readlane(start + k, 0);  // non-string slots come first
    if (lane < kStagedClasses) cnt[lane] = start;
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const uint32_t s = (uint32_t)(c * 64 + lane);
        if (s < ns) {
            const uint32_t pos = __hip_atomic_fetch_add(&cnt[cls[c]], 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WAVEFRONT);
            perm[pos] = (uint16_t)s;
        }
    }
    wave_lds_sync();

    // ---- 4. hash: non-strings (lean), then class-sorted string passes ---------
    bool bad = false;
    uint64_t* parked = reinterpret_cast<uint64_t*>(desc);
    for (uint32_t t = (uint32_t)lane; t < ns; t += 64) {
        const uint32_t s = perm[t];
        const StDesc d = desc[s];
        const uint32_t o = div_small(s, args.a_magic);
        const uint32_t j = s - o * A;
        const uint32_t cd = codes[j];
        uint64_t h;
        if (t < n0) {
            h = staged ? hash_numeric_lds(w, cd, d.off, d.len, bad)
                       : hash_numeric_slot(cd, args.blob + obase[o] + d.off, d.len, bad);
        } else if (staged) {
            h = hash_string_lds(w, d.off, d.len);
        } else {
            const uint8_t* p = args.blob + obase[o] + d.off;
            h = hash_blk<false, false, true>(CODE_STRING, p, d.len,
                                             consume_any<true>(issue_any<true>(CODE_STRING, p, d.len)), bad);
        }
        parked[s] = h;  // over its own, consumed, descriptor
    }
    wave_lds_sync();

    // ---- 5. coalesced stores in slot order ------------------------------------
    for (uint32_t s = (uint32_t)lane; s < ns; s += 64) __builtin_nontemporal_store(parked[s], args.coords + q0 + s);
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}

// K objects per wave so that K * A <= slots (<= 256), window win_bytes.
template <int NCH>
static hipError_t launch_staged_nch(BatchArgs args, hipStream_t stream) {
    const uint64_t waves = (args.n + args.K - 1) / args.K;
    if (waves == 0) return hipSuccess;
    if (waves > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_staged_kernel<NCH>), dim3((uint32_t)waves), dim3(64), staged_lds_bytes(args.win_bytes),
                       stream, args);
    return hipGetLastError();
}

hipError_t launch_hash_staged(const BatchArgs& a, hipStream_t stream, uint32_t slots, uint32_t win_bytes) {
    BatchArgs args = a;
    if (args.n == 0) return hipSuccess;
    if (slots > kStagedSlotsMax || win_bytes % 1024 || win_bytes > 65536) return hipErrorInvalidValue;
    if (args.A > 64) return launch_hash_batch_variant(args, stream, 44);  // wider schemas: the regroup kernel
    args.K = slots / args.A;
    if (args.K == 0) args.K = 1;
    if (args.K > 64) args.K = 64;
    args.win_bytes = win_bytes;
    const uint32_t nch = (args.K * args.A + 63) / 64;
    switch (nch) {
        case 1: return launch_staged_nch<1>(args, stream);
        case 2: return launch_staged_nch<2>(args, stream);
        case 3: return launch_staged_nch<3>(args, stream);
        default: return launch_staged_nch<4>(args, stream);
    }
}

}  // namespace hdx
