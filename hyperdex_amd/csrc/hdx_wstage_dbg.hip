// hdx_wstage_dbg.hip — the wave-staged kernel's A/B forms (debug library
// only, libhdxhash_dbg.so): window sizes and passes per wave, the class sort
// over the workgroup (hash_wgstage_kernel), debug shapes.  Results: DESIGN.md
// §4.5 (round 3), profiles/r3/ab_wstage_*.jsonl.
#include "hdx_wstage.h"

namespace hdx {

template <int NCH, uint32_t WB>
__global__ void __launch_bounds__(256)
hash_wgstage_kernel(const BatchArgs args) {
    static_assert(NCH >= 1 && NCH <= 2 && WB % 16 == 0, "slot ids are 9 bits");
    constexpr uint32_t SL = NCH * 64;  // slots per wave
    __shared__ __attribute__((aligned(16))) uint8_t win_all[4][WB + 64];
    __shared__ uint64_t desc_all[4 * SL];  // {absolute window offset, length}; then the parked coordinate
    __shared__ uint16_t perm[4 * SL];      // workgroup slot | code << 9, in class order
    __shared__ uint32_t wcnt[4][kClasses]; // per wave: staged slots per class
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    uint64_t* desc = desc_all + w * SL;
    const ldsw_t lw_all = as_ldsw(&win_all[0][0]);
    const uint32_t win_off = (uint32_t)w * (WB + 64);

    const uint64_t o0 = ((uint64_t)blockIdx.x * 4 + w) * args.K;
    const bool live = o0 < args.n;  // (every wave reaches every barrier)
    Group<NCH> g{};
    if (live) g = describe_group<NCH, WB, 0>(args, o0, win_all[w], win_off, desc);
    const bool sorted = live && g.staged;
    bool bad = false;
    if (live && !g.staged) {  // hashed here, from global memory, in slot order
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t s = (uint32_t)(c * 64 + lane);
            desc[s] = hash_slot<0>(args, lw_all, false, g.mybase, s, g.code[c], desc[s], bad);
        }
    }
    // per-class counts of this wave's staged slots
    uint32_t mine[kClasses];
#pragma unroll
    for (int k = 0; k < kClasses; ++k) {
        uint32_t n = 0;
#pragma unroll
        for (int c = 0; c < NCH; ++c)
            n += (uint32_t)__popcll(__ballot(sorted && (uint32_t)(c * 64 + lane) < g.ns && g.cls[c] == (uint32_t)k));
        mine[k] = n;
    }
    if (lane < kClasses) {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < kClasses; ++k) v = lane == k ? mine[k] : v;
        wcnt[w][lane] = v;
    }
    __syncthreads();  // (1) counts published, descriptors written

    // class bases over the workgroup, and this wave's offset inside each class
    uint32_t tot = 0, before = 0;  // lane k < kClasses: class k's total, waves < w's share
    if (lane < kClasses) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const uint32_t x = wcnt[v][lane];
            tot += x;
            before += v < w ? x : 0u;
        }
    }
    const uint32_t cbase = wave_scan_dpp(tot) - tot;  // lanes >= kClasses add 0
    const uint32_t T = __builtin_amdgcn_readlane(cbase + tot, kClasses - 1);
    const uint32_t start = cbase + before;  // lane k: this wave's first position in class k
    uint32_t seen[kClasses];  // per class: this wave's next position (read with every lane active:
#pragma unroll                // a ds_bpermute from an inactive lane returns 0)
    for (int k = 0; k < kClasses; ++k) seen[k] = (uint32_t)__shfl((int)start, k, 64);
    if (sorted) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t s = (uint32_t)(c * 64 + lane);
            const bool in = s < g.ns;
#pragma unroll
            for (int k = 0; k < kClasses; ++k) {
                const uint64_t m = __ballot(in && g.cls[c] == (uint32_t)k);
                if (in && g.cls[c] == (uint32_t)k) {
                    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    const uint32_t pos = seen[k] + rank;
                    perm[pos] = (uint16_t)((uint32_t)(w * SL + s) | (g.code[c] << 9));
                }
                seen[k] += (uint32_t)__popcll(m);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's window has landed
    __syncthreads();  // (2) permutation complete, every window landed

    // passes of 64 class-sorted slots of the workgroup: wave w takes w, w+4, ...
    const uint32_t passes = (T + 63) / 64;
    for (uint32_t p = (uint32_t)w; p < passes; p += 4) {
        const uint32_t idx = p * 64 + (uint32_t)lane;
        if (idx < T) {
            const uint32_t e = perm[idx];
            const uint32_t gs = e & 0x1ffu, cd = e >> 9;
            desc_all[gs] = hash_slot<0>(args, lw_all, true, 0, gs, cd, desc_all[gs], bad);
        }
    }
    __syncthreads();  // (3) every parked coordinate written

    if (live) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const uint32_t s = (uint32_t)(c * 64 + lane);
            if (s < g.ns) __builtin_nontemporal_store(desc[s], args.coords + g.q0 + s);
        }
    }
    if (bad && args.status) atomicOr(args.status, 1u << 2 /* HDX_E_BADSIZE */);
}


template <int NCH, uint32_t WB>
static hipError_t launch_wgstage_t(BatchArgs args, hipStream_t stream) {
    args.K = std::min<uint32_t>((uint32_t)(64 * NCH) / args.A, 63u);
    if (args.K == 0) return hipErrorInvalidValue;
    const uint64_t waves = (args.n + args.K - 1) / args.K;
    const uint64_t blocks = (waves + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (blocks > 0x7fffffffULL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((hash_wgstage_kernel<NCH, WB>), dim3((uint32_t)blocks), dim3(256), 0, stream, args);
    return hipGetLastError();
}


// form: 0 = 2 passes / 10 KiB windows; 1 = 3 / 14 KiB; 2 = 2 / 8 KiB;
// 3 = 1 / 5 KiB; 4 = 4 / 18 KiB; 5 = 2 / 8832 B (four workgroups per CU);
// 6 = form 5 with at most 6 objects per wave.  A wider schema than the form's
// passes hold (K = 0) returns hipErrorInvalidValue.
hipError_t launch_hash_wstage(const BatchArgs& args, hipStream_t stream, int form) {
    if (args.n == 0) return hipSuccess;
    switch (form) {
        case 0: return launch_wstage_t<2, 10240>(args, stream);
        case 1: return launch_wstage_t<3, 14336>(args, stream);
        case 2: return launch_wstage_t<2, 8192>(args, stream);
        case 3: return launch_wstage_t<1, 5120>(args, stream);
        case 4: return launch_wstage_t<4, 18432>(args, stream);
        case 5: return launch_wstage_t<2, 8832>(args, stream);
        case 6: return launch_wstage_t<2, 8832, 6>(args, stream);
        case 7: return launch_wstage_t<2, 8832, 63, 1>(args, stream);  // debug shape: no hash
        case 8: return launch_wstage_t<2, 8832, 63, 2>(args, stream);  // debug shape: no DMA
        case 9: return launch_wstage_t<2, 8832, 3>(args, stream);  // <= 3 objects: per-regime costs on uniform batches
        // head/tail window hashing (hash_slot_window)
        case 12: return launch_wstage_t<2, 8832, 63, 0, true>(args, stream);
        case 13: return launch_wstage_t<2, 8832, 3, 0, true>(args, stream);  // <= 3 objects (per-regime costs)
        case 14: return launch_wstage_t<3, 14336, 63, 0, true>(args, stream);
        case 15: return launch_wstage_t<2, 8832, 63, 0, true, 3>(args, stream);  // 12 in class order 3
        case 16: return launch_wstage_t<2, 8832, 63, 0, true, 1, true>(args, stream);  // 12 with b128 window reads
        case 18: return launch_wstage_t<2, 8832, 63, 1, true>(args, stream);  // debug shape of 12: no hash (WRONG coordinates)
        case 19: return launch_wstage_t<2, 8832, 63, 0, 2, 1>(args, stream);  // the product without the pass-boundary gap
        case 39: return launch_wstage_t<2, 8832, 63, 0, 1, 4, false, false, true, true>(args, stream);  // the product with the one-block loop
        case 40: return launch_wstage_t<2, 8832, 63, 0, 2, 1, false, false, true>(args, stream);  // the product with the DMA as the builtin
        case 41: return launch_wstage_t<2, 8832, 63, 1, 2, 1, false, false, true, true>(args, stream);  // debug shape of the product: no hash
        case 42: return launch_wstage_t<2, 8832, 63, 0, 3, 4, false, false, true, true>(args, stream);  // the product with the shared final mix16
        case 44: return launch_wstage_t<2, 8832, 63, 0, 2, 4, false, false, true, true, false>(args, stream);  // the product, pass loop not unrolled
        case 45: return launch_wstage_t<2, 8832, 63, 0, 5, 1, false, false, true, true>(args, stream);  // the product with the branchy class (ORDER 1)
        case 46: return launch_wstage_t<2, 8832, 63, 0, 2, 4, false, false, true, true>(args, stream);  // the product without TNUM
        case 48: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 2, false, true, true>(args, stream);  // debug shape: the product's LDS reads conflict-free (WRONG coordinates)
        case 49: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 3, false, true, true>(args, stream);  // debug shape: no funnel shifts (WRONG coordinates)
        case 55: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, true>(args, stream);  // the product with round 3's per-KiB span copy
        case 56: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 1>(args, stream);  // the product (one wave per workgroup)
        case 57: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 2>(args, stream);  // the product, two waves per workgroup
        case 58: return launch_wstage_t<2, 7680, 6, 0, 5, 4, 0, false, true, true, true, false, 1>(args, stream);  // <= 6 objects, 7.5 KiB windows: 18 waves per CU
        case 59: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 4>(args, stream);  // round 4's product: four waves per workgroup
        case 70: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true>(args, stream);  // the product (XCD-aware block order)
        case 73: return launch_wstage_t<3, 14336, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true>(args, stream);  // 3 passes, 11 objects, 14 KiB
        case 75: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true, true>(args, stream);  // descriptors in registers (17 waves per CU)
        case 76: return launch_wstage_t<2, 8704, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true, true>(args, stream);  // ... with 8.5 KiB windows (18 waves per CU)
        case 74: return launch_wstage_t<3, 13312, 10, 0, 5, 4, 0, false, true, true, true, false, 1, true>(args, stream);  // 3 passes, 10 objects, 13 KiB
        case 79: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true, false, true>(args, stream);  // 70 with non-temporal loads (the product before its wave priorities)
        case 78: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 1, false, true, true, true, false, 1, true, false, true>(args, stream);  // the product with dword-aligned ds_read_b128 window reads
        case 87: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true, false, true, 1>(args, stream);  // the product: 79 with the loads at high wave priority
        // round 6: the per-schema slot plan (PLAN), numerics by selects (NUM2), the class table (ORDER 5)
        case 93: return launch_wstage_t<2, 8832, 63, 0, 5, 5, 0, false, true, true, true, false, 1, true, false, true, 1, true, true>(args, stream);  // all three
        case 94: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true, false, true, 1, true, false>(args, stream);  // the plan alone
        case 95: return launch_wstage_t<2, 8832, 63, 0, 5, 4, 0, false, true, true, true, false, 1, true, false, true, 1, false, true>(args, stream);  // NUM2 alone
        case 96: return launch_wstage_t<2, 8832, 63, 0, 5, 5, 0, false, true, true, true, false, 1, true, false, true, 1, false, false>(args, stream);  // the class table alone
        case 97: return launch_wstage_t<2, 8832, 63, 1, 5, 5, 0, false, true, true, true, false, 1, true, false, true, 1, true, true>(args, stream);  // debug shape of 93: no hash (WRONG coordinates)
        case 98: return launch_wstage_t<2, 8832, 63, 0, 5, 5, 0, false, true, true, true, false, 1, true, false, true, 1, true, true>(args, stream);  // the product before LOOP 4 (= 93)
        // the slots class-sorted over the workgroup
        case 10: return launch_wgstage_t<2, 8832>(args, stream);
        case 11: return launch_wgstage_t<1, 4352>(args, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace hdx
