// hdx_wsweep_dbg.hip — the wave-staged sweep's A/B forms and debug shapes
// (hdx_wsweep.h), built into libhdxhash_dbg.so only (Makefile SRCS_DBG).
#include "hdx_wsweep.h"

namespace hdx {

// A/B forms (debug library): 0 = the product's, 1 = 7 objects, 2 = 3 passes /
// 11 objects / 14 KiB, 6 = the product's without the pass-boundary gap,
// 7 / 8 debug shapes (WRONG coordinates), 9 = the product's with the one-block
// > 64-byte loop, 12 without the shared final mix16, 13 with the DMA as
// inline asm (4.24 vs 4.20 ms per 10 M: the builtin stays)
hipError_t launch_hash_wsweep(const EncodedArgs& a, hipStream_t stream, int form) {
    if (a.n == 0) return hipSuccess;
    if (!a.coords) return hipErrorInvalidValue;
    switch (form) {
        case 0: return launch_hash_wsweep_product(a, stream);
        case 1: return launch_wsweep_t<2, 8704, 7>(a, stream);
        case 2: return launch_wsweep_t<3, 14336, 11>(a, stream);
        case 6: return launch_wsweep_t<2, 8704, 6, false, false, 0, 2>(a, stream);
        case 7: return launch_wsweep_t<2, 8704, 6, false, true, 1>(a, stream);  // debug shape: no hash
        case 8: return launch_wsweep_t<2, 8704, 6, false, true, 2>(a, stream);  // debug shape: no hash, no walk
        case 9: return launch_wsweep_t<2, 8704, 6, false, true, 0, 1>(a, stream);  // the one-block loop
        case 12: return launch_wsweep_t<2, 8704, 6, false, true, 0, 2, false>(a, stream);  // without the shared final mix16
        case 13: return launch_wsweep_t<2, 8704, 6, false, true, 0, 3, true>(a, stream);  // the DMA as inline asm
        case 14: return launch_wsweep_t<2, 8704, 6, false, true, 0, 3, false, false, true>(a, stream);  // pass loop not unrolled
        case 15: return launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, false>(a, stream);  // the branchy class, guarded loads
        case 16: return launch_wsweep_t<2, 8704, 6, false, true, 0, 3, false, true, true>(a, stream);  // without TNUM
        case 17: return launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, false>(a, stream);  // without the record span
        case 18: return launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, false, false>(a, stream);  // keys in place gathered by dwords (round 3)
        case 19: return launch_wsweep_t<2, 8704, 6, false, true, 3, 13, false, true, true, false>(a, stream);  // debug shape: no copy, no walk, the hash
        case 20: return launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, false, true, true>(a, stream);  // round 3's span copy (per KiB)
        case 21: return launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, true, true, true>(a, stream);  // the record form, round 3's span copy
        case 22: return launch_wsweep_t<2, 8704, 6, false, true, 4, 13, false, true, true, false>(a, stream);  // the walk's reads as dword pairs + v_alignbyte (round 3)
        case 23: return a.keys == a.vals  // the product, one wave per workgroup
                        ? launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, true, true, false, 1>(a, stream)
                        : launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, false, true, false, 1>(a, stream);
        case 24: return a.keys == a.vals  // the product, two waves per workgroup
                        ? launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, true, true, false, 2>(a, stream)
                        : launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, false, true, false, 2>(a, stream);
        case 25: return a.keys == a.vals  // 7.75 KiB windows, one wave per workgroup: 17 waves per CU
                        ? launch_wsweep_t<2, 7936, 6, false, true, 0, 13, false, true, true, true, true, false, 1>(a, stream)
                        : launch_wsweep_t<2, 7936, 6, false, true, 0, 13, false, true, true, false, true, false, 1>(a, stream);
        case 27: return a.keys == a.vals  // the product, XCD-aware block order
                        ? launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, true, true, false, 1, true>(a, stream)
                        : launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, false, true, false, 1, true>(a, stream);
        case 28: return a.keys == a.vals  // 7 objects per wave in 9.5 KiB windows (one wave per workgroup, XCD order)
                        ? launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, true, true, false, 1, true>(a, stream)
                        : launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, false, true, false, 1, true>(a, stream);
        case 29: return a.keys == a.vals  // 7 objects per wave in 9 KiB windows (one wave per workgroup, XCD order)
                        ? launch_wsweep_t<2, 9216, 7, false, true, 0, 13, false, true, true, true, true, false, 1, true>(a, stream)
                        : launch_wsweep_t<2, 9216, 7, false, true, 0, 13, false, true, true, false, true, false, 1, true>(a, stream);
        case 30: return a.keys == a.vals  // 3 passes, 11 objects per wave in 14 KiB windows
                        ? launch_wsweep_t<3, 14336, 11, false, true, 0, 13, false, true, true, true, true, false, 1, true>(a, stream)
                        : launch_wsweep_t<3, 14336, 11, false, true, 0, 13, false, true, true, false, true, false, 1, true>(a, stream);
        case 31: return a.keys == a.vals  // the product without wave priorities (round 5 before)
                        ? launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, true, true, false, 1, true, 0>(a, stream)
                        : launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, false, true, false, 1, true, 0>(a, stream);
        case 36: return a.keys == a.vals  // round 6: the product with NUM2 (numerics by selects, the class table)
                        ? launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, true, true, false, 1, true, 4, true>(a, stream)
                        : launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, false, true, false, 1, true, 4, true>(a, stream);
        // the product's debug shapes (WRONG coordinates): 38 no hash, 39 no hash and no walk, 40 no copy and no walk
        case 38: return launch_wsweep_t<2, 9728, 7, false, true, 1, 14, false, true, true, false, true, false, 1, true, 4, true>(a, stream);
        case 39: return launch_wsweep_t<2, 9728, 7, false, true, 2, 14, false, true, true, false, true, false, 1, true, 4, true>(a, stream);
        case 40: return launch_wsweep_t<2, 9728, 7, false, true, 3, 14, false, true, true, false, true, false, 1, true, 4, true>(a, stream);
        case 37: return a.keys == a.vals  // the product before LOOP 4 (two head reads per divergent pass; = 36)
                        ? launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, true, true, false, 1, true, 4, true>(a, stream)
                        : launch_wsweep_t<2, 9728, 7, false, true, 0, 13, false, true, true, false, true, false, 1, true, 4, true>(a, stream);
        case 26: return a.keys == a.vals  // round 4's product: four waves per workgroup
                        ? launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, true, true, false, 4>(a, stream)
                        : launch_wsweep_t<2, 8704, 6, false, true, 0, 13, false, true, true, false, true, false, 4>(a, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace hdx
