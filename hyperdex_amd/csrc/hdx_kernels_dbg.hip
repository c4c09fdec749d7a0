// hdx_kernels_dbg.hip — the batch hash's A/B alternatives and debug shapes
// (DESIGN.md §4), built into libhdxhash_dbg.so only (Makefile SRCS_DBG): the
// regroup / chunk kernels' other template forms, the wave-staged kernel's
// forms and debug shapes, the fused forms' alternatives, and the
// process-wide variant selection (hdxdbg_set_kernel_variant /
// HDX_KERNEL_VARIANT).  Every form here writes the reference's coordinates
// (except the named debug shapes) and is parity-tested in tests/; none is
// reachable from the product library.  Round 5 removed the retired
// experiments no A/B still used (occupancy caps, quad loads, late heads,
// register descriptors, grid striding, the column / typed / workgroup-sorted /
// LDS-staged / streamed kernels: variants 60-99, 140-191, 220-227); their
// results are in DESIGN.md Appendix A and profiles/r1-r3.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

#include "hdx_regroup.h"

namespace hdx {

hipError_t launch_debug_variant(const BatchArgs& args, hipStream_t stream, int variant) {
    switch (variant) {
        // alternatives for interleaved A/B (scripts/ab_variants.py), bit-exact
        case 18: return launch_regroup<4, true>(args, stream);
        case 19: return launch_regroup<8, true>(args, stream);
        case 26: return launch_regroup<2, true>(args, stream);
        case 30: return launch_chunk<true, true>(args, stream);
        case 31: return launch_chunk<true, false, 0, true>(args, stream);
        case 35: return launch_regroup<2, true, true, true, true>(args, stream);
        case 37: return launch_regroup<2, true, true, true, true, true>(args, stream);
        case 38: return launch_regroup<2, true, true, true, true, false, true>(args, stream);
        case 39: return launch_regroup<8, true, true, true, false, false, true>(args, stream);
        case 45: return launch_regroup<2, true, true, true, true, false, true, 2>(args, stream);
        // one wave per workgroup (round 5): 260 = 21, 261 = 25, 262 = 12, 263 = 20, 264 = 46, 265 = 44
        case 260: return launch_regroup<4, true, false, true, false, false, false, 0, 1>(args, stream);
        case 261: return launch_regroup<16, true, false, false, false, false, false, 0, 1>(args, stream);
        case 262: return launch_chunk<true, false, 0, false, 1>(args, stream);
        case 263: return launch_regroup<8, true, false, true, false, false, false, 0, 1>(args, stream);
        case 264: return launch_regroup<8, true, true, true, false, false, true, 1, 1>(args, stream);
        case 265: return launch_regroup<2, true, true, true, true, false, true, 1, 1>(args, stream);
        // deferred strings (round 5, hash_regroup_defer_kernel): 280 = 21 with the strings
        // first, 281 = ... with cached stores, 282 = strings last, 283 = 8 chunks, 284 = A4 loads,
        // 285 = strings last with cached stores, 286 = 8 chunks with cached stores
        case 280: return launch_regroup_defer<4, true, false, 1>(args, stream);
        case 281: return launch_regroup_defer<4, false, false, 1>(args, stream);
        case 282: return launch_regroup_defer<4, true, false, 2>(args, stream);
        case 283: return launch_regroup_defer<8, true, false, 1>(args, stream);
        case 284: return launch_regroup_defer<4, true, true, 1>(args, stream);
        case 285: return launch_regroup_defer<4, false, false, 2>(args, stream);
        case 286: return launch_regroup_defer<8, false, false, 1>(args, stream);
        // wave-staged (hdx_wstage.hip): 200 2 passes / 10 KiB, 201 3 / 14 KiB, 202 2 / 8 KiB,
        // 203 1 / 5 KiB, 204 4 / 18 KiB, 205 2 / 8832 B, 206 = 205 with <= 6 objects
        case 200: case 201: case 202: case 203: case 204: case 205: case 206: case 207: case 208:
        case 209: case 210: case 211: case 213: case 214: case 215: case 216: case 218: case 219: case 239: case 240: case 241: case 242: case 244: case 245: case 246: case 248: case 249: case 255: case 256: case 257: case 258: case 259: case 270: case 273: case 274: case 275: case 276: case 278: case 279: case 287: case 293: case 294: case 295: case 296: case 297: case 298: {
            const hipError_t e = launch_hash_wstage(args, stream, variant - 200);
            return e == hipErrorInvalidValue ? launch_hash_batch_variant(args, stream, 44) : e;
        }
        // debug shapes: WRONG coordinates, debug library only
        case 40: return launch_chunk<true, false, 1>(args, stream);  // loads only
        case 41: return launch_chunk<true, false, 2>(args, stream);  // arithmetic only
        default: return hipErrorInvalidValue;
    }
}

// Debug library only: the fused forms for interleaved A/B (variants 100-119).
hipError_t launch_fused_debug(const BatchArgs& args, hipStream_t stream, int v) {
    switch (v) {
        case 100: return launch_regroup_regions<4, false, false, false, 0, false>(args, stream);
        case 101: return launch_regroup_regions<4, false, false, false, 0, true>(args, stream);
        case 102: return launch_regroup_regions<2, false, false, false, 0, true>(args, stream);
        case 103: return launch_regroup_regions<8, false, false, false, 0, true>(args, stream);
        case 104: return launch_regroup_regions<4, false, false, false, 0, true>(args, stream, false);
        case 105: return launch_regroup_regions<3, true, true, true, 1, false>(args, stream);
        case 106: return launch_regroup_regions<3, true, true, true, 1, true>(args, stream);
        case 107: return launch_regroup_regions<2, true, true, true, 1, true>(args, stream);
        case 108: return launch_regroup_regions<8, false, false, false, 0, false>(args, stream);
        case 109: return launch_regroup_regions<8, false, false, false, 0, true>(args, stream);
        case 110: return launch_regroup_regions<1, false, false, false, 0, true>(args, stream);
        case 111: return launch_regroup_regions<4, true, true, true, 1, true>(args, stream);
        default: return hipErrorInvalidValue;
    }
}

// Debug library only (libhdxhash_dbg.so): a process-wide kernel selection for
// interleaved A/B runs, from hdxdbg_set_kernel_variant or HDX_KERNEL_VARIANT.
// 33 / 43 / 47 / 48 select the stored-object sweep's alternative forms, 57 / 58
// its walk-only and loads-only debug shapes (hdx_encoded.hip).
static bool known_variant(int v) {
    switch (v) {
        case -1: case 12: case 18: case 19: case 20: case 21: case 25: case 26: case 30: case 31: case 35: case 37:
        case 38: case 39: case 44: case 45: case 46:
        case 260: case 261: case 262: case 263: case 264: case 265:  // 21 / 25 / 12 / 20 / 46 / 44, one wave per workgroup
        case 280: case 281: case 282: case 283: case 284: case 285: case 286:  // 21 with the string slots deferred to passes of their own
        case 300:  // the wide kernel (hdx_wide.hip), at any A
        case 301:  // the wide sweep (hdx_wide.hip), at any A
        case 304: case 305: case 306:  // the wide sweep streamed through an LDS ring in 4 / 2 / 8 KiB chunks (hdx_wide.hip)
        case 307: case 308:  // debug shapes of 304: no hash / no walk (WRONG coordinates)
        case 309: case 310:  // the wide sweep's walk storing its descriptors one / 8 per step group (hdx_wide.hip)
        case 311:  // the wide sweep's hash class-sorted per 256 attributes
        case 312:  // the wide sweep in one launch, a lane per object (walk and hash fused)
        case 313: case 314: case 315:  // the product sweep's debug shapes: no hash / no hash, no walk / no copy, no walk (WRONG coordinates)
        case 100: case 101: case 102: case 103: case 104: case 105: case 106: case 107: case 108: case 109:
        case 110: case 111:  // fused hash + lookup_region forms (launch_fused_debug)
        case 170: case 171: case 172: case 173: case 174:  // the sweep's numeric walk (hdx_encoded.hip)
        case 200: case 201: case 202: case 203: case 204: case 205: case 206:  // wave-staged (hdx_wstage.hip)
        case 207: case 208:  // its debug shapes: no hash / no DMA (WRONG coordinates)
        case 209:  // <= 3 objects per wave (per-regime VALU on uniform batches)
        case 212: case 213: case 214: case 215: case 216:  // wave-staged, head/tail window hashing
        case 217:  // wave-staged with the fused region lookup (hdx_hash_batch_regions_device)
        case 218:  // debug shape of 212: no hash (WRONG coordinates)
        case 219:  // 212 without the pass-boundary gap (class_sort)
        case 239:  // 212 / 230 with the one-block > 64-byte loop (city_gt64_lds LOOP 1)
        case 240:  // 212 with the DMA as the builtin (describe_group ADMA off)
        case 241:  // debug shape of 212: no hash (WRONG coordinates)
        case 242:  // 212 with / 230 without one final mix16 for the > 64 and 8..32-byte regimes (LOOP 3)
        case 243:  // 230 with the DMA as inline asm
        case 244:  // 212 / 230 with the pass loop not unrolled
        case 245:  // 212 / 230 with the branchy work class (and, 230, guarded loads)
        case 246:  // 212 / 230 without TNUM (numerics read apart from the strings' tail)
        case 230: case 231: case 232: case 233: case 234:  // wave-staged sweep (hdx_wsweep_dbg.hip; 233: fused regions; 234: the gather sweep's fused regions)
        case 236:  // 230 without the pass-boundary gap
        case 237: case 238:  // 230's debug shapes: no hash / no hash, no walk (WRONG coordinates)
        case 235:  // regions by hash + separate lookups at any n, 64 MiB chunks (hdx_regions.hip)
        case 247:  // 235 with the scratch allocation failing: the fused fallback
        case 248:  // debug shape of 212: its LDS reads at conflict-free addresses (WRONG coordinates)
        case 249:  // debug shape of 212: no funnel shifts on its LDS reads (WRONG coordinates)
        case 250:  // the product sweep (230) without the record span
        case 251:  // ... and with round 3's dword-by-dword key gather
        case 252:  // debug shape of 250: no copy, no walk, the hash on made-up descriptors (WRONG coordinates)
        case 253: case 254:  // the product sweep's non-record / record forms with round 3's per-KiB span copy
        case 255:  // 212 with round 3's per-KiB span copy; the sweep with round 3's walk reads
        case 256: case 257:  // 212 / the product sweep with one / two waves per workgroup
        case 258:  // 212 with <= 6 objects and 7.5 KiB windows / the sweep with 7.75 KiB windows (one wave per workgroup)
        case 293: case 294: case 295: case 296:  // 287 with the slot plan + select numerics + class table / each alone; 293: the sweep with NUM2
        case 297:  // debug shape of 293: no hash (WRONG coordinates)
        case 298:  // the wave-staged kernel / the sweep as before LOOP 4 (two head reads, separate mix16s)
        case 259:  // 212 / the sweep as in round 4: four waves per workgroup
        case 270:  // 212 / the product sweep with the XCD-aware block order
        case 271:  // the sweep with 7 objects per wave (9.5 KiB windows)
        case 272:  // the sweep with 7 objects per wave (9 KiB windows)
        case 273:  // 212 / the sweep with 3 passes, 11 objects per wave, 14 KiB windows
        case 274:  // 212 with 3 passes, 10 objects per wave, 13 KiB windows
        case 275: case 276:  // 212 with its descriptors in registers (8832 / 8704-byte windows)
        case 279:  // 270 with non-temporal loads (lengths, bases, span)
        case 278:  // 279 with dword-aligned ds_read_b128 window reads (W128 1)
        case 277:  // the sweep without wave priorities (the product before round 5's s_setprio)
        case 287:  // 279 with wave priorities: loads high (the product in round 5)
        case 210: case 211:  // wave-staged, sorted over the workgroup
        case 40: case 41:
        case 33: case 43: case 47: case 48: case 49: case 57: case 58:  // stored-object sweep forms (hdx_encoded.hip)
            return true;
        default:
            return false;
    }
}

static int g_variant = [] {
    const char* e = getenv("HDX_KERNEL_VARIANT");
    return e && *e && known_variant(atoi(e)) ? atoi(e) : -1;
}();

int hash_variant() { return __atomic_load_n(&g_variant, __ATOMIC_RELAXED); }

int set_hash_variant(int v) {
    if (!known_variant(v)) return -2;
    return __atomic_exchange_n(&g_variant, v, __ATOMIC_RELAXED);
}

}  // namespace hdx
