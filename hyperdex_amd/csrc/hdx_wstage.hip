// hdx_wstage.hip — the product instantiation of the wave-staged batch hash
// (hdx_wstage.h): two class-sorted passes per wave, 8832-byte windows, one
// wave per workgroup (16 per CU by LDS; round 5: 2.597 vs 2.658 ms for four
// waves per workgroup, whose 40 KiB stayed allocated until the slowest of the
// four finished, profiles/r5/ab_wpb.jsonl), slots hashed from the window with
// the head/tail reads of hash_slot_window (hdx_lds_hash.h).  The automatic policy
// runs it for mixed string / int64 / float schemas (config 3b: 2.92 vs 3.32 ms
// for variant 44, profiles/r3/ab_wstage_ht.jsonl).  The A/B forms are in
// hdx_wstage_dbg.hip (debug library only).
// Round 5: the bases, lengths and span loaded non-temporal (each byte is read
// once): 2.556 / 2.561 / 2.554 vs 2.573 / 2.628 / 2.602 ms on three boxes
// (variant 279 vs 270/212, profiles/r5/ab_nt_misaligned.jsonl,
// ab_persistent_prefetch.jsonl); and the load phase at high wave priority, the
// passes at low (s_setprio, PRIO 1): a wave that has just started gets its
// loads and span DMA out ahead of the waves that are hashing — 2.500 vs 2.555
// ms on a fast box, 2.711–2.729 vs 2.716–2.746 on a slow one (variant 287 vs
// 279, profiles/r5/ab_priority.jsonl).
// Round 6 (variant 293): the per-schema slot plan (each slot's object,
// attribute and code from the launcher's table, BatchArgs::plan), numerics by
// selects for schemas of strings, int64 and floats only (NUM2), and the work
// class from a table (ORDER 5): 862.6 -> 841.6 VALU and 264.9 -> 238.9 SALU
// per wave, 2.666 vs 2.709 ms (profiles/r6/ab_plan.jsonl,
// pmc_lds_cfg3b_plan.txt).  Other schemas (timestamps, non-hashable types:
// forced debug variants only — the policy gives them the regroup kernel) keep
// the round-5 instantiation.  Late round 6 (HT 6, hash_slot_window LOOP 4): a
// pass holding long and short strings reads each slot's head once and runs one
// final mix16 (also for 4..7-byte strings): 2.447 vs 2.462 and 2.663 vs 2.681
// ms on two boxes (debug 298 = the form before it, profiles/r6/ab_loop4.jsonl).
#include "hdx_wstage.h"

namespace hdx {

hipError_t launch_hash_wstage_product(const BatchArgs& args, hipStream_t stream) {
    if (args.n == 0) return hipSuccess;
    if (num2_schema(args))
        return launch_wstage_t<2, 8832, 63, 0, 6, 5, 0, false, true, true, true, false, 1, true, false, true, 1, true,
                               true>(args, stream);
    return launch_wstage_t<2, 8832, 63, 0, 6, 4, 0, false, true, true, true, false, 1, true, false, true, 1>(args, stream);
}

// ... with the fused region lookup (args.T tables; args.coords may be NULL)
hipError_t launch_hash_wstage_regions(const BatchArgs& args, hipStream_t stream) {
    if (args.n == 0) return hipSuccess;
    if (num2_schema(args))
        return launch_wstage_t<2, 8832, 63, 0, 6, 5, 0, true, true, true, true, false, 1, true, false, true, 1, true,
                               true>(args, stream);
    return launch_wstage_t<2, 8832, 63, 0, 6, 4, 0, true, true, true, true, false, 1, true, false, true, 1>(args, stream);
}

}  // namespace hdx
