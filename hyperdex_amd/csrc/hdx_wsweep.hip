// hdx_wsweep.hip — the product instantiation of the wave-staged reindex sweep
// (hdx_wsweep.h); its A/B forms are in hdx_wsweep_dbg.hip (debug library only).
#include "hdx_wsweep.h"

namespace hdx {

// The product form: 2 passes, 6 objects per wave, 8.5 KiB windows (four
// workgroups of four waves per CU).  With a.T tables, the fused region lookup
// (coords may then be NULL): debug variant 233 only — the sweep + separate
// lookups is faster (hdx_encoded.hip).  A <= kWsweepMaxAttrs.
// The record span is compiled in only when keys and values are one store (the
// check costs the other layouts ~1 %: 3.78 vs 3.74 ms per 10 M on a key column).
// One wave per workgroup (round 5: 3.466 vs 3.626 ms per 10 M on the key
// column for four, whose 40 KiB stayed allocated until the slowest of the four
// finished; profiles/r5/ab_wpb.jsonl), in the XCD-aware block order
// (xcd_block: 3.412 vs 3.447 ms, profiles/r5/ab_xcd.jsonl), 7 objects per
// wave in 9.5 KiB windows (the per-wave skeleton over one more object:
// 3.301 vs 3.415 ms for 6 in 8.5 KiB; 9 KiB windows 3.343 — a group of 7
// then overflows the window more often; profiles/r5/ab_sweep_k7.jsonl).
// Round 5: wave priorities (s_setprio, PRIO 4): the load phase (offsets,
// lengths, the span DMA) high, the walk and the class sort — chains of
// dependent LDS reads and atomics — medium, the passes low: a wave that has
// just started gets its loads out, and a walking wave its next read, ahead of
// the waves that are hashing.  3.198 vs 3.274 ms per 10 M on the key column,
// 3.357 vs 3.424 keys in place, 3.146 vs 3.213 records; the walk at high
// priority 3.211 / 3.369 / 3.155; loads high alone −0.3 to −1.2 %
// (profiles/r5/ab_priority.jsonl).
// Round 6: NUM2 for schemas of strings, int64 and floats (numerics by
// selects, the class from the table): 3.258 vs 3.304 ms per 10 M on the key
// column, VALU 971.8 -> 956.8 and SALU 401.1 -> 370.1 per wave
// (profiles/r6/ab_sweep_num2.jsonl, pmc_lds_cfg5k_num2.txt); other schemas keep
// the round-5 form.  Late round 6: LOOP 14 (hash_slot_window LOOP 4, one head
// read per slot in a pass holding long and short strings): 3.247 vs 3.266 and
// 3.261 vs 3.287 ms per 10 M on the key column (debug 298 = LOOP 13,
// profiles/r6/ab_loop4.jsonl).
template <bool REG, bool RECS>
static hipError_t launch_wsweep_product_t(const EncodedArgs& a, hipStream_t stream) {
    if (num2_codes(a))
        return launch_wsweep_t<2, 9728, 7, REG, true, 0, 14, false, true, true, RECS, true, false, 1, true, 4, true>(a, stream);
    return launch_wsweep_t<2, 9728, 7, REG, true, 0, 14, false, true, true, RECS, true, false, 1, true, 4>(a, stream);
}

hipError_t launch_hash_wsweep_product(const EncodedArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    const bool recs = a.keys == a.vals;
    if (a.T) return recs ? launch_wsweep_product_t<true, true>(a, stream) : launch_wsweep_product_t<true, false>(a, stream);
    if (!a.coords) return hipErrorInvalidValue;
    return recs ? launch_wsweep_product_t<false, true>(a, stream) : launch_wsweep_product_t<false, false>(a, stream);
}

}  // namespace hdx
