// hyperdex_amd/hash.h — drop-in replacement for HyperDex's common/hash.h.
//
// Same namespace, names and signatures as the reference (common/hash.h:43-55),
// implemented inline over the C-ABI of libhdxhash.so (include/hdxhash.h), so
// the daemon's callers — key_state::hash_objects (daemon/key_state.cc:1477,
// 1478,1495,1517), configuration::point_leader (common/configuration.cc:438,
// 475), configuration::lookup_search (:819,833,843) — compile unchanged.
// Integration: INTEGRATION.md.  It is written against the daemon's own types:
// e::slice (libe), hyperdex::schema / attribute (common/schema.h,
// common/attribute.h) and enum hyperdatatype (include/hyperdex.h).
//
// These are the per-object calls of the client (point_leader), the search
// planner (lookup_search) and the daemon's write path: they run on the host
// CPU inside libhdxhash.so (hyperdex_amd/csrc/hdx_cpu.cpp), pure, reentrant,
// with no allocation and no GPU needed — a client host without an MI355X
// links this header unchanged.  Bulk work goes to the batched C-ABI
// (hdx_hash_batch_device / _host, hdx_batcher_*), which runs the gfx950
// kernels.
//
// Semantics are the reference's bit for bit.  Where the reference asserts —
// unknown type (hash.cc:38), int64/float/timestamp value not 0 or 8 bytes
// (datatype_int64.cc:233, datatype_float.cc:204) — these functions print the
// library's message and abort(), in every build (the reference's asserts
// compile out under NDEBUG; then it reads the wrong-sized value anyway).
#ifndef hyperdex_common_hash_h_
#define hyperdex_common_hash_h_

// C
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

// STL
#include <vector>

// e
#include <e/slice.h>

// HyperDex
#include "namespace.h"
#include "common/schema.h"

// hdxhash
#include "hdxhash.h"

BEGIN_HYPERDEX_NAMESPACE

namespace hdx_dropin {
inline void
check(hdx_status s, const char* what)
{
    if (s != HDX_OK)
    {
        fprintf(stderr, "hyperdex::%s: %s\n", what, hdx_last_error());
        abort();
    }
}
} // namespace hdx_dropin

inline uint64_t
hash(hyperdatatype t, const e::slice& v)
{
    uint64_t h = 0;
    hdx_dropin::check(hdx_hash_value(static_cast<uint32_t>(t), v.data(), v.size(), &h), "hash(type, value)");
    return h;
}

inline void
hash(const schema& sc,
     const e::slice& key,
     uint64_t* h)
{
    *h = hash(sc.attrs[0].type, key);
}

inline void
hash(const schema& sc,
     const e::slice& key,
     const std::vector<e::slice>& value,
     uint64_t* hs)
{
    // common/hash.cc:63-67: hs[0] from the key, hs[i] from value[i - 1]
    hs[0] = hash(sc.attrs[0].type, key);

    for (size_t i = 1; i < sc.attrs_sz; ++i)
    {
        hs[i] = hash(sc.attrs[i].type, value[i - 1]);
    }
}

END_HYPERDEX_NAMESPACE

#endif // hyperdex_common_hash_h_
