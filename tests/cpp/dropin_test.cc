// Drives include/hyperdex_amd/hash.h exactly as the daemon and the client
// would, on the reference-produced values of tests/golden/reference_values.json
// (SURVEY §8c).  Built against the reference's own common/schema.h,
// common/attribute.h, include/hyperdex.h and namespace.h when /root/reference
// is present (only libe's e/slice.h is a stand-in, tests/cpp/shim_e), else
// against tests/cpp/shim_types.  Needs no GPU: the per-object signatures run on
// the host CPU.  Exit 0 = all equal.
//
//   dropin_test            check the reference values
//   dropin_test bench N    also time N config-3b-shaped objects through
//                          hash(schema, key, value, hs); prints ns/object
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hyperdex_amd/hash.h"

static int failures = 0;

static void expect(const char* what, uint64_t got, uint64_t want) {
    if (got != want) {
        fprintf(stderr, "%s: got %016llx want %016llx\n", what, (unsigned long long)got,
                (unsigned long long)want);
        ++failures;
    }
}

// The reference's attribute and schema are classes with out-of-line
// constructors (common/attribute.cc, common/schema.cc, not linked here); their
// data members are public and standard-layout, so a layout-identical
// aggregate stands in for construction.
struct raw_attribute {
    const char* name;
    hyperdatatype type;
};
struct raw_schema {
    uint16_t attrs_sz;
    const void* attrs;  // const hyperdex::attribute*
    bool authorization;
};

static const hyperdex::schema& make_schema(raw_schema* rs, const raw_attribute* ra, uint16_t n) {
    rs->attrs_sz = n;
    rs->attrs = ra;
    rs->authorization = false;
    return *reinterpret_cast<const hyperdex::schema*>(rs);
}

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

static int bench(long n) {
    // config 3b: key STRING 64 B, 10 STRING U{0..195}, 3 INT64, 3 FLOAT
    raw_attribute ra[17];
    ra[0] = {"k", HYPERDATATYPE_STRING};
    for (int i = 1; i <= 10; ++i) ra[i] = {"s", HYPERDATATYPE_STRING};
    for (int i = 11; i <= 13; ++i) ra[i] = {"i", HYPERDATATYPE_INT64};
    for (int i = 14; i <= 16; ++i) ra[i] = {"f", HYPERDATATYPE_FLOAT};
    raw_schema rs;
    const hyperdex::schema& sc = make_schema(&rs, ra, 17);
    const long pool = 4096;  // distinct objects, cycled
    uint64_t seed = 0x4859504552444558ULL;
    std::vector<uint8_t> bytes(pool * 1400);
    for (size_t i = 0; i < bytes.size(); ++i) bytes[i] = (uint8_t)splitmix(&seed);
    std::vector<std::vector<e::slice> > values(pool);
    std::vector<e::slice> keys(pool);
    size_t off = 0, payload = 0;
    for (long o = 0; o < pool; ++o) {
        keys[o] = e::slice(&bytes[off], 64);
        off += 64;
        for (int a = 1; a < 17; ++a) {
            const size_t len = a <= 10 ? splitmix(&seed) % 196 : 8;
            values[o].push_back(e::slice(&bytes[off], len));
            off += len;
        }
    }
    payload = off;
    uint64_t hs[17], sink = 0;
    timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (long i = 0; i < n; ++i) {
        hyperdex::hash(sc, keys[i % pool], values[i % pool], hs);
        sink ^= hs[i % 17];
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double ns = ((t1.tv_sec - t0.tv_sec) * 1e9 + (t1.tv_nsec - t0.tv_nsec)) / (double)n;
    printf("bench ns_per_object %.1f bytes_per_object %.1f sink %016llx\n", ns, payload / (double)pool,
           (unsigned long long)sink);
    return 0;
}

int main(int argc, char** argv) {
    using hyperdex::hash;
    const char* key = "hello world, this is a 64 byte key padded out to the full length";
    int64_t i42 = 42;
    double f35 = 3.5;
    const raw_attribute ra[3] = {{"k", HYPERDATATYPE_STRING}, {"a", HYPERDATATYPE_INT64},
                                 {"b", HYPERDATATYPE_FLOAT}};
    raw_schema rs;
    const hyperdex::schema& sc = make_schema(&rs, ra, 3);
    std::vector<e::slice> value;
    value.push_back(e::slice(reinterpret_cast<const uint8_t*>(&i42), 8));
    value.push_back(e::slice(reinterpret_cast<const uint8_t*>(&f35), 8));
    uint64_t hs[3];
    hash(sc, e::slice(key), value, hs);
    expect("object[0]", hs[0], 0x6221bfe1aade394cULL);
    expect("object[1]", hs[1], 0x800000000000002aULL);
    expect("object[2]", hs[2], 0xc00c000000000002ULL);
    uint64_t h = 0;
    hash(sc, e::slice(key), &h);
    expect("key", h, 0x6221bfe1aade394cULL);
    expect("empty string", hash(HYPERDATATYPE_STRING, e::slice()), 0x9ae16a3b2f90404fULL);
    expect("empty int64", hash(HYPERDATATYPE_INT64, e::slice()), 0x8000000000000000ULL);
    expect("list", hash(HYPERDATATYPE_LIST_STRING, e::slice("abc")), 0);
    int64_t ts = 1420666849000000LL;
    expect("ts second", hash(HYPERDATATYPE_TIMESTAMP_SECOND, e::slice(reinterpret_cast<const uint8_t*>(&ts), 8)),
           0xd3f9d92bcba0484fULL);
    expect("ts month", hash(HYPERDATATYPE_TIMESTAMP_MONTH, e::slice(reinterpret_cast<const uint8_t*>(&ts), 8)),
           0xefed25ccac6fc125ULL);
    if (failures) return 1;
    printf("dropin ok\n");
    if (argc > 2 && strcmp(argv[1], "bench") == 0) return bench(atol(argv[2]));
    return 0;
}
