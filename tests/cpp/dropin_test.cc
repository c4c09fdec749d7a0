// Drives include/hyperdex_amd/hash.h exactly as the daemon would, on the
// reference-produced values of tests/golden/reference_values.json.
// Exit 0 = all equal.  Needs a gfx950 GPU (the header aborts without one).
#include <stdio.h>
#include <string.h>

#include "hyperdex_amd/hash.h"

static int failures = 0;

static void expect(const char* what, uint64_t got, uint64_t want) {
    if (got != want) {
        fprintf(stderr, "%s: got %016llx want %016llx\n", what, (unsigned long long)got,
                (unsigned long long)want);
        ++failures;
    }
}

int main() {
    using hyperdex::hash;
    const char* key = "hello world, this is a 64 byte key padded out to the full length";
    int64_t i42 = 42;
    double f35 = 3.5;
    hyperdex::attribute attrs[3] = {{"k", HYPERDATATYPE_STRING}, {"a", HYPERDATATYPE_INT64},
                                    {"b", HYPERDATATYPE_FLOAT}};
    hyperdex::schema sc = {3, attrs, false};
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
    if (failures == 0) printf("dropin ok\n");
    return failures ? 1 : 0;
}
