// ref_ordered_shim.cc — TEST INFRASTRUCTURE ONLY.
//
// Exports the reference's own ordered encodings (common/ordered_encoding.cc,
// compiled unmodified from /root/reference by oracle/Makefile) under C
// linkage so tests can compare oracle/hdx_oracle.c against them.  The
// reference declares them with hidden visibility (namespace.h), hence this
// thin wrapper.  Output goes to oracle/_ref/ only.
#include "common/ordered_encoding.h"

extern "C" __attribute__((visibility("default"))) uint64_t
ref_ordered_encode_int64(int64_t x) { return hyperdex::ordered_encode_int64(x); }

extern "C" __attribute__((visibility("default"))) int64_t
ref_ordered_decode_int64(uint64_t x) { return hyperdex::ordered_decode_int64(x); }

extern "C" __attribute__((visibility("default"))) uint64_t
ref_ordered_encode_double(double x) { return hyperdex::ordered_encode_double(x); }
