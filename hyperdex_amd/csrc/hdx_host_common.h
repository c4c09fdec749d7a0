// hdx_host_common.h — declarations the host translation units share that need
// no HIP header (the CPU per-object path, hdx_cpu.cpp, includes only this).
#pragma once

#include <stdint.h>

#include "../../include/hdxhash.h"

#define HDX_EXPORT extern "C" __attribute__((visibility("default")))

namespace hdx {

// Attribute classes the kernels and the CPU path dispatch on (the host maps
// hyperdatatype -> code, type_code).
enum : uint32_t {
    CODE_ZERO = 0,     // not hashable: document/list/set/map/macaroon -> 0
    CODE_STRING = 1,
    CODE_INT64 = 2,
    CODE_FLOAT = 3,
    CODE_TS_SECOND = 4,  // .. CODE_TS_MONTH = 9, in hyperdatatype order
    CODE_TS_MONTH = 9,
};

// hyperdatatype -> CODE_* (-1: the reference's datatype_info::lookup returns
// NULL); include/hyperdex.h:53-102, datatype_info.cc:72-141.  Inline: the
// per-object CPU entry points call it once per attribute.
inline int type_code(uint32_t t) {
    switch (t) {
        case 9217: return CODE_STRING;
        case 9218: return CODE_INT64;
        case 9219: return CODE_FLOAT;
        case 9473: case 9474: case 9475: case 9476: case 9477: case 9478:
            return CODE_TS_SECOND + (int)(t - 9473);
        // lookup() returns a datatype whose hashable() is false (hash.cc:40-43)
        case 9223:                                   // document
        case 9281: case 9282: case 9283:             // list string/int64/float
        case 9345: case 9346: case 9347:             // set string/int64/float
        case 9417: case 9418: case 9419:             // map string->*
        case 9425: case 9426: case 9427:             // map int64->*
        case 9433: case 9434: case 9435:             // map float->*
        case 9664:                                   // macaroon secret
            return CODE_ZERO;
        default:  // generic, *_GENERIC, *_KEYONLY, garbage, anything else: lookup() == NULL
            return -1;
    }
}
// Sets the calling thread's hdx_last_error() text and returns s.
hdx_status fail(hdx_status s, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace hdx
