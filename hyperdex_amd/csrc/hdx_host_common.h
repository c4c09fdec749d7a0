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

// hyperdatatype -> CODE_* (-1: the reference's datatype_info::lookup returns NULL).
int type_code(uint32_t type);
// Sets the calling thread's hdx_last_error() text and returns s.
hdx_status fail(hdx_status s, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace hdx
