// hdx_cpu.h — the host CPU implementation of the per-object hash (hdx_cpu.cpp).
#pragma once

#include <stdint.h>

#include "hdx_host_common.h"

namespace hdx {
namespace cpu {

uint64_t cityhash64(const uint8_t* s, uint64_t n);            // city.cc:361-397
uint64_t ordered_int64(uint64_t bits);                         // ordered_encoding.cc:43-49
uint64_t ordered_double(uint64_t bits);                        // ordered_encoding.cc:114-161
uint64_t timestamp_hash(unsigned granularity, uint64_t t);    // datatype_timestamp.cc:138-219
// hash(type, slice) on a dispatch code; HDX_E_BADSIZE for a numeric value not 0 or 8 bytes
hdx_status hash_code(int code, const uint8_t* p, uint64_t n, uint64_t* out);

}  // namespace cpu
}  // namespace hdx
