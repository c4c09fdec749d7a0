// hdx_cpu.cpp — the per-object entry points of libhdxhash.so on the host CPU.
//
// The reference's hash() is an in-process CPU leaf (common/hash.cc:34-68),
// reached per object from the client library (client/client.cc:1240 ->
// configuration::point_leader, common/configuration.cc:438,475), from
// configuration::lookup_search (:819,833,843) and from the daemon's
// key_state::hash_objects (daemon/key_state.cc:1477-1517) — on hosts with or
// without an MI355X, one object per call, from every network thread at once.
// A GPU round trip per object would cost tens of microseconds against a
// fraction of one on a core, so these signatures are served here, by design:
//
//   hdx_hash_value   hash(hyperdatatype, const e::slice&)      common/hash.cc:34-46
//   hdx_hash_key     hash(const schema&, key, uint64_t* h)     common/hash.cc:48-54
//   hdx_hash_object  hash(const schema&, key, value, hs)       common/hash.cc:56-68
//
// Every batch entry point (hdx_hash_batch_*, the sweep, the fused lookups, the
// batcher) runs the gfx950 kernels only; nothing here is a fallback for them.
// Pure, reentrant, lock-free, no allocation, no HIP call: works on a host with
// no GPU.  Bit-exact with the kernels (hdx_device_hash.h) and the reference:
//   CityHash64 v1.1         cityhash/city.cc:255-397, city.h:100-109
//   ordered_encode_int64    common/ordered_encoding.cc:43-49
//   ordered_encode_double   common/ordered_encoding.cc:114-161
//   timestamp calendar hash common/datatype_timestamp.cc:117-219
// Built without -ffast-math: the timestamp hash needs an IEEE division.
#include <stdint.h>
#include <string.h>

#include "hdx_cpu.h"
#include "hdx_host_common.h"

namespace hdx {
namespace cpu {
namespace {

constexpr uint64_t kK0 = 0xc3a5c85c97cb3127ULL;
constexpr uint64_t kK1 = 0xb492b66fbe98f273ULL;
constexpr uint64_t kK2 = 0x9ae16a3b2f90404fULL;
constexpr uint64_t kMul128 = 0x9ddfea08eb382d69ULL;  // Hash128to64, city.h:100-109

// Little-endian loads at any alignment (Fetch64/Fetch32, city.cc:107-113 on x86/arm64 LE)
inline uint64_t le64(const uint8_t* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
inline uint32_t le32(const uint8_t* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
inline uint64_t rotr(uint64_t v, unsigned r) { return (v >> r) | (v << ((64 - r) & 63)); }
inline uint64_t fold47(uint64_t v) { return v ^ (v >> 47); }

// HashLen16(u, v, mul) (city.cc:268-276); with kMul128 it is Hash128to64(u, v)
inline uint64_t murmur2x64(uint64_t u, uint64_t v, uint64_t mul) {
    const uint64_t a = fold47((u ^ v) * mul);
    return fold47((v ^ a) * mul) * mul;
}

// city.cc:278-301
inline uint64_t len_upto16(const uint8_t* s, uint64_t n) {
    if (n >= 8) {
        const uint64_t mul = kK2 + 2 * n;
        const uint64_t a = le64(s) + kK2;
        const uint64_t b = le64(s + n - 8);
        return murmur2x64(rotr(b, 37) * mul + a, (rotr(a, 25) + b) * mul, mul);
    }
    if (n >= 4) {
        const uint64_t mul = kK2 + 2 * n;
        return murmur2x64(n + ((uint64_t)le32(s) << 3), le32(s + n - 4), mul);
    }
    if (n == 0) return kK2;
    const uint32_t lo = (uint32_t)s[0] | ((uint32_t)s[n >> 1] << 8);  // unsigned bytes (:293-297)
    const uint32_t hi = (uint32_t)n + ((uint32_t)s[n - 1] << 2);
    return fold47((uint64_t)lo * kK2 ^ (uint64_t)hi * kK0) * kK2;
}

// city.cc:305-313
inline uint64_t len_17to32(const uint8_t* s, uint64_t n) {
    const uint64_t mul = kK2 + 2 * n;
    const uint64_t a = le64(s) * kK1, b = le64(s + 8);
    const uint64_t c = le64(s + n - 8) * mul, d = le64(s + n - 16) * kK2;
    return murmur2x64(rotr(a + b, 43) + rotr(c, 30) + d, a + rotr(b + kK2, 18) + c, mul);
}

// city.cc:340-359
inline uint64_t len_33to64(const uint8_t* s, uint64_t n) {
    const uint64_t mul = kK2 + 2 * n;
    uint64_t a = le64(s) * kK2;
    uint64_t b = le64(s + 8);
    const uint64_t c = le64(s + n - 24), d = le64(s + n - 32);
    const uint64_t e = le64(s + 16) * kK2, f = le64(s + 24) * 9;
    const uint64_t g = le64(s + n - 8), h = le64(s + n - 16) * mul;
    const uint64_t u = rotr(a + g, 43) + (rotr(b, 30) + c) * 9;
    const uint64_t v = ((a + g) ^ d) + f + 1;
    const uint64_t w = __builtin_bswap64((u + v) * mul) + h;
    const uint64_t x = rotr(e + f, 42) + c;
    const uint64_t y = (__builtin_bswap64((v + w) * mul) + g) * mul;
    const uint64_t z = e + f + c;
    a = __builtin_bswap64((x + z) * mul + y) + b;
    b = fold47((z + a) * mul + d + h) * mul;
    return b + x;
}

// WeakHashLen32WithSeeds on the 32 bytes at s (city.cc:317-337)
struct Pair {
    uint64_t first, second;
};
inline Pair weak_seeded32(const uint8_t* s, uint64_t a, uint64_t b) {
    const uint64_t w = le64(s), x = le64(s + 8), y = le64(s + 16), z = le64(s + 24);
    a += w;
    b = rotr(b + a + z, 21);
    const uint64_t c = a;
    a += x + y;
    b += rotr(a, 44);
    return Pair{a + z, b + c};
}

}  // namespace

// CityHash64 v1.1, city.cc:361-397
uint64_t cityhash64(const uint8_t* s, uint64_t n) {
    if (n <= 16) return len_upto16(s, n);
    if (n <= 32) return len_17to32(s, n);
    if (n <= 64) return len_33to64(s, n);
    uint64_t x = le64(s + n - 40);
    uint64_t y = le64(s + n - 16) + le64(s + n - 56);
    uint64_t z = murmur2x64(le64(s + n - 48) + n, le64(s + n - 24), kMul128);
    Pair v = weak_seeded32(s + n - 64, n, z);
    Pair w = weak_seeded32(s + n - 32, y + kK1, x);
    x = x * kK1 + le64(s);
    for (uint64_t blocks = (n - 1) >> 6; blocks; --blocks, s += 64) {
        x = rotr(x + y + v.first + le64(s + 8), 37) * kK1;
        y = rotr(y + v.second + le64(s + 48), 42) * kK1;
        x ^= w.second;
        y += v.first + le64(s + 40);
        z = rotr(z + w.first, 33) * kK1;
        v = weak_seeded32(s, v.second * kK1, x + w.first);
        w = weak_seeded32(s + 32, z + w.second, y + le64(s + 16));
        const uint64_t t = z;
        z = x;
        x = t;
    }
    return murmur2x64(murmur2x64(v.first, w.first, kMul128) + fold47(y) * kK1 + z,
                      murmur2x64(v.second, w.second, kMul128) + x, kMul128);
}

// ordered_encoding.cc:43-49: (u64)x + (x >= 0 ? 2^63 : INT64_MIN) == x ^ 2^63
uint64_t ordered_int64(uint64_t bits) { return bits ^ 0x8000000000000000ULL; }

// ordered_encoding.cc:114-161, tested on the bit pattern in the reference's
// order: inf, NaN, zero (either sign -> the same code), then finite values
// (subnormals keep their fraction).
uint64_t ordered_double(uint64_t bits) {
    const uint64_t exp = (bits >> 52) & 0x7ff, frac = bits & 0x000fffffffffffffULL;
    if (exp == 0x7ff) return frac ? 0xfff0000000000003ULL : (bits >> 63) ? 0ULL : 0xfff0000000000002ULL;
    if ((bits << 1) == 0) return 0x8000000000000001ULL;
    if (bits >> 63) return (~bits & 0x7fffffffffffffffULL) + 1;
    return (bits | 0x8000000000000000ULL) + 2;
}

// datatype_timestamp.cc:138-219; g = 0..5 for second..month.  The digit
// visiting order TABLE_* (:131-136) is g, g-1, .., 0, then g+1 .. 6.
uint64_t timestamp_hash(unsigned g, uint64_t t) {
    static const uint64_t kIntervals[6] = {60, 60, 24, 7, 4, 12};  // :117-129
    uint64_t x = (uint64_t)((double)t / 1000000.);                 // :198 (u64 -> f64, IEEE divide)
    uint64_t digit[7];
    for (int i = 0; i < 6; ++i) {
        digit[i] = x % kIntervals[i];
        x /= kIntervals[i];
    }
    digit[6] = x;
    uint64_t y = ~0ULL, h = 0;
    for (unsigned i = 0; i < 6; ++i) {
        const unsigned k = i <= g ? g - i : i;
        y /= kIntervals[k];
        h += digit[k] * y;
    }
    return h + digit[6];
}

// hash(hyperdatatype, slice), hash.cc:34-46, on a dispatch code (type_code)
hdx_status hash_code(int code, const uint8_t* p, uint64_t n, uint64_t* out) {
    switch (code) {
        case CODE_STRING:
            *out = cityhash64(p, n);
            return HDX_OK;
        case CODE_ZERO:  // hashable() == false (datatype_info.cc:169-180)
            *out = 0;
            return HDX_OK;
        default:
            break;
    }
    // int64 / float / timestamp: 8 bytes LE, empty = 0 (datatype_int64.cc:46-59,
    // datatype_float.cc:44-57, datatype_timestamp.cc:43-56); other sizes assert
    if (n != 0 && n != 8) return HDX_E_BADSIZE;
    const uint64_t bits = n ? le64(p) : 0;
    if (code == CODE_INT64) *out = ordered_int64(bits);
    else if (code == CODE_FLOAT) *out = ordered_double(bits);
    else *out = timestamp_hash((unsigned)(code - CODE_TS_SECOND), bits);
    return HDX_OK;
}

}  // namespace cpu
}  // namespace hdx

using namespace hdx;

HDX_EXPORT hdx_status hdx_hash_value(uint32_t type, const uint8_t* data, size_t len, uint64_t* out) {
    const int code = type_code(type);
    if (code < 0) return fail(HDX_E_BADTYPE, "unknown hyperdatatype %u", type);
    if (!out || (!data && len)) return fail(HDX_E_INVALID, "NULL pointer");
    const hdx_status st = cpu::hash_code(code, data, len, out);
    if (st != HDX_OK) return fail(st, "hyperdatatype %u: numeric value of %zu bytes", type, len);
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_hash_key(const uint32_t* types, uint32_t attrs_sz, const uint8_t* key,
                                   size_t key_len, uint64_t* h) {
    if (!types || attrs_sz == 0) return fail(HDX_E_INVALID, "empty schema");
    return hdx_hash_value(types[0], key, key_len, h);
}

HDX_EXPORT hdx_status hdx_hash_object(const uint32_t* types, uint32_t attrs_sz, const uint8_t* key,
                                      size_t key_len, const uint8_t* const* values, const size_t* value_lens,
                                      uint64_t* hs) {
    if (!types) return fail(HDX_E_INVALID, "types is NULL");
    if (attrs_sz == 0 || attrs_sz > HDX_MAX_ATTRS)
        return fail(HDX_E_INVALID, "attrs_sz=%u outside [1, %d]", attrs_sz, HDX_MAX_ATTRS);
    if (!hs || (!key && key_len) || (attrs_sz > 1 && (!values || !value_lens)))
        return fail(HDX_E_INVALID, "NULL pointer");
    // the reference asserts on the first bad attribute (hash.cc:38, :233/:204);
    // here nothing is written unless the whole object hashes
    for (uint32_t j = 0; j < attrs_sz; ++j) {
        const int code = type_code(types[j]);
        if (code < 0) return fail(HDX_E_BADTYPE, "attribute %u: unknown hyperdatatype %u", j, types[j]);
        const size_t n = j ? value_lens[j - 1] : key_len;
        if (code >= (int)CODE_INT64 && n != 0 && n != 8) {
            if (j) return fail(HDX_E_BADSIZE, "attribute %u: numeric value of %zu bytes", j, n);
            return fail(HDX_E_BADSIZE, "key: numeric value of %zu bytes", n);
        }
        if (j > 0 && !values[j - 1] && n) return fail(HDX_E_INVALID, "value %u is NULL", j - 1);
    }
    (void)cpu::hash_code(type_code(types[0]), key, key_len, &hs[0]);
    for (uint32_t j = 1; j < attrs_sz; ++j)
        (void)cpu::hash_code(type_code(types[j]), values[j - 1], value_lens[j - 1], &hs[j]);
    return HDX_OK;
}
