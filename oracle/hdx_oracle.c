/*
 * hdx_oracle.c — plain-C restatement of the reference hashing path.
 *
 * TEST INFRASTRUCTURE ONLY (see hdx_oracle.h).  Compiled -O2 without
 * -ffast-math so the IEEE comparisons and the timestamp's double division
 * behave exactly as in the reference build.
 *
 * Each function names the reference file:line it restates.
 */
#define _GNU_SOURCE
#include "hdx_oracle.h"


#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* include/hyperdex.h:53-102 */
enum {
    T_GENERIC = 9216, T_STRING = 9217, T_INT64 = 9218, T_FLOAT = 9219,
    T_DOCUMENT = 9223,
    T_LIST_GENERIC = 9280, T_LIST_STRING = 9281, T_LIST_INT64 = 9282, T_LIST_FLOAT = 9283,
    T_SET_GENERIC = 9344, T_SET_STRING = 9345, T_SET_INT64 = 9346, T_SET_FLOAT = 9347,
    T_MAP_GENERIC = 9408,
    T_MAP_SS = 9417, T_MAP_SI = 9418, T_MAP_SF = 9419,
    T_MAP_IS = 9425, T_MAP_II = 9426, T_MAP_IF = 9427,
    T_MAP_FS = 9433, T_MAP_FI = 9434, T_MAP_FF = 9435,
    T_TS_GENERIC = 9472,
    T_TS_SECOND = 9473, T_TS_MINUTE = 9474, T_TS_HOUR = 9475,
    T_TS_DAY = 9476, T_TS_WEEK = 9477, T_TS_MONTH = 9478,
    T_MACAROON = 9664
};

/* ---- CityHash v1.1 (cityhash/city.cc) --------------------------------- */

#define K0 0xc3a5c85c97cb3127ULL /* city.cc:116 */
#define K1 0xb492b66fbe98f273ULL /* city.cc:117 */
#define K2 0x9ae16a3b2f90404fULL /* city.cc:118 */
#define KMUL 0x9ddfea08eb382d69ULL /* city.h:102 */

/* city.cc:45-55,107-113: unaligned little-endian loads */
static inline uint64_t ld64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t ld32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }

/* city.cc:255-258 (never called with r == 0 on this path) */
static inline uint64_t ror64(uint64_t v, int r) { return r == 0 ? v : (v >> r) | (v << (64 - r)); }
/* city.cc:260-262 */
static inline uint64_t smix(uint64_t v) { return v ^ (v >> 47); }

/* city.cc:268-276: murmur-style 128->64 with an explicit multiplier */
static uint64_t mix2(uint64_t u, uint64_t v, uint64_t mul) {
    uint64_t a = (u ^ v) * mul;
    a ^= a >> 47;
    uint64_t b = (v ^ a) * mul;
    b ^= b >> 47;
    return b * mul;
}
/* city.cc:264-266 -> city.h:100-109 (Hash128to64) */
static uint64_t mix2k(uint64_t u, uint64_t v) { return mix2(u, v, KMUL); }

/* city.cc:278-301 */
static uint64_t city_0to16(const uint8_t* s, size_t n) {
    if (n >= 8) {
        uint64_t m = K2 + (uint64_t)n * 2;
        uint64_t a = ld64(s) + K2;
        uint64_t b = ld64(s + n - 8);
        uint64_t c = ror64(b, 37) * m + a;
        uint64_t d = (ror64(a, 25) + b) * m;
        return mix2(c, d, m);
    }
    if (n >= 4) {
        uint64_t m = K2 + (uint64_t)n * 2;
        uint64_t a = ld32(s);
        return mix2((uint64_t)n + (a << 3), ld32(s + n - 4), m);
    }
    if (n > 0) {
        uint32_t y = (uint32_t)s[0] + ((uint32_t)s[n >> 1] << 8);
        uint32_t z = (uint32_t)n + ((uint32_t)s[n - 1] << 2);
        return smix((uint64_t)y * K2 ^ (uint64_t)z * K0) * K2;
    }
    return K2;
}

/* city.cc:305-313 */
static uint64_t city_17to32(const uint8_t* s, size_t n) {
    uint64_t m = K2 + (uint64_t)n * 2;
    uint64_t a = ld64(s) * K1;
    uint64_t b = ld64(s + 8);
    uint64_t c = ld64(s + n - 8) * m;
    uint64_t d = ld64(s + n - 16) * K2;
    return mix2(ror64(a + b, 43) + ror64(c, 30) + d, a + ror64(b + K2, 18) + c, m);
}

/* city.cc:317-337: weak 32-byte mix with two seeds, returns (lo, hi) */
static void weak32(const uint8_t* s, uint64_t a, uint64_t b, uint64_t* lo, uint64_t* hi) {
    uint64_t w = ld64(s), x = ld64(s + 8), y = ld64(s + 16), z = ld64(s + 24);
    a += w;
    b = ror64(b + a + z, 21);
    uint64_t c = a;
    a += x;
    a += y;
    b += ror64(a, 44);
    *lo = a + z;
    *hi = b + c;
}

/* city.cc:340-359 */
static uint64_t city_33to64(const uint8_t* s, size_t n) {
    uint64_t m = K2 + (uint64_t)n * 2;
    uint64_t a = ld64(s) * K2;
    uint64_t b = ld64(s + 8);
    uint64_t c = ld64(s + n - 24);
    uint64_t d = ld64(s + n - 32);
    uint64_t e = ld64(s + 16) * K2;
    uint64_t f = ld64(s + 24) * 9;
    uint64_t g = ld64(s + n - 8);
    uint64_t h = ld64(s + n - 16) * m;
    uint64_t u = ror64(a + g, 43) + (ror64(b, 30) + c) * 9;
    uint64_t v = ((a + g) ^ d) + f + 1;
    uint64_t w = __builtin_bswap64((u + v) * m) + h;
    uint64_t x = ror64(e + f, 42) + c;
    uint64_t y = (__builtin_bswap64((v + w) * m) + g) * m;
    uint64_t z = e + f + c;
    a = __builtin_bswap64((x + z) * m + y) + b;
    b = smix((z + a) * m + d + h) * m;
    return b + x;
}

/* city.cc:361-397 */
uint64_t hdxo_cityhash64(const uint8_t* s, size_t n) {
    if (n <= 16) return city_0to16(s, n);
    if (n <= 32) return city_17to32(s, n);
    if (n <= 64) return city_33to64(s, n);

    uint64_t x = ld64(s + n - 40);
    uint64_t y = ld64(s + n - 16) + ld64(s + n - 56);
    uint64_t z = mix2k(ld64(s + n - 48) + n, ld64(s + n - 24));
    uint64_t v0, v1, w0, w1;
    weak32(s + n - 64, n, z, &v0, &v1);
    weak32(s + n - 32, y + K1, x, &w0, &w1);
    x = x * K1 + ld64(s);

    size_t left = (n - 1) & ~(size_t)63;
    do {
        x = ror64(x + y + v0 + ld64(s + 8), 37) * K1;
        y = ror64(y + v1 + ld64(s + 48), 42) * K1;
        x ^= w1;
        y += v0 + ld64(s + 40);
        z = ror64(z + w0, 33) * K1;
        uint64_t nv0, nv1, nw0, nw1;
        weak32(s, v1 * K1, x + w0, &nv0, &nv1);
        weak32(s + 32, z + w1, y + ld64(s + 16), &nw0, &nw1);
        v0 = nv0; v1 = nv1; w0 = nw0; w1 = nw1;
        uint64_t t = z; z = x; x = t;
        s += 64;
        left -= 64;
    } while (left != 0);
    return mix2k(mix2k(v0, w0) + smix(y) * K1 + z, mix2k(v1, w1) + x);
}

/* ---- ordered encodings (common/ordered_encoding.cc) ------------------- */

/* ordered_encoding.cc:43-49 */
uint64_t hdxo_encode_int64(int64_t x) {
    uint64_t out = (uint64_t)x;
    out += x >= 0 ? 0x8000000000000000ULL : (uint64_t)INT64_MIN;
    return out;
}

/* ordered_encoding.cc:114-161 (ieee_double bitfields: common/ieee.h:107) */
uint64_t hdxo_encode_double(double x) {
    if (isinf(x)) return x > 0 ? 0xfff0000000000000ULL + 2 : 0;
    if (isnan(x)) return 0xfff0000000000000ULL + 3;
    if (x == 0) return 0x8000000000000000ULL + 1;
    uint64_t bits;
    memcpy(&bits, &x, 8);
    uint64_t sign = (bits >> 63) ^ 1;
    uint64_t ex = (bits >> 52) & 0x7ff;
    uint64_t frac = bits & 0xfffffffffffffULL;
    uint64_t shift = 2;
    if (x < 0) {
        ex ^= 0x7ff;
        frac ^= 0xfffffffffffffULL;
        shift = 1;
    }
    return ((sign << 63) | (ex << 52) | frac) + shift;
}

/* ---- timestamp (common/datatype_timestamp.cc:117-219) ----------------- */

static const uint64_t TS_INTERVALS[6] = {60, 60, 24, 7, 4, 12};
/* datatype_timestamp.cc:131-136: permutation per granularity */
static const unsigned TS_ORDER[6][7] = {
    {0, 1, 2, 3, 4, 5, 6}, /* second */
    {1, 0, 2, 3, 4, 5, 6}, /* minute */
    {2, 1, 0, 3, 4, 5, 6}, /* hour */
    {3, 2, 1, 0, 4, 5, 6}, /* day */
    {4, 3, 2, 1, 0, 5, 6}, /* week */
    {5, 4, 3, 2, 1, 0, 6}, /* month */
};

uint64_t hdxo_hash_timestamp(uint32_t type, int64_t ts) {
    uint64_t t = (uint64_t)ts; /* :141 unsigned view of the signed value */
    if (type < T_TS_SECOND || type > T_TS_MONTH) return t; /* :174-176 default */
    const unsigned* ord = TS_ORDER[type - T_TS_SECOND];
    uint64_t x = (uint64_t)((double)t / 1000000.); /* :198 */
    uint64_t digit[7];
    for (int i = 0; i < 6; ++i) {
        digit[i] = x % TS_INTERVALS[i];
        x /= TS_INTERVALS[i];
    }
    digit[6] = x;
    uint64_t y = UINT64_MAX, h = 0;
    for (int i = 0; i < 6; ++i) {
        y /= TS_INTERVALS[ord[i]];
        h += digit[ord[i]] * y;
    }
    return h + digit[ord[6]];
}

/* ---- dispatch (common/hash.cc:34-46, datatype_info.cc:72-141,169-180) -- */

static int known_type(uint32_t t) {
    switch (t) {
        case T_STRING: case T_INT64: case T_FLOAT: case T_DOCUMENT:
        case T_LIST_STRING: case T_LIST_INT64: case T_LIST_FLOAT:
        case T_SET_STRING: case T_SET_INT64: case T_SET_FLOAT:
        case T_MAP_SS: case T_MAP_SI: case T_MAP_SF:
        case T_MAP_IS: case T_MAP_II: case T_MAP_IF:
        case T_MAP_FS: case T_MAP_FI: case T_MAP_FF:
        case T_TS_SECOND: case T_TS_MINUTE: case T_TS_HOUR:
        case T_TS_DAY: case T_TS_WEEK: case T_TS_MONTH:
        case T_MACAROON:
            return 1;
        default:
            return 0;
    }
}

uint64_t hdxo_hash_value(uint32_t type, const uint8_t* p, size_t len, int* err) {
    *err = 0;
    if (!known_type(type)) { *err = 1; return 0; }
    switch (type) {
        case T_STRING: /* datatype_string.cc:181-185 */
            return hdxo_cityhash64(p, len);
        case T_INT64: { /* datatype_int64.cc:46-59,230-235 */
            if (len != 0 && len != 8) { *err = 2; return 0; }
            int64_t v = 0;
            if (len) memcpy(&v, p, 8);
            return hdxo_encode_int64(v);
        }
        case T_FLOAT: { /* datatype_float.cc:44-57,201-207 */
            if (len != 0 && len != 8) { *err = 2; return 0; }
            double v = 0;
            if (len) memcpy(&v, p, 8);
            return hdxo_encode_double(v);
        }
        case T_TS_SECOND: case T_TS_MINUTE: case T_TS_HOUR:
        case T_TS_DAY: case T_TS_WEEK: case T_TS_MONTH: { /* datatype_timestamp.cc:43-56 */
            if (len != 0 && len != 8) { *err = 2; return 0; }
            int64_t v = 0;
            if (len) memcpy(&v, p, 8);
            return hdxo_hash_timestamp(type, v);
        }
        default: /* hashable() == false */
            return 0;
    }
}

/* ---- batch over the packed layout ------------------------------------- */

struct job {
    const uint32_t* types; uint32_t A; const uint8_t* blob;
    const uint64_t* obj_base; const uint32_t* attr_len;
    uint64_t lo, hi; uint64_t* coords; int err;
};

static void* run_job(void* arg) {
    struct job* jb = (struct job*)arg;
    for (uint64_t i = jb->lo; i < jb->hi; ++i) {
        const uint8_t* p = jb->blob + jb->obj_base[i];
        const uint32_t* lens = jb->attr_len + i * jb->A;
        uint64_t* out = jb->coords + i * jb->A;
        for (uint32_t j = 0; j < jb->A; ++j) {
            int e;
            out[j] = hdxo_hash_value(jb->types[j], p, lens[j], &e);
            if (e && !jb->err) jb->err = e;
            p += lens[j];
        }
    }
    return NULL;
}

int hdxo_hash_batch(const uint32_t* types, uint32_t A, const uint8_t* blob,
                    const uint64_t* obj_base, const uint32_t* attr_len,
                    uint64_t n, uint64_t* coords, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
    struct job* jobs = (struct job*)calloc((size_t)nthreads, sizeof(struct job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (struct job){types, A, blob, obj_base, attr_len,
                               n * (uint64_t)t / nthreads, n * (uint64_t)(t + 1) / nthreads,
                               coords, 0};
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, run_job, &jobs[t]);
    run_job(&jobs[0]);
    int err = jobs[0].err;
    for (int t = 1; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (!err) err = jobs[t].err;
    }
    free(jobs);
    free(th);
    return err;
}

/* ---- region grid (admin/partition.cc) --------------------------------- */

/* partition.cc:36-55 */
static void points(uint64_t intervals, uint64_t* lbs, uint64_t* ubs) {
    uint64_t interval = (0x8000000000000000ULL / intervals) * 2;
    for (uint64_t i = 0; i < intervals; ++i) lbs[i] = i * interval;
    for (uint64_t i = 1; i < intervals; ++i) ubs[i - 1] = lbs[i] - 1;
    ubs[intervals - 1] = UINT64_MAX;
}

/* partition.cc:102-135 (recursively_generate :57-100 as an odometer over the
 * dimensions, first dimension outermost) */
uint64_t hdxo_partition(uint32_t num_attrs, uint32_t num_servers, uint64_t* lower,
                        uint64_t* upper, uint64_t max_regions) {
    if (num_attrs == 0) return 0;
    double per_dim = pow((double)num_servers, 1 / (double)num_attrs);
    uint64_t* dims = (uint64_t*)calloc(num_attrs, sizeof(uint64_t));
    for (uint32_t i = 0; i < num_attrs; ++i) dims[i] = (uint64_t)per_dim;
    uint64_t partitions = num_attrs * dims[0]; /* sic: partition.cc:109 */
    for (uint32_t i = 0; partitions < num_servers && i < num_attrs; ++i) {
        partitions = partitions / dims[i];
        ++dims[i];
        partitions = partitions * dims[i];
    }
    uint64_t bigger = dims[0], smaller = dims[num_attrs - 1];
    uint64_t *blb = (uint64_t*)calloc(bigger, 8), *bub = (uint64_t*)calloc(bigger, 8);
    uint64_t *slb = (uint64_t*)calloc(smaller, 8), *sub = (uint64_t*)calloc(smaller, 8);
    points(bigger, blb, bub);
    points(smaller, slb, sub);
    uint64_t total = 1;
    for (uint32_t i = 0; i < num_attrs; ++i) total *= dims[i];
    uint64_t* idx = (uint64_t*)calloc(num_attrs, 8);
    for (uint64_t r = 0; r < total; ++r) {
        if (r < max_regions) {
            for (uint32_t a = 0; a < num_attrs; ++a) {
                const int big = dims[a] == bigger;
                lower[r * num_attrs + a] = big ? blb[idx[a]] : slb[idx[a]];
                upper[r * num_attrs + a] = big ? bub[idx[a]] : sub[idx[a]];
            }
        }
        for (int a = (int)num_attrs - 1; a >= 0; --a) { /* last dimension fastest */
            if (++idx[a] < dims[a]) break;
            idx[a] = 0;
        }
    }
    free(dims); free(blb); free(bub); free(slb); free(sub); free(idx);
    return total;
}

/* ---- region lookup (common/configuration.cc:698-735) ------------------- */

void hdxo_lookup_region(uint32_t D, uint32_t R, const uint16_t* attrs, const uint64_t* lower,
                        const uint64_t* upper, const uint64_t* ids, const uint64_t* coords,
                        uint32_t A, uint64_t n, uint64_t* out) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t* hs = coords + i * A;
        uint64_t rid = 0; /* region_id() */
        for (uint32_t r = 0; r < R; ++r) {
            int matches = 1;
            for (uint32_t a = 0; matches && a < D; ++a) {
                const uint64_t h = hs[attrs[a]];
                matches &= lower[(uint64_t)r * D + a] <= h && h <= upper[(uint64_t)r * D + a];
            }
            if (matches) {
                rid = ids[r];
                break;
            }
        }
        out[i] = rid;
    }
}

/* ---- point_leader (common/configuration.cc:427-458; :460-497 is the same
 * scan after finding the region) --------------------------------------------
 * h = hash(sc, key) (hash.cc:48-54: the key's own type), then the first
 * subspace-0 region with lower_coord[0] <= h <= upper_coord[0]: its first
 * replica's virtual server (replicas[0].vsi), or virtual_server_id() == 0 when
 * the region has no replicas (:446-449).  No region: the reference abort()s
 * (:453); here *aborted = 1 and the result is 0. */
uint64_t hdxo_point_leader(uint32_t key_type, const uint8_t* key, size_t len, uint32_t R,
                           const uint64_t* lower0, const uint64_t* upper0, const uint64_t* leader_vsi,
                           const uint8_t* has_replicas, int* aborted) {
    int err = 0;
    const uint64_t h = hdxo_hash_value(key_type, key, len, &err);
    *aborted = 0;
    for (uint32_t pl = 0; pl < R; ++pl) {
        if (lower0[pl] <= h && h <= upper0[pl]) return has_replicas[pl] ? leader_vsi[pl] : 0;
    }
    *aborted = 1;
    return 0;
}

/* ---- stored objects (daemon/datalayer_encodings.cc:139-217) ------------ */

static uint64_t be64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
    return v;
}
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

int64_t hdxo_hash_encoded(const uint32_t* types, uint32_t A, const uint8_t* keys,
                          const uint64_t* key_off, const uint32_t* key_len, const uint8_t* vals,
                          const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                          uint64_t* coords, uint64_t* versions, uint8_t* bad) {
    int64_t nbad = 0;
    /* any schema width (the reference's attrs_sz is a u16, common/schema.h:49) */
    const uint8_t** attr_p = (const uint8_t**)malloc(sizeof(*attr_p) * (A ? A : 1));
    uint32_t* attr_n = (uint32_t*)malloc(sizeof(*attr_n) * (A ? A : 1));
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t* hs = coords + i * A;
        const uint8_t* v = vals + val_off[i];
        const uint8_t* end = v + val_len[i];
        const uint8_t* ptr = v;
        int ok = 1;
        uint64_t version = 0;
        /* :174-181 version, :185-192 count */
        if (ptr + 8 <= end) { version = be64(ptr); ptr += 8; } else ok = 0;
        uint32_t count = 0;
        if (ok && ptr + 2 <= end) { count = ((uint32_t)ptr[0] << 8) | ptr[1]; ptr += 2; } else ok = 0;
        if (ok && count != A - 1) ok = 0; /* the schema's value attributes */
        for (uint32_t k = 0; ok && k < count; ++k) {
            /* :198-213; unlike the reference, the attribute must end inside the value */
            if (ptr + 4 > end) { ok = 0; break; }
            attr_n[k] = be32(ptr);
            ptr += 4;
            if ((uint64_t)(end - ptr) < attr_n[k]) { ok = 0; break; }
            attr_p[k] = ptr;
            ptr += attr_n[k];
        }
        if (versions) versions[i] = ok ? version : 0;
        bad[i] = !ok;
        if (!ok) {
            for (uint32_t j = 0; j < A; ++j) hs[j] = 0;
            ++nbad;
            continue;
        }
        int e;
        hs[0] = hdxo_hash_value(types[0], keys + key_off[i], key_len[i], &e);
        if (e) { nbad = -1; break; }
        for (uint32_t k = 0; k + 1 < A && !e; ++k) hs[k + 1] = hdxo_hash_value(types[k + 1], attr_p[k], attr_n[k], &e);
        if (e) { nbad = -1; break; }
    }
    free(attr_p);
    free(attr_n);
    return nbad;
}

/* ---- secondary-index keys (daemon/index_*.cc) --------------------------- */

static void put_be64(uint8_t* o, uint64_t v) {
    for (int i = 0; i < 8; ++i) o[i] = (uint8_t)(v >> (56 - 8 * i));
}

size_t hdxo_index_encode(uint32_t type, const uint8_t* p, size_t len, uint8_t* out, int* err) {
    int is_float = type == 9219;
    int is_int = type == 9218 || (type >= 9473 && type <= 9478); /* index_info.cc:87-93 */
    *err = 0;
    if (!is_float && !is_int) return 0;
    const size_t size = is_float ? 16 : 8;
    memset(out, 0, size);
    if (len != 0 && len != 8) {
        *err = 2;
        return size;
    }
    /* index_int64.cc:76-79 and index_timestamp.cc:79-82 (m_iei is the int64
     * encoding, so timestamps are keyed by hash(INT64, v), not the calendar
     * hash) */
    int e = 0;
    const uint64_t h = hdxo_hash_value(is_float ? 9219 : 9218, p, len, &e);
    put_be64(out, h);
    if (is_float && len == 8) memcpy(out + 8, p, 8); /* packdoublele(number) */
    return size;
}

/* ---- search pruning (common/configuration.cc:736-858) ------------------- */

static int slice_eq(const uint8_t* a, uint64_t al, const uint8_t* b, uint64_t bl) {
    return al == bl && (al == 0 || memcmp(a, b, al) == 0);
}

int hdxo_search_regions(uint32_t D, uint32_t R, const uint16_t* attrs, const uint64_t* lower,
                        const uint64_t* upper, const uint8_t* has_replicas, const hdxo_range* ranges,
                        uint32_t nranges, uint8_t* include) {
    for (uint32_t i = 0; i < nranges; ++i) /* :761-768 */
        if (ranges[i].invalid) {
            memset(include, 0, R);
            return 1;
        }
    for (uint32_t j = 0; j < R; ++j) { /* :777 */
        int exclude = 0;
        if (has_replicas && !has_replicas[j]) { /* :782-785: skipped before any test */
            include[j] = 0;
            continue;
        }
        for (uint32_t k = 0; !exclude && k < nranges; ++k) { /* :789 */
            const hdxo_range* rg = &ranges[k];
            uint32_t attr = UINT16_MAX;
            for (uint32_t l = 0; l < D; ++l) /* :794-801 */
                if (attrs[l] == rg->attr) {
                    attr = l;
                    break;
                }
            if (attr == UINT16_MAX) continue;
            const uint64_t lo = lower[(uint64_t)j * D + attr], hi = upper[(uint64_t)j * D + attr];
            if (lo > hi) { /* :810-815 */
                memset(include, 0, R);
                return 1;
            }
            int e = 0;
            if (rg->type == 9217 && rg->has_start && rg->has_end &&
                slice_eq(rg->start, rg->start_len, rg->end, rg->end_len)) { /* :817-829 */
                const uint64_t h = hdxo_hash_value(9217, rg->start, rg->start_len, &e);
                if (lo > h || hi < h) exclude = 1;
            }
            if (rg->type == 9218 || rg->type == 9219) { /* :831-852 */
                if (rg->has_start) {
                    const uint64_t h = hdxo_hash_value(rg->type, rg->start, rg->start_len, &e);
                    if (e) return -1;
                    if (hi < h) exclude = 1;
                }
                if (rg->has_end) {
                    const uint64_t h = hdxo_hash_value(rg->type, rg->end, rg->end_len, &e);
                    if (e) return -1;
                    if (lo > h) exclude = 1;
                }
            }
        }
        include[j] = exclude ? 0 : 1;
    }
    return 0;
}

int hdxo_search_space(uint32_t ntables, const uint32_t* D, const uint32_t* R, const uint16_t* const* attrs,
                      const uint64_t* const* lower, const uint64_t* const* upper,
                      const uint8_t* const* has_replicas, const hdxo_range* ranges, uint32_t nranges,
                      uint8_t* include, int* cleared) {
    int initialized = 0, chosen = -1; /* :771-772 */
    uint32_t smallest = 0;
    *cleared = 0;
    for (uint32_t k = 0; k < nranges; ++k) { /* :761-768, before any subspace */
        if (ranges[k].invalid) {
            *cleared = 1;
            return -1;
        }
    }
    for (uint32_t i = 0; i < ntables; ++i) { /* :774 */
        uint8_t* mine = (uint8_t*)calloc(R[i] ? R[i] : 1, 1);
        int rc = hdxo_search_regions(D[i], R[i], attrs[i], lower[i], upper[i],
                                     has_replicas ? has_replicas[i] : NULL, ranges, nranges, mine);
        if (rc != 0) { /* servers->clear(); return (:766, :811), or a bad endpoint */
            free(mine);
            *cleared = rc == 1;
            return rc == 1 ? -1 : -2;
        }
        uint32_t size = 0; /* one server per included region (:853-856) */
        for (uint32_t r = 0; r < R[i]; ++r) size += mine[r];
        if (!initialized || (size != 0 && size <= smallest)) { /* :859-865 */
            smallest = size;
            chosen = (int)i;
            initialized = 1;
            memcpy(include, mine, R[i]);
        }
        free(mine);
    }
    return chosen;
}
