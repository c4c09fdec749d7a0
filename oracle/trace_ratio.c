/* oracle/trace_ratio.c — TEST INFRASTRUCTURE ONLY (built into oracle/_ref/).
 *
 * SURVEY §8d asks for the reference and the restatement timed single-threaded
 * on identical inputs in this container, so the GPU box's CPU baseline (the
 * restatement, oracle/hdx_oracle.c) is traceable to the reference.  The only
 * part of the path the reference lets us build unmodified is
 * common/ordered_encoding.cc, so:
 *   1. ordered_encode_int64 / ordered_encode_double: the reference
 *      (oracle/_ref/libref_ordered.so) vs the oracle, the same 2^24 values;
 *   2. whole config-3b objects (key + 10 strings U{0..195} + 3 int64 + 3
 *      double): the oracle's hdxo_hash_value per attribute vs the product's
 *      per-object CPU entry point hdx_hash_object (libhdxhash.so), checked
 *      equal.
 * Prints one JSON object.  Usage: trace_ratio [objects]
 */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "hdx_oracle.h"

typedef uint64_t (*enc_i64_fn)(int64_t);
typedef uint64_t (*enc_f64_fn)(double);
typedef int (*hash_object_fn)(const uint32_t*, uint32_t, const uint8_t*, size_t, const uint8_t* const*,
                              const size_t*, uint64_t*);

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const char* here = argc > 2 ? argv[2] : ".";
    char path[4096];
    snprintf(path, sizeof path, "%s/_ref/libref_ordered.so", here);
    void* ref = dlopen(path, RTLD_NOW);
    snprintf(path, sizeof path, "%s/../hyperdex_amd/libhdxhash.so", here);
    void* prod = dlopen(path, RTLD_NOW);
    if (!ref || !prod) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 2;
    }
    enc_i64_fn ref_i64 = (enc_i64_fn)dlsym(ref, "ref_ordered_encode_int64");
    enc_f64_fn ref_f64 = (enc_f64_fn)dlsym(ref, "ref_ordered_encode_double");
    hash_object_fn prod_obj = (hash_object_fn)dlsym(prod, "hdx_hash_object");
    if (!ref_i64 || !ref_f64 || !prod_obj) return 2;

    /* 1. ordered encodings */
    const size_t N = 1u << 24;
    int64_t* xi = malloc(N * sizeof *xi);
    double* xd = malloc(N * sizeof *xd);
    uint64_t s = 0x4859504552444558ull;
    for (size_t i = 0; i < N; ++i) {
        xi[i] = (int64_t)splitmix(&s);
        uint64_t b = splitmix(&s);
        memcpy(&xd[i], &b, 8);
    }
    uint64_t acc[4] = {0, 0, 0, 0};
    double t0 = now();
    for (size_t i = 0; i < N; ++i) acc[0] += ref_i64(xi[i]) ^ ref_f64(xd[i]);
    double t_ref = now() - t0;
    t0 = now();
    for (size_t i = 0; i < N; ++i) acc[1] += hdxo_encode_int64(xi[i]) ^ hdxo_encode_double(xd[i]);
    double t_orc = now() - t0;
    if (acc[0] != acc[1]) {
        fprintf(stderr, "ordered encodings differ\n");
        return 1;
    }

    /* 2. config-3b objects */
    const uint32_t A = 17;
    uint32_t types[17];
    for (uint32_t j = 0; j < A; ++j) types[j] = j <= 10 ? 9217 : j <= 13 ? 9218 : 9219;
    const size_t n = argc > 1 ? (size_t)atol(argv[1]) : 200000;
    uint32_t* len = malloc(n * A * sizeof *len);
    uint64_t* off = malloc(n * sizeof *off);
    size_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        off[i] = total;
        for (uint32_t j = 0; j < A; ++j) {
            len[i * A + j] = j == 0 ? 64 : j <= 10 ? (uint32_t)(splitmix(&s) % 196) : 8;
            total += len[i * A + j];
        }
    }
    uint8_t* blob = malloc(total + 1);
    for (size_t k = 0; k < total; ++k) blob[k] = (uint8_t)splitmix(&s);
    uint64_t* h1 = malloc(n * A * sizeof *h1);
    uint64_t* h2 = malloc(n * A * sizeof *h2);
    double t_orc_obj = 0, t_prod_obj = 0;
    const uint8_t* vp[16];
    size_t vl[16];
    for (int rep = 0; rep < 2; ++rep) {  /* the second pass of each is kept */
    t0 = now();
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* p = blob + off[i];
        for (uint32_t j = 0; j < A; ++j) {
            int e = 0;
            h1[i * A + j] = hdxo_hash_value(types[j], p, len[i * A + j], &e);
            p += len[i * A + j];
        }
    }
    t_orc_obj = now() - t0;
    t0 = now();
    for (size_t i = 0; i < n; ++i) {
        const uint8_t* p = blob + off[i] + len[i * A];
        for (uint32_t j = 1; j < A; ++j) {
            vp[j - 1] = p;
            vl[j - 1] = len[i * A + j];
            p += len[i * A + j];
        }
        if (prod_obj(types, A, blob + off[i], len[i * A], vp, vl, h2 + i * A) != 0) return 1;
    }
    t_prod_obj = now() - t0;
    }
    if (memcmp(h1, h2, n * A * sizeof *h1) != 0) {
        fprintf(stderr, "per-object hashes differ\n");
        return 1;
    }
    printf("{\"tool\": \"trace_ratio\", \"threads\": 1, "
           "\"ordered_values\": %zu, \"reference_ordered_ns\": %.3f, \"oracle_ordered_ns\": %.3f, "
           "\"oracle_over_reference\": %.3f, "
           "\"cfg3b_objects\": %zu, \"bytes_per_object\": %.1f, \"oracle_ns_per_object\": %.1f, "
           "\"product_cpu_ns_per_object\": %.1f, \"product_over_oracle\": %.3f}\n",
           N, 1e9 * t_ref / N, 1e9 * t_orc / N, t_orc / t_ref, n, (double)total / n, 1e9 * t_orc_obj / n,
           1e9 * t_prod_obj / n, t_prod_obj / t_orc_obj);
    return 0;
}
