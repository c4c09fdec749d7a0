/*
 * hdx_oracle.h — CPU restatement of HyperDex's attribute-hashing path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in hyperdex_amd/ may include, link or
 * call this.  It is the parity checker for the HIP kernels (tests/,
 * __graft_entry__.smoke()) and the timed CPU baseline in bench.py
 * ("cpu_baseline.kind" = "port").
 *
 * Pinning:
 *   - CityHash64 v1.1: every column-0 vector of the reference KAT
 *     cityhash/test/city.cc:63-1265 (tests/golden/cityhash64_kat.json).
 *   - ordered encodings: exact cases of common/test/ordered_encoding.cc:42-69
 *     and, when oracle/_ref is built, 2^20+ random inputs against the
 *     reference's own ordered_encoding.cc compiled unmodified.
 *   - timestamp hash and whole-object hash: the reference-produced values
 *     recorded in SURVEY.md §8c (survey-time reference build).
 */
#ifndef HDX_ORACLE_H
#define HDX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CityHash v1.1 CityHash64 (reference cityhash/city.cc:361-397). */
uint64_t hdxo_cityhash64(const uint8_t* s, size_t len);

/* common/ordered_encoding.cc:43-49 */
uint64_t hdxo_encode_int64(int64_t x);
/* common/ordered_encoding.cc:114-161 */
uint64_t hdxo_encode_double(double x);
/* common/datatype_timestamp.cc:138-219; type = HYPERDATATYPE_TIMESTAMP_* */
uint64_t hdxo_hash_timestamp(uint32_t type, int64_t ts);

/* common/hash.cc:34-46.  *err: 0 ok, 1 unknown type (reference asserts),
 * 2 bad size for int64/float/timestamp (reference asserts). */
uint64_t hdxo_hash_value(uint32_t type, const uint8_t* p, size_t len, int* err);

/* Whole batch in the packed layout of include/hdxhash.h:
 *   attr i,j lives at blob + obj_base[i] + sum_{k<j} attr_len[i*A+k].
 * Returns 0, or the first error code.  nthreads <= 1 runs on the caller. */
int hdxo_hash_batch(const uint32_t* types, uint32_t A, const uint8_t* blob,
                    const uint64_t* obj_base, const uint32_t* attr_len,
                    uint64_t n, uint64_t* coords, int nthreads);

/* admin/partition.cc:36-135: the rectilinear region grid HyperDex builds for a
 * subspace of num_attrs dimensions and num_servers partitions.  Writes up to
 * max_regions boxes (lower/upper row-major, num_attrs per region) and returns
 * the number of regions the reference would create. */
uint64_t hdxo_partition(uint32_t num_attrs, uint32_t num_servers, uint64_t* lower,
                        uint64_t* upper, uint64_t max_regions);

/* common/configuration.cc:698-735 (lookup_region) for a batch: region r of the
 * table matches object i when lower[r*D+a] <= coords[i*A+attrs[a]] <=
 * upper[r*D+a] for every a < D; the first match's id is written, 0
 * (region_id()) when none matches. */
uint64_t hdxo_point_leader(uint32_t key_type, const uint8_t* key, size_t len, uint32_t R,
                           const uint64_t* lower0, const uint64_t* upper0, const uint64_t* leader_vsi,
                           const uint8_t* has_replicas, int* aborted);
void hdxo_lookup_region(uint32_t D, uint32_t R, const uint16_t* attrs, const uint64_t* lower,
                        const uint64_t* upper, const uint64_t* ids, const uint64_t* coords,
                        uint32_t A, uint64_t n, uint64_t* out);

/* daemon/datalayer_encodings.cc:168-217 (decode_value) + common/hash.cc:56-68
 * over stored objects: value i = vals[val_off[i], +val_len[i]) encoded as
 * [u64 BE version][u16 BE count]{[u32 BE len][bytes]}*count, key i =
 * keys[key_off[i], +key_len[i]).  coords[i*A+0] = hash(types[0], key),
 * coords[i*A+1+k] = hash(types[1+k], attribute k).  versions may be NULL.
 * bad[i] = 1 (and coords 0) when the value does not decode into A-1
 * attributes inside its bytes; returns the number of such objects, or -1 on
 * an unknown type / mis-sized numeric. */
int64_t hdxo_hash_encoded(const uint32_t* types, uint32_t A, const uint8_t* keys,
                          const uint64_t* key_off, const uint32_t* key_len, const uint8_t* vals,
                          const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                          uint64_t* coords, uint64_t* versions, uint8_t* bad);

/* daemon/index_int64.cc:76-79, index_timestamp.cc:79-82, index_float.cc:75-90:
 * the secondary-index key of one value.  INT64 and TIMESTAMP_* write 8 bytes
 * (big-endian hash(INT64, v)); FLOAT writes 16 (big-endian hash(FLOAT, v),
 * then the double's little-endian bytes or 0.0 when not 8 bytes long).
 * Returns the key size, 0 for other types; *err = 2 (and an all-zero key)
 * when the value's size is not 0 or 8 (the reference asserts). */
size_t hdxo_index_encode(uint32_t type, const uint8_t* p, size_t len, uint8_t* out, int* err);

/* common/range.h:40-55 after range_searches(); same layout as hdx_range. */
typedef struct hdxo_range {
    uint32_t attr, type;
    const uint8_t* start;
    uint64_t start_len;
    const uint8_t* end;
    uint64_t end_len;
    uint32_t has_start, has_end, invalid, reserved;
} hdxo_range;

/* common/configuration.cc:736-858 (lookup_search), the region loop of one
 * subspace whose attributes are attrs[D] and boxes lower/upper[R*D]:
 * include[r] = 1 unless a range excludes region r.  Returns 1 (and all-zero
 * include) when the reference clears the server list, else 0; -1 when a
 * numeric endpoint's size is not 0 or 8. */
int hdxo_search_regions(uint32_t D, uint32_t R, const uint16_t* attrs, const uint64_t* lower,
                        const uint64_t* upper, const uint8_t* has_replicas, const hdxo_range* ranges,
                        uint32_t nranges, uint8_t* include);

/* common/configuration.cc:771-868 (lookup_search's choice over subspaces):
 * subspace i has D[i] attributes attrs[i], R[i] boxes lower[i]/upper[i] and
 * replica flags has_replicas[i] (may be NULL).  Returns the chosen subspace
 * (its include mask in include[0..R[chosen])) or -1 (none, or cleared: then
 * *cleared = 1); -2 on a bad numeric endpoint. */
int hdxo_search_space(uint32_t ntables, const uint32_t* D, const uint32_t* R, const uint16_t* const* attrs,
                      const uint64_t* const* lower, const uint64_t* const* upper,
                      const uint8_t* const* has_replicas, const hdxo_range* ranges, uint32_t nranges,
                      uint8_t* include, int* cleared);

#ifdef __cplusplus
}
#endif

#endif
