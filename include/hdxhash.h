/*
 * hdxhash.h — C-ABI of the MI355X hyperspace-hashing engine (libhdxhash.so).
 *
 * Replaces the per-object attribute hashing of HyperDex:
 *   uint64_t hyperdex::hash(hyperdatatype, const e::slice&)          common/hash.h:43-44, hash.cc:34-46
 *   void     hyperdex::hash(const schema&, const e::slice& key, uint64_t* h)
 *                                                                  common/hash.h:46-49, hash.cc:48-54
 *   void     hyperdex::hash(const schema&, const e::slice& key,
 *                           const std::vector<e::slice>& value, uint64_t* hs)
 *                                                                  common/hash.h:51-55, hash.cc:56-68
 * with (a) C entry points of the same meaning (hdx_hash_value / hdx_hash_key /
 * hdx_hash_object) and (b) a batched entry point over a packed layout that
 * runs the hand-written gfx950 kernels (hdx_hash_batch_device / _host).
 * The C++ signatures themselves are provided header-only by
 * include/hyperdex_amd/hash.h on top of these functions.
 *
 * Plain pointers and sizes only.  Type ids are the reference's
 * enum hyperdatatype values (include/hyperdex.h:53-102).
 *
 * Packed batch layout (all arrays caller-owned):
 *   types[A]        u32 hyperdatatype per attribute position; attr 0 = key
 *                   (schema.attrs[i].type, common/schema.h:40-51)
 *   blob            bytes; object i's attributes are stored back to back
 *                   starting at blob + obj_base[i] (any alignment)
 *   obj_base[n]     u64 byte offset of object i in blob (objects may have gaps
 *                   between them and may appear in any order)
 *   attr_len[n*A]   u32 length of attribute j of object i at [i*A + j]
 *   coords[n*A]     u64 output, row-major: coords[i*A + j] = hash of attr j
 *                   (= hs[j] of the reference's whole-object hash)
 * Limits: 1 <= A <= HDX_MAX_ATTRS (65535, the reference's u16 attrs_sz);
 * each object's attributes total < 4 GiB.
 *
 * Errors: the reference asserts on an unknown type (hash.cc:38) and on an
 * int64/float/timestamp value whose size is not 0 or 8
 * (datatype_int64.cc:233, datatype_float.cc:204, datatype_timestamp.cc:46);
 * this library returns HDX_E_BADTYPE / HDX_E_BADSIZE instead and never
 * aborts.  Non-hashable types (document, list, set, map, macaroon) hash to 0
 * exactly as in the reference (hash.cc:40-43).
 *
 * Threading: every entry point is thread-safe.  Device work is issued on the
 * caller's stream (batch API; NULL = null stream) or on library streams
 * (host-resident and multi-device API).
 *
 * Two implementations, split by call shape: the per-object entry points
 * (hdx_hash_value / hdx_hash_key / hdx_hash_object, the C forms of
 * common/hash.h) run on the host CPU, bit-exact, with no device and no
 * allocation; every batch entry point runs the gfx950 kernels, with no CPU
 * substitute — without a usable gfx950 device it returns HDX_E_DEVICE.
 */
#ifndef HDXHASH_H
#define HDXHASH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HDX_ABI_VERSION 4
/* The reference's schema::attrs_sz is a u16 (common/schema.h:49). */
#define HDX_MAX_ATTRS 65535

typedef enum hdx_status {
    HDX_OK = 0,
    HDX_E_BADTYPE = 1,     /* unknown hyperdatatype (reference: assert(di)) */
    HDX_E_BADSIZE = 2,     /* int64/float/timestamp value of size not in {0, 8} */
    HDX_E_DEVICE = 3,      /* no usable device, or a HIP runtime error */
    HDX_E_INVALID = 4,     /* bad argument: NULL pointer, A == 0, A > HDX_MAX_ATTRS */
    HDX_E_NOMEM = 5,       /* device or pinned allocation failed */
    HDX_E_BADENC = 6       /* a stored value does not decode (hdx_hash_encoded_device) */
} hdx_status;

/* An opaque hipStream_t.  NULL is the HIP null (default) stream. */
typedef void* hdx_stream;
/* A subspace's region table (hdx_region_table_create, below). */
typedef struct hdx_region_table_s* hdx_region_table;

/* ---- library state ---------------------------------------------------- */

/* ABI version and a human-readable build string. */
int hdx_abi_version(void);
const char* hdx_version(void);
/* Binds the calling thread to `device` (a HIP ordinal) and checks it is a
 * gfx950 part.  Optional: every entry point initialises lazily on device 0
 * or on the thread's current HIP device. */
hdx_status hdx_init(int device);
/* The process's device set (hdx_init(device_mask)).  Checks that
 * every device in device_mask (bit d = HIP ordinal d) is a visible gfx950
 * part, binds the calling thread to the lowest one, and creates per device
 * one worker thread (with its own streams and pinned / device staging) and
 * one stream; the RCCL communicator over the set is created on the first
 * gathering hdx_hash_batch_device_multi.  From then on hdx_hash_batch_host
 * splits every batch over the set, and hdx_hash_batch_device_multi takes one
 * shard per device.  Calling it again with the same mask does nothing; with
 * another mask it replaces the set (no call may be in progress). */
hdx_status hdx_init_mask(uint64_t device_mask);
/* The device set's HIP ordinals, ascending, into devices[0..max_devices);
 * returns how many devices it has (0: no hdx_init_mask yet). */
int hdx_device_set(int* devices, int max_devices);
/* Tears the device set down (joins its workers, destroys its streams and
 * communicator) and frees every thread's library scratch (streams, pinned
 * and device staging) after waiting for the work queued on it.  No call may
 * be in progress; region tables and batchers are the caller's to destroy.
 * Threads rebind lazily on their next call; the host-resident path runs on
 * the calling thread's device again until the next hdx_init_mask. */
hdx_status hdx_shutdown(void);
/* Number of HIP devices visible (0 without a GPU; never initialises one). */
int hdx_device_count(void);
/* Message for the last non-OK status returned on this thread. */
const char* hdx_last_error(void);
/* hipStreamSynchronize on `stream` (NULL: the null stream). */
hdx_status hdx_sync(hdx_stream stream);

/* ---- schema ------------------------------------------------------------ */

/* HDX_OK if every type id is a hyperdatatype the reference's
 * datatype_info::lookup accepts (datatype_info.cc:72-141), else
 * HDX_E_BADTYPE.  Host only; no device needed. */
hdx_status hdx_schema_check(const uint32_t* types, uint32_t attrs_sz);
/* 1 if datatype_info::lookup(type)->hashable() (string, int64, float,
 * timestamp second..month), 0 otherwise (including unknown). */
int hdx_type_hashable(uint32_t type);

/* ---- batched hashing (the GPU path) -------------------------------------- */

/* All of blob, obj_base, attr_len, coords are DEVICE pointers; `types` is a
 * HOST array.  Asynchronous on `stream`: returns after the launch.  If
 * `status_dev` (a device u32, may be NULL) is given, the kernel ORs
 * (1u << HDX_E_BADSIZE) into it for any mis-sized numeric attribute (whose
 * coordinate is then written as 0).  Returns HDX_E_BADTYPE / HDX_E_INVALID
 * before launching anything. */
hdx_status hdx_hash_batch_device(const uint32_t* types, uint32_t attrs_sz,
                                 const uint8_t* blob, const uint64_t* obj_base,
                                 const uint32_t* attr_len, uint64_t n,
                                 uint64_t* coords, uint32_t* status_dev,
                                 hdx_stream stream);

/* Same batch with every array in HOST memory (pageable or pinned).
 * Synchronous.  Any thread; the calling thread runs its own device's share
 * itself.  The library streams the batch through the device in chunks,
 * overlapping H2D copies, kernels and D2H copies on two streams, and
 * validates numeric sizes and object extents on the host chunk by chunk
 * ahead of the copies.  blob_bytes is the size of the blob allocation (every
 * object must lie inside it).  After hdx_init_mask the batch is split into
 * one contiguous object range per device of the set, balanced by payload
 * bytes (hdx_shard_ranges with no equal-count tolerance), and each device's
 * worker pipelines its range into its rows of coords; without a device set
 * the calling thread's device takes the whole batch.  On HDX_E_BADSIZE /
 * HDX_E_INVALID nothing is in flight when the call returns and the status
 * is the first failing range's (in device order); coordinates of other
 * objects may have been written. */
hdx_status hdx_hash_batch_host(const uint32_t* types, uint32_t attrs_sz,
                               const uint8_t* blob, uint64_t blob_bytes,
                               const uint64_t* obj_base, const uint32_t* attr_len,
                               uint64_t n, uint64_t* coords);

/* The same host-resident batch for the ingest path: every object's region in
 * ntables (1..4) subspaces, region_ids[t*n + i] = lookup_region(tables[t],
 * hash(schema, key, value) of object i) — the values hdx_lookup_region_device
 * gives on hdx_hash_batch_host's coordinates — with only 8 bytes per table
 * per object crossing PCIe back (key_state::hash_objects consumes only
 * regions, daemon/key_state.cc:1482-1534).  coords (host, may be NULL) also
 * receives the coordinates.  Split over the device set like
 * hdx_hash_batch_host; the tables are replicated to each device on first use.
 * Synchronous. */
hdx_status hdx_hash_batch_regions_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* blob,
                                       uint64_t blob_bytes, const uint64_t* obj_base, const uint32_t* attr_len,
                                       uint64_t n, const hdx_region_table* tables, uint32_t ntables,
                                       uint64_t* region_ids, uint64_t* coords);

/* ---- multi-device (the device set of hdx_init_mask) ---------------------- */

/* Contiguous object ranges, one per shard, balanced by payload bytes (SURVEY
 * §8e; the rule of hyperdex_amd/dist.py shard_ranges): object i's size is
 * the sum of attr_len[i*attrs_sz .. +attrs_sz), and shard k starts at the
 * first object whose byte prefix reaches k/world of the total.  With
 * equal_count_tol > 0 the equal-count cuts (n*k/world) are taken instead
 * whenever every shard's bytes stay within that fraction of the mean share
 * (so the gather needs no padding).  attr_len NULL: equal counts.  Output:
 * first[0..world], first[world] = n.  Host only; no device needed. */
hdx_status hdx_shard_ranges(const uint32_t* attr_len, uint32_t attrs_sz, uint64_t n, uint32_t world,
                            double equal_count_tol, uint64_t* first);

/* One device's shard of a device-resident batch (the packed layout above;
 * device pointers on that device). */
typedef struct hdx_shard {
    const uint8_t* blob;
    const uint64_t* obj_base;   /* offsets into this shard's blob */
    const uint32_t* attr_len;   /* n * attrs_sz */
    uint64_t n;                 /* objects in this shard (may be 0) */
    uint64_t* coords;           /* gather: the whole (N x attrs_sz) matrix on this
                                   device, N = the shards' total; else this
                                   shard's own (n x attrs_sz) rows */
    uint32_t* status_dev;       /* may be NULL; as hdx_hash_batch_device */
} hdx_shard;
/* Hashes shards[k] on the k-th device of the set (nshards = the set's size)
 * on the library's per-device streams.  gather != 0: shard k is hashed into
 * rows [first_k, first_k + n_k) of its device's matrix (first_k = the
 * earlier shards' total), then the rows are exchanged over the devices' RCCL
 * communicator (ncclCommInitAll over the set, xGMI) in ONE group: an
 * in-place all-gather when every shard has the same count, else one in-place
 * broadcast per shard — no staging memory either way — so every device ends
 * with all N rows.  Synchronous: returns when every device is done. */
hdx_status hdx_hash_batch_device_multi(const uint32_t* types, uint32_t attrs_sz, const hdx_shard* shards,
                                       uint32_t nshards, int gather);

/* The region-id form of the same: each shard is hashed and
 * looked up in ntables (1..4) region tables on its device; with gather, ONLY
 * the region ids are exchanged — 8 bytes per table per object instead of the
 * 8 * attrs_sz of the coordinates (config 3b: 16 vs 136 bytes with two
 * tables).  The tables are replicated to each device on first use. */
typedef struct hdx_region_shard {
    const uint8_t* blob;
    const uint64_t* obj_base;
    const uint32_t* attr_len;
    uint64_t n;
    uint64_t* region_ids;       /* gather: ntables x N on this device, table t's id of object i at
                                   [t*N + i] (N = the shards' total); else ntables x n, [t*n + i] */
    uint64_t* coords;           /* may be NULL: this shard's own (n x attrs_sz) coordinates,
                                   never exchanged */
    uint32_t* status_dev;       /* may be NULL; as hdx_hash_batch_device */
} hdx_region_shard;
hdx_status hdx_hash_batch_regions_device_multi(const uint32_t* types, uint32_t attrs_sz,
                                               const hdx_region_shard* shards, uint32_t nshards,
                                               const hdx_region_table* tables, uint32_t ntables, int gather);

/* Reindex sweep over stored objects: value i is
 * vals[val_off[i], +val_len[i]) in the daemon's on-disk encoding
 * [u64 BE version][u16 BE count]{[u32 BE len][bytes]}*count
 * (daemon/datalayer_encodings.cc:139-217), key i is keys[key_off[i],
 * +key_len[i]).  Decodes and hashes every object in one launch:
 * coords[i*A + 0] = hash(types[0], key), coords[i*A + 1 + k] =
 * hash(types[1+k], attribute k); versions[i] (may be NULL) = the value's
 * version.  An object whose value does not decode into exactly A-1
 * attributes lying inside its bytes gets zero coordinates (and version 0)
 * and (1u << HDX_E_BADENC) is ORed into status_dev (may be NULL).  The
 * reference's decode_value does not check that the last attribute ends
 * inside the value (:201-213); this does.  Any placement of keys and values
 * is exact; keys back to back, values back to back, or — keys == vals —
 * records [key][value] back to back are read with coalesced span copies.
 * Device pointers, asynchronous.  Any attrs_sz up to HDX_MAX_ATTRS (above 128
 * a wave per object, hdx_wide.hip). */
hdx_status hdx_hash_encoded_device(const uint32_t* types, uint32_t attrs_sz,
                                   const uint8_t* keys, const uint64_t* key_off,
                                   const uint32_t* key_len, const uint8_t* vals,
                                   const uint64_t* val_off, const uint32_t* val_len,
                                   uint64_t n, uint64_t* coords, uint64_t* versions,
                                   uint32_t* status_dev, hdx_stream stream);

/* The reindex sweep from HOST memory (datalayer::indexer_thread reads the
 * region's stored objects from LevelDB into host buffers, daemon/
 * datalayer_indexer_thread.cc:161-176, daemon/datalayer.cc:853-882): the
 * arrays of hdx_hash_encoded_device, all in host memory (pageable or pinned),
 * keys_bytes / vals_bytes the sizes of the two stores (keys == vals: records
 * [key][value] in one store).  The call is cut into contiguous object ranges
 * balanced by key + value bytes, one per device of the set (the calling
 * thread's device without one); each device pipelines its range through PCIe
 * in 128 MiB chunks (H2D of each chunk's key and value spans, the sweep, D2H
 * of its coordinates and versions) into the caller's arrays.  versions may be
 * NULL.  Synchronous.  Returns HDX_E_BADENC when a value does not decode
 * (those objects get zero coordinates and version 0, every other object is
 * hashed) and HDX_E_BADSIZE for a numeric value of neither 0 nor 8 bytes
 * (coordinate 0), naming the device and the object range; HDX_E_INVALID for
 * a key or value outside its store, before anything of its chunk is copied. */
hdx_status hdx_hash_encoded_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* keys,
                                 uint64_t keys_bytes, const uint64_t* key_off, const uint32_t* key_len,
                                 const uint8_t* vals, uint64_t vals_bytes, const uint64_t* val_off,
                                 const uint32_t* val_len, uint64_t n, uint64_t* coords, uint64_t* versions);
/* ... and each object's region under ntables (1..4) subspaces (the
 * indexer's purpose), region_ids[t*n + i], host memory; coords may be NULL. */
hdx_status hdx_hash_encoded_regions_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* keys,
                                         uint64_t keys_bytes, const uint64_t* key_off, const uint32_t* key_len,
                                         const uint8_t* vals, uint64_t vals_bytes, const uint64_t* val_off,
                                         const uint32_t* val_len, uint64_t n, const hdx_region_table* tables,
                                         uint32_t ntables, uint64_t* region_ids, uint64_t* coords,
                                         uint64_t* versions);

/* ---- per-value / per-object (the reference signatures, C form) ---------- */

/* hash(hyperdatatype, slice)  — common/hash.cc:34-46 */
hdx_status hdx_hash_value(uint32_t type, const uint8_t* data, size_t len, uint64_t* out);
/* hash(schema, key, &h)       — common/hash.cc:48-54 (uses types[0] only) */
hdx_status hdx_hash_key(const uint32_t* types, uint32_t attrs_sz,
                        const uint8_t* key, size_t key_len, uint64_t* h);
/* hash(schema, key, value, hs) — common/hash.cc:56-68.  values[k] /
 * value_lens[k] are attribute k+1, k in [0, attrs_sz-1). */
hdx_status hdx_hash_object(const uint32_t* types, uint32_t attrs_sz,
                           const uint8_t* key, size_t key_len,
                           const uint8_t* const* values, const size_t* value_lens,
                           uint64_t* hs);

/* ---- coordinates -> regions ------------------------------ */

/* A subspace's region table on the device: `dims` = subspace.attrs.size()
 * (<= 16), attrs[dims] the schema attribute indices of the subspace
 * (common/hyperspace.h:99-113), lower/upper[regions*dims] the boxes and
 * ids[regions] the region ids (region.id, common/hyperspace.h:122-137), all
 * host arrays, copied at creation. */
hdx_status hdx_region_table_create(uint32_t dims, uint32_t regions, const uint16_t* attrs,
                                   const uint64_t* lower, const uint64_t* upper,
                                   const uint64_t* ids, hdx_region_table* out);
hdx_status hdx_region_table_destroy(hdx_region_table table);
/* configuration::lookup_region (common/configuration.cc:698-735) for n
 * objects: region_ids[i] = id of the first region whose box holds
 * coords[i*attrs_sz + attrs[a]] for every a (bounds inclusive), else 0
 * (region_id()).  Device pointers; asynchronous on `stream`.  With a table
 * of subspace 0 (attrs = {0}) this is point_leader's region (:427-497). */
hdx_status hdx_lookup_region_device(hdx_region_table table, const uint64_t* coords,
                                    uint32_t attrs_sz, uint64_t n, uint64_t* region_ids,
                                    hdx_stream stream);

/* The sweep's purpose (daemon/datalayer_indexer_thread.cc): every stored
 * object's region under a new subspace configuration.  One launch decodes,
 * hashes and looks up: region_ids[t*n + i] = lookup_region(tables[t], the
 * coordinates of object i) for t < ntables (1..4) — the values
 * hdx_lookup_region_device would give on the coordinates hdx_hash_encoded_device
 * computes (an undecodable object's are zero).  coords may be NULL.  The
 * tables' subspace attributes must be < attrs_sz.  Device pointers,
 * asynchronous; any attrs_sz (above 128 always hash + lookups).
 * Implementation note: below 2^20 objects this is one fused launch; from
 * 2^20 on, the hash and one lookup launch per table (faster there: the hash
 * kernels are VALU-bound), and with coords NULL the coordinates then pass
 * through device scratch of at most 2 GiB per chunk, allocated and freed
 * stream-ordered on `stream` from a memory pool the library keeps per device
 * (one chunk cached between calls; hdx_shutdown trims it). */
hdx_status hdx_hash_encoded_regions_device(const uint32_t* types, uint32_t attrs_sz,
                                           const uint8_t* keys, const uint64_t* key_off,
                                           const uint32_t* key_len, const uint8_t* vals,
                                           const uint64_t* val_off, const uint32_t* val_len,
                                           uint64_t n, const hdx_region_table* tables,
                                           uint32_t ntables, uint64_t* region_ids, uint64_t* coords,
                                           uint64_t* versions, uint32_t* status_dev, hdx_stream stream);

/* The batch form of the same fusion, for objects in the packed layout of
 * hdx_hash_batch_device (blob / obj_base / attr_len): one launch hashes every
 * object and looks it up in ntables (1..4) region tables — region_ids[t*n + i]
 * = lookup_region(tables[t], hash(schema, key, value) of object i), what
 * hdx_lookup_region_device gives on hdx_hash_batch_device's coordinates.
 * coords may be NULL (the ingest path key_state::hash_objects -> point_leader
 * / lookup_region needs only the region).  Device pointers, asynchronous;
 * any attrs_sz (above 128: hash + lookups, and with coords NULL the
 * coordinates' scratch is required: HDX_E_NOMEM without it); status_dev
 * (may be NULL) gets HDX_E_BADSIZE's bit for a
 * numeric value not 0 or 8 bytes long.  Mixed string / numeric schemas from
 * 2^20 objects on take hash + per-table lookups, with the scratch of
 * hdx_hash_encoded_regions_device's note when coords is NULL. */
hdx_status hdx_hash_batch_regions_device(const uint32_t* types, uint32_t attrs_sz, const uint8_t* blob,
                                         const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n,
                                         const hdx_region_table* tables, uint32_t ntables,
                                         uint64_t* region_ids, uint64_t* coords, uint32_t* status_dev,
                                         hdx_stream stream);

/* ---- secondary-index keys and search pruning ------------ */

/* Bytes of one index key for `type`: 8 for INT64 and TIMESTAMP_*, 16 for
 * FLOAT, 0 for types whose index key is not a fixed-size hash encoding. */
size_t hdx_index_key_size(uint32_t type);
/* index_encoding_{int64,timestamp,float}::encode (daemon/index_int64.cc:76-79,
 * daemon/index_timestamp.cc:79-82, daemon/index_float.cc:75-90) for n values
 * of one attribute: value i is len[i] bytes at blob + off[i]; key i is
 * written at out + i * hdx_index_key_size(type):
 *   INT64, TIMESTAMP_*: big-endian ordered_encode_int64 (the int64 hash);
 *   FLOAT:              big-endian ordered_encode_double ++ the double's
 *                       little-endian bytes (0.0 when the value is empty).
 * A value whose size is not 0 or 8 gets an all-zero key and sets bit
 * (1 << HDX_E_BADSIZE) in *status_dev (the reference asserts).  Device
 * pointers; asynchronous on `stream`. */
hdx_status hdx_index_encode_device(uint32_t type, const uint8_t* blob, const uint64_t* off,
                                   const uint32_t* len, uint64_t n, uint8_t* out,
                                   uint32_t* status_dev, hdx_stream stream);

/* One range of a search, as range_searches() leaves it (common/range.h:40-55,
 * common/range_searches.cc:151-202): inclusive, at most one per attribute. */
typedef struct hdx_range {
    uint32_t attr;        /* schema attribute index */
    uint32_t type;        /* hyperdatatype of the attribute */
    const uint8_t* start; /* host bytes */
    uint64_t start_len;
    const uint8_t* end;
    uint64_t end_len;
    uint32_t has_start;
    uint32_t has_end;
    uint32_t invalid;
    uint32_t reserved;
} hdx_range;
/* The region test of configuration::lookup_search (common/configuration.cc:
 * 736-858) for one subspace: include[r] = 0 when region r of `table` has no
 * replicas (has_replicas[r] == 0; skipped before any test, :782-785) or a
 * range excludes it (a STRING range with start == end whose hash lies outside
 * the region's box on that dimension; an INT64/FLOAT range whose hashed start
 * is above the box or hashed end below it), else 1.  *cleared = 1 when the
 * reference would return an empty server list (an invalid range, or a region
 * with replicas whose box has lower > upper on a ranged dimension reached
 * before the region is excluded, :808-813); include[] is then all 0.
 * has_replicas may be NULL (every region has replicas).  Endpoint hashes are
 * computed on the device.  Host pointers; synchronous. */
hdx_status hdx_search_regions(hdx_region_table table, const hdx_range* ranges, uint32_t nranges,
                              const uint8_t* has_replicas, uint8_t* include, int* cleared);

/* The whole of configuration::lookup_search (common/configuration.cc:737-868)
 * over a space's subspaces tables[0..ntables) (in the space's order): each
 * subspace's server set is its hdx_search_regions include mask (one server per
 * included region, region.replicas.back(), :853-856); the first subspace
 * initialises the choice and a later one replaces it only when its set is
 * non-empty and no larger than the current one (:859-865; so the last of equal
 * sizes wins, and an empty first subspace is never replaced).  Outputs:
 * *chosen = the chosen subspace index (-1 when ntables == 0 or cleared),
 * include[0..max R) = its mask (zero beyond its R), *servers = its set size,
 * *cleared = 1 when the reference returns an empty list outright (an invalid
 * range, or an ill-formed box reached in any subspace).  has_replicas may be
 * NULL, or hold one per-table flag array (entries may be NULL).  Host
 * pointers; synchronous. */
hdx_status hdx_search_space(const hdx_region_table* tables, uint32_t ntables, const hdx_range* ranges,
                            uint32_t nranges, const uint8_t* const* has_replicas, int32_t* chosen,
                            uint8_t* include, uint32_t* servers, int* cleared);

/* ---- daemon batching shim --------------------------------- */

/* key_state::hash_objects (daemon/key_state.cc:1455-1543) hashes one or two
 * objects per replicated op, from every daemon::loop thread at once.  A
 * batcher keeps that synchronous per-object call.  By default every object is
 * hashed on the calling thread by the per-object CPU path (hdx_hash_object)
 * and looked up in the batcher's tables on the host (configuration::
 * lookup_region's scan): a core hashes a config-3b object in ~0.15 us, a
 * device round trip costs ~36 us, and CityHash is serial within a string, so
 * no device batch of synchronous callers beats their own cores at any object
 * size.  Objects above host_max_bytes, or every object with
 * HDX_BATCHER_DEVICE_ONLY (hosts whose cores are needed elsewhere: the
 * callers sleep while the device works), are coalesced into device batches:
 * each caller copies its object into a pinned staging buffer and blocks; a
 * flush thread ships a batch as soon as the previous one has completed, when
 * it is full, or `max_delay_us` after its first object, runs the hash kernel
 * (and the region lookups of the batcher's tables) and wakes the callers.
 * One batcher per space (schema). */
typedef struct hdx_batcher_s* hdx_batcher;
typedef struct hdx_batcher_config {
    uint32_t max_objects;    /* objects per device batch; 0 = 4096 */
    uint32_t max_delay_us;   /* flush a partial batch this long after its first object; 0 = 50 */
    uint64_t max_bytes;      /* payload bytes per device batch; 0 = 8 MiB */
    uint32_t slots;          /* staging buffers in rotation (>= 2); 0 = 4 */
    int32_t device;          /* -1 = the creating thread's current device */
    const hdx_region_table* tables; /* optional: subspaces to look every object up in */
    uint32_t ntables;        /* <= 16 */
    uint32_t flags;          /* HDX_BATCHER_* */
    uint64_t host_max_bytes; /* objects of at most this many payload bytes are hashed on the
                                calling thread; 0 = every object */
} hdx_batcher_config;
/* Stage batches through device memory (H2D, kernels, D2H) instead of letting
 * the kernels read and write the pinned staging buffers in place (default,
 * fewer operations per batch; best for the small batches of a daemon). */
#define HDX_BATCHER_STAGE_DEVICE 1u
/* Every object goes to the device, whatever its size (the calling threads'
 * cores stay free for the rest of the daemon). */
#define HDX_BATCHER_DEVICE_ONLY 2u
typedef struct hdx_batcher_stats {
    uint64_t objects;        /* objects hashed */
    uint64_t batches;        /* device batches shipped */
    uint64_t full_batches;   /* batches shipped because they were full */
    uint64_t direct;         /* objects larger than max_bytes, hashed on the device on their own */
    uint64_t host;           /* objects hashed on the calling thread */
} hdx_batcher_stats;
/* cfg may be NULL (all defaults).  The tables must outlive the batcher. */
hdx_status hdx_batcher_create(const uint32_t* types, uint32_t attrs_sz, const hdx_batcher_config* cfg,
                              hdx_batcher* out);
/* Waits for in-flight batches, then frees everything.  No call may be in
 * progress on the batcher. */
hdx_status hdx_batcher_destroy(hdx_batcher b);
/* hdx_hash_object through the batcher: returns once the object is hashed
 * (on the calling thread, or after its device batch has run).  Thread-safe;
 * any number of threads.  When the batcher has tables, region_ids[t]
 * receives lookup_region(tables[t], hs) (region_ids may be NULL to skip).  A
 * numeric attribute whose size is not 0 or 8 returns HDX_E_BADSIZE before
 * anything is hashed. */
hdx_status hdx_batcher_hash_object(hdx_batcher b, const uint8_t* key, size_t key_len,
                                   const uint8_t* const* values, const size_t* value_lens,
                                   uint64_t* hs, uint64_t* region_ids);
hdx_status hdx_batcher_get_stats(hdx_batcher b, hdx_batcher_stats* out);

/* ---- pinned host memory ------------------------------------------------- */

hdx_status hdx_alloc_pinned(size_t bytes, void** out);
hdx_status hdx_free_pinned(void* p);

/* ---- synthetic batches (benchmark tooling; see hyperdex_amd/synth.py) ---- */

/* Per-attribute synthetic rule, one per attribute position. */
typedef struct hdx_synth_rule {
    uint32_t type;   /* hyperdatatype */
    uint32_t kind;   /* 0 fixed len lo; 1 uniform len in [lo, hi]; 2 numeric (8 B, 1% empty) */
    uint32_t lo;
    uint32_t hi;
} hdx_synth_rule;

/* attr_len[n*A] for objects [first, first+n) of the synthetic stream `seed`. */
hdx_status hdx_synth_lengths(const hdx_synth_rule* rules, uint32_t attrs_sz, uint64_t seed,
                             uint64_t first, uint64_t n, uint32_t* attr_len_dev,
                             hdx_stream stream);
/* Fills blob_dev[0, bytes) with the seed's byte stream (position-keyed), then
 * writes the numeric attributes (int64/float/timestamp values incl. special
 * values) at their offsets.  obj_base_dev must already hold the offsets. */
hdx_status hdx_synth_fill(const hdx_synth_rule* rules, uint32_t attrs_sz, uint64_t seed,
                          uint64_t first, uint64_t n, const uint64_t* obj_base_dev,
                          const uint32_t* attr_len_dev, uint8_t* blob_dev, uint64_t bytes,
                          hdx_stream stream);

/* Encode objects of a packed batch into stored values (the encode_value
 * format above), version first_version + i, at vals_dev + val_off_dev[i];
 * val_off must hold room for 10 + sum_{j>=1}(4 + attr_len[i*A+j]) bytes each. */
hdx_status hdx_synth_encode_values(const uint8_t* blob_dev, const uint64_t* obj_base_dev,
                                   const uint32_t* attr_len_dev, uint32_t attrs_sz, uint64_t n,
                                   uint64_t first_version, const uint64_t* val_off_dev,
                                   uint8_t* vals_dev, hdx_stream stream);

/* The same, with every key (attribute 0 of object i) also copied to
 * keys_dev + key_off_dev[i]: a key column beside the values, or — keys_dev ==
 * vals_dev and key_off = val_off - key_len — records [key][value] in one
 * store (the adjacency of a LevelDB block's entries). */
hdx_status hdx_synth_encode_store(const uint8_t* blob_dev, const uint64_t* obj_base_dev,
                                  const uint32_t* attr_len_dev, uint32_t attrs_sz, uint64_t n,
                                  uint64_t first_version, const uint64_t* val_off_dev, uint8_t* vals_dev,
                                  const uint64_t* key_off_dev, uint8_t* keys_dev, hdx_stream stream);

#ifdef __cplusplus
}
#endif

#endif /* HDXHASH_H */
