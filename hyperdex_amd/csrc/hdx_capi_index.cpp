// hdx_capi_index.cpp — C-ABI for the index-key encoders and the search
// region test (include/hdxhash.h).  Host work here is argument
// checking and packing the search endpoints; the hashing and the per-region
// tests run in hdx_index.hip / hdx_kernels.hip.
#include <hip/hip_runtime.h>

#include <cstring>
#include <functional>
#include <vector>

#include "hdx_host.h"

using namespace hdx;

namespace {

// Index key code for a hyperdatatype (daemon/index_info.cc:77-118 routes
// TIMESTAMP_* to index_encoding_timestamp, which is the int64 encoding).
int index_code(uint32_t type) {
    if (type == 9218) return CODE_INT64;
    if (type == 9219) return CODE_FLOAT;
    if (type >= 9473 && type <= 9478) return CODE_INT64;
    return -1;
}

// Per-thread staging for hdx_search_regions: one pinned block
// [endpoints | obj_base | attr_len | hashes | include | cleared/status] and
// its device twin, so a search is one H2D, two launches and one D2H.
struct SearchStage : Scratch {
    int device = -1;
    bool tracked = false;
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    std::function<void()> detach() {
        if (device < 0) return {};
        const int d = device;
        uint8_t *h = host, *g = dev;
        host = dev = nullptr;
        cap = 0;
        device = -1;
        return [d, h, g] {
            (void)hipSetDevice(d);
            (void)hipHostFree(h);
            (void)hipFree(g);
        };
    }
    void release() override {
        if (auto f = detach()) f();
    }
    ~SearchStage() {  // no HIP call at thread exit (hdx_capi.cpp, park_orphan)
        if (tracked) untrack_scratch(this);
        if (auto f = detach()) park_orphan(std::move(f));
    }
};
thread_local SearchStage t_search;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

HDX_EXPORT size_t hdx_index_key_size(uint32_t type) {
    const int c = index_code(type);
    return c < 0 ? 0 : (c == CODE_FLOAT ? 16 : 8);
}

HDX_EXPORT hdx_status hdx_index_encode_device(uint32_t type, const uint8_t* blob, const uint64_t* off,
                                              const uint32_t* len, uint64_t n, uint8_t* out,
                                              uint32_t* status_dev, hdx_stream stream) {
    const int c = index_code(type);
    if (c < 0) {
        if (type_code(type) < 0) return fail(HDX_E_BADTYPE, "unknown hyperdatatype %u", type);
        return fail(HDX_E_INVALID, "hyperdatatype %u has no fixed-size index key", type);
    }
    if (n == 0) return HDX_OK;
    if (!blob || !off || !len || !out) return fail(HDX_E_INVALID, "NULL device pointer");
    hdx_status st = bind_device(-1);
    if (st != HDX_OK) return st;
    IndexArgs a{};
    a.blob = blob;
    a.off = off;
    a.len = len;
    a.out = out;
    a.status = status_dev;
    a.n = n;
    a.code = (uint32_t)c;
    HIP_TRY(launch_index_encode(a, (hipStream_t)stream));
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_search_regions(hdx_region_table t, const hdx_range* ranges, uint32_t nranges,
                                         const uint8_t* has_replicas, uint8_t* include, int* cleared) {
    if (!t || !cleared || (nranges && !ranges) || (t->R && !include))
        return fail(HDX_E_INVALID, "NULL pointer");
    *cleared = 0;
    // configuration.cc:761-768: any invalid range clears the server list
    for (uint32_t k = 0; k < nranges; ++k)
        if (ranges[k].invalid) {
            *cleared = 1;
            if (t->R) std::memset(include, 0, t->R);
            return HDX_OK;
        }
    // :792-803 — the subspace dimension each range names; the rest `continue`
    SearchArgs a{};
    uint64_t ep_bytes = 0;
    const hdx_range* used[kMaxSearchRanges];
    for (uint32_t k = 0; k < nranges; ++k) {
        uint32_t l = UINT32_MAX;
        for (uint32_t d = 0; d < t->D; ++d)
            if (t->attrs[d] == ranges[k].attr) {
                l = d;
                break;
            }
        if (l == UINT32_MAX) continue;
        if (a.m == kMaxSearchRanges)
            return fail(HDX_E_INVALID, "more than %u ranges name subspace attributes", kMaxSearchRanges);
        const hdx_range& r = ranges[k];
        if ((r.has_start && !r.start && r.start_len) || (r.has_end && !r.end && r.end_len))
            return fail(HDX_E_INVALID, "range %u: NULL endpoint", k);
        uint8_t kind = SEARCH_NONE;
        if (r.type == 9217) {  // :817-829 — point query on a string
            if (r.has_start && r.has_end && r.start_len == r.end_len &&
                (r.start_len == 0 || std::memcmp(r.start, r.end, r.start_len) == 0))
                kind = SEARCH_STRING_EQ;
        } else if (r.type == 9218 || r.type == 9219) {  // :831-852
            kind = SEARCH_ORDERED;
            if ((r.has_start && r.start_len != 0 && r.start_len != 8) ||
                (r.has_end && r.end_len != 0 && r.end_len != 8))
                return fail(HDX_E_BADSIZE, "range %u: numeric endpoint not 0 or 8 bytes", k);
        }
        a.dim[a.m] = (uint8_t)l;
        a.kind[a.m] = kind;
        a.flags[a.m] = (r.has_start ? 1 : 0) | (r.has_end ? 2 : 0);
        used[a.m] = &r;
        if (kind == SEARCH_STRING_EQ) ep_bytes += r.start_len;
        if (kind == SEARCH_ORDERED) ep_bytes += (r.has_start ? r.start_len : 0) + (r.has_end ? r.end_len : 0);
        ++a.m;
    }
    if (t->R == 0) return HDX_OK;
    if (a.m == 0) {  // no range names this subspace: every region with replicas
        for (uint32_t r = 0; r < t->R; ++r) include[r] = has_replicas ? (has_replicas[r] != 0) : 1;
        return HDX_OK;
    }
    hdx_status st = bind_device(t->device);
    if (st != HDX_OK) return st;
    hipStream_t s;
    if ((st = thread_stream(&s)) != HDX_OK) return st;

    // staging layout (one object of 2m attributes: start_k, end_k)
    const uint32_t A = 2 * a.m;
    const size_t o_base = align_up(ep_bytes + 16, 16);
    const size_t o_len = o_base + 8;
    const size_t o_hash = align_up(o_len + 4 * A, 16);
    const size_t o_rep = o_hash + 8 * A;
    const size_t o_incl = align_up(o_rep + (has_replicas ? t->R : 0), 16);
    const size_t o_flag = align_up(o_incl + t->R, 16);
    const size_t need = o_flag + 16;
    SearchStage& g = t_search;
    if (g.cap < need) {
        (void)hipHostFree(g.host);
        (void)hipFree(g.dev);
        g.host = g.dev = nullptr;
        g.cap = 0;
        const size_t cap = std::max<size_t>(need, 64 << 10);
        if (hipHostMalloc((void**)&g.host, cap, hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void**)&g.dev, cap) != hipSuccess) {
            (void)hipGetLastError();
            return fail(HDX_E_NOMEM, "search staging of %zu bytes", cap);
        }
        g.cap = cap;
        g.device = t->device;
        if (!g.tracked) {
            track_scratch(&g);
            g.tracked = true;
        }
    }
    BatchArgs b{};
    uint64_t pos = 0;
    uint32_t* lens = reinterpret_cast<uint32_t*>(g.host + o_len);
    for (uint32_t k = 0; k < a.m; ++k) {
        const hdx_range& r = *used[k];
        uint64_t ls = 0, le = 0;
        uint8_t cs = CODE_ZERO, ce = CODE_ZERO;
        if (a.kind[k] == SEARCH_STRING_EQ) {
            ls = r.start_len;
            cs = CODE_STRING;
        } else if (a.kind[k] == SEARCH_ORDERED) {
            cs = ce = r.type == 9218 ? CODE_INT64 : CODE_FLOAT;
            ls = r.has_start ? r.start_len : 0;
            le = r.has_end ? r.end_len : 0;
        }
        if (ls) std::memcpy(g.host + pos, r.start, ls);
        if (le) std::memcpy(g.host + pos + ls, r.end, le);
        pos += ls + le;
        lens[2 * k] = (uint32_t)ls;
        lens[2 * k + 1] = (uint32_t)le;
        b.codes[2 * k] = cs;
        b.codes[2 * k + 1] = ce;
    }
    *reinterpret_cast<uint64_t*>(g.host + o_base) = 0;
    if (has_replicas) std::memcpy(g.host + o_rep, has_replicas, t->R);
    std::memset(g.host + o_flag, 0, 16);
    HIP_TRY(hipMemcpyAsync(g.dev, g.host, need, hipMemcpyHostToDevice, s));
    b.blob = g.dev;
    b.obj_base = reinterpret_cast<const uint64_t*>(g.dev + o_base);
    b.attr_len = reinterpret_cast<const uint32_t*>(g.dev + o_len);
    b.coords = reinterpret_cast<uint64_t*>(g.dev + o_hash);
    b.status = reinterpret_cast<uint32_t*>(g.dev + o_flag + 4);
    b.n = 1;
    b.A = A;
    finalize_args(b);
    HIP_TRY(launch_hash_batch(b, s));
    a.lower = t->d_lower;
    a.upper = t->d_upper;
    a.hashes = b.coords;
    a.include = g.dev + o_incl;
    a.replicas = has_replicas ? g.dev + o_rep : nullptr;
    a.cleared = reinterpret_cast<uint32_t*>(g.dev + o_flag);
    a.R = t->R;
    a.D = t->D;
    HIP_TRY(launch_search_regions(a, s));
    HIP_TRY(hipMemcpyAsync(g.host + o_incl, g.dev + o_incl, need - o_incl, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint32_t* flags = reinterpret_cast<const uint32_t*>(g.host + o_flag);
    if (flags[1]) return fail(HDX_E_BADSIZE, "numeric search endpoint not 0 or 8 bytes");
    if (flags[0]) {
        *cleared = 1;
        std::memset(include, 0, t->R);
        return HDX_OK;
    }
    std::memcpy(include, g.host + o_incl, t->R);
    return HDX_OK;
}

HDX_EXPORT hdx_status hdx_search_space(const hdx_region_table* tables, uint32_t ntables, const hdx_range* ranges,
                                       uint32_t nranges, const uint8_t* const* has_replicas, int32_t* chosen,
                                       uint8_t* include, uint32_t* servers, int* cleared) {
    if (!chosen || !servers || !cleared || (ntables && !tables) || (nranges && !ranges))
        return fail(HDX_E_INVALID, "NULL pointer");
    *chosen = -1;
    *servers = 0;
    *cleared = 0;
    uint32_t rmax = 0;
    for (uint32_t i = 0; i < ntables; ++i) {
        if (!tables[i]) return fail(HDX_E_INVALID, "table %u is NULL", i);
        rmax = std::max(rmax, tables[i]->R);
    }
    if (rmax && !include) return fail(HDX_E_INVALID, "NULL include");
    // configuration.cc:761-768: an invalid range clears the server list before
    // any subspace is looked at (so also with no subspaces at all)
    for (uint32_t k = 0; k < nranges; ++k) {
        if (ranges[k].invalid) {
            *cleared = 1;
            if (rmax) std::memset(include, 0, rmax);
            return HDX_OK;
        }
    }
    // configuration.cc:771-866: subspaces in order; the first initialises the
    // choice, a later one replaces it only if its server set is non-empty and
    // no larger (so the last of equal non-empty sizes wins); a cleared server
    // list (:766, :811) ends the whole search empty.
    std::vector<uint8_t> mask(rmax ? rmax : 1);
    bool initialized = false;
    uint32_t best = 0;
    for (uint32_t i = 0; i < ntables; ++i) {
        int cl = 0;
        hdx_status st = hdx_search_regions(tables[i], ranges, nranges, has_replicas ? has_replicas[i] : nullptr,
                                           mask.data(), &cl);
        if (st != HDX_OK) return st;
        if (cl) {
            *chosen = -1;
            *servers = 0;
            *cleared = 1;
            if (rmax) std::memset(include, 0, rmax);
            return HDX_OK;
        }
        uint32_t cnt = 0;
        for (uint32_t r = 0; r < tables[i]->R; ++r) cnt += mask[r] != 0;
        if (!initialized || (cnt != 0 && cnt <= best)) {
            initialized = true;
            best = cnt;
            *chosen = (int32_t)i;
            if (rmax) std::memset(include, 0, rmax);
            if (tables[i]->R) std::memcpy(include, mask.data(), tables[i]->R);
        }
    }
    *servers = best;
    return HDX_OK;
}
