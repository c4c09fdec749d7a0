// hdx_hostpath.cpp — the host-resident entry points (include/hdxhash.h):
// batches and stored objects that arrive in host memory and whose outputs go
// back to host memory, as in the daemon: objects come from network buffers
// (daemon/key_state.cc:1455-1543 -> hyperdex::hash) and the reindex sweep
// reads LevelDB values on the host (daemon/datalayer_indexer_thread.cc:
// 161-176 -> datalayer::get_from_iterator -> decode_value,
// daemon/datalayer.cc:853-882).
//
// One device's pipeline (hash_host, hash_encoded_host) streams the call
// through its two slots in chunks of at most kChunkBytes: host validation of
// the chunk, H2D of its span(s) and rebased offsets, the kernel(s), D2H of the
// outputs — the two slots' streams overlap one chunk's copies with the
// other's kernel.  hdx_multi.cpp splits a call over the device set and runs
// one pipeline per device (hash_host_any / hash_encoded_host_any).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "hdx_host.h"

namespace hdx {

static constexpr uint64_t kChunkBytes = 128ull << 20;  // payload bytes per in-flight chunk
// A chunk packed on the device (hdx_gather.hip) grows to this: its two slots'
// kernels share one hardware queue, so each chunk pays ~0.5 ms of queue
// turnaround between its gather and the next (profiles/r6/host_order_trace.txt);
// larger chunks amortise it (device staging only: no pinned copy)
static constexpr uint64_t kPackChunkBytes = 512ull << 20;
// A call's first chunk: small, so the first copy starts after a few
// milliseconds less of host-side validation (later chunks are validated while
// the previous ones move)
static constexpr uint64_t kFirstChunkBytes = 16ull << 20;

void free_host_slot(HostSlot& s) {
    if (s.s) (void)hipStreamSynchronize(s.s);
    for (void* p : {(void*)s.d_blob.p, (void*)s.d_keys.p, (void*)s.d_base.p, (void*)s.d_coords.p, (void*)s.d_ids.p,
                    (void*)s.d_koff.p, (void*)s.d_voff.p, (void*)s.d_ver.p, (void*)s.d_len.p, (void*)s.d_klen.p,
                    (void*)s.d_vlen.p, (void*)s.d_status.p, (void*)s.d_src.p, (void*)s.d_src2.p, (void*)s.d_sz.p,
                    (void*)s.d_sz2.p})
        (void)hipFree(p);
    for (void* p : {(void*)s.h_blob.p, (void*)s.h_keys.p, (void*)s.h_base.p, (void*)s.h_coords.p, (void*)s.h_ids.p,
                    (void*)s.h_koff.p, (void*)s.h_voff.p, (void*)s.h_ver.p, (void*)s.h_len.p, (void*)s.h_klen.p,
                    (void*)s.h_vlen.p, (void*)s.h_status.p, (void*)s.h_src.p, (void*)s.h_src2.p, (void*)s.h_sz.p,
                    (void*)s.h_sz2.p})
        (void)hipHostFree(p);
    if (s.s) (void)hipStreamDestroy(s.s);
    s = HostSlot{};
}

static bool is_numeric_code(uint8_t c) { return c >= CODE_INT64; }

const uint8_t* device_view(const uint8_t* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return (const uint8_t*)a.devicePointer + (p - (const uint8_t*)a.hostPointer);
}

// A chunk whose objects' byte span is no more than this much over their
// payload goes as one span copy (no gather); otherwise its objects are packed
// in index order (hdx_gather.hip for pinned sources, a host copy per object
// for pageable ones), so a batch in any order moves only its own bytes.
static bool span_pays(uint64_t span, uint64_t payload) {
    return span <= kChunkBytes && span <= payload + payload / 8 + (64u << 10);
}

// In the pipelines' loops: a HIP error lets the copies in flight land first.
#define DRAIN_TRY(expr)                                          \
    do {                                                         \
        hipError_t e_ = (expr);                                  \
        if (e_ != hipSuccess) return drain(hip_fail(e_, #expr)); \
    } while (0)

namespace {

// One chunk in flight on a slot: where its outputs go once it lands.
struct Pending {
    bool live = false;
    uint64_t first = 0, cnt = 0;
};

// The outputs common to both pipelines: coordinates, region ids (staged
// through pinned memory when the caller's arrays are pageable).
struct Outputs {
    uint32_t A;
    uint64_t* coords;  // may be NULL
    bool coords_pinned;
    const HostRegions* R;  // may be NULL
    bool ids_pinned;
    uint64_t* versions = nullptr;  // stored objects only
    bool versions_pinned = false;

    uint32_t T() const { return R ? R->T : 0; }
    // D2H of a chunk's outputs on the slot's stream
    hdx_status copy_back(HostSlot& sl, uint64_t i, uint64_t cnt) const {
        hdx_status st;
        if (coords) {
            uint64_t* dst = coords + i * A;
            if (!coords_pinned) {
                if ((st = sl.h_coords.need(cnt * A)) != HDX_OK) return st;
                dst = sl.h_coords.p;
            }
            HIP_TRY(hipMemcpyAsync(dst, sl.d_coords.p, cnt * A * 8, hipMemcpyDeviceToHost, sl.s));
        }
        if (T()) {
            if (!ids_pinned && (st = sl.h_ids.need(cnt * T())) != HDX_OK) return st;
            for (uint32_t t = 0; t < T(); ++t) {
                uint64_t* dst = ids_pinned ? R->ids + t * R->stride + i : sl.h_ids.p + t * cnt;
                HIP_TRY(hipMemcpyAsync(dst, sl.d_ids.p + t * cnt, cnt * 8, hipMemcpyDeviceToHost, sl.s));
            }
        }
        if (versions) {
            uint64_t* dst = versions + i;
            if (!versions_pinned) {
                if ((st = sl.h_ver.need(cnt)) != HDX_OK) return st;
                dst = sl.h_ver.p;
            }
            HIP_TRY(hipMemcpyAsync(dst, sl.d_ver.p, cnt * 8, hipMemcpyDeviceToHost, sl.s));
        }
        return HDX_OK;
    }
    // after the slot's stream synchronised: the staged outputs into place
    void land(HostSlot& sl, uint64_t i, uint64_t cnt) const {
        if (coords && !coords_pinned) std::memcpy(coords + i * A, sl.h_coords.p, cnt * A * 8);
        if (T() && !ids_pinned)
            for (uint32_t t = 0; t < T(); ++t) std::memcpy(R->ids + t * R->stride + i, sl.h_ids.p + t * cnt, cnt * 8);
        if (versions && !versions_pinned) std::memcpy(versions + i, sl.h_ver.p, cnt * 8);
    }
};

}  // namespace

// ---- packed batches ---------------------------------------------------------------

hdx_status hash_host(const uint8_t* codes, uint32_t A, const uint8_t* blob, uint64_t blob_bytes,
                     const uint64_t* obj_base, const uint32_t* attr_len, uint64_t n, uint64_t* coords,
                     const HostRegions* R) {
    HostSlot* slots;
    hdx_status st = thread_slots(&slots);
    if (st != HDX_OK) return st;
    const int dev = thread_device();

    // Host-side validation (the reference asserts here) and the object's byte
    // extent, done chunk by chunk as the pipeline below reaches each object, so
    // the first copies start after one chunk's validation, not the batch's.
    auto extent = [&](uint64_t i, uint64_t* out) -> hdx_status {
        uint64_t s = 0;
        for (uint32_t j = 0; j < A; ++j) {
            const uint32_t L = attr_len[i * A + j];
            if (is_numeric_code(codes[j]) && L != 0 && L != 8)
                return fail(HDX_E_BADSIZE, "object %llu attribute %u: numeric value of %u bytes",
                            (unsigned long long)i, j, L);
            s += L;
        }
        if (s >= (1ull << 32))
            return fail(HDX_E_INVALID, "object %llu is %llu bytes (limit 4 GiB)", (unsigned long long)i,
                        (unsigned long long)s);
        if (obj_base[i] > blob_bytes || s > blob_bytes - obj_base[i])
            return fail(HDX_E_INVALID, "object %llu [%llu,+%llu) outside blob of %llu bytes", (unsigned long long)i,
                        (unsigned long long)obj_base[i], (unsigned long long)s, (unsigned long long)blob_bytes);
        *out = s;
        return HDX_OK;
    };

    const bool blob_pinned = is_pinned(blob);
    const bool len_pinned = is_pinned(attr_len);
    Outputs out{A, coords, coords && is_pinned(coords), R, R && R->T && is_pinned(R->ids)};
    const uint32_t T = out.T();

    Pending pend[2];
    auto finish = [&](int k) -> hdx_status {
        if (!pend[k].live) return HDX_OK;
        pend[k].live = false;
        HIP_TRY(hipStreamSynchronize(slots[k].s));
        out.land(slots[k], pend[k].first, pend[k].cnt);
        return HDX_OK;
    };
    auto drain = [&](hdx_status err) {  // an error: let every copy in flight land before returning
        for (int q = 0; q < 2; ++q) {
            (void)finish(q);
            (void)hipStreamSynchronize(slots[q].s);
        }
        return err;
    };

    const uint8_t* blob_dev = blob_pinned ? device_view(blob) : nullptr;  // the gather kernel's view
    std::vector<uint32_t> sizes;  // the chunk's object sizes (validated as the chunk grows)
    uint64_t i = 0, next_size = 0;
    int k = 0;
    if ((st = extent(0, &next_size)) != HDX_OK) return st;
    while (i < n) {
        // Grow the chunk while its payload stays under kChunkBytes (an object
        // that does not fit starts the next chunk; its extent is kept), then
        // move it as one span when its objects lie (nearly) back to back, else
        // packed in index order.
        uint64_t lo = obj_base[i], hi = obj_base[i] + next_size, payload = next_size, e = i + 1;
        sizes.assign(1, (uint32_t)next_size);
        uint64_t limit = i == 0 ? kFirstChunkBytes : kChunkBytes;
        while (e < n) {
            if ((st = extent(e, &next_size)) != HDX_OK) return drain(st);
            if (payload + next_size > limit) {
                // a chunk the device will pack grows further
                if (limit == kChunkBytes && blob_dev && !span_pays(hi - lo, payload)) limit = kPackChunkBytes;
                if (payload + next_size > limit) break;
            }
            lo = std::min(lo, obj_base[e]);
            hi = std::max(hi, obj_base[e] + next_size);
            payload += next_size;
            sizes.push_back((uint32_t)next_size);
            ++e;
        }
        const uint64_t cnt = e - i;
        const bool span = cnt == 1 || span_pays(hi - lo, payload);  // one object: its own bytes, however large
        const uint64_t bytes = span ? hi - lo : payload;
        HostSlot& sl = slots[k];
        if ((st = finish(k)) != HDX_OK) return drain(st);
        if ((st = sl.d_blob.need(std::max<uint64_t>(bytes, 1))) != HDX_OK || (st = sl.d_base.need(cnt)) != HDX_OK ||
            (st = sl.d_len.need(cnt * A)) != HDX_OK || (st = sl.d_coords.need(cnt * A)) != HDX_OK ||
            (T && (st = sl.d_ids.need(cnt * T)) != HDX_OK) || (st = sl.h_base.need(cnt)) != HDX_OK)
            return drain(st);
        const bool gather = !span && blob_dev;  // pinned objects out of order: packed on the device
        const uint8_t* src_blob = blob + lo;
        if (span) {
            for (uint64_t t = 0; t < cnt; ++t) sl.h_base.p[t] = obj_base[i + t] - lo;
            if (!blob_pinned) {
                if ((st = sl.h_blob.need(std::max<uint64_t>(bytes, 1))) != HDX_OK) return drain(st);
                std::memcpy(sl.h_blob.p, blob + lo, bytes);
                src_blob = sl.h_blob.p;
            }
        } else {
            uint64_t at = 0;  // packed offsets, index order
            for (uint64_t t = 0; t < cnt; ++t) {
                sl.h_base.p[t] = at;
                at += sizes[t];
            }
            if (gather) {
                if ((st = sl.h_src.need(cnt)) != HDX_OK || (st = sl.h_sz.need(cnt)) != HDX_OK ||
                    (st = sl.d_src.need(cnt)) != HDX_OK || (st = sl.d_sz.need(cnt)) != HDX_OK)
                    return drain(st);
                std::memcpy(sl.h_src.p, obj_base + i, cnt * 8);
                std::memcpy(sl.h_sz.p, sizes.data(), cnt * 4);
            } else {  // pageable: each object copied into the pinned staging
                if ((st = sl.h_blob.need(std::max<uint64_t>(bytes, 1))) != HDX_OK) return drain(st);
                for (uint64_t t = 0; t < cnt; ++t) std::memcpy(sl.h_blob.p + sl.h_base.p[t], blob + obj_base[i + t], sizes[t]);
                src_blob = sl.h_blob.p;
            }
        }
        const uint32_t* src_len = attr_len + i * A;
        if (!len_pinned) {
            if ((st = sl.h_len.need(cnt * A)) != HDX_OK) return drain(st);
            std::memcpy(sl.h_len.p, attr_len + i * A, cnt * A * sizeof(uint32_t));
            src_len = sl.h_len.p;
        }
        if (gather) {
            // every input of the chunk moved by the compute queue: the small
            // arrays by one copy kernel (pinned staging or the caller's pinned
            // lengths, through their device views), the objects by the gather
            const void* lsrc[4] = {device_view((const uint8_t*)sl.h_base.p), device_view((const uint8_t*)sl.h_src.p),
                                   device_view((const uint8_t*)sl.h_sz.p), device_view((const uint8_t*)src_len)};
            void* ldst[4] = {sl.d_base.p, sl.d_src.p, sl.d_sz.p, sl.d_len.p};
            const uint64_t lbytes[4] = {cnt * 8, cnt * 8, cnt * 4, cnt * A * 4};
            if (lsrc[0] && lsrc[1] && lsrc[2] && lsrc[3]) {
                DRAIN_TRY(launch_copy_linear(lsrc, ldst, lbytes, 4, sl.s));
            } else {
                DRAIN_TRY(hipMemcpyAsync(sl.d_base.p, sl.h_base.p, cnt * 8, hipMemcpyHostToDevice, sl.s));
                DRAIN_TRY(hipMemcpyAsync(sl.d_src.p, sl.h_src.p, cnt * 8, hipMemcpyHostToDevice, sl.s));
                DRAIN_TRY(hipMemcpyAsync(sl.d_sz.p, sl.h_sz.p, cnt * 4, hipMemcpyHostToDevice, sl.s));
                DRAIN_TRY(hipMemcpyAsync(sl.d_len.p, src_len, cnt * A * 4, hipMemcpyHostToDevice, sl.s));
            }
            DRAIN_TRY(launch_gather_extents(blob_dev, sl.d_src.p, sl.d_sz.p, sl.d_base.p, sl.d_blob.p, cnt, sl.s));
        } else {
            DRAIN_TRY(hipMemcpyAsync(sl.d_base.p, sl.h_base.p, cnt * 8, hipMemcpyHostToDevice, sl.s));
            DRAIN_TRY(hipMemcpyAsync(sl.d_len.p, src_len, cnt * A * 4, hipMemcpyHostToDevice, sl.s));
            DRAIN_TRY(hipMemcpyAsync(sl.d_blob.p, src_blob, bytes, hipMemcpyHostToDevice, sl.s));
        }
        BatchArgs args;
        // status: none (sizes validated above); the coordinates always land in
        // device staging, so the regions form needs no scratch of its own
        if ((st = batch_args(args, codes, A, sl.d_blob.p, sl.d_base.p, sl.d_len.p, cnt, sl.d_coords.p, nullptr,
                             R ? R->tables : nullptr, T, sl.d_ids.p, cnt, dev)) != HDX_OK)
            return drain(st);
        if (T) {
            const hipError_t e2 = launch_hash_batch_regions(args, sl.s);
            if (e2 != hipSuccess) return drain(hip_fail(e2, "launch_hash_batch_regions"));
        } else {
            const hipError_t e2 = launch_hash_batch(args, sl.s);
            if (e2 != hipSuccess) return drain(hip_fail(e2, "launch_hash_batch"));
        }
        if ((st = out.copy_back(sl, i, cnt)) != HDX_OK) return drain(st);
        pend[k] = {true, i, cnt};
        i = e;
        k ^= 1;
    }
    if ((st = finish(k)) != HDX_OK) return drain(st);
    return finish(k ^ 1);
}

// ---- stored objects (the reindex sweep from host memory) ----------------------------

hdx_status hash_encoded_host(const uint8_t* codes, uint32_t A, const uint8_t* keys, uint64_t keys_bytes,
                             const uint64_t* key_off, const uint32_t* key_len, const uint8_t* vals,
                             uint64_t vals_bytes, const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                             uint64_t* coords, uint64_t* versions, const HostRegions* R, uint32_t* status_bits) {
    *status_bits = 0;
    HostSlot* slots;
    hdx_status st = thread_slots(&slots);
    if (st != HDX_OK) return st;
    const int dev = thread_device();
    // records [key][value] in one store (keys == vals, a LevelDB block's
    // adjacency): one span per chunk, and the kernel sees keys == vals
    const bool records = keys == vals;

    auto check = [&](uint64_t i) -> hdx_status {
        const uint32_t kl = key_len[i];
        if (is_numeric_code(codes[0]) && kl != 0 && kl != 8)
            return fail(HDX_E_BADSIZE, "object %llu: numeric key of %u bytes", (unsigned long long)i, kl);
        if (key_off[i] > keys_bytes || kl > keys_bytes - key_off[i])
            return fail(HDX_E_INVALID, "object %llu: key [%llu,+%u) outside keys of %llu bytes", (unsigned long long)i,
                        (unsigned long long)key_off[i], kl, (unsigned long long)keys_bytes);
        if (val_off[i] > vals_bytes || val_len[i] > vals_bytes - val_off[i])
            return fail(HDX_E_INVALID, "object %llu: value [%llu,+%u) outside values of %llu bytes",
                        (unsigned long long)i, (unsigned long long)val_off[i], val_len[i],
                        (unsigned long long)vals_bytes);
        return HDX_OK;
    };

    const bool keys_pinned = is_pinned(keys), vals_pinned = is_pinned(vals);
    const bool klen_pinned = is_pinned(key_len), vlen_pinned = is_pinned(val_len);
    Outputs out{A, coords, coords && is_pinned(coords), R, R && R->T && is_pinned(R->ids)};
    out.versions = versions;
    out.versions_pinned = versions && is_pinned(versions);
    const uint32_t T = out.T();

    Pending pend[2];
    auto finish = [&](int k) -> hdx_status {
        if (!pend[k].live) return HDX_OK;
        pend[k].live = false;
        HIP_TRY(hipStreamSynchronize(slots[k].s));
        out.land(slots[k], pend[k].first, pend[k].cnt);
        *status_bits |= *slots[k].h_status.p;
        return HDX_OK;
    };
    auto drain = [&](hdx_status err) {  // an error: let every copy in flight land before returning
        for (int q = 0; q < 2; ++q) {
            (void)finish(q);
            (void)hipStreamSynchronize(slots[q].s);
        }
        return err;
    };
    // a span's host source: the caller's pinned bytes, or a pinned copy
    auto stage = [&](PinBuf<uint8_t>& buf, const uint8_t* base, bool pinned, uint64_t lo, uint64_t bytes,
                     const uint8_t** src) -> hdx_status {
        if (pinned) {
            *src = base + lo;
            return HDX_OK;
        }
        hdx_status s2 = buf.need(std::max<uint64_t>(bytes, 1));
        if (s2 != HDX_OK) return s2;
        std::memcpy(buf.p, base + lo, bytes);
        *src = buf.p;
        return HDX_OK;
    };

    // keys and values out of order: packed as records [key][value] in index
    // order (hdx_gather.hip from pinned stores, a host copy per object from
    // pageable ones), so the kernel sees the record layout
    const uint8_t* keys_dev = keys_pinned ? device_view(keys) : nullptr;
    const uint8_t* vals_dev = vals_pinned ? device_view(vals) : nullptr;
    uint64_t i = 0;
    int k = 0;
    if ((st = check(0)) != HDX_OK) return st;
    while (i < n) {
        uint64_t klo = key_off[i], khi = key_off[i] + key_len[i];
        uint64_t vlo = val_off[i], vhi = val_off[i] + val_len[i];
        uint64_t payload = (uint64_t)key_len[i] + val_len[i];
        if (records) {
            klo = vlo = std::min(klo, vlo);
            khi = vhi = std::max(khi, vhi);
        }
        auto span_bytes = [&](uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
            return records ? d - c : (b - a) + (d - c);
        };
        uint64_t e = i + 1;
        uint64_t limit = i == 0 ? kFirstChunkBytes : kChunkBytes;
        while (e < n) {
            if ((st = check(e)) != HDX_OK) return drain(st);
            const uint64_t pe = (uint64_t)key_len[e] + val_len[e];
            if (payload + pe > limit) {
                if (limit == kChunkBytes && keys_dev && vals_dev && !span_pays(span_bytes(klo, khi, vlo, vhi), payload))
                    limit = kPackChunkBytes;  // packed on the device: larger chunks
                if (payload + pe > limit) break;
            }
            uint64_t nklo = std::min(klo, key_off[e]), nkhi = std::max(khi, key_off[e] + key_len[e]);
            uint64_t nvlo = std::min(vlo, val_off[e]), nvhi = std::max(vhi, val_off[e] + val_len[e]);
            if (records) {
                nklo = nvlo = std::min(nklo, nvlo);
                nkhi = nvhi = std::max(nkhi, nvhi);
            }
            klo = nklo; khi = nkhi; vlo = nvlo; vhi = nvhi;
            payload += pe;
            ++e;
        }
        const uint64_t cnt = e - i;
        // one object whose spans hold nothing else moves as spans, however large
        const bool span = span_pays(span_bytes(klo, khi, vlo, vhi), payload) ||
                          (cnt == 1 && span_bytes(klo, khi, vlo, vhi) == payload);
        const bool gather = !span && keys_dev && vals_dev;
        const bool packed = !span;  // the chunk's device layout is then records
        HostSlot& sl = slots[k];
        if ((st = finish(k)) != HDX_OK) return drain(st);
        if ((st = sl.d_blob.need(std::max<uint64_t>(span ? vhi - vlo : payload, 1))) != HDX_OK ||
            (span && !records && (st = sl.d_keys.need(std::max<uint64_t>(khi - klo, 1))) != HDX_OK) ||
            (st = sl.d_koff.need(cnt)) != HDX_OK || (st = sl.d_voff.need(cnt)) != HDX_OK ||
            (st = sl.d_klen.need(cnt)) != HDX_OK || (st = sl.d_vlen.need(cnt)) != HDX_OK ||
            (st = sl.d_coords.need(cnt * A)) != HDX_OK || (st = sl.d_ver.need(cnt)) != HDX_OK ||
            (st = sl.d_status.need(1)) != HDX_OK || (st = sl.h_status.need(1)) != HDX_OK ||
            (T && (st = sl.d_ids.need(cnt * T)) != HDX_OK) || (st = sl.h_koff.need(cnt)) != HDX_OK ||
            (st = sl.h_voff.need(cnt)) != HDX_OK)
            return drain(st);
        const uint8_t *src_vals = nullptr, *src_keys = nullptr;
        if (span) {
            for (uint64_t t = 0; t < cnt; ++t) {
                sl.h_koff.p[t] = key_off[i + t] - klo;
                sl.h_voff.p[t] = val_off[i + t] - vlo;
            }
            if ((st = stage(sl.h_blob, vals, vals_pinned, vlo, vhi - vlo, &src_vals)) != HDX_OK) return drain(st);
            if (!records && (st = stage(sl.h_keys, keys, keys_pinned, klo, khi - klo, &src_keys)) != HDX_OK)
                return drain(st);
        } else {
            uint64_t at = 0;  // record t: its key at h_koff, its value right after
            for (uint64_t t = 0; t < cnt; ++t) {
                sl.h_koff.p[t] = at;
                sl.h_voff.p[t] = at + key_len[i + t];
                at += (uint64_t)key_len[i + t] + val_len[i + t];
            }
            if (gather) {  // 2 extents per object, absolute device-view sources
                if ((st = sl.h_src.need(2 * cnt)) != HDX_OK || (st = sl.h_sz.need(2 * cnt)) != HDX_OK ||
                    (st = sl.h_src2.need(2 * cnt)) != HDX_OK || (st = sl.d_src.need(2 * cnt)) != HDX_OK ||
                    (st = sl.d_sz.need(2 * cnt)) != HDX_OK || (st = sl.d_src2.need(2 * cnt)) != HDX_OK)
                    return drain(st);
                for (uint64_t t = 0; t < cnt; ++t) {
                    sl.h_src.p[2 * t] = (uint64_t)(uintptr_t)keys_dev + key_off[i + t];
                    sl.h_sz.p[2 * t] = key_len[i + t];
                    sl.h_src2.p[2 * t] = sl.h_koff.p[t];
                    sl.h_src.p[2 * t + 1] = (uint64_t)(uintptr_t)vals_dev + val_off[i + t];
                    sl.h_sz.p[2 * t + 1] = val_len[i + t];
                    sl.h_src2.p[2 * t + 1] = sl.h_voff.p[t];
                }
            } else {  // pageable: each key and value copied into the pinned staging
                if ((st = sl.h_blob.need(std::max<uint64_t>(payload, 1))) != HDX_OK) return drain(st);
                for (uint64_t t = 0; t < cnt; ++t) {
                    std::memcpy(sl.h_blob.p + sl.h_koff.p[t], keys + key_off[i + t], key_len[i + t]);
                    std::memcpy(sl.h_blob.p + sl.h_voff.p[t], vals + val_off[i + t], val_len[i + t]);
                }
                src_vals = sl.h_blob.p;
            }
        }
        const uint32_t* src_klen = key_len + i;
        const uint32_t* src_vlen = val_len + i;
        if (!klen_pinned) {
            if ((st = sl.h_klen.need(cnt)) != HDX_OK) return drain(st);
            std::memcpy(sl.h_klen.p, key_len + i, cnt * 4);
            src_klen = sl.h_klen.p;
        }
        if (!vlen_pinned) {
            if ((st = sl.h_vlen.need(cnt)) != HDX_OK) return drain(st);
            std::memcpy(sl.h_vlen.p, val_len + i, cnt * 4);
            src_vlen = sl.h_vlen.p;
        }
        const void* lsrc[7] = {device_view((const uint8_t*)sl.h_koff.p), device_view((const uint8_t*)sl.h_voff.p),
                               device_view((const uint8_t*)src_klen), device_view((const uint8_t*)src_vlen),
                               gather ? device_view((const uint8_t*)sl.h_src.p) : nullptr,
                               gather ? device_view((const uint8_t*)sl.h_sz.p) : nullptr,
                               gather ? device_view((const uint8_t*)sl.h_src2.p) : nullptr};
        if (gather && lsrc[0] && lsrc[1] && lsrc[2] && lsrc[3] && lsrc[4] && lsrc[5] && lsrc[6]) {
            // every input of the chunk moved by the compute queue (one copy
            // kernel, then the gather): no SDMA copy for the gather to wait on
            void* ldst[7] = {sl.d_koff.p, sl.d_voff.p, sl.d_klen.p, sl.d_vlen.p, sl.d_src.p, sl.d_sz.p, sl.d_src2.p};
            const uint64_t lbytes[7] = {cnt * 8, cnt * 8, cnt * 4, cnt * 4, 2 * cnt * 8, 2 * cnt * 4, 2 * cnt * 8};
            DRAIN_TRY(launch_copy_linear(lsrc, ldst, lbytes, 7, sl.s));
        } else {
            DRAIN_TRY(hipMemcpyAsync(sl.d_koff.p, sl.h_koff.p, cnt * 8, hipMemcpyHostToDevice, sl.s));
            DRAIN_TRY(hipMemcpyAsync(sl.d_voff.p, sl.h_voff.p, cnt * 8, hipMemcpyHostToDevice, sl.s));
            DRAIN_TRY(hipMemcpyAsync(sl.d_klen.p, src_klen, cnt * 4, hipMemcpyHostToDevice, sl.s));
            DRAIN_TRY(hipMemcpyAsync(sl.d_vlen.p, src_vlen, cnt * 4, hipMemcpyHostToDevice, sl.s));
            if (gather) {
                DRAIN_TRY(hipMemcpyAsync(sl.d_src.p, sl.h_src.p, 2 * cnt * 8, hipMemcpyHostToDevice, sl.s));
                DRAIN_TRY(hipMemcpyAsync(sl.d_sz.p, sl.h_sz.p, 2 * cnt * 4, hipMemcpyHostToDevice, sl.s));
                DRAIN_TRY(hipMemcpyAsync(sl.d_src2.p, sl.h_src2.p, 2 * cnt * 8, hipMemcpyHostToDevice, sl.s));
            }
        }
        if (gather) {
            DRAIN_TRY(launch_gather_extents(nullptr, sl.d_src.p, sl.d_sz.p, sl.d_src2.p, sl.d_blob.p, 2 * cnt, sl.s));
        } else {
            DRAIN_TRY(hipMemcpyAsync(sl.d_blob.p, src_vals, span ? vhi - vlo : payload, hipMemcpyHostToDevice, sl.s));
            if (span && !records)
                DRAIN_TRY(hipMemcpyAsync(sl.d_keys.p, src_keys, khi - klo, hipMemcpyHostToDevice, sl.s));
        }
        DRAIN_TRY(hipMemsetAsync(sl.d_status.p, 0, 4, sl.s));
        EncodedArgs a{};
        if ((st = set_codes(a, codes, A)) != HDX_OK) return drain(st);
        a.keys = records || packed ? sl.d_blob.p : sl.d_keys.p;
        a.key_off = sl.d_koff.p;
        a.key_len = sl.d_klen.p;
        a.vals = sl.d_blob.p;
        a.val_off = sl.d_voff.p;
        a.val_len = sl.d_vlen.p;
        a.coords = sl.d_coords.p;  // always staged: no scratch for the regions form
        a.versions = sl.d_ver.p;
        a.status = sl.d_status.p;
        a.n = cnt;
        a.A = A;
        a.T = T;
        for (uint32_t t = 0; t < T; ++t)
            if ((st = fill_sweep_table(a.t[t], R->tables[t], dev, sl.d_ids.p + t * cnt)) != HDX_OK) return drain(st);
        const hipError_t e2 = launch_hash_encoded(a, sl.s);
        if (e2 != hipSuccess) return drain(hip_fail(e2, "launch_hash_encoded"));
        if ((st = out.copy_back(sl, i, cnt)) != HDX_OK) return drain(st);
        DRAIN_TRY(hipMemcpyAsync(sl.h_status.p, sl.d_status.p, 4, hipMemcpyDeviceToHost, sl.s));
        pend[k] = {true, i, cnt};
        i = e;
        k ^= 1;
    }
    if ((st = finish(k)) != HDX_OK) return drain(st);
    return finish(k ^ 1);
}

}  // namespace hdx

using namespace hdx;

// ---- exported -----------------------------------------------------------------------

static const uint8_t g_empty = 0;  // a blob / store of 0 bytes

HDX_EXPORT hdx_status hdx_hash_batch_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* blob,
                                          uint64_t blob_bytes, const uint64_t* obj_base, const uint32_t* attr_len,
                                          uint64_t n, uint64_t* coords) {
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    hdx_status st = check_schema(types, attrs_sz, codes.data());
    if (st != HDX_OK) return st;
    if (n == 0) return HDX_OK;
    if (!obj_base || !attr_len || !coords || (!blob && blob_bytes)) return fail(HDX_E_INVALID, "NULL host pointer");
    return hash_host_any(codes.data(), attrs_sz, blob ? blob : &g_empty, blob_bytes, obj_base, attr_len, n, coords,
                         nullptr);
}

HDX_EXPORT hdx_status hdx_hash_batch_regions_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* blob,
                                                  uint64_t blob_bytes, const uint64_t* obj_base,
                                                  const uint32_t* attr_len, uint64_t n, const hdx_region_table* tables,
                                                  uint32_t ntables, uint64_t* region_ids, uint64_t* coords) {
    if (ntables == 0) return fail(HDX_E_INVALID, "no region tables");
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    hdx_status st = check_schema(types, attrs_sz, codes.data());
    if (st != HDX_OK) return st;
    if ((st = check_tables(tables, ntables, attrs_sz, region_ids)) != HDX_OK) return st;
    if (n == 0) return HDX_OK;
    if (!obj_base || !attr_len || (!blob && blob_bytes)) return fail(HDX_E_INVALID, "NULL host pointer");
    const HostRegions R{tables, ntables, region_ids, n};
    return hash_host_any(codes.data(), attrs_sz, blob ? blob : &g_empty, blob_bytes, obj_base, attr_len, n, coords,
                         &R);
}

static hdx_status encoded_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* keys, uint64_t keys_bytes,
                               const uint64_t* key_off, const uint32_t* key_len, const uint8_t* vals,
                               uint64_t vals_bytes, const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                               const hdx_region_table* tables, uint32_t ntables, uint64_t* region_ids,
                               uint64_t* coords, uint64_t* versions) {
    std::vector<uint8_t> codes(attrs_sz ? attrs_sz : 1);
    hdx_status st = check_schema(types, attrs_sz, codes.data());
    if (st != HDX_OK) return st;
    if ((st = check_tables(tables, ntables, attrs_sz, region_ids)) != HDX_OK) return st;
    if (n == 0) return HDX_OK;
    if (!key_off || !key_len || !val_off || !val_len || (!coords && !ntables) || (!keys && keys_bytes) ||
        (!vals && vals_bytes))
        return fail(HDX_E_INVALID, "NULL host pointer");
    const HostRegions R{tables, ntables, region_ids, n};
    return hash_encoded_host_any(codes.data(), attrs_sz, keys ? keys : &g_empty, keys_bytes, key_off, key_len,
                                 vals ? vals : &g_empty, vals_bytes, val_off, val_len, n, coords, versions,
                                 ntables ? &R : nullptr);
}

HDX_EXPORT hdx_status hdx_hash_encoded_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* keys,
                                            uint64_t keys_bytes, const uint64_t* key_off, const uint32_t* key_len,
                                            const uint8_t* vals, uint64_t vals_bytes, const uint64_t* val_off,
                                            const uint32_t* val_len, uint64_t n, uint64_t* coords,
                                            uint64_t* versions) {
    return encoded_host(types, attrs_sz, keys, keys_bytes, key_off, key_len, vals, vals_bytes, val_off, val_len, n,
                        nullptr, 0, nullptr, coords, versions);
}

HDX_EXPORT hdx_status hdx_hash_encoded_regions_host(const uint32_t* types, uint32_t attrs_sz, const uint8_t* keys,
                                                    uint64_t keys_bytes, const uint64_t* key_off,
                                                    const uint32_t* key_len, const uint8_t* vals, uint64_t vals_bytes,
                                                    const uint64_t* val_off, const uint32_t* val_len, uint64_t n,
                                                    const hdx_region_table* tables, uint32_t ntables,
                                                    uint64_t* region_ids, uint64_t* coords, uint64_t* versions) {
    if (ntables == 0) return fail(HDX_E_INVALID, "no region tables");
    return encoded_host(types, attrs_sz, keys, keys_bytes, key_off, key_len, vals, vals_bytes, val_off, val_len, n,
                        tables, ntables, region_ids, coords, versions);
}
