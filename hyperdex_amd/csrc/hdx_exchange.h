// hdx_exchange.h — the device set's gather as a host-only plan: which
// collectives run, and which rows of which device's matrix each one moves
// (hdx_multi.cpp issues the plan over RCCL; tests/cpp/sanitize_test.cc
// applies it to per-device matrices in host memory under ASan/UBSan).
//
// Shard k (k < world) holds counts[k] objects, rows [first_k, first_k +
// counts[k]) of an N-object matrix, N = the counts' total.  A matrix is
// `sections` blocks of `stride` u64 elements each (coordinates: one section
// of N * A elements, row = A; region ids: one section per table of N
// elements, row = 1).  Before the exchange device k holds only its own rows
// of every section; after it, every device holds every row.
//   * equal counts: one in-place all-gather per section (device k's rows are
//     its send buffer, at offset + k * count of the receive buffer);
//   * unequal counts: one in-place broadcast per non-empty shard and
//     section, rooted at the shard's device.
// No staging memory either way (hyperdex_amd/dist.py pads instead: torch has
// no grouped broadcast).  Host-only, no HIP.
#pragma once

#include <stdint.h>

#include <cstring>
#include <vector>

namespace hdx {

struct ExchangeOp {
    enum Kind : uint8_t { kAllGather = 0, kBroadcast = 1 } kind;
    uint32_t root;    // broadcast: the shard whose rows are sent
    uint64_t offset;  // first element of the op's region in every device's matrix
    uint64_t count;   // all-gather: elements per device; broadcast: elements
};

inline std::vector<ExchangeOp> exchange_plan(const uint64_t* counts, uint32_t world, uint64_t row,
                                             uint32_t sections, uint64_t stride) {
    std::vector<ExchangeOp> plan;
    uint64_t total = 0;
    bool equal = true;
    for (uint32_t k = 0; k < world; ++k) {
        total += counts[k];
        equal = equal && counts[k] == counts[0];
    }
    if (total == 0 || row == 0) return plan;
    for (uint32_t s = 0; s < sections; ++s) {
        if (equal) {
            plan.push_back({ExchangeOp::kAllGather, 0, s * stride, counts[0] * row});
            continue;
        }
        uint64_t first = 0;
        for (uint32_t k = 0; k < world; ++k) {
            if (counts[k]) plan.push_back({ExchangeOp::kBroadcast, k, s * stride + first * row, counts[k] * row});
            first += counts[k];
        }
    }
    return plan;
}

// Bytes one device receives over the fabric for this plan.
inline uint64_t exchange_bytes_in(const std::vector<ExchangeOp>& plan, uint32_t world, uint32_t k) {
    uint64_t b = 0;
    for (const ExchangeOp& op : plan)
        b += op.kind == ExchangeOp::kAllGather ? (uint64_t)(world - 1) * op.count * 8 : (op.root == k ? 0 : op.count * 8);
    return b;
}

// The plan's collectives with RCCL's in-place semantics, on host matrices
// (mats[k] = device k's matrix).  The test harness of the plan.
inline void exchange_apply(const std::vector<ExchangeOp>& plan, std::vector<std::vector<uint64_t>>& mats) {
    const uint32_t world = (uint32_t)mats.size();
    for (const ExchangeOp& op : plan) {
        if (op.kind == ExchangeOp::kAllGather) {
            // receive buffer [offset, offset + world * count); device r sends
            // its own block at offset + r * count
            std::vector<uint64_t> sent((size_t)world * op.count);
            for (uint32_t r = 0; r < world; ++r)
                std::memcpy(sent.data() + (size_t)r * op.count, mats[r].data() + op.offset + (size_t)r * op.count,
                            op.count * 8);
            for (uint32_t k = 0; k < world; ++k)
                std::memcpy(mats[k].data() + op.offset, sent.data(), sent.size() * 8);
        } else {
            const std::vector<uint64_t> src(mats[op.root].begin() + op.offset,
                                            mats[op.root].begin() + op.offset + op.count);
            for (uint32_t k = 0; k < world; ++k) std::memcpy(mats[k].data() + op.offset, src.data(), op.count * 8);
        }
    }
}

}  // namespace hdx
