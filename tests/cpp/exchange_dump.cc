// exchange_dump — the device set's exchange plan (hyperdex_amd/csrc/
// hdx_exchange.h) applied to per-device matrices in host memory, for
// tests/test_dist.py to compare with hyperdex_amd.dist.allgather_coords (the
// one-process-per-GPU path's padded / in-place gather) on the same shards.
//
//   exchange_dump OUT ROW COUNT0 [COUNT1 ...]
//
// The full matrix is N x ROW u64 with element e = mix64(e + 1) (synth.mix64);
// device k starts with only its own rows (the rest poisoned), the plan runs,
// and OUT receives the world matrices back to back (world x N x ROW u64).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "hdx_exchange.h"

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s OUT ROW COUNT0 [COUNT1 ...]\n", argv[0]);
        return 2;
    }
    const uint64_t row = strtoull(argv[2], nullptr, 10);
    const uint32_t world = (uint32_t)(argc - 3);
    std::vector<uint64_t> counts(world);
    uint64_t N = 0;
    for (uint32_t k = 0; k < world; ++k) N += counts[k] = strtoull(argv[3 + k], nullptr, 10);
    std::vector<std::vector<uint64_t>> mats(world, std::vector<uint64_t>(N * row, 0xdeadbeefdeadbeefull));
    uint64_t first = 0;
    for (uint32_t k = 0; k < world; ++k) {
        for (uint64_t e = first * row; e < (first + counts[k]) * row; ++e) mats[k][e] = mix64(e + 1);
        first += counts[k];
    }
    hdx::exchange_apply(hdx::exchange_plan(counts.data(), world, row, 1, N * row), mats);
    FILE* f = fopen(argv[1], "wb");
    if (!f) return 1;
    for (const auto& m : mats)
        if (!m.empty() && fwrite(m.data(), 8, m.size(), f) != m.size()) return 1;
    return fclose(f) == 0 ? 0 : 1;
}
