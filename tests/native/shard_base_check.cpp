// shard_base (spt_internal.h): the segments of a sharded queue partition the
// producer's items exactly — segment j is as long as shard j's threads (blocks
// b = j, j + 8, ..., the last block short).  Host-only; tests/test_host.py builds it.
#include "spt_internal.h"
#include <cstdio>
int main() {
    using namespace spt;
    long bad = 0, cases = 0;
    for (uint32_t block : {64u, 128u, 512u})
        for (uint32_t items = 0; items < 20000; items += (items < 3000 ? 1 : 97)) {
            cases++;
            const uint32_t nb = (items + block - 1) / block;
            uint32_t cnt[kShards] = {};
            for (uint32_t b = 0; b < nb; b++) cnt[b % kShards] += (b + 1 == nb) ? items - b * block : block;
            uint32_t acc = 0;
            for (uint32_t j = 0; j <= kShards; j++) {
                if (shard_base(j, items, block) != acc) bad++;
                if (j < kShards) acc += cnt[j];
            }
        }
    std::printf("{\"cases\": %ld, \"bad\": %ld}\n", cases, bad);
    return bad ? 1 : 0;
}
