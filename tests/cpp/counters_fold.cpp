// counters_fold.cpp — the node-wide counter fold (cts_counters_read_multi, cts_host_util.cpp) over two and
// more engines, built with g++ against the link-time fakes of tests/cpp/engine_stub.cpp (a counter block is
// host memory with the device layout). Run under ASan/UBSan and TSan by tests/test_host_sanitizers.py.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "cts_engine.h"

#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                             \
        }                                                             \
    } while (0)

int main()
{
    // fake engine handles: the fold only passes them through to cts_counters_read
    std::vector<char> handles(8);
    for (uint32_t n : {1u, 2u, 8u}) {
        std::vector<std::vector<uint64_t>> blocks(n, std::vector<uint64_t>(CTS_COUNTER_SHARDS * 8, 0));
        std::vector<cts_engine*> eng(n);
        std::vector<const void*> ptrs(n);
        uint64_t want[5] = {0, 0, 0, 0, 0};
        for (uint32_t g = 0; g < n; ++g) {
            eng[g] = reinterpret_cast<cts_engine*>(&handles[g]);
            ptrs[g] = blocks[g].data();
            for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh)
                for (int k = 0; k < 8; ++k) {
                    // slots 5..7 of a shard are not counters and must not be folded in
                    const uint64_t v = (uint64_t)(g + 1) * 1000003ull * (sh + 1) + (uint64_t)k * 7919ull;
                    blocks[g][sh * 8 + k] = v;
                    if (k < 5) want[k] += v;
                }
        }
        cts_counters c{};
        CHECK(cts_counters_read_multi(eng.data(), ptrs.data(), nullptr, n, &c) == CTS_OK);
        CHECK(c.bytes_checked == want[0] && c.bytes_ok == want[1] && c.buffers_checked == want[2]);
        CHECK(c.buffers_failed == want[3] && c.mismatched_bytes == want[4]);
    }
    cts_counters c{};
    CHECK(cts_counters_read_multi(nullptr, nullptr, nullptr, 0, &c) == CTS_OK && c.bytes_checked == 0);
    CHECK(cts_counters_read_multi(nullptr, nullptr, nullptr, 1, &c) == CTS_E_INVALID);
    const void* nullblock[1] = {nullptr};
    cts_engine* e1[1] = {reinterpret_cast<cts_engine*>(&handles[0])};
    CHECK(cts_counters_read_multi(e1, nullblock, nullptr, 1, &c) == CTS_E_INVALID);
    CHECK(cts_counters_read_multi(e1, nullblock, nullptr, 1, nullptr) == CTS_E_INVALID);
    std::printf("counters_fold: ok\n");
    return 0;
}
