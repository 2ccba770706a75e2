// counters_fold.cpp — the node-wide counters of one process's engines, both ways:
//   cts_counters_read_multi (cts_host_util.cpp): each block read and summed on the host;
//   cts_counters_allreduce (cts_collective.cpp): each block folded on its device, then an RCCL all-reduce.
// Built with g++ against the link-time fakes of tests/cpp/engine_stub.cpp, with a working fake device here (host
// memory stands in for device memory, a thread-local current device, the fold done on the host) and a stub RCCL
// (tests/cpp/rccl_stub.cpp) that the collective loads through $CTS_RCCL_LIBRARY. Run under ASan/UBSan and TSan by
// tests/test_host_sanitizers.py.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "cts_engine.h"
#include "cts_internal.hpp"

#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                             \
        }                                                             \
    } while (0)

// ---- the fake device ------------------------------------------------------------------------------------
namespace {
constexpr int kDevices = 8;
thread_local int t_cur = 0;
std::mutex g_mu;
std::map<const void*, int> g_alloc_dev;  // fake device allocations -> their device
char g_handles[64];                      // fake engine handles
int g_dev_of[64];                        // engine handle i -> its device
int g_folds = 0;
int g_syncs = 0;
}  // namespace

extern "C" {
hipError_t hipGetDevice(int* d)
{
    *d = t_cur;
    return hipSuccess;
}
hipError_t hipSetDevice(int d)
{
    if (d < 0 || d >= kDevices) return hipErrorInvalidDevice;
    t_cur = d;
    return hipSuccess;
}
// the clique's slots are stream-ordered on the device's null stream (a plain hipFree would synchronize the device)
hipError_t hipMallocAsync(void** p, size_t bytes, hipStream_t s)
{
    if (s != nullptr) return hipErrorInvalidValue;
    *p = std::calloc(1, bytes);
    std::lock_guard<std::mutex> lk(g_mu);
    g_alloc_dev[*p] = t_cur;
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFreeAsync(void* p, hipStream_t s)
{
    if (s != nullptr) return hipErrorInvalidValue;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_alloc_dev.find(p);
        if (it == g_alloc_dev.end() || it->second != t_cur) return hipErrorInvalidValue;  // freed on its device
        g_alloc_dev.erase(it);
    }
    std::free(p);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void* dst, int v, size_t bytes, hipStream_t)
{
    std::memset(dst, v, bytes);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind, hipStream_t)
{
    std::memcpy(dst, src, bytes);
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t)
{
    std::lock_guard<std::mutex> lk(g_mu);
    ++g_syncs;
    return hipSuccess;
}
int cts_engine_device(const cts_engine* e)
{
    const char* h = reinterpret_cast<const char*>(e);
    if (h < g_handles || h >= g_handles + 64) return CTS_E_INVALID;
    return g_dev_of[h - g_handles];
}
}  // extern "C"

namespace cts {
hipError_t launch_counters_fold(const void* block, uint64_t* out, bool accumulate, hipStream_t)
{
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_alloc_dev.find(out);
        if (it == g_alloc_dev.end() || it->second != t_cur) return hipErrorInvalidValue;  // launched on its device
        ++g_folds;
    }
    const uint64_t* h = static_cast<const uint64_t*>(block);
    for (int k = 0; k < kCounterCount; ++k) {
        uint64_t s = accumulate ? out[k] : 0;
        for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh) s += h[sh * kCounterSlots + k];
        out[k] = s;
    }
    return hipSuccess;
}
}  // namespace cts

// ---- the test ---------------------------------------------------------------------------------------------
struct Node {
    std::vector<std::vector<uint64_t>> blocks;
    std::vector<cts_engine*> eng;
    std::vector<const void*> ptrs;
    uint64_t want[cts::kCounterCount] = {};
};

// n engines, engine g on device dev(g); block values distinct per engine, shard and slot
template <typename DevOf>
Node make_node(uint32_t n, DevOf dev)
{
    Node x;
    x.blocks.assign(n, std::vector<uint64_t>(CTS_COUNTER_SHARDS * 8, 0));
    for (uint32_t g = 0; g < n; ++g) {
        g_dev_of[g] = dev(g);
        x.eng.push_back(reinterpret_cast<cts_engine*>(&g_handles[g]));
        x.ptrs.push_back(x.blocks[g].data());
        for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh)
            for (int k = 0; k < 8; ++k) {
                // slots kCounterCount..7 of a shard are not counters and must not be folded in
                const uint64_t v = (uint64_t)(g + 1) * 1000003ull * (sh + 1) + (uint64_t)k * 7919ull;
                x.blocks[g][sh * 8 + k] = v;
                if (k < cts::kCounterCount) x.want[k] += v;
            }
    }
    return x;
}

bool equal(const cts_counters& c, const uint64_t* w)
{
    return c.bytes_checked == w[0] && c.bytes_ok == w[1] && c.buffers_checked == w[2] && c.buffers_failed == w[3] &&
           c.mismatched_bytes == w[4];
}
bool equal(const cts_counters_ex& c, const uint64_t* w)
{
    return c.bytes_checked == w[0] && c.bytes_ok == w[1] && c.buffers_checked == w[2] && c.buffers_failed == w[3] &&
           c.mismatched_bytes == w[4] && c.connections_failed == w[5];
}

int main(int argc, char** argv)
{
    // 1. the host fold
    for (uint32_t n : {1u, 2u, 8u}) {
        Node x = make_node(n, [](uint32_t g) { return (int)g; });
        cts_counters c{};
        CHECK(cts_counters_read_multi(x.eng.data(), x.ptrs.data(), nullptr, n, &c) == CTS_OK);
        CHECK(equal(c, x.want));
    }
    cts_counters c{};
    CHECK(cts_counters_read_multi(nullptr, nullptr, nullptr, 0, &c) == CTS_OK && c.bytes_checked == 0);
    CHECK(cts_counters_read_multi(nullptr, nullptr, nullptr, 1, &c) == CTS_E_INVALID);
    const void* nullblock[1] = {nullptr};
    cts_engine* e1[1] = {reinterpret_cast<cts_engine*>(&g_handles[0])};
    CHECK(cts_counters_read_multi(e1, nullblock, nullptr, 1, &c) == CTS_E_INVALID);
    CHECK(cts_counters_read_multi(e1, nullblock, nullptr, 1, nullptr) == CTS_E_INVALID);

    // 2. the all-reduce: argument checks need no RCCL
    CHECK(argc == 2);  // the stub RCCL library
    CHECK(cts_counters_allreduce(nullptr, nullptr, nullptr, 0, nullptr) == CTS_E_INVALID);
    c.bytes_checked = 7;
    CHECK(cts_counters_allreduce(nullptr, nullptr, nullptr, 0, &c) == CTS_OK && c.bytes_checked == 0);
    CHECK(cts_counters_allreduce(nullptr, nullptr, nullptr, 1, &c) == CTS_E_INVALID);
    CHECK(cts_counters_allreduce(e1, nullblock, nullptr, 1, &c) == CTS_E_INVALID);
    cts_engine* bogus[1] = {reinterpret_cast<cts_engine*>(&c)};  // cts_engine_device < 0
    const void* oneblock[1] = {&c};
    CHECK(cts_counters_allreduce(bogus, oneblock, nullptr, 1, &c) == CTS_E_INVALID);
    // no RCCL to load: unavailable, and nothing was cached
    setenv("CTS_RCCL_LIBRARY", "/nonexistent/librccl.so.1", 1);
    {
        Node x = make_node(2, [](uint32_t g) { return (int)g; });
        CHECK(cts_counters_allreduce(x.eng.data(), x.ptrs.data(), nullptr, 2, &c) == CTS_E_UNAVAILABLE);
    }
    setenv("CTS_RCCL_LIBRARY", argv[1], 1);
    void* stub = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);  // the same handle the collective gets
    CHECK(stub != nullptr);
    auto live = reinterpret_cast<int (*)()>(dlsym(stub, "stub_rccl_live_comms"));
    CHECK(live != nullptr);
    // communicator creation failing: an error, and the next call tries again
    setenv("STUB_RCCL_FAIL_INIT", "1", 1);
    {
        Node x = make_node(2, [](uint32_t g) { return (int)g; });
        CHECK(cts_counters_allreduce(x.eng.data(), x.ptrs.data(), nullptr, 2, &c) == CTS_E_HIP);
        CHECK(live() == 0);
    }
    unsetenv("STUB_RCCL_FAIL_INIT");
    // one engine per device, several engines per device (one rank per distinct device), every device set twice
    // (the second call reuses the cached clique)
    struct Case {
        uint32_t n;
        int per_dev;  // engines per device
    } cases[] = {{1, 1}, {2, 1}, {8, 1}, {2, 2}, {8, 2}, {16, 2}, {3, 3}, {8, 8}};
    int comms_expected = 0;
    for (const Case& k : cases) {
        Node x = make_node(k.n, [&](uint32_t g) { return (int)(g / (uint32_t)k.per_dev) % kDevices; });
        const int ndev = (int)((k.n + k.per_dev - 1) / k.per_dev);
        for (int rep = 0; rep < 2; ++rep) {
            t_cur = 3;
            const int folds0 = g_folds, live0 = live();
            cts_counters a{};
            CHECK(cts_counters_allreduce(x.eng.data(), x.ptrs.data(), nullptr, k.n, &a) == CTS_OK);
            CHECK(equal(a, x.want));
            CHECK(t_cur == 3);                          // the caller's current device is restored
            // every block folded once, on its own device, plus one dry-run fold per device of a new clique
            CHECK(g_folds - folds0 == (int)k.n + (live() - live0));
            cts_counters h{};
            CHECK(cts_counters_read_multi(x.eng.data(), x.ptrs.data(), nullptr, k.n, &h) == CTS_OK);
            CHECK(std::memcmp(&a, &h, sizeof(a)) == 0);  // the two ways agree
        }
        (void)ndev;
    }
    // distinct device sets so far: {0}, {0,1}, {0..7}, {0..3}, {0..7} again, {0} (3 on one device), {0}
    comms_expected = 1 + 2 + 8 + 4;
    CHECK(live() == comms_expected);
    // per-engine streams: engines sharing a device on other streams are synchronised before the fold
    {
        Node x = make_node(4, [](uint32_t g) { return (int)(g / 2); });
        int s_tokens[4];
        void* streams[4] = {&s_tokens[0], &s_tokens[1], &s_tokens[2], &s_tokens[3]};
        const int syncs0 = g_syncs;
        cts_counters a{};
        CHECK(cts_counters_allreduce(x.eng.data(), x.ptrs.data(), streams, 4, &a) == CTS_OK && equal(a, x.want));
        CHECK(g_syncs - syncs0 == 2 + 2);  // engines 1 and 3 (non-leading), then one read-back per device
    }
    // concurrent callers (TSan): the calls are serialised inside
    {
        Node x = make_node(8, [](uint32_t g) { return (int)g; });
        std::vector<std::thread> th;
        int bad = 0;
        std::mutex bm;
        for (int t = 0; t < 4; ++t)
            th.emplace_back([&] {
                for (int r = 0; r < 50; ++r) {
                    cts_counters a{};
                    if (cts_counters_allreduce(x.eng.data(), x.ptrs.data(), nullptr, 8, &a) != CTS_OK ||
                        !equal(a, x.want)) {
                        std::lock_guard<std::mutex> lk(bm);
                        ++bad;
                    }
                }
            });
        for (auto& t : th) t.join();
        CHECK(bad == 0);
    }
    CHECK(cts_counters_allreduce_release() == CTS_OK);
    CHECK(live() == 0);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        CHECK(g_alloc_dev.empty());  // every device slot freed, each on its own device
    }
    // after a release the clique is created again
    {
        Node x = make_node(2, [](uint32_t g) { return (int)g; });
        cts_counters a{};
        CHECK(cts_counters_allreduce(x.eng.data(), x.ptrs.data(), nullptr, 2, &a) == CTS_OK && equal(a, x.want));
        CHECK(live() == 2);
    }
    CHECK(cts_counters_allreduce_release() == CTS_OK && live() == 0);

    // 3. the DataError count (slot kConnectionsFailed) through the _ex reads, both ways
    for (uint32_t n : {1u, 3u, 8u}) {
        Node x = make_node(n, [](uint32_t g) { return (int)g; });
        cts_counters_ex a{}, h{};
        CHECK(cts_counters_read_multi_ex(x.eng.data(), x.ptrs.data(), nullptr, n, &h) == CTS_OK && equal(h, x.want));
        CHECK(cts_counters_allreduce_ex(x.eng.data(), x.ptrs.data(), nullptr, n, &a) == CTS_OK && equal(a, x.want));
        CHECK(std::memcmp(&a, &h, sizeof(a)) == 0);
        cts_counters five{};  // the five-field reads are the _ex reads' first five fields
        CHECK(cts_counters_allreduce(x.eng.data(), x.ptrs.data(), nullptr, n, &five) == CTS_OK && equal(five, x.want));
    }
    CHECK(cts_counters_read_multi_ex(nullptr, nullptr, nullptr, 1, nullptr) == CTS_E_INVALID);
    CHECK(cts_counters_allreduce_ex(nullptr, nullptr, nullptr, 1, nullptr) == CTS_E_INVALID);
    CHECK(cts_counters_allreduce_release() == CTS_OK && live() == 0);

    // 4. prepare: the clique (slots, communicators, a first all-reduce) is built before any counter read, once
    CHECK(cts_counters_allreduce_prepare(nullptr, 0) == CTS_OK);
    CHECK(cts_counters_allreduce_prepare(nullptr, 2) == CTS_E_INVALID);
    CHECK(cts_counters_allreduce_prepare(bogus, 1) == CTS_E_INVALID);
    CHECK(cts_counters_allreduce_setup_times(nullptr) == CTS_E_INVALID);
    {
        Node x = make_node(6, [](uint32_t g) { return (int)(g / 2); });  // devices 0, 1, 2: two engines each
        t_cur = 5;
        const int folds_before = g_folds;
        CHECK(cts_counters_allreduce_prepare(x.eng.data(), 6) == CTS_OK);
        CHECK(t_cur == 5 && live() == 3);
        CHECK(g_folds - folds_before == 3);  // the dry run: one fold of a zeroed block per device
        {
            std::lock_guard<std::mutex> lk(g_mu);
            CHECK(g_alloc_dev.size() == 3);  // one slot per device
        }
        cts_allreduce_setup st{};
        CHECK(cts_counters_allreduce_setup_times(&st) == CTS_OK);
        CHECK(st.devices == 3 && st.prepared == 1 && st.slots_ms >= 0.0 && st.comm_init_ms >= 0.0 &&
              st.first_allreduce_ms >= 0.0 && st.rccl_load_ms == 0.0);  // RCCL was loaded by an earlier call
        CHECK(cts_counters_allreduce_prepare(x.eng.data(), 6) == CTS_OK && live() == 3);  // idempotent
        const int folds0 = g_folds;
        cts_counters_ex a{};
        CHECK(cts_counters_allreduce_ex(x.eng.data(), x.ptrs.data(), nullptr, 6, &a) == CTS_OK && equal(a, x.want));
        CHECK(live() == 3 && g_folds - folds0 == 6);  // the prepared clique is the one used: no dry run again
        cts_allreduce_setup st2{};
        CHECK(cts_counters_allreduce_setup_times(&st2) == CTS_OK);
        // the set-up part unchanged; the last call's phases are the all-reduce's own
        CHECK(st2.rccl_load_ms == st.rccl_load_ms && st2.slots_ms == st.slots_ms && st2.comm_init_ms == st.comm_init_ms &&
              st2.first_allreduce_ms == st.first_allreduce_ms && st2.devices == st.devices && st2.prepared == 1);
        CHECK(st2.last_fold_us >= 0.0 && st2.last_allreduce_us >= 0.0 && st2.last_readback_us >= 0.0 &&
              st2.last_total_us >= st2.last_fold_us + st2.last_allreduce_us + st2.last_readback_us);
    }
    // a clique built lazily by a first all-reduce says so
    {
        Node x = make_node(2, [](uint32_t g) { return (int)g + 4; });
        cts_counters_ex a{};
        CHECK(cts_counters_allreduce_ex(x.eng.data(), x.ptrs.data(), nullptr, 2, &a) == CTS_OK && equal(a, x.want));
        cts_allreduce_setup st{};
        CHECK(cts_counters_allreduce_setup_times(&st) == CTS_OK && st.devices == 2 && st.prepared == 0);
    }
    // communicator creation failing in prepare: an error, nothing kept, a later prepare succeeds
    CHECK(cts_counters_allreduce_release() == CTS_OK && live() == 0);
    setenv("STUB_RCCL_FAIL_INIT", "1", 1);
    {
        Node x = make_node(2, [](uint32_t g) { return (int)g; });
        CHECK(cts_counters_allreduce_prepare(x.eng.data(), 2) == CTS_E_HIP && live() == 0);
        std::lock_guard<std::mutex> lk(g_mu);
        CHECK(g_alloc_dev.empty());
    }
    unsetenv("STUB_RCCL_FAIL_INIT");
    {
        Node x = make_node(2, [](uint32_t g) { return (int)g; });
        CHECK(cts_counters_allreduce_prepare(x.eng.data(), 2) == CTS_OK && live() == 2);
    }
    CHECK(cts_counters_allreduce_release() == CTS_OK && live() == 0);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        CHECK(g_alloc_dev.empty());
    }
    dlclose(stub);
    std::printf("counters_fold: ok\n");
    return 0;
}
