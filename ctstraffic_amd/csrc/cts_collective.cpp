// cts_collective.cpp — cts_counters_allreduce (include/cts_engine.h): the node-wide ctsStatsTracking counters
// (ctsStatistics.hpp:87-198) of ONE process that drives one engine per GPU, reduced over RCCL on the GPUs.
//
// ctsTraffic is one process per host with many IO threads; its byte/error statistics are process-global atomics
// (ctsStatistics.hpp:87-198, read by ctsConfig::TcpStatusDetails, ctsConfig.h:415-417). With the verify on N GPUs
// each engine's counters live in its own device block. This entry point folds every block on its own device (one
// 64-thread launch, counters_fold_kernel), reduces the six sums (ctsStatsTracking's bytes and buffers, and the
// DataError count of ConnectionStatusDetails, ctsSocketState.cpp:221-228) across the devices with one ncclAllReduce
// (sum, ncclUint64, count 6) per device inside ncclGroupStart/End over the xGMI links, and
// reads the result back. Every device's copy is read and compared: a reduction that disagrees is an error.
//
// RCCL is loaded on first use (dlopen of librccl.so.1, or $CTS_RCCL_LIBRARY), so the engine library itself does
// not pull the 570 MB RCCL image into every process that only verifies; inside a PyTorch process the soname
// resolves to the RCCL torch already loaded. One communicator clique (ncclCommInitAll) is kept per set of
// devices and reused until cts_counters_allreduce_release; cts_counters_allreduce_prepare builds it (and runs its
// first all-reduce, which carries RCCL's own first-collective set-up) before the status timer's first tick. Calls
// are serialised by one lock (a counter read happens once per status interval, not per IO).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "cts_engine.h"
#include "cts_internal.hpp"

namespace {

struct Rccl {
    void* handle = nullptr;
    ncclResult_t (*comm_init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
};

// One communicator per device of a device set, plus a device slot each: kCounterSlots u64 (the fold's output and the
// all-reduce's in-place buffer), then a zeroed counter block of the device layout that the set-up's dry run folds.
struct Clique {
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;
    std::vector<uint64_t*> sums;
};

std::mutex g_mu;  // guards everything below
Rccl g_rccl;
std::vector<std::unique_ptr<Clique>> g_cliques;
cts_allreduce_setup g_setup{0.0, 0.0, 0.0, 0.0, 0u, 0u, 0.0, 0.0, 0.0, 0.0};  // the newest clique's set-up, the last call

double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = (prev == dev) || (hipSetDevice(dev) == hipSuccess);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// Resolves the RCCL entry points once; a failed load is retried on the next call. *load_ms: the time this call
// spent loading (0 when RCCL was already loaded).
bool load_rccl(double* load_ms)
{
    *load_ms = 0.0;
    if (g_rccl.handle != nullptr) return true;
    const auto t0 = std::chrono::steady_clock::now();
    const char* env = std::getenv("CTS_RCCL_LIBRARY");
    void* h = nullptr;
    if (env != nullptr && *env != 0) {
        h = dlopen(env, RTLD_NOW | RTLD_LOCAL);
    } else {
        h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (h == nullptr) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    }
    if (h == nullptr) return false;
    Rccl r;
    r.handle = h;
    r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    if (!r.comm_init_all || !r.comm_destroy || !r.all_reduce || !r.group_start || !r.group_end) {
        dlclose(h);
        return false;
    }
    g_rccl = r;
    *load_ms = ms_since(t0);
    return true;
}

void destroy_clique(Clique& c)
{
    for (size_t k = 0; k < c.comms.size(); ++k) {
        if (c.comms[k] != nullptr) (void)g_rccl.comm_destroy(c.comms[k]);
        if (c.sums[k] != nullptr) {
            DeviceGuard g(c.devices[k]);
            (void)hipFreeAsync(c.sums[k], nullptr);  // stream-ordered: hipFree would wait for every kernel on the device
        }
    }
    c.comms.clear();
    c.sums.clear();
}

// One grouped all-reduce (sum, u64 x kCounterCount, in place on every device's slot), each device's op on
// streams[k]. One thread drives every rank of the clique, so a multi-rank clique must be grouped.
int grouped_allreduce(Clique& c, const std::vector<hipStream_t>& streams)
{
    if (g_rccl.group_start() != ncclSuccess) return CTS_E_HIP;
    ncclResult_t r = ncclSuccess;
    for (size_t k = 0; k < c.devices.size() && r == ncclSuccess; ++k)
        r = g_rccl.all_reduce(c.sums[k], c.sums[k], cts::kCounterCount, ncclUint64, ncclSum, c.comms[k], streams[k]);
    const ncclResult_t re = g_rccl.group_end();
    return (r != ncclSuccess || re != ncclSuccess) ? CTS_E_HIP : CTS_OK;
}

constexpr size_t kSlotWords = cts::kCounterSlots + (size_t)CTS_COUNTER_SHARDS * cts::kCounterSlots;

// The clique of exactly these devices (in this order), created on first use: slots, communicators, and one dry run
// of a counter read on each device's null stream (the fold of a zeroed block, the grouped all-reduce, the copy back):
// RCCL sets up its first collective's channels and kernels in it, and the fold kernel and the device-to-host copy
// have run once, so the first real read costs what every later one does. Each step is timed into g_setup. load_ms:
// what this call spent loading RCCL.
int clique_for(const std::vector<int>& devices, double load_ms, bool prepared, Clique** out)
{
    for (auto& c : g_cliques)
        if (c->devices == devices) {
            *out = c.get();
            return CTS_OK;
        }
    cts_allreduce_setup t{load_ms, 0.0, 0.0, 0.0, (uint32_t)devices.size(), prepared ? 1u : 0u, 0.0, 0.0, 0.0, 0.0};
    std::unique_ptr<Clique> c(new (std::nothrow) Clique());
    if (!c) return CTS_E_NOMEM;
    c->devices = devices;
    c->comms.assign(devices.size(), nullptr);
    c->sums.assign(devices.size(), nullptr);
    auto t0 = std::chrono::steady_clock::now();
    for (size_t k = 0; k < devices.size(); ++k) {
        DeviceGuard g(devices[k]);
        void* p = nullptr;
        // on the device's null stream, which the engines' non-blocking streams never wait for; the caller's
        // leading stream uses the slot only after the synchronize below
        if (!g.ok || hipMallocAsync(&p, kSlotWords * sizeof(uint64_t), nullptr) != hipSuccess) {
            destroy_clique(*c);
            return g.ok ? CTS_E_NOMEM : CTS_E_HIP;
        }
        c->sums[k] = static_cast<uint64_t*>(p);
        if (hipMemsetAsync(p, 0, kSlotWords * sizeof(uint64_t), nullptr) != hipSuccess ||
            hipStreamSynchronize(nullptr) != hipSuccess) {
            destroy_clique(*c);
            return CTS_E_HIP;
        }
    }
    t.slots_ms = ms_since(t0);
    int prev = -1;
    (void)hipGetDevice(&prev);
    t0 = std::chrono::steady_clock::now();
    const ncclResult_t r = g_rccl.comm_init_all(c->comms.data(), (int)devices.size(), devices.data());
    t.comm_init_ms = ms_since(t0);
    if (prev >= 0) (void)hipSetDevice(prev);
    if (r != ncclSuccess) {
        std::fill(c->comms.begin(), c->comms.end(), nullptr);
        destroy_clique(*c);
        return CTS_E_HIP;
    }
    t0 = std::chrono::steady_clock::now();
    int rc = CTS_OK;
    for (size_t k = 0; k < devices.size() && rc == CTS_OK; ++k) {
        DeviceGuard g(devices[k]);
        if (!g.ok || cts::launch_counters_fold(c->sums[k] + cts::kCounterSlots, c->sums[k], false, nullptr) != hipSuccess)
            rc = CTS_E_HIP;
    }
    if (rc == CTS_OK) rc = grouped_allreduce(*c, std::vector<hipStream_t>(devices.size(), nullptr));
    for (size_t k = 0; k < devices.size() && rc == CTS_OK; ++k) {
        DeviceGuard g(devices[k]);
        uint64_t h[cts::kCounterCount];
        if (!g.ok || hipMemcpyAsync(h, c->sums[k], sizeof(h), hipMemcpyDeviceToHost, nullptr) != hipSuccess ||
            hipStreamSynchronize(nullptr) != hipSuccess)
            rc = CTS_E_HIP;
        for (int j = 0; j < cts::kCounterCount && rc == CTS_OK; ++j)
            if (h[j] != 0) rc = CTS_E_HIP;  // zeros folded and summed must stay zeros
    }
    t.first_allreduce_ms = ms_since(t0);
    if (rc != CTS_OK) {
        destroy_clique(*c);
        return rc;
    }
    g_setup = t;
    *out = c.get();
    g_cliques.push_back(std::move(c));
    return CTS_OK;
}

// engines grouped by device: devices in first-appearance order, leader[k] = index of device k's first engine
int group_by_device(cts_engine* const* engines, uint32_t n, std::vector<int>& dev_of, std::vector<int>& devices,
                    std::vector<uint32_t>& leader)
{
    dev_of.assign(n, -1);
    for (uint32_t i = 0; i < n; ++i) {
        if (engines[i] == nullptr) return CTS_E_INVALID;
        const int d = cts_engine_device(engines[i]);
        if (d < 0) return CTS_E_INVALID;
        dev_of[i] = d;
        if (std::find(devices.begin(), devices.end(), d) == devices.end()) {
            devices.push_back(d);
            leader.push_back(i);
        }
    }
    return CTS_OK;
}

}  // namespace

extern "C" {

int cts_counters_allreduce_ex(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                              uint32_t n, cts_counters_ex* out)
{
    const auto t_entry = std::chrono::steady_clock::now();
    if (out == nullptr || (n > 0 && (engines == nullptr || dev_counters == nullptr))) return CTS_E_INVALID;
    if (n == 0) {
        *out = cts_counters_ex{0, 0, 0, 0, 0, 0};
        return CTS_OK;
    }
    // the first engine of a device leads (its stream carries the device's folds and its all-reduce); the others'
    // blocks are folded into the same slot
    std::vector<int> dev_of, devices;
    std::vector<uint32_t> leader;
    for (uint32_t i = 0; i < n; ++i)
        if (dev_counters[i] == nullptr) return CTS_E_INVALID;
    int rc = group_by_device(engines, n, dev_of, devices, leader);
    if (rc != CTS_OK) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    double load_ms = 0.0;
    if (!load_rccl(&load_ms)) return CTS_E_UNAVAILABLE;
    Clique* c = nullptr;
    if ((rc = clique_for(devices, load_ms, false, &c)) != CTS_OK) return rc;
    const size_t D = devices.size();
    std::vector<hipStream_t> lead_stream(D);
    for (size_t k = 0; k < D; ++k) lead_stream[k] = streams ? static_cast<hipStream_t>(streams[leader[k]]) : nullptr;
    // 1. fold every engine's shard block into its device's slot, on the device's leading stream
    auto t0 = std::chrono::steady_clock::now();
    for (size_t k = 0; k < D; ++k) {
        DeviceGuard g(devices[k]);
        if (!g.ok) return CTS_E_HIP;
        bool first = true;
        for (uint32_t i = 0; i < n; ++i) {
            if (dev_of[i] != devices[k]) continue;
            const hipStream_t s = streams ? static_cast<hipStream_t>(streams[i]) : nullptr;
            // another stream's verifies must be complete before the leading stream reads this block
            if (s != lead_stream[k] && hipStreamSynchronize(s) != hipSuccess) return CTS_E_HIP;
            if (cts::launch_counters_fold(dev_counters[i], c->sums[k], !first, lead_stream[k]) != hipSuccess)
                return CTS_E_HIP;
            first = false;
        }
    }
    const double fold_us = ms_since(t0) * 1e3;
    // 2. one all-reduce per device, grouped
    t0 = std::chrono::steady_clock::now();
    if ((rc = grouped_allreduce(*c, lead_stream)) != CTS_OK) return rc;
    const double allreduce_us = ms_since(t0) * 1e3;
    // 3. every device's copy back; they must agree
    t0 = std::chrono::steady_clock::now();
    uint64_t first_copy[cts::kCounterCount] = {};
    for (size_t k = 0; k < D; ++k) {
        DeviceGuard g(devices[k]);
        uint64_t h[cts::kCounterCount];
        if (!g.ok || hipMemcpyAsync(h, c->sums[k], sizeof(h), hipMemcpyDeviceToHost, lead_stream[k]) != hipSuccess ||
            hipStreamSynchronize(lead_stream[k]) != hipSuccess)
            return CTS_E_HIP;
        if (k == 0) std::memcpy(first_copy, h, sizeof(h));
        else if (std::memcmp(first_copy, h, sizeof(h)) != 0) return CTS_E_HIP;
    }
    g_setup.last_fold_us = fold_us;
    g_setup.last_allreduce_us = allreduce_us;
    g_setup.last_readback_us = ms_since(t0) * 1e3;
    *out = cts::counters_ex_of(first_copy);
    g_setup.last_total_us = ms_since(t_entry) * 1e3;
    return CTS_OK;
}

int cts_counters_allreduce(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                           uint32_t n, cts_counters* out)
{
    if (out == nullptr) return CTS_E_INVALID;
    cts_counters_ex x{};
    const int rc = cts_counters_allreduce_ex(engines, dev_counters, streams, n, &x);
    if (rc == CTS_OK) *out = cts::counters_of(x);
    return rc;
}

int cts_counters_allreduce_prepare(cts_engine* const* engines, uint32_t n)
{
    if (n > 0 && engines == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    std::vector<int> dev_of, devices;
    std::vector<uint32_t> leader;
    int rc = group_by_device(engines, n, dev_of, devices, leader);
    if (rc != CTS_OK) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    double load_ms = 0.0;
    if (!load_rccl(&load_ms)) return CTS_E_UNAVAILABLE;
    Clique* c = nullptr;
    return clique_for(devices, load_ms, true, &c);
}

int cts_counters_allreduce_setup_times(cts_allreduce_setup* out)
{
    if (out == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::mutex> lk(g_mu);
    *out = g_setup;
    return CTS_OK;
}

int cts_counters_allreduce_release(void)
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto& c : g_cliques) destroy_clique(*c);
    g_cliques.clear();
    return CTS_OK;
}

}  // extern "C"
