// first_read_probe.cpp — where a status tick's first counter read (cts_counters_allreduce_ex after
// cts_counters_allreduce_prepare) spends more than the steady 25-35 us, with no Python in the process. Each case is
// timed around the C ABI call (steady_clock) and by the library itself (cts_allreduce_setup.last_total_us):
//   same_thread_after_idle : the thread that called prepare, after 1 s asleep (a status timer's next tick)
//   same_thread_hot        : the same thread again at once
//   new_thread_first       : a thread that never called HIP; its first call, then its second
//   new_thread_after_hip   : a new thread whose first HIP call (hipGetDevice) is timed apart, then the read
//   new_thread_after_malloc: a new thread whose first malloc is timed apart, then the read
//   new_thread_after_idle  : a new thread that sleeps 1 s first
//   same_thread_idle_N     : the first thread after N us asleep (0 .. 1 s)
// Three rounds; one JSON line per case and round. Diagnostic only (profiles/r06/s/).
//   build: make tools/first_read_probe      run: tools/first_read_probe
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#include "cts_engine.h"

namespace {

double us_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

struct Node {
    cts_engine* e[1] = {nullptr};
    const void* blk[1] = {nullptr};
};

cts_allreduce_setup g_last{};  // the phases of the newest read

// one all-reduce: {wall us around the call, the library's own last_total_us, rc}
void read_once(const Node& n, double* wall, double* lib, int* rc)
{
    cts_counters_ex out{};
    const auto t0 = std::chrono::steady_clock::now();
    *rc = cts_counters_allreduce_ex(n.e, n.blk, nullptr, 1, &out);
    *wall = us_since(t0);
    (void)cts_counters_allreduce_setup_times(&g_last);
    *lib = g_last.last_total_us;
}

void emit(int round, const char* name, double wall, double lib, int rc, double hip_us = -1.0)
{
    std::printf("{\"round\": %d, \"case\": \"%s\", \"wall_us\": %.1f, \"c_abi_us\": %.1f, \"rc\": %d", round, name, wall,
                lib, rc);
    if (hip_us >= 0) std::printf(", \"first_call_us\": %.1f", hip_us);
    // before_fold_us: entry to the first fold launch (argument checks, device grouping, lock, clique lookup)
    std::printf(", \"before_fold_us\": %.1f, \"fold_us\": %.1f, \"allreduce_us\": %.1f, \"readback_us\": %.1f}\n",
                g_last.last_total_us - g_last.last_fold_us - g_last.last_allreduce_us - g_last.last_readback_us,
                g_last.last_fold_us, g_last.last_allreduce_us, g_last.last_readback_us);
    std::fflush(stdout);
}

}  // namespace

int main()
{
    Node n;
    if (cts_engine_create(0, &n.e[0]) != CTS_OK) return 1;
    void* ctr = nullptr;
    if (hipMalloc(&ctr, cts_counters_device_bytes()) != hipSuccess) return 1;
    if (cts_counters_reset(n.e[0], ctr, nullptr) != CTS_OK || hipDeviceSynchronize() != hipSuccess) return 1;
    n.blk[0] = ctr;
    const auto t0 = std::chrono::steady_clock::now();
    if (cts_counters_allreduce_prepare(n.e, 1) != CTS_OK) return 1;
    std::printf("{\"prepare_ms\": %.1f}\n", us_since(t0) / 1e3);
    for (int round = 0; round < 3; ++round) {
        double w = 0, l = 0;
        int rc = 0;
        std::this_thread::sleep_for(std::chrono::seconds(1));
        read_once(n, &w, &l, &rc);
        emit(round, "same_thread_after_idle", w, l, rc);
        read_once(n, &w, &l, &rc);
        emit(round, "same_thread_hot", w, l, rc);
        std::thread([&] {
            double w1, l1;
            int r1;
            read_once(n, &w1, &l1, &r1);
            emit(round, "new_thread_first", w1, l1, r1);
            read_once(n, &w1, &l1, &r1);
            emit(round, "new_thread_second", w1, l1, r1);
        }).join();
        std::thread([&] {
            int dev = -1;
            const auto th = std::chrono::steady_clock::now();
            (void)hipGetDevice(&dev);
            const double hip_us = us_since(th);
            double w1, l1;
            int r1;
            read_once(n, &w1, &l1, &r1);
            emit(round, "new_thread_after_hip", w1, l1, r1, hip_us);
        }).join();
        std::thread([&] {
            const auto tm = std::chrono::steady_clock::now();
            void* volatile q = std::malloc(64);
            std::free(q);
            const double malloc_us = us_since(tm);
            double w1, l1;
            int r1;
            read_once(n, &w1, &l1, &r1);
            emit(round, "new_thread_after_malloc", w1, l1, r1, malloc_us);
        }).join();
        std::thread([&] {
            std::this_thread::sleep_for(std::chrono::seconds(1));
            double w1, l1;
            int r1;
            read_once(n, &w1, &l1, &r1);
            emit(round, "new_thread_after_idle", w1, l1, r1);
        }).join();
    }
    // the same thread after 0 / 0.1 / 1 / 10 / 100 / 1000 ms asleep, three times each
    for (int round = 0; round < 3; ++round)
        for (int idle_us : {0, 100, 1000, 10000, 100000, 1000000}) {
            std::this_thread::sleep_for(std::chrono::microseconds(idle_us));
            double w = 0, l = 0;
            int rc = 0;
            read_once(n, &w, &l, &rc);
            char name[64];
            std::snprintf(name, sizeof(name), "same_thread_idle_%dus", idle_us);
            emit(round, name, w, l, rc);
        }
    (void)cts_counters_allreduce_release();
    (void)hipFree(ctr);
    (void)cts_engine_destroy(n.e[0]);
    return 0;
}
