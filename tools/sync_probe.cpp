// sync_probe.cpp — latency of one SYNC-mode verify (ctsIOPattern.cpp:745-775 called per CompleteIo):
// a 64 KiB buffer in pinned, device-mapped host memory verified in place over PCIe and waited for,
// exactly as cts_pattern.cpp VerifyNow does (cts_verify on the pattern's own stream + synchronize).
// Variants: the buffer described as S slices (S descriptors of 64 KiB / S, expected offsets advanced,
// so S workgroups/waves issue their PCIe reads at once) and T threads, each with its own stream,
// buffer, descriptor and result (T connections completing concurrently). Wait = hipStreamSynchronize
// or a hipStreamQuery spin, or cts_verify_mapped (posted to the engine's resident mailbox grid: no launch per
// verify). Prints one JSON line per variant: us per verify (mean, min and max over threads) and GB/s over the
// wall time from the first thread's start to the last one's end (the timed loops start together).
//   build: make tools/sync_probe      run: tools/sync_probe [iters [mailbox]]  (mailbox: waits 2-4 only)
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <sched.h>

#include <fstream>
#include <sstream>
#include <string>

#include "cts_engine.h"

// CTS_PIN_NEAR_GPU=1: restrict the process to the CPUs of the GPU's NUMA node (PCI device -> numa_node ->
// cpulist) before any pinned allocation or thread; prints the node and CPU count it used.
static void pin_near_gpu()
{
    const char* v = std::getenv("CTS_PIN_NEAR_GPU");
    if (v == nullptr || std::atoi(v) == 0) return;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), 0) != hipSuccess) return;
    std::string id(bus);
    for (auto& c : id) c = (char)std::tolower((unsigned char)c);
    int node = -1;
    std::ifstream(std::string("/sys/bus/pci/devices/") + id + "/numa_node") >> node;
    if (node < 0) {
        std::printf("{\"pin\": \"no numa node for %s\"}\n", id.c_str());
        return;
    }
    std::string list;
    std::ifstream(std::string("/sys/devices/system/node/node") + std::to_string(node) + "/cpulist") >> list;
    cpu_set_t set;
    CPU_ZERO(&set);
    int count = 0;
    std::stringstream ss(list);
    std::string part;
    while (std::getline(ss, part, ',')) {
        const size_t dash = part.find('-');
        const int lo = std::atoi(part.substr(0, dash).c_str());
        const int hi = dash == std::string::npos ? lo : std::atoi(part.substr(dash + 1).c_str());
        for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c, ++count) CPU_SET(c, &set);
    }
    const int rc = sched_setaffinity(0, sizeof(set), &set);
    std::printf("{\"pin\": \"%s\", \"numa_node\": %d, \"cpus\": %d, \"rc\": %d}\n", id.c_str(), node, count, rc);
    std::fflush(stdout);
}

// All threads of a variant start their timed loops together (gate) and report their start/end times, so the
// variant's throughput is all verifies / (last end - first start), fair or not.
struct Gate {
    std::atomic<uint32_t> ready{0};
    uint32_t threads = 1;
};
using Clock = std::chrono::steady_clock;

static int run_thread(cts_engine* e, uint32_t slices, bool spin, bool mapped, int iters, double* us_out, int* bad,
                      bool host_copy, Gate* gate, Clock::time_point* start, Clock::time_point* end)
{
    void* stream = nullptr;
    if (cts_engine_stream_create(e, &stream) != CTS_OK) return 1;
    const uint32_t len = 65536, per = len / slices;
    void *host = nullptr, *dev = nullptr, *hd = nullptr, *dd = nullptr;
    if (cts_host_alloc(e, len, &host, &dev) != CTS_OK) return 1;
    if (cts_host_alloc(e, 4096 + slices * 64, &hd, &dd) != CTS_OK) return 1;
    for (uint32_t b = 0; b < len; ++b) static_cast<uint8_t*>(host)[b] = cts_pattern_byte(b + 1000);
    auto* desc = static_cast<cts_buf_desc*>(hd);
    for (uint32_t k = 0; k < slices; ++k)
        desc[k] = cts_buf_desc{(uint64_t)k * per, per, (1000 + k * per) % CTS_PATTERN_PERIOD, k, 0};
    auto* res_h = reinterpret_cast<cts_verify_result*>(static_cast<uint8_t*>(hd) + 2048);
    auto* res_d = reinterpret_cast<cts_verify_result*>(static_cast<uint8_t*>(dd) + 2048);
    hipStream_t s = static_cast<hipStream_t>(stream);
    std::vector<uint8_t> pageable;
    if (host_copy) pageable.assign(static_cast<uint8_t*>(host), static_cast<uint8_t*>(host) + len);
    auto once = [&]() {
        if (host_copy) {  // cts_verify_host: a pageable buffer (the Level-1 VerifyBuffer drop-in)
            cts_verify_result r{};
            return cts_verify_host(e, pageable.data(), len, 1000, &r) == CTS_OK && r.pass && r.first_mismatch == len;
        }
        if (mapped) {  // cts_verify_mapped: the mailbox grid
            cts_verify_result r{};
            return cts_verify_mapped(e, dev, len, 1000, &r) == CTS_OK && r.pass && r.first_mismatch == len;
        }
        if (cts_verify(e, dev, len, static_cast<cts_buf_desc*>(dd), slices, per, res_d, nullptr, nullptr, 0, stream) !=
            CTS_OK)
            return false;
        if (spin) {
            while (hipStreamQuery(s) == hipErrorNotReady) {
            }
        } else if (hipStreamSynchronize(s) != hipSuccess) {
            return false;
        }
        for (uint32_t k = 0; k < slices; ++k)
            if (!res_h[k].pass) return false;
        return true;
    };
    for (int i = 0; i < 50; ++i)
        if (!once()) ++*bad;
    gate->ready.fetch_add(1);
    while (gate->ready.load() < gate->threads) std::this_thread::yield();
    const auto t0 = Clock::now();
    for (int i = 0; i < iters; ++i)
        if (!once()) ++*bad;
    const auto t1 = Clock::now();
    *start = t0;
    *end = t1;
    *us_out = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    cts_host_free(e, host);
    cts_host_free(e, hd);
    cts_engine_stream_destroy(e, stream);
    return 0;
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    const bool mailbox_only = argc > 2 && std::strcmp(argv[2], "mailbox") == 0;
    pin_near_gpu();
    cts_engine* e = nullptr;
    if (cts_engine_create(0, &e) != CTS_OK) return 1;
    // wait: 0 stream_sync, 1 query_spin, 2 cts_verify_mapped (mailbox; slices = its 4 KiB pieces, reported as 64)
    // wait 3/4: cts_verify_host (copy of a pageable buffer) through the mailbox / through a launch + sync
    for (int spin = mailbox_only ? 2 : 0; spin < 5; ++spin)
        for (uint32_t threads : {1u, 8u, 16u})
            for (uint32_t slices : {1u, 2u, 4u, 8u, 16u, 32u, 64u}) {
                if (spin >= 2 && slices != 64) continue;
                if (threads == 16 && slices != 64) continue;
                std::vector<double> us(threads, 0.0);
                std::vector<int> bad(threads, 0), rc(threads, 0);
                std::vector<Clock::time_point> t_start(threads), t_end(threads);
                Gate gate;
                gate.threads = threads;
                std::vector<std::thread> th;
                if (spin >= 3) (void)cts_engine_set_attr(e, CTS_ATTR_SYNC_MAILBOX, spin == 3 ? 1 : 0);
                for (uint32_t t = 0; t < threads; ++t)
                    th.emplace_back([&, t] { rc[t] = run_thread(e, slices, spin == 1, spin == 2, iters, &us[t], &bad[t], spin >= 3, &gate,
                                                            &t_start[t], &t_end[t]); });
                for (auto& x : th) x.join();
                double mean = 0, lo = 1e30, hi = 0;
                int nbad = 0, nrc = 0;
                Clock::time_point first = t_start[0], last = t_end[0];
                for (uint32_t t = 0; t < threads; ++t) {
                    mean += us[t] / threads;
                    lo = std::min(lo, us[t]);
                    hi = std::max(hi, us[t]);
                    nbad += bad[t];
                    nrc += rc[t];
                    first = std::min(first, t_start[t]);
                    last = std::max(last, t_end[t]);
                }
                const double wall_s = std::chrono::duration<double>(last - first).count();
                std::printf("{\"wait\": \"%s\", \"threads\": %u, \"slices\": %u, \"us_per_verify\": %.2f, "
                            "\"us_min_thread\": %.2f, \"us_max_thread\": %.2f, \"GBps_wall\": %.2f, \"bad\": %d, \"rc\": %d}\n",
                            spin == 4 ? "host_launch" : spin == 3 ? "host_mailbox" : spin == 2 ? "mailbox" : spin ? "query_spin" : "stream_sync",
                            threads, slices, mean, lo, hi,
                            threads * (double)iters * 65536.0 / (wall_s * 1e9), nbad, nrc);
                std::fflush(stdout);
            }
    cts_engine_destroy(e);
    return 0;
}
