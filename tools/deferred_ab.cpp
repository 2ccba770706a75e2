// deferred_ab.cpp — why does config 1 with GPU DEFERRED verify receive ~12 % slower than with verify off, while the
// receive threads spend the same CPU per GiB? (VERDICT r03 "Next round" 6)
//
// Two suspects, each switched on alone, in one process, legs alternated over several rounds (config 1: loopback TCP
// push, 8 connections x 1 GiB, 64 KiB IO, through the product library's cts_loopback_run):
//   - the GPU's reads of the pinned recv ring over PCIe (host DRAM traffic beside the socket copies): verify off
//     with a background stream of zero-copy verifies of another pinned host arena (cts_verify_strided on its device
//     view) at full rate, against verify off alone;
//   - the recv ring's footprint (2 x batch + 2 slots of 64 KiB per connection: 64 MiB at the loopback default of 512,
//     against one reused 64 KiB buffer with verify off): DEFERRED at batch 512 against batch 16 (2.1 MiB).
// Every verify is a real one; nothing in the product changes. Prints one JSON line per leg and round.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "cts_engine.h"
#include "cts_loopback.h"
#include "cts_pattern.h"

namespace {

struct Background {
    cts_engine* e = nullptr;
    void* host = nullptr;
    void* dev = nullptr;
    uint32_t* lens = nullptr;
    void* stream = nullptr;
    static constexpr uint32_t kN = 1024;  // 64 MiB of 64 KiB buffers in pinned host memory
    std::atomic<bool> stop{false};
    std::atomic<uint64_t> bytes{0};
    std::thread th;
    bool init(cts_engine* eng)
    {
        e = eng;
        if (cts_host_alloc(e, (uint64_t)kN << 16, &host, &dev) != CTS_OK) return false;
        if (cts_engine_stream_create(e, &stream) != CTS_OK) return false;
        std::vector<cts_buf_desc> d(kN);
        for (uint32_t i = 0; i < kN; ++i) d[i] = cts_buf_desc{(uint64_t)i << 16, 65536u, 0u, 0u, 0u};
        cts_buf_desc* dd = nullptr;
        if (hipMalloc((void**)&dd, kN * sizeof(cts_buf_desc)) != hipSuccess) return false;
        if (hipMalloc((void**)&lens, kN * 4) != hipSuccess) return false;
        std::vector<uint32_t> l(kN, 65536u);
        if (hipMemcpy(dd, d.data(), kN * sizeof(cts_buf_desc), hipMemcpyHostToDevice) != hipSuccess) return false;
        if (hipMemcpy(lens, l.data(), kN * 4, hipMemcpyHostToDevice) != hipSuccess) return false;
        // the pinned arena holds the pattern (written through its device view), so every verify passes
        if (cts_fill(e, dev, (uint64_t)kN << 16, dd, kN, 65536u, stream) != CTS_OK) return false;
        if (hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess) return false;
        (void)hipFree(dd);
        return true;
    }
    void start()
    {
        stop = false;
        bytes = 0;
        th = std::thread([this] {
            while (!stop.load(std::memory_order_relaxed)) {
                if (cts_verify_strided(e, dev, (uint64_t)kN << 16, 65536u, lens, kN, 0u, 0u, 0u, nullptr, nullptr, nullptr,
                                       0u, stream) != CTS_OK)
                    break;
                if (hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess) break;
                bytes += (uint64_t)kN << 16;
            }
        });
    }
    void finish()
    {
        stop = true;
        th.join();
    }
};

void leg(const char* name, int round, cts_engine* e, uint32_t verify, uint32_t mode, uint32_t batch, Background* bg)
{
    cts_loopback_config c{};
    c.connections = 8;
    c.io_pattern = 0;  // Push
    c.buffer_size = 65536;
    c.verify_buffers = verify;
    c.transfer_size = 1ull << 30;
    c.verify_mode = mode;
    c.batch_buffers = batch;
    c.corrupt_connection = ~0u;
    cts_loopback_result r{};
    std::vector<cts_loopback_side> sides(2 * c.connections);
    if (bg != nullptr) bg->start();
    const auto t0 = std::chrono::steady_clock::now();
    cts_engine* engines[1] = {e};
    const int rc = cts_loopback_run_detailed(&c, verify ? engines : nullptr, verify ? 1u : 0u, nullptr, nullptr, &r,
                                             sides.data());
    const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double bg_gbps = 0;
    if (bg != nullptr) {
        bg->finish();
        bg_gbps = (double)bg->bytes.load() / wall / 1e9;
    }
    const double gib = (double)r.bytes_recv / (double)(1ull << 30);
    double wait_s = 0;  // the receiving (server) sides' waits for device verdicts
    for (uint32_t i = c.connections; i < 2 * c.connections; ++i) wait_s += (double)sides[i].stats.verify_wait_ns * 1e-9;
    const double thread_s = r.seconds * c.connections;  // wall time of the receive threads
    std::printf("{\"leg\":\"%s\",\"round\":%d,\"rc\":%d,\"hw_queues\":\"%s\",\"connections_ok\":%u,"
                "\"GBps_recv\":%.3f,\"recv_busy_frac\":%.3f,\"send_busy_frac\":%.3f,\"recv_verify_wait_frac\":%.3f,"
                "\"recv_verify_wait_s_per_GiB\":%.4f,"
                "\"recv_cpu_s_per_GiB\":%.4f,\"recv_socket_cpu_s_per_GiB\":%.4f,\"recv_pattern_cpu_s_per_GiB\":%.4f,"
                "\"send_cpu_s_per_GiB\":%.4f,\"batch_buffers\":%u,\"ring_MiB_per_connection\":%.2f,"
                "\"background_pcie_read_GBps\":%.1f}\n",
                name, round, rc, std::getenv("GPU_MAX_HW_QUEUES") ? std::getenv("GPU_MAX_HW_QUEUES") : "default",
                r.connections_ok, (double)r.bytes_recv / r.seconds / 1e9, r.recv_cpu_seconds / thread_s,
                r.send_cpu_seconds / thread_s, wait_s / thread_s, wait_s / gib, r.recv_cpu_seconds / gib,
                r.recv_io_cpu_seconds / gib, (r.recv_cpu_seconds - r.recv_io_cpu_seconds) / gib, r.send_cpu_seconds / gib,
                batch, mode == CTS_VERIFY_DEFERRED && verify ? (2.0 * batch + 2.0) * 65536.0 / (1 << 20) : 0.0, bg_gbps);
    std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 3;
    cts_engine* e = nullptr;
    if (cts_engine_create(0, &e) != CTS_OK) return 1;
    // g_senderSharedBuffer from the fill kernel before any leg (the verify-off legs create patterns without an engine)
    if (cts_shared_buffer_init(e, 65536) != CTS_OK) return 2;
    Background bg;
    if (!bg.init(e)) return 2;
    for (int r = 0; r < rounds; ++r) {
        // the legs in a rotated order each round, so no leg always follows the same one
        for (int k = 0; k < 5; ++k) {
            switch ((k + r) % 5) {
            case 0: leg("verify_off", r, e, 0, CTS_VERIFY_SYNC, 0, nullptr); break;
            case 1: leg("verify_off_plus_pcie_reads", r, e, 0, CTS_VERIFY_SYNC, 0, &bg); break;
            case 2: leg("gpu_deferred_batch512", r, e, 1, CTS_VERIFY_DEFERRED, 512, nullptr); break;
            case 3: leg("gpu_deferred_batch2048", r, e, 1, CTS_VERIFY_DEFERRED, 2048, nullptr); break;
            case 4: leg("gpu_deferred_batch64", r, e, 1, CTS_VERIFY_DEFERRED, 64, nullptr); break;
            }
        }
    }
    (void)cts_engine_destroy(e);
    return 0;
}
