// bench_multi.cpp — the timed launches of bench.py's single-process leg (`--engines N`) in native threads.
//
// ctsTraffic verifies from many native threads of ONE process (IOCP / RIO completion threads calling
// CompleteIo -> VerifyBuffer, ctsSendRecvIocp.cpp:60,97, ctsRioIocp.cpp:589,687). bench.py's single-process leg
// models that with one engine per GPU; launching from Python threads put every launch behind the GIL
// (~6 us of Python per cts_verify call), so at 8 GPUs the host, not the GPUs, set the rate. Here one
// std::thread per GPU issues its launches through the C ABI (cts_verify) onto its engine's streams, round
// robin; Python only prepares the batches and reads the clocks. The headline leg (one GPU) issues its launches
// through the same call in the calling thread, so both legs pay the same host cost per launch.
//
// build: make tools/libcts_bench_multi.so (links libcts_engine.so; bench.py loads it after the engine library,
// so both share one HIP runtime and the engine handles are the ones Python created).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "cts_engine.h"

extern "C" {

// One GPU's work: R rotated arenas of one batch (same descriptors), per-arena outputs, S streams.
struct cts_bench_gpu {
    cts_engine* engine;
    int device;
    uint32_t arenas;                      // R
    const void* const* arena;             // [R] device arenas
    uint64_t arena_bytes;
    const cts_buf_desc* descs;            // device descriptors (n)
    uint32_t n;
    uint32_t max_length_hint;
    cts_verify_result* const* results;    // [R] device result records (n each)
    void* counters;                       // device counter block
    uint32_t* const* conn_first_fail;     // [R] device first-failure slots (n_conns each)
    uint32_t n_conns;
    void* const* streams;                 // [S] engine streams
    uint32_t nstreams;
};

// Every GPU's thread waits at a common start, then issues `launches` cts_verify calls (launch i: arena i % R on
// stream i % S) and, with `sync`, synchronises its streams. t0[g] / t1[g] = that thread's start / end (end of
// its launches, or of its streams with `sync`), in seconds on one steady clock; *t_start = when the start was
// released. G == 1 runs in the calling thread (no thread start inside a timed region). Returns the first non-zero
// status of any call.
int cts_bench_run_multi(const cts_bench_gpu* gpus, uint32_t G, uint32_t launches, double* t0, double* t1,
                        double* t_start, int sync)
{
    if (gpus == nullptr || G == 0 || t0 == nullptr || t1 == nullptr) return CTS_E_INVALID;
    for (uint32_t g = 0; g < G; ++g)
        if (gpus[g].arenas == 0 || gpus[g].nstreams == 0 || gpus[g].arena == nullptr || gpus[g].streams == nullptr)
            return CTS_E_INVALID;
    using clk = std::chrono::steady_clock;
    const auto secs = [](clk::time_point t) { return std::chrono::duration<double>(t.time_since_epoch()).count(); };
    std::atomic<uint32_t> ready{0};
    std::atomic<bool> go{false};
    std::vector<int> rc(G, CTS_OK);
    const auto work = [&](uint32_t g) {
        const cts_bench_gpu& w = gpus[g];
        int r = hipSetDevice(w.device) == hipSuccess ? CTS_OK : CTS_E_HIP;
        ready.fetch_add(1, std::memory_order_acq_rel);
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
        t0[g] = secs(clk::now());
        for (uint32_t i = 0; i < launches && r == CTS_OK; ++i) {
            const uint32_t a = i % w.arenas;
            r = cts_verify(w.engine, w.arena[a], w.arena_bytes, w.descs, w.n, w.max_length_hint,
                           w.results ? w.results[a] : nullptr, w.counters,
                           w.conn_first_fail ? w.conn_first_fail[a] : nullptr, w.n_conns,
                           w.streams[i % w.nstreams]);
        }
        for (uint32_t s = 0; sync && s < w.nstreams; ++s)
            if (hipStreamSynchronize(static_cast<hipStream_t>(w.streams[s])) != hipSuccess && r == CTS_OK)
                r = CTS_E_HIP;
        t1[g] = secs(clk::now());
        rc[g] = r;
    };
    if (G == 1) {
        if (t_start) *t_start = secs(clk::now());
        go.store(true, std::memory_order_release);
        work(0);
        return rc[0];
    }
    std::vector<std::thread> th;
    th.reserve(G);
    for (uint32_t g = 0; g < G; ++g) th.emplace_back(work, g);
    while (ready.load(std::memory_order_acquire) < G) std::this_thread::yield();
    if (t_start) *t_start = secs(clk::now());
    go.store(true, std::memory_order_release);
    for (auto& t : th) t.join();
    for (uint32_t g = 0; g < G; ++g)
        if (rc[g] != CTS_OK) return rc[g];
    return CTS_OK;
}

}  // extern "C"
