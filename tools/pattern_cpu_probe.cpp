// pattern_cpu_probe.cpp — receive-thread CPU inside the ctsIoPattern calls, without sockets: a Push server
// pattern (ctsIOPattern.cpp:796-886) receives `gib` GiB in 64 KiB completions whose bytes are copied from the
// shared sender buffer (the copy stands in for recv(); it is timed on its own: copy_cpu_s_per_GiB). Every cts_io_pattern_initiate_io and
// cts_io_pattern_complete_io call is bracketed with CLOCK_THREAD_CPUTIME_ID; completions that took more than
// 20 us are tallied apart (the DEFERRED batch rotations: retire + launch). One JSON line per run.
//   build: make tools/pattern_cpu_probe
//   run:   tools/pattern_cpu_probe {sync|deferred|off} [gib [batch_buffers [threads]]]
// threads > 1: that many connections at once, one thread and one pattern each (the loopback feeder's shape,
// without its sockets); the figures are summed over the threads.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <thread>
#include <vector>

#include "cts_engine.h"
#include "cts_pattern.h"

static double cpu_now()
{
    timespec ts{};
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

static double wall_now()
{
    timespec ts{};
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

struct Run {
    double t_init = 0, t_complete = 0, t_slow = 0, t_copy = 0;
    uint64_t n_complete = 0, n_slow = 0, recvs = 0, bytes = 0, verified = 0;
    int st = CTS_IO_CONTINUE;
    uint32_t last_error = 0;
};

static void run_one(cts_engine* e, const char* mode, uint64_t gib, uint32_t batch, Run* out)
{
    const uint32_t buf = 65536;
    Run& r = *out;
    cts_pattern_config c{};
    c.io_pattern = CTS_PATTERN_PUSH;
    c.protocol = CTS_PROTOCOL_TCP;
    c.listening = 1;
    c.verify_buffers = std::strcmp(mode, "off") != 0;
    c.verify_mode = std::strcmp(mode, "sync") == 0 ? CTS_VERIFY_SYNC : CTS_VERIFY_DEFERRED;
    c.batch_buffers = batch;
    c.pre_post_recvs = 1;
    c.pre_post_sends = 1;
    c.buffer_size_low = buf;
    c.tcp_shutdown = CTS_SHUTDOWN_GRACEFUL;
    c.transfer_size = gib << 30;
    cts_io_pattern* p = nullptr;
    if (cts_io_pattern_create(&c, e, &p) != CTS_OK) {
        r.st = -1;
        return;
    }
    const char* sender = cts_shared_buffer();
    while (r.st == CTS_IO_CONTINUE) {
        cts_task t{};
        double c0 = cpu_now();
        if (cts_io_pattern_initiate_io(p, &t) != CTS_OK) {
            r.st = CTS_IO_FAILED;
            break;
        }
        r.t_init += cpu_now() - c0;
        uint32_t done = t.buffer_length;
        if (t.io_action == CTS_TASK_RECV) {
            if (r.bytes >= c.transfer_size) {
                done = 0;  // the transfer is in: the client's FIN after the server's DONE
            } else {
                const double m0 = cpu_now();
                std::memcpy(t.buffer + t.buffer_offset, sender + t.expected_pattern_offset, t.buffer_length);
                r.t_copy += cpu_now() - m0;
                ++r.recvs;
                r.bytes += t.buffer_length;
            }
        } else if (t.io_action == CTS_TASK_NONE) {
            r.st = cts_io_pattern_flush(p);
            break;
        }
        c0 = cpu_now();
        r.st = cts_io_pattern_complete_io(p, &t, done, 0);
        const double dt = cpu_now() - c0;
        r.t_complete += dt;
        ++r.n_complete;
        if (dt > 20e-6) {
            r.t_slow += dt;
            ++r.n_slow;
        }
    }
    cts_pattern_stats s{};
    (void)cts_io_pattern_get_stats(p, &s);
    r.verified = s.buffers_verified;
    r.last_error = cts_io_pattern_last_error(p);
    cts_io_pattern_destroy(p);
}

int main(int argc, char** argv)
{
    const char* mode = argc > 1 ? argv[1] : "deferred";
    const uint64_t gib = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1;
    const uint32_t batch = argc > 3 ? (uint32_t)std::strtoul(argv[3], nullptr, 10) : 0;
    const uint32_t buf = 65536;
    cts_engine* e = nullptr;
    if (cts_engine_create(0, &e) != CTS_OK) {
        std::fprintf(stderr, "engine\n");
        return 1;
    }
    if (cts_shared_buffer_init(e, buf) != CTS_OK) {
        std::fprintf(stderr, "shared buffer\n");
        return 1;
    }
    const uint32_t threads = argc > 4 ? (uint32_t)std::strtoul(argv[4], nullptr, 10) : 1;
    std::vector<Run> runs(threads);
    const double w0 = wall_now();
    {
        std::vector<std::thread> ts;
        for (uint32_t i = 0; i < threads; ++i) ts.emplace_back(run_one, e, mode, gib, batch, &runs[i]);
        for (auto& t : ts) t.join();
    }
    const double wall = wall_now() - w0;
    Run r;
    int st = CTS_IO_COMPLETED;
    for (const Run& x : runs) {
        r.t_init += x.t_init;
        r.t_complete += x.t_complete;
        r.t_slow += x.t_slow;
        r.t_copy += x.t_copy;
        r.n_complete += x.n_complete;
        r.n_slow += x.n_slow;
        r.recvs += x.recvs;
        r.bytes += x.bytes;
        r.verified += x.verified;
        if (x.st != CTS_IO_COMPLETED) st = x.st;
        if (x.last_error != 0) r.last_error = x.last_error;
    }
    const double g = (double)r.bytes / (double)(1ull << 30);
    std::printf("{\"mode\": \"%s\", \"batch_buffers\": %u, \"threads\": %u, \"status\": %d, \"last_error\": %u, "
                "\"recvs\": %llu, \"buffers_verified\": %llu, \"wall_s\": %.4f, \"initiate_cpu_s_per_GiB\": %.5f, "
                "\"complete_cpu_s_per_GiB\": %.5f, \"complete_us_mean\": %.3f, \"slow_completes\": %llu, "
                "\"slow_cpu_s_per_GiB\": %.5f, \"complete_us_mean_fast\": %.3f, \"copy_cpu_s_per_GiB\": %.5f}\n",
                mode, batch, threads, st, r.last_error, (unsigned long long)r.recvs, (unsigned long long)r.verified,
                wall, r.t_init / g, r.t_complete / g, 1e6 * r.t_complete / (double)r.n_complete,
                (unsigned long long)r.n_slow, r.t_slow / g,
                1e6 * (r.t_complete - r.t_slow) / (double)(r.n_complete - r.n_slow), r.t_copy / g);
    cts_shared_buffer_release();
    cts_engine_destroy(e);
    return st == CTS_IO_COMPLETED ? 0 : 2;
}
