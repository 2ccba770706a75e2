// thread_start_failure.cpp — no C++ exception crosses the C ABI when a thread cannot start. This program defines
// pthread_create itself (it interposes on libc's for libstdc++'s std::thread), fails it on demand with EAGAIN, and
// drives every host component that starts a thread:
//   - the MediaStream client's timer thread (its first InitiateIo): a latched FAIL_FAST, no timer left armed, later
//     calls fail instead of rendering nothing forever;
//   - the TCP loopback feeder's side threads and the UDP feeder's threads: their connections fail, the run returns.
// Built with g++ against tests/cpp/engine_stub.cpp (no sanitizer: the sanitizers intercept pthread_create
// themselves); run by tests/test_host_sanitizers.py.
#include <dlfcn.h>
#include <pthread.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "cts_loopback.h"
#include "cts_oracle.h"
#include "cts_pattern.h"

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

namespace {
std::atomic<int> g_fail{0};
std::atomic<int> g_refused{0};
}  // namespace

extern "C" int pthread_create(pthread_t* t, const pthread_attr_t* a, void* (*fn)(void*), void* arg)
{
    using real_fn = int (*)(pthread_t*, const pthread_attr_t*, void* (*)(void*), void*);
    static real_fn real = reinterpret_cast<real_fn>(dlsym(RTLD_NEXT, "pthread_create"));
    if (g_fail.load()) {
        g_refused.fetch_add(1);
        return EAGAIN;
    }
    return real(t, a, fn, arg);
}

namespace {

cts_pattern_config ms_client(uint32_t mode)
{
    cts_pattern_config c{};
    c.io_pattern = CTS_PATTERN_MEDIA_STREAM;
    c.protocol = CTS_PROTOCOL_UDP;
    c.verify_buffers = 1;
    c.pre_post_recvs = 2;
    c.buffer_size_low = 3000;
    c.transfer_size = 3000ull * 10;
    c.verify_mode = mode;
    c.ms_frames_per_second = 100;
    c.ms_datagram_max_size = 1400;
    c.ms_buffered_frames = 4;
    c.ms_stream_length_frames = 10;
    return c;
}

void media_stream_client_timer_thread(uint32_t mode)
{
    const cts_pattern_config c = ms_client(mode);
    cts_io_pattern* p = nullptr;
    CHECK(cts_io_pattern_create(&c, nullptr, &p) == CTS_OK);
    CHECK(cts_io_pattern_set_verifier(p, reinterpret_cast<cts_batch_verifier>(ora_batch_verifier), nullptr) == CTS_OK);
    const int refused = g_refused.load();
    g_fail = 1;
    cts_task t{};
    const int rc = cts_io_pattern_initiate_io(p, &t);  // starts the timers: std::system_error inside
    g_fail = 0;
    CHECK(rc == CTS_OK);
    CHECK(g_refused.load() == refused + 1);
    CHECK(t.io_action == CTS_TASK_NONE);
    CHECK(cts_io_pattern_last_error(p) == CTS_PATTERN_E_FAIL_FAST);
    const char* why = cts_io_pattern_fail_fast_reason(p);
    CHECK(why != nullptr && std::string(why).find("timer thread") != std::string::npos);
    int64_t start_due = 0, render_due = 0;
    CHECK(cts_io_pattern_media_stream_timers(p, &start_due, &render_due) == CTS_OK);
    CHECK(start_due == -1 && render_due == -1);  // nothing armed that no thread would ever fire
    // the latch holds: no task, every completion fails
    CHECK(cts_io_pattern_initiate_io(p, &t) == CTS_OK && t.io_action == CTS_TASK_NONE);
    cts_task r{};
    r.io_action = CTS_TASK_RECV;
    CHECK(cts_io_pattern_complete_io(p, &r, 0, 0) == CTS_IO_FAILED);
    CHECK(cts_io_pattern_destroy(p) == CTS_OK);  // no thread to join
}

void tcp_feeder()
{
    cts_loopback_config c{};
    c.connections = 2;
    c.io_pattern = CTS_PATTERN_PUSH;
    c.buffer_size = 4096;
    c.verify_buffers = 1;
    c.transfer_size = 1 << 20;
    c.corrupt_connection = ~0u;
    for (const uint32_t functor : {(uint32_t)CTS_LOOPBACK_FUNCTOR_SYNC, (uint32_t)CTS_LOOPBACK_FUNCTOR_ASYNC}) {
        c.functor = functor;
        cts_loopback_result r{};
        g_fail = 1;
        const int rc = cts_loopback_run(&c, nullptr, reinterpret_cast<cts_batch_verifier>(ora_batch_verifier), nullptr, &r);
        g_fail = 0;
        CHECK(rc == CTS_OK);
        CHECK(r.connections_ok == 0 && r.connections_failed == 2);
        // and the feeder still works once threads can start again
        r = cts_loopback_result{};
        CHECK(cts_loopback_run(&c, nullptr, reinterpret_cast<cts_batch_verifier>(ora_batch_verifier), nullptr, &r) ==
              CTS_OK);
        CHECK(r.connections_ok == 2 && r.connections_failed == 0);
    }
}

void udp_feeder()
{
    cts_media_stream_loopback_config c{};
    c.connections = 2;
    c.frame_size_bytes = 3000;
    c.frames_per_second = 200;
    c.stream_length_frames = 10;
    c.buffered_frames = 5;
    c.verify_buffers = 1;
    c.corrupt_connection = ~0u;
    cts_media_stream_loopback_result r{};
    g_fail = 1;
    const int rc =
        cts_loopback_media_stream_run(&c, nullptr, reinterpret_cast<cts_batch_verifier>(ora_batch_verifier), nullptr, &r);
    g_fail = 0;
    CHECK(rc == CTS_OK);
    CHECK(r.connections_ok == 0 && r.connections_failed == 2);
}

}  // namespace

int main()
{
    std::vector<uint8_t> sender(ora_sender_buffer_size(65536));
    ora_build_sender_buffer(sender.data(), 65536);
    CHECK(cts_shared_buffer_attach(sender.data(), sender.size()) == CTS_OK);
    // the interposer is the one std::thread reaches
    g_fail = 1;
    bool threw = false;
    try {
        std::thread([] {}).join();
    } catch (const std::system_error&) {
        threw = true;
    }
    g_fail = 0;
    CHECK(threw);
    media_stream_client_timer_thread(CTS_VERIFY_SYNC);
    media_stream_client_timer_thread(CTS_VERIFY_DEFERRED);
    tcp_feeder();
    udp_feeder();
    cts_shared_buffer_release();
    std::puts("thread_start_failure: ok");
    return 0;
}
