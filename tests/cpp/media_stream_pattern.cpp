// media_stream_pattern.cpp — the MediaStream patterns of the ctsIoPattern mirror (cts_pattern.cpp) under the
// sanitizers. Each run pairs a server pattern with a client pattern, as ctsMediaStreamServer and ctsMediaStreamClient
// drive them: the server's connection-id datagram and frame tasks become the client's datagrams (split by
// cts_media_stream_split, header + sender-buffer payload, a few dropped or repeated), delivered by a receive thread
// while the client's own timer thread runs StartCallback / TimerCallback on the real clock and hands Abort to the
// registered callback, which completes it from inside the callback (the reference functor's re-entrant path). Several
// connections run at once, so TSan sees the timer threads, the receive threads and the pattern locks together; a
// corrupt payload must fail its stream with DATA_DID_NOT_MATCH. The oracle's C verifier is every pattern's hook.
// Built with g++ against tests/cpp/engine_stub.cpp; run by tests/test_host_sanitizers.py.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "cts_loopback.h"
#include "cts_media_stream.h"
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

constexpr uint32_t kFrame = 3000, kMaxDgram = 1400, kFps = 200, kFrames = 12;

cts_pattern_config config(bool listening, uint32_t mode = CTS_VERIFY_SYNC)
{
    cts_pattern_config c{};
    c.io_pattern = CTS_PATTERN_MEDIA_STREAM;
    c.protocol = CTS_PROTOCOL_UDP;
    c.listening = listening ? 1 : 0;
    c.verify_buffers = 1;
    c.pre_post_recvs = 2;
    c.buffer_size_low = kFrame;
    c.transfer_size = (uint64_t)kFrame * kFrames;
    c.verify_mode = mode;
    c.batch_buffers = 5;  // DEFERRED: small batches, so batches fill between ticks as well as at them
    c.ms_frames_per_second = kFps;
    c.ms_datagram_max_size = kMaxDgram;
    c.ms_buffered_frames = kFrames;  // the whole stream fits the jitter window
    c.ms_stream_length_frames = kFrames;
    return c;
}

struct Conn {
    cts_io_pattern* client = nullptr;
    std::atomic<int> finished{0};  // the status CompleteIo(Abort / FatalAbort) returned + 1
};

void on_task(void* ctx, const cts_task* t)
{
    Conn* c = static_cast<Conn*>(ctx);
    if (t->io_action == CTS_TASK_ABORT || t->io_action == CTS_TASK_FATAL_ABORT) {
        const int st = cts_io_pattern_complete_io(c->client, t, 0, 0);  // from inside the callback
        c->finished.store(st + 1);
    } else if (t->io_action == CTS_TASK_SEND) {
        CHECK(t->buffer_length == 5 && std::memcmp(t->buffer, "START", 5) == 0);
        CHECK(cts_io_pattern_complete_io(c->client, t, 5, 0) == CTS_IO_CONTINUE);
    }
}

// one connection: returns the client's final cts_io_status; `corrupt` flips one payload byte of one datagram
int run_connection(uint64_t seed, bool corrupt, uint32_t mode)
{
    std::mt19937_64 rng(seed);
    cts_pattern_config sc = config(true), cc = config(false, mode);
    cts_io_pattern *server = nullptr, *client = nullptr;
    CHECK(cts_io_pattern_create(&sc, nullptr, &server) == CTS_OK);
    CHECK(cts_io_pattern_set_verifier(server, reinterpret_cast<cts_batch_verifier>(ora_batch_verifier), nullptr) == CTS_OK);
    CHECK(cts_io_pattern_create(&cc, nullptr, &client) == CTS_OK);
    CHECK(cts_io_pattern_set_verifier(client, reinterpret_cast<cts_batch_verifier>(ora_batch_verifier), nullptr) == CTS_OK);
    Conn conn;
    conn.client = client;
    CHECK(cts_io_pattern_register_callback(client, on_task, &conn) == CTS_OK);

    // the server's datagrams: the connection id, then every frame split into data datagrams
    std::vector<std::vector<char>> wire;
    cts_task t{};
    CHECK(cts_io_pattern_initiate_io(server, &t) == CTS_OK && t.buffer_type == CTS_BUFFER_UDP_CONNECTION_ID);
    wire.emplace_back(t.buffer, t.buffer + t.buffer_length);
    CHECK(cts_io_pattern_complete_io(server, &t, t.buffer_length, 0) == CTS_IO_CONTINUE);
    uint32_t lens[8];
    const uint64_t per = cts_media_stream_split(kFrame, kMaxDgram, lens, 8);
    CHECK(per > 0 && per <= 8);
    for (uint32_t f = 1; f <= kFrames; ++f) {
        CHECK(cts_io_pattern_initiate_io(server, &t) == CTS_OK && t.io_action == CTS_TASK_SEND);
        CHECK(t.buffer_length == kFrame);
        for (uint64_t k = 0; k < per; ++k) {
            std::vector<char> d(lens[k]);
            const uint16_t flag = CTS_UDP_FLAG_DATA;
            const int64_t h[3] = {(int64_t)f, 0, 0};
            std::memcpy(d.data(), &flag, 2);
            std::memcpy(d.data() + 2, h, sizeof h);
            std::memcpy(d.data() + 26, t.buffer, lens[k] - 26);  // the frame's payload: the sender buffer's base
            const uint32_t r = (uint32_t)(rng() % 100);
            if (r < 3) continue;  // dropped
            wire.push_back(d);
            if (r > 97) wire.push_back(d);  // repeated
        }
        CHECK(cts_io_pattern_complete_io(server, &t, kFrame, 0) == (f == kFrames ? CTS_IO_COMPLETED : CTS_IO_CONTINUE));
    }
    if (corrupt) wire[wire.size() / 2][26 + rng() % 100] ^= 0x21;

    // the client: a receive thread posts recvs and completes them with the wire's datagrams
    std::thread rx([&] {
        std::vector<cts_task> posted;
        for (int i = 0; i < 2; ++i) {
            cts_task r{};
            CHECK(cts_io_pattern_initiate_io(client, &r) == CTS_OK && r.io_action == CTS_TASK_RECV);
            posted.push_back(r);
        }
        for (size_t i = 0; i < wire.size() && !posted.empty(); ++i) {
            cts_task r = posted.front();
            posted.erase(posted.begin());
            CHECK(wire[i].size() <= r.buffer_length);
            std::memcpy(r.buffer, wire[i].data(), wire[i].size());
            const int st = cts_io_pattern_complete_io(client, &r, (uint32_t)wire[i].size(), 0);
            CHECK(st >= 0);
            if (st != CTS_IO_CONTINUE) break;
            cts_task n{};
            CHECK(cts_io_pattern_initiate_io(client, &n) == CTS_OK);
            if (n.io_action == CTS_TASK_RECV) posted.push_back(n);
            if (i % 7 == 0) std::this_thread::sleep_for(std::chrono::microseconds(200));
        }
    });
    rx.join();
    int status = CTS_IO_CONTINUE;
    if (cts_io_pattern_last_error(client) == CTS_STATUS_IO_RUNNING) {
        // the renderer finishes the stream on its own (kFrames frames at 5 ms) and hands Abort to the callback
        const auto t0 = std::chrono::steady_clock::now();
        while (conn.finished.load() == 0) {
            CHECK(std::chrono::steady_clock::now() - t0 < std::chrono::seconds(20));
            std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
        status = conn.finished.load() - 1;
        cts_media_stream_stats s{};
        CHECK(cts_io_pattern_media_stream_stats(client, &s) == CTS_OK);
        CHECK(s.finished == 1 && s.last_error == 0);
        CHECK(s.successful_frames + s.dropped_frames + s.duplicate_frames == kFrames);
    } else {
        status = CTS_IO_FAILED;
        CHECK(cts_io_pattern_last_error(client) == CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN);
    }
    cts_io_pattern_destroy(client);  // joins the timer thread
    cts_io_pattern_destroy(server);
    return status;
}

}  // namespace

int main()
{
    std::vector<uint8_t> sender(ora_sender_buffer_size(kFrame));
    ora_build_sender_buffer(sender.data(), kFrame);
    CHECK(cts_shared_buffer_attach(sender.data(), sender.size()) == CTS_OK);
    cts_udp_status_details_reset();
    std::vector<std::thread> conns;
    std::atomic<int> completed{0}, failed{0};
    for (int c = 0; c < 6; ++c)
        conns.emplace_back([&, c] {
            // connections alternate per-datagram (SYNC) and batched (DEFERRED) verify
            const int st = run_connection(0xC0FFEEull + (uint64_t)c, c >= 4,
                                          c % 2 ? (uint32_t)CTS_VERIFY_DEFERRED : (uint32_t)CTS_VERIFY_SYNC);
            (st == CTS_IO_COMPLETED ? completed : failed).fetch_add(1);
        });
    for (auto& th : conns) th.join();
    CHECK(completed.load() == 4 && failed.load() == 2);
    cts_udp_status_details u{};
    CHECK(cts_udp_status_details_read(&u) == CTS_OK && u.successful_frames > 0);
    // the same over loopback UDP sockets (cts_loopback_udp.cpp): server and client threads per connection, the
    // clients' timer threads, one corrupt datagram
    cts_media_stream_loopback_config lc{};
    lc.connections = 3;
    lc.frame_size_bytes = kFrame;
    lc.frames_per_second = kFps;
    lc.stream_length_frames = 20;
    lc.buffered_frames = 10;
    lc.pre_post_recvs = 2;
    lc.verify_buffers = 1;
    lc.corrupt_connection = 2;
    lc.corrupt_datagram = 9;
    for (const uint32_t mode : {(uint32_t)CTS_VERIFY_SYNC, (uint32_t)CTS_VERIFY_DEFERRED}) {
        lc.verify_mode = mode;
        cts_media_stream_loopback_result lr{};
        CHECK(cts_loopback_media_stream_run(&lc, nullptr, reinterpret_cast<cts_batch_verifier>(ora_batch_verifier),
                                            nullptr, &lr) == CTS_OK);
        CHECK(lr.connections_ok == 2 && lr.connections_failed == 1 && lr.data_errors == 1);
    }
    cts_shared_buffer_release();
    std::puts("media_stream_pattern: ok");
    return 0;
}
