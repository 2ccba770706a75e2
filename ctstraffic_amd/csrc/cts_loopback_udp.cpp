// cts_loopback_udp.cpp — MediaStream over loopback UDP (include/cts_loopback.h,
// cts_loopback_media_stream_run): blocking POSIX UDP sockets driving the MediaStream patterns of the
// ctsIoPattern mirror as the reference's functors drive them.
//   client (run_client): ctsMediaStreamClientConnect sends START (ctsMediaStreamClient.cpp:152-210), then the
//          receive loop posts the pattern's recv tasks and completes each datagram into the pattern
//          (:230-300, 380-420); the pattern's timer thread hands START resends and Abort / FatalAbort to the
//          registered callback, which sends or completes them (:300-340).
//   server (run_server): the listening socket's START (ctsMediaStreamServer.cpp:420-510) starts the stream;
//          ConnectedSocketIo (:510-600) sends the connection-id datagram as it is and splits every frame task
//          into datagrams stamped {flag 0, ++sequence number, QPC, QPF} ahead of g_senderSharedBuffer's bytes,
//          after the task's time offset (ctsMediaStreamServerConnectedSocket.cpp:60-140), then completes it.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <deque>
#include <system_error>
#include <thread>
#include <vector>

#include "cts_loopback.h"
#include "cts_media_stream.h"
#include "cts_teardown.hpp"

namespace {

using Clock = std::chrono::steady_clock;

uint32_t wsa_error(int err) { return err == ECONNREFUSED ? 10061u : 20000u + (uint32_t)err; }  // WSAECONNREFUSED

double thread_cpu_s()
{
    rusage u{};
    if (::getrusage(RUSAGE_THREAD, &u) != 0) return 0;
    return (double)u.ru_utime.tv_sec + (double)u.ru_stime.tv_sec + 1e-6 * (double)(u.ru_utime.tv_usec + u.ru_stime.tv_usec);
}

void recv_timeout(int fd, int ms)
{
    timeval tv{ms / 1000, (ms % 1000) * 1000};
    (void)::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

struct Conn {
    int sfd = -1, cfd = -1;  // server / client socket
    cts_io_pattern* server = nullptr;
    cts_io_pattern* client = nullptr;
    std::atomic<bool> client_done{false};
    std::atomic<int> client_status{CTS_IO_CONTINUE};
    int server_status = CTS_IO_CONTINUE;
    bool socket_error = false;
    uint64_t sent = 0, received = 0;
    double recv_cpu = 0;
    Clock::time_point end;
};

// the functor's handling of the tasks the client pattern's timers hand out
void on_client_task(void* ctx, const cts_task* t)
{
    Conn* c = static_cast<Conn*>(ctx);
    int st = CTS_IO_CONTINUE;
    if (t->io_action == CTS_TASK_SEND) {  // START resend
        const ssize_t k = ::send(c->cfd, t->buffer + t->buffer_offset, t->buffer_length, MSG_NOSIGNAL);
        st = cts_io_pattern_complete_io(c->client, t, k < 0 ? 0u : (uint32_t)k, k < 0 ? wsa_error(errno) : 0u);
    } else if (t->io_action == CTS_TASK_ABORT || t->io_action == CTS_TASK_FATAL_ABORT) {
        st = cts_io_pattern_complete_io(c->client, t, 0, 0);
    }
    if (st != CTS_IO_CONTINUE) {
        c->client_status.store(st);
        c->client_done.store(true);
    }
}

void pump(cts_io_pattern* p, std::deque<cts_task>& posted)
{
    for (;;) {
        cts_task t{};
        if (cts_io_pattern_initiate_io(p, &t) != CTS_OK || t.io_action != CTS_TASK_RECV) return;
        posted.push_back(t);
    }
}

void run_client(Conn* c)
{
    const double cpu0 = thread_cpu_s();
    std::deque<cts_task> posted;
    pump(c->client, posted);  // arms the pattern's timers (the first InitiateIo)
    static const char kStart[] = "START";
    if (::send(c->cfd, kStart, sizeof(kStart) - 1, MSG_NOSIGNAL) < 0) c->socket_error = true;
    recv_timeout(c->cfd, 20);
    while (!c->client_done.load()) {
        if (posted.empty()) {
            pump(c->client, posted);
            if (posted.empty()) {
                std::this_thread::sleep_for(std::chrono::milliseconds(1));
                continue;
            }
        }
        cts_task t = posted.front();
        const ssize_t k = ::recv(c->cfd, t.buffer + t.buffer_offset, t.buffer_length, 0);
        if (k < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) continue;  // look at client_done again
            posted.pop_front();
            const int st = cts_io_pattern_complete_io(c->client, &t, 0, wsa_error(errno));
            c->socket_error = true;
            c->client_status.store(st < 0 ? CTS_IO_FAILED : st);
            break;
        }
        posted.pop_front();
        ++c->received;
        const int st = cts_io_pattern_complete_io(c->client, &t, (uint32_t)k, 0);
        if (st != CTS_IO_CONTINUE) {
            c->client_status.store(st < 0 ? CTS_IO_FAILED : st);
            break;
        }
        pump(c->client, posted);
    }
    c->recv_cpu = thread_cpu_s() - cpu0;
    c->end = Clock::now();
}

void run_server(Conn* c, uint32_t frame, uint32_t max_dgram, bool inject, uint32_t inject_index)
{
    // the START that opens the stream (5 s at most)
    sockaddr_in from{};
    socklen_t flen = sizeof(from);
    char buf[64];
    recv_timeout(c->sfd, 100);
    const auto deadline = Clock::now() + std::chrono::seconds(5);
    bool started = false;
    while (!started && Clock::now() < deadline) {
        const ssize_t k = ::recvfrom(c->sfd, buf, sizeof(buf), 0, (sockaddr*)&from, &flen);
        started = k == 5 && std::memcmp(buf, "START", 5) == 0;
    }
    if (!started || ::connect(c->sfd, (sockaddr*)&from, flen) != 0) {
        c->socket_error = true;
        c->server_status = CTS_IO_FAILED;
        return;
    }
    std::vector<uint32_t> lens(frame / 27 + 2);
    lens.resize(cts_media_stream_split(frame, max_dgram, lens.data(), lens.size()));
    std::vector<char> scratch(max_dgram);
    int64_t sequence = 0;
    uint64_t data_index = 0;
    for (;;) {
        cts_task t{};
        if (cts_io_pattern_initiate_io(c->server, &t) != CTS_OK || t.io_action == CTS_TASK_NONE) break;
        const auto issued = Clock::now();
        uint32_t sent = 0, err = 0;
        if (t.buffer_type == CTS_BUFFER_UDP_CONNECTION_ID) {
            const ssize_t k = ::send(c->sfd, t.buffer + t.buffer_offset, t.buffer_length, MSG_NOSIGNAL);
            if (k < 0) err = wsa_error(errno);
            else sent = (uint32_t)k;
        } else {
            if (t.time_offset_ms > 0) std::this_thread::sleep_until(issued + std::chrono::milliseconds(t.time_offset_ms));
            const int64_t seq = ++sequence;
            const int64_t qpc = std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
            const int64_t qpf = 1000000000LL;
            char header[CTS_UDP_DATA_HEADER_LENGTH];
            const uint16_t flag = CTS_UDP_FLAG_DATA;
            std::memcpy(header, &flag, 2);
            std::memcpy(header + 2, &seq, 8);
            std::memcpy(header + 10, &qpc, 8);
            std::memcpy(header + 18, &qpf, 8);
            for (const uint32_t len : lens) {
                // every datagram's payload is the first bytes of the sender buffer (ctsMediaStreamProtocol.hpp:242)
                const char* payload = t.buffer;
                if (inject && data_index == inject_index) {
                    std::memcpy(scratch.data(), t.buffer, len - CTS_UDP_DATA_HEADER_LENGTH);
                    scratch[(len - CTS_UDP_DATA_HEADER_LENGTH) / 2] ^= 0x10;
                    payload = scratch.data();
                }
                iovec iov[2] = {{header, CTS_UDP_DATA_HEADER_LENGTH},
                                {const_cast<char*>(payload), len - CTS_UDP_DATA_HEADER_LENGTH}};
                msghdr m{};
                m.msg_iov = iov;
                m.msg_iovlen = 2;
                ssize_t k;
                while ((k = ::sendmsg(c->sfd, &m, MSG_NOSIGNAL)) < 0 && (errno == EINTR || errno == ENOBUFS))
                    std::this_thread::yield();
                if (k < 0) {
                    err = wsa_error(errno);
                    break;
                }
                sent += (uint32_t)k;
                ++data_index;
                ++c->sent;
            }
        }
        c->server_status = cts_io_pattern_complete_io(c->server, &t, sent, err);
        if (err != 0) c->socket_error = true;
        if (c->server_status != CTS_IO_CONTINUE) break;
    }
}

}  // namespace

extern "C" int cts_loopback_media_stream_run(const cts_media_stream_loopback_config* cfg, cts_engine* engine,
                                             cts_batch_verifier hook, void* hook_ctx,
                                             cts_media_stream_loopback_result* out)
{
    if (cfg == nullptr || out == nullptr || cfg->connections == 0 || cfg->frame_size_bytes < 40 ||
        cfg->frames_per_second == 0 || cfg->stream_length_frames == 0 || cfg->buffered_frames == 0)
        return CTS_E_INVALID;
    if (engine == nullptr && hook == nullptr && cfg->verify_buffers) return CTS_E_INVALID;
    if (cfg->verify_mode > CTS_VERIFY_DEFERRED) return CTS_E_INVALID;
    const uint32_t max_dgram = cfg->datagram_max_size ? cfg->datagram_max_size : 1400u;
    if (max_dgram <= CTS_UDP_DATA_HEADER_LENGTH || max_dgram > 65507u) return CTS_E_INVALID;
    *out = cts_media_stream_loopback_result{};
    const uint32_t n = cfg->connections;
    auto make_cfg = [&](bool listening) {
        cts_pattern_config c{};
        c.io_pattern = CTS_PATTERN_MEDIA_STREAM;
        c.protocol = CTS_PROTOCOL_UDP;
        c.listening = listening ? 1u : 0u;
        c.verify_buffers = cfg->verify_buffers;
        c.pre_post_recvs = cfg->pre_post_recvs ? cfg->pre_post_recvs : 1u;
        c.buffer_size_low = cfg->frame_size_bytes;
        c.transfer_size = (uint64_t)cfg->frame_size_bytes * cfg->stream_length_frames;
        c.verify_mode = listening ? CTS_VERIFY_SYNC : cfg->verify_mode;
        c.ms_frames_per_second = cfg->frames_per_second;
        c.ms_datagram_max_size = max_dgram;
        c.ms_buffered_frames = cfg->buffered_frames;
        c.ms_stream_length_frames = cfg->stream_length_frames;
        c.batch_buffers = listening ? 0u : cfg->batch_buffers;
        return c;
    };
    std::vector<Conn> conns(n);
    int rc = CTS_OK;
    for (uint32_t i = 0; i < n && rc == CTS_OK; ++i) {
        const cts_pattern_config sc = make_cfg(true), cc = make_cfg(false);
        rc = cts_io_pattern_create(&sc, engine, &conns[i].server);
        if (rc == CTS_OK) rc = cts_io_pattern_create(&cc, engine, &conns[i].client);
        if (rc == CTS_OK && hook != nullptr) rc = cts_io_pattern_set_verifier(conns[i].server, hook, hook_ctx);
        if (rc == CTS_OK && hook != nullptr) rc = cts_io_pattern_set_verifier(conns[i].client, hook, hook_ctx);
        if (rc == CTS_OK) rc = cts_io_pattern_register_callback(conns[i].client, on_client_task, &conns[i]);
    }
    // one UDP socket pair per connection on 127.0.0.1: the client connects to its server's port
    const int sbuf = (int)(cfg->socket_buffer_bytes ? cfg->socket_buffer_bytes : (8u << 20));
    for (uint32_t i = 0; i < n && rc == CTS_OK; ++i) {
        Conn& c = conns[i];
        c.sfd = ::socket(AF_INET, SOCK_DGRAM, 0);
        c.cfd = ::socket(AF_INET, SOCK_DGRAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        socklen_t alen = sizeof(a);
        if (c.sfd < 0 || c.cfd < 0 || ::bind(c.sfd, (sockaddr*)&a, sizeof(a)) != 0 ||
            ::getsockname(c.sfd, (sockaddr*)&a, &alen) != 0 || ::connect(c.cfd, (sockaddr*)&a, sizeof(a)) != 0) {
            rc = CTS_E_INVALID;
            break;
        }
        for (const int fd : {c.sfd, c.cfd}) {
            (void)::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sbuf, sizeof(sbuf));
            (void)::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &sbuf, sizeof(sbuf));
        }
    }
    if (rc == CTS_OK) {
        cts_udp_status_details before{};
        (void)cts_udp_status_details_read(&before);
        std::vector<std::thread> threads;
        const auto t0 = Clock::now();
        threads.reserve(2 * n);
        for (uint32_t i = 0; i < n; ++i) {
            // a side whose thread cannot start fails its connection, never std::terminate: a server without its
            // client gives up on START after 5 s; a client without its server drops every frame and finishes
            try {
                threads.emplace_back(run_server, &conns[i], cfg->frame_size_bytes, max_dgram,
                                     i == cfg->corrupt_connection, cfg->corrupt_datagram);
            } catch (const std::system_error&) {
                conns[i].socket_error = true;
                conns[i].server_status = CTS_IO_FAILED;
            }
            try {
                threads.emplace_back(run_client, &conns[i]);
            } catch (const std::system_error&) {
                // (the server thread may be running: nothing is written here; client_status never reaches
                // CTS_IO_COMPLETED, so the connection counts as failed)
            }
        }
        for (auto& t : threads) t.join();
        auto t1 = t0;
        for (const Conn& c : conns) t1 = std::max(t1, c.end);
        out->seconds = std::chrono::duration<double>(t1 - t0).count();
        for (Conn& c : conns) {
            const int st = c.client_status.load();
            const uint32_t le = cts_io_pattern_last_error(c.client);
            if (st == CTS_IO_COMPLETED && !c.socket_error) ++out->connections_ok;
            else ++out->connections_failed;
            if (le == CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN) ++out->data_errors;
            out->datagrams_sent += c.sent;
            out->datagrams_received += c.received;
            out->recv_cpu_seconds += c.recv_cpu;
            cts_media_stream_stats s{};
            if (cts_io_pattern_media_stream_stats(c.client, &s) == CTS_OK) {
                out->clients.bits_received += s.bits_received;
                out->clients.successful_frames += s.successful_frames;
                out->clients.dropped_frames += s.dropped_frames;
                out->clients.duplicate_frames += s.duplicate_frames;
                out->clients.error_frames += s.error_frames;
                out->clients.datagrams += s.datagrams;
            }
        }
    }
    for (Conn& c : conns) {
        // (the client's timer thread is stopped by its first destroy call); a teardown failure fails a run that
        // had not failed already
        const int dc = cts::destroy_pattern(c.client), ds = cts::destroy_pattern(c.server);
        if (rc == CTS_OK) rc = dc != CTS_OK ? dc : ds;
        if (c.sfd >= 0) ::close(c.sfd);
        if (c.cfd >= 0) ::close(c.cfd);
    }
    return rc;
}
