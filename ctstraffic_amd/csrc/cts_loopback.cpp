// cts_loopback.cpp — loopback-TCP feeder (include/cts_loopback.h): blocking
// POSIX sockets driving a cts_io_pattern exactly as the reference's IOCP functor
// drives ctsIoPattern: InitiateIo -> post the IO -> CompleteIo(task, transferred,
// status) (ctsTraffic/ctsSendRecvIocp.cpp:130-300, 335-415).
//   sync functor  (run_side): one thread per connection side, one IO at a time
//                 (PrePostRecvs = PrePostSends = 1, what -Verify:data requires for
//                 TCP, ctsConfig.cpp:3440-3446) — Push, Pull, PushPull.
//   async functor (AsyncSide): a send thread and a recv thread per side, so a send
//                 and a recv are in flight together (Duplex). Completions run under
//                 the connection's lock and re-pump InitiateIo until it returns
//                 None, as ctsSendRecvCompletionCallback / ctsSendRecvIocp do
//                 (:47-127, :335-415); the side is done when its IO count drops to 0.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <ctime>
#include <deque>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

#include "cts_loopback.h"
#include "cts_teardown.hpp"

namespace {

// Winsock codes the pattern's state machine distinguishes (ctsIOPatternState.hpp:269-275)
uint32_t wsa_status(int err)
{
    switch (err) {
    case ECONNRESET: return 10054;    // WSAECONNRESET
    case ECONNABORTED: return 10053;  // WSAECONNABORTED
    case ETIMEDOUT: return 10060;     // WSAETIMEDOUT
    case EPIPE: return 10054;
    default: return 20000u + (uint32_t)err;
    }
}

// returns 0 or a wsa_status
// A send the pattern deferred (rate limit / burst delay: ctsTask::m_timeOffsetMilliseconds) goes out that
// many ms later, as ctsSendRecvIocp.cpp:378-383 schedules it on the socket's threadpool timer.
void pace(const cts_task& t)
{
    if (t.time_offset_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(t.time_offset_ms));
}

uint32_t send_all(int fd, const char* p, uint32_t n)
{
    while (n > 0) {
        const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            return wsa_status(errno);
        }
        p += k;
        n -= (uint32_t)k;
    }
    return 0;
}

// one recv (partial completions are part of the path: they shift the next buffer's phase)
uint32_t recv_some(int fd, char* p, uint32_t n, uint32_t* got, bool wait_all)
{
    *got = 0;
    for (;;) {
        const ssize_t k = ::recv(fd, p + *got, n - *got, 0);
        if (k < 0) {
            if (errno == EINTR) continue;
            return wsa_status(errno);
        }
        *got += (uint32_t)k;
        if (k == 0 || !wait_all || *got == n) return 0;
    }
}

struct SideResult {
    int status = CTS_IO_FAILED;
    uint32_t last_error = 0;
    cts_pattern_stats stats{};
    double recv_cpu_s = 0;  // CPU time (user + sys) of the thread that ran this side's recvs
    double send_cpu_s = 0;  // ... and of its send thread (the same thread in the sync functor)
    double recv_io_cpu_s = 0;  // the part of recv_cpu_s spent inside the socket calls (send/recv syscalls)
};

// this thread's CPU seconds so far (user + system)
double thread_cpu_s()
{
    rusage u{};
    if (::getrusage(RUSAGE_THREAD, &u) != 0) return 0;
    return (double)u.ru_utime.tv_sec + (double)u.ru_utime.tv_usec * 1e-6 + (double)u.ru_stime.tv_sec +
           (double)u.ru_stime.tv_usec * 1e-6;
}

// the same at nanosecond resolution, cheap enough to bracket every socket call (one clock_gettime)
double thread_cpu_ns_s()
{
    timespec ts{};
    if (::clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts) != 0) return 0;
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

// The diagnostic recv ring (cts_loopback_config.recv_ring_buffers): data recvs land in its slots round robin.
struct RecvRing {
    char* base = nullptr;
    uint32_t slots = 0, slot_bytes = 0, next = 0;
    char* take() { return base + (size_t)(next++ % slots) * slot_bytes; }
};

void run_side(int* fdslot, cts_io_pattern* p, bool inject, uint32_t inject_index, bool recv_whole, SideResult* out,
              RecvRing ring = {})
{
    const double cpu0 = thread_cpu_s();
    const int fd = *fdslot;
    std::vector<char> scratch;
    uint32_t data_sends = 0;
    int st = CTS_IO_CONTINUE;
    double io_cpu = 0;  // CPU inside the socket calls; the rest of the thread's time is the pattern's
    for (;;) {
        cts_task t{};
        if (cts_io_pattern_initiate_io(p, &t) != CTS_OK) {
            st = CTS_IO_FAILED;
            break;
        }
        uint32_t transferred = 0, status = 0;
        switch (t.io_action) {
        case CTS_TASK_SEND: {
            pace(t);
            const char* src = t.buffer + t.buffer_offset;
            if (inject && t.track_io && data_sends++ == inject_index && t.buffer_length > 0) {
                scratch.assign(src, src + t.buffer_length);  // fault injection: one flipped byte on the wire
                scratch[t.buffer_length / 2] ^= 0x5A;
                src = scratch.data();
            }
            const double c0 = thread_cpu_ns_s();
            status = send_all(fd, src, t.buffer_length);
            io_cpu += thread_cpu_ns_s() - c0;
            transferred = status == 0 ? t.buffer_length : 0;
            break;
        }
        case CTS_TASK_RECV: {
            // protocol messages are fixed-size; data recvs complete with whatever arrived
            // (or, with recv_whole, with the whole posted length: deterministic completions)
            const bool whole = recv_whole || t.buffer_type == CTS_BUFFER_TCP_CONNECTION_ID ||
                               t.buffer_type == CTS_BUFFER_COMPLETION_MESSAGE;
            char* dst = t.buffer + t.buffer_offset;
            if (ring.base != nullptr && t.buffer_type == CTS_BUFFER_DYNAMIC && t.track_io &&
                t.buffer_length <= ring.slot_bytes)
                dst = ring.take();  // verify is off: the pattern never reads the bytes
            const double c0 = thread_cpu_ns_s();
            status = recv_some(fd, dst, t.buffer_length, &transferred, whole);
            io_cpu += thread_cpu_ns_s() - c0;
            break;
        }
        case CTS_TASK_GRACEFUL_SHUTDOWN:
            if (::shutdown(fd, SHUT_WR) != 0) status = wsa_status(errno);
            break;
        case CTS_TASK_HARD_SHUTDOWN: {
            linger l{1, 0};  // RST on close
            (void)::setsockopt(fd, SOL_SOCKET, SO_LINGER, &l, sizeof(l));
            break;
        }
        case CTS_TASK_NONE:
            // one IO at a time: nothing to post means the pattern is waiting on nothing -> done
            break;
        default: break;
        }
        if (t.io_action == CTS_TASK_NONE) {
            st = cts_io_pattern_flush(p);
            break;
        }
        st = cts_io_pattern_complete_io(p, &t, transferred, status);
        if (st != CTS_IO_CONTINUE) break;
    }
    // the side closes its socket as soon as its pattern is done (ctsSocketState
    // Closing, ctsSocketState.cpp:213-264): gracefully after CompletedIo — the
    // peer may still be waiting for this FIN — and with RST after a failure, which
    // unblocks a peer stuck in send/recv
    if (st != CTS_IO_COMPLETED) {
        linger l{1, 0};
        (void)::setsockopt(fd, SOL_SOCKET, SO_LINGER, &l, sizeof(l));
    }
    ::close(fd);
    *fdslot = -1;
    out->status = st;
    out->last_error = cts_io_pattern_last_error(p);
    (void)cts_io_pattern_get_stats(p, &out->stats);
    out->recv_cpu_s = out->send_cpu_s = thread_cpu_s() - cpu0;  // one thread runs both directions
    out->recv_io_cpu_s = io_cpu;
}

// ---- async functor (Duplex): one send and one recv thread per connection side -----------------
struct AsyncSide {
    int fd;
    cts_io_pattern* p;
    bool inject;
    uint32_t inject_index;
    bool recv_whole = false;
    uint32_t data_sends = 0;
    std::mutex mu;  // the ctsSocket lock: every pattern call runs under it (ctsSocket.h:189)
    std::condition_variable cv;
    std::deque<cts_task> sends, recvs;
    uint32_t io = 0;       // posted IOs + the pump's own hold (sharedSocket->IncrementIo)
    bool finished = false; // io dropped to 0 (CompleteState)
    bool aborted = false;  // the pattern failed: queued IO completes as aborted, blocked IO is unblocked
    int status = CTS_IO_CONTINUE;

    void fail_socket()
    {
        aborted = true;
        (void)::shutdown(fd, SHUT_RDWR);  // wakes a send/recv blocked in the other thread
    }
    void on_status(int st)
    {
        if (st == CTS_IO_FAILED) {
            status = CTS_IO_FAILED;
            fail_socket();
        } else if (st == CTS_IO_COMPLETED && status != CTS_IO_FAILED) {
            status = CTS_IO_COMPLETED;
        }
    }
    void release()  // DecrementIo; at 0 the side is done
    {
        if (--io == 0) {
            finished = true;
            cv.notify_all();
        }
    }
    // ctsSendRecvIocp (:335-415): post IO until InitiateIo returns None. Shutdown tasks run inline.
    void pump()
    {
        ++io;
        while (!aborted) {
            cts_task t{};
            if (cts_io_pattern_initiate_io(p, &t) != CTS_OK) {
                on_status(CTS_IO_FAILED);
                break;
            }
            if (t.io_action == CTS_TASK_NONE) break;
            if (t.io_action == CTS_TASK_SEND || t.io_action == CTS_TASK_RECV) {
                (t.io_action == CTS_TASK_SEND ? sends : recvs).push_back(t);
                ++io;
                cv.notify_all();
                continue;
            }
            uint32_t err = 0;
            if (t.io_action == CTS_TASK_GRACEFUL_SHUTDOWN) {
                if (::shutdown(fd, SHUT_WR) != 0) err = wsa_status(errno);
            } else if (t.io_action == CTS_TASK_HARD_SHUTDOWN) {
                linger l{1, 0};  // RST on close
                (void)::setsockopt(fd, SOL_SOCKET, SO_LINGER, &l, sizeof(l));
            }
            const int st = cts_io_pattern_complete_io(p, &t, 0, err);
            on_status(st);
            if (st != CTS_IO_CONTINUE) break;
        }
        release();
    }
    double cpu_s[2] = {0, 0};  // CPU seconds of the recv (0) and send (1) worker
    double recv_io_cpu_s = 0;  // the recv worker's CPU inside recv()
    void worker(bool sending)
    {
        const double cpu0 = thread_cpu_s();
        struct Done {
            AsyncSide* a;
            bool sending;
            double cpu0;
            ~Done() { a->cpu_s[sending ? 1 : 0] = thread_cpu_s() - cpu0; }
        } done{this, sending, cpu0};
        std::deque<cts_task>& q = sending ? sends : recvs;
        std::vector<char> scratch;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return finished || !q.empty(); });
            if (q.empty()) return;  // finished
            cts_task t = q.front();
            q.pop_front();
            uint32_t transferred = 0, err = 0;
            if (aborted) {
                err = 10053;  // WSAECONNABORTED: the socket was closed under this IO
            } else {
                const bool inj = sending && inject && t.track_io && data_sends++ == inject_index && t.buffer_length > 0;
                lk.unlock();
                if (sending) {
                    pace(t);
                    const char* src = t.buffer + t.buffer_offset;
                    if (inj) {  // fault injection: one flipped byte on the wire
                        scratch.assign(src, src + t.buffer_length);
                        scratch[t.buffer_length / 2] ^= 0x5A;
                        src = scratch.data();
                    }
                    err = send_all(fd, src, t.buffer_length);
                    transferred = err == 0 ? t.buffer_length : 0;
                } else {
                    const bool whole = recv_whole || t.buffer_type == CTS_BUFFER_TCP_CONNECTION_ID ||
                                       t.buffer_type == CTS_BUFFER_COMPLETION_MESSAGE;
                    const double c0 = thread_cpu_ns_s();
                    err = recv_some(fd, t.buffer + t.buffer_offset, t.buffer_length, &transferred, whole);
                    recv_io_cpu_s += thread_cpu_ns_s() - c0;
                }
                lk.lock();
            }
            // ctsSendRecvCompletionCallback (:47-127): CompleteIo, then more IO if it asks for it
            const int st = cts_io_pattern_complete_io(p, &t, transferred, err);
            on_status(st);
            if (st == CTS_IO_CONTINUE) pump();
            release();
        }
    }
};

void run_side_async(int* fdslot, cts_io_pattern* p, bool inject, uint32_t inject_index, bool recv_whole,
                    SideResult* out)
{
    AsyncSide a;
    a.fd = *fdslot;
    a.p = p;
    a.inject = inject;
    a.inject_index = inject_index;
    a.recv_whole = recv_whole;
    {
        std::lock_guard<std::mutex> lk(a.mu);
        a.pump();
    }
    std::thread ts([&] { a.worker(true); });
    a.worker(false);
    ts.join();
    int st = a.status;
    if (st == CTS_IO_CONTINUE) st = cts_io_pattern_flush(p);  // nothing left to post: settle the pattern
    if (st != CTS_IO_COMPLETED) {
        linger l{1, 0};
        (void)::setsockopt(a.fd, SOL_SOCKET, SO_LINGER, &l, sizeof(l));
    }
    ::close(a.fd);
    *fdslot = -1;
    out->status = st;
    out->last_error = cts_io_pattern_last_error(p);
    (void)cts_io_pattern_get_stats(p, &out->stats);
    out->recv_cpu_s = a.cpu_s[0];
    out->send_cpu_s = a.cpu_s[1];
    out->recv_io_cpu_s = a.recv_io_cpu_s;
}

}  // namespace

extern "C" int cts_loopback_run(const cts_loopback_config* cfg, cts_engine* engine, cts_batch_verifier hook,
                                void* hook_ctx, cts_loopback_result* out)
{
    return cts_loopback_run_multi(cfg, engine ? &engine : nullptr, engine ? 1u : 0u, hook, hook_ctx, out);
}

extern "C" int cts_loopback_run_multi(const cts_loopback_config* cfg, cts_engine* const* engines, uint32_t n_engines,
                                      cts_batch_verifier hook, void* hook_ctx, cts_loopback_result* out)
{
    return cts_loopback_run_detailed(cfg, engines, n_engines, hook, hook_ctx, out, nullptr);
}

extern "C" int cts_loopback_run_detailed(const cts_loopback_config* cfg, cts_engine* const* engines,
                                         uint32_t n_engines, cts_batch_verifier hook, void* hook_ctx,
                                         cts_loopback_result* out, cts_loopback_side* sides)
{
    if (cfg == nullptr || out == nullptr || cfg->connections == 0 || cfg->buffer_size == 0 ||
        (cfg->buffer_size_high != 0 && cfg->buffer_size_high < cfg->buffer_size))
        return CTS_E_INVALID;
    const uint32_t max_buffer = cfg->buffer_size_high ? cfg->buffer_size_high : cfg->buffer_size;  // GetMaxBufferSize
    if (n_engines > 0 && engines == nullptr) return CTS_E_INVALID;
    for (uint32_t k = 0; k < n_engines; ++k)
        if (engines[k] == nullptr) return CTS_E_INVALID;
    cts_engine* const engine = n_engines ? engines[0] : nullptr;  // fills the process-wide sender buffer
    const uint32_t pattern = cfg->io_pattern ? cfg->io_pattern : CTS_PATTERN_PUSH;
    if (pattern < CTS_PATTERN_PUSH || pattern > CTS_PATTERN_DUPLEX || cfg->functor > CTS_LOOPBACK_FUNCTOR_ASYNC)
        return CTS_E_INVALID;
    // one blocking IO per side cannot run Duplex (a send and a recv in flight together)
    const bool async = cfg->functor == CTS_LOOPBACK_FUNCTOR_ASYNC ||
                       (cfg->functor == CTS_LOOPBACK_FUNCTOR_AUTO && pattern == CTS_PATTERN_DUPLEX);
    if (pattern == CTS_PATTERN_DUPLEX && !async) return CTS_E_INVALID;
    if (engine == nullptr && hook == nullptr && cfg->verify_buffers) return CTS_E_INVALID;
    *out = cts_loopback_result{};
    if (engine != nullptr) {
        const int rc = cts_shared_buffer_init(engine, max_buffer);
        if (rc != CTS_OK) return rc;
    }
    const int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (lfd < 0) return CTS_E_INVALID;
    int one = 1;
    (void)::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    addr.sin_port = 0;
    socklen_t alen = sizeof(addr);
    if (::bind(lfd, (sockaddr*)&addr, sizeof(addr)) != 0 || ::listen(lfd, (int)cfg->connections) != 0 ||
        ::getsockname(lfd, (sockaddr*)&addr, &alen) != 0) {
        ::close(lfd);
        return CTS_E_INVALID;
    }
    const uint32_t n = cfg->connections;
    auto make_cfg = [&](bool listening, uint32_t side) {
        cts_pattern_config c{};
        c.io_pattern = pattern;
        c.push_bytes = cfg->push_bytes ? cfg->push_bytes : cfg->buffer_size;  // PushPull segments
        c.pull_bytes = cfg->pull_bytes ? cfg->pull_bytes : cfg->buffer_size;
        c.protocol = CTS_PROTOCOL_TCP;
        c.listening = listening ? 1u : 0u;
        c.verify_buffers = cfg->verify_buffers;
        c.pre_post_recvs = 1;
        c.pre_post_sends = 1;
        c.buffer_size_low = cfg->buffer_size;
        c.buffer_size_high = cfg->buffer_size_high;
        c.random_seed = (uint64_t)cfg->random_seed + side;
        c.tcp_shutdown = CTS_SHUTDOWN_GRACEFUL;
        c.transfer_size = cfg->transfer_size;
        c.verify_mode = cfg->verify_mode;
        c.batch_buffers = cfg->batch_buffers ? cfg->batch_buffers : 512u;  // (DEFERRED launches halves of 256)
        c.tcp_bytes_per_second = cfg->tcp_bytes_per_second;  // both sides pace their own sends
        c.burst_count = cfg->burst_count;
        c.burst_delay = cfg->burst_delay;
        c.batch_bytes = (uint64_t)c.batch_buffers * max_buffer;
        return c;
    };
    std::vector<cts_io_pattern*> pats(2 * n, nullptr);
    int rc = CTS_OK;
    for (uint32_t i = 0; i < 2 * n && rc == CTS_OK; ++i) {
        const cts_pattern_config c = make_cfg(i >= n, i);  // [0,n) clients, [n,2n) servers
        cts_engine* const eng = n_engines ? engines[cts_shard_of(i % n, n_engines)] : nullptr;
        rc = cts_io_pattern_create(&c, eng, &pats[i]);
        if (rc == CTS_OK && hook != nullptr) rc = cts_io_pattern_set_verifier(pats[i], hook, hook_ctx);
    }
    if (rc != CTS_OK) {
        (void)cts::destroy_patterns(pats);  // (the creation error is the one reported)
        ::close(lfd);
        return rc;
    }
    // the diagnostic recv ring: one per side that receives data, verify off and the sync functor only
    std::vector<RecvRing> rings(2 * n);
    std::vector<std::vector<char>> ring_pageable;
    std::vector<void*> ring_pinned;
    auto free_rings = [&] {
        for (void* q : ring_pinned) (void)cts_host_free(engine, q);
        ring_pinned.clear();
    };
    if (cfg->recv_ring_buffers) {
        if (cfg->verify_buffers || async || (cfg->recv_ring_pinned && engine == nullptr)) {
            (void)cts::destroy_patterns(pats);
            ::close(lfd);
            return CTS_E_INVALID;
        }
        const uint64_t bytes = (uint64_t)cfg->recv_ring_buffers * max_buffer;
        for (uint32_t i = 0; i < 2 * n && rc == CTS_OK; ++i) {
            const bool receives = pattern == CTS_PATTERN_PUSH ? i >= n : (pattern == CTS_PATTERN_PULL ? i < n : true);
            if (!receives) continue;
            char* base = nullptr;
            if (cfg->recv_ring_pinned) {
                void* h = nullptr;
                void* d = nullptr;
                rc = cts_host_alloc(engine, bytes, &h, &d);
                if (rc == CTS_OK) ring_pinned.push_back(h);
                base = static_cast<char*>(h);
            } else {
                ring_pageable.emplace_back(bytes);
                base = ring_pageable.back().data();
            }
            rings[i] = RecvRing{base, cfg->recv_ring_buffers, max_buffer, 0};
        }
        if (rc != CTS_OK) {
            free_rings();
            (void)cts::destroy_patterns(pats);
            ::close(lfd);
            return rc;
        }
    }
    cts_status_details before{};
    (void)cts_status_details_read(&before);
    std::vector<SideResult> res(2 * n);
    std::vector<int> fds(2 * n, -1);
    std::vector<std::thread> threads;
    const auto t0 = std::chrono::steady_clock::now();
    auto tune = [&](int fd) {
        (void)::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        if (cfg->socket_buffer_bytes) {
            const int b = (int)cfg->socket_buffer_bytes;
            (void)::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &b, sizeof(b));
            (void)::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &b, sizeof(b));
        }
    };
    for (uint32_t i = 0; i < n; ++i) {  // clients connect; the listen backlog holds them
        const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0 || ::connect(fd, (sockaddr*)&addr, sizeof(addr)) != 0) {
            if (fd >= 0) ::close(fd);
            continue;
        }
        tune(fd);
        fds[i] = fd;
    }
    for (uint32_t i = 0; i < n; ++i) {  // servers accept in connect order
        const int fd = ::accept(lfd, nullptr, nullptr);
        if (fd < 0) break;
        tune(fd);
        fds[n + i] = fd;
    }
    std::vector<bool> connected0(2 * n);
    for (uint32_t i = 0; i < 2 * n; ++i) connected0[i] = fds[i] >= 0;
    threads.reserve(2 * n);
    for (uint32_t i = 0; i < 2 * n; ++i) {
        if (fds[i] < 0) continue;
        const bool inject = i % n == cfg->corrupt_connection;  // whichever side(s) send data
        try {
            if (async)
                threads.emplace_back(run_side_async, &fds[i], pats[i], inject, cfg->corrupt_send_index,
                                     cfg->recv_whole != 0, &res[i]);
            else
                threads.emplace_back(run_side, &fds[i], pats[i], inject, cfg->corrupt_send_index, cfg->recv_whole != 0,
                                     &res[i], rings[i]);
        } catch (const std::system_error&) {
            // no thread for this side: its connection fails (the peer sees the reset), the others run on
            ::shutdown(fds[i], SHUT_RDWR);
            connected0[i] = false;
        }
    }
    const std::vector<bool>& connected = connected0;
    for (auto& t : threads) t.join();
    const auto t1 = std::chrono::steady_clock::now();
    for (int fd : fds)
        if (fd >= 0) ::close(fd);
    ::close(lfd);
    cts_status_details after{};
    (void)cts_status_details_read(&after);
    out->seconds = std::chrono::duration<double>(t1 - t0).count();
    out->bytes_sent = after.bytes_sent - before.bytes_sent;
    out->bytes_recv = after.bytes_recv - before.bytes_recv;
    for (uint32_t i = 0; i < n; ++i) {
        const SideResult& c = res[i];
        const SideResult& s = res[n + i];
        const bool ok = connected[i] && connected[n + i] && c.status == CTS_IO_COMPLETED && s.status == CTS_IO_COMPLETED;
        if (ok) ++out->connections_ok;
        else ++out->connections_failed;
        if (c.last_error == CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN ||
            s.last_error == CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN)
            ++out->data_errors;
        out->buffers_verified += c.stats.buffers_verified + s.stats.buffers_verified;
    }
    for (uint32_t i = 0; i < 2 * n; ++i) {  // the threads that received the data / sent it
        const cts_pattern_stats& st = res[i].stats;
        if (async) {  // a recv worker and a send worker per side
            if (st.bytes_recv != 0) {
                out->recv_cpu_seconds += res[i].recv_cpu_s;
                out->recv_io_cpu_seconds += res[i].recv_io_cpu_s;
            }
            if (st.bytes_sent != 0) out->send_cpu_seconds += res[i].send_cpu_s;
        } else if (st.bytes_recv > st.bytes_sent) {  // one thread per side: by the direction it mostly ran
            out->recv_cpu_seconds += res[i].recv_cpu_s;
            out->recv_io_cpu_seconds += res[i].recv_io_cpu_s;
        } else {
            out->send_cpu_seconds += res[i].send_cpu_s;
        }
    }
    if (sides != nullptr)
        for (uint32_t i = 0; i < 2 * n; ++i) {
            sides[i].stats = res[i].stats;
            sides[i].status = connected[i] ? (uint32_t)res[i].status : (uint32_t)CTS_IO_FAILED;
            sides[i].last_error = res[i].last_error;
        }
    // a pattern whose final verify failed or whose kernels outlived every bounded wait is a failed run
    const int drc = cts::destroy_patterns(pats);
    free_rings();
    return drc;
}
