// cts_pattern.cpp — host-side ctsIoPattern mirror (include/cts_pattern.h): the
// caller of the gfx950 fill/verify engine, restated from the reference
// (microsoft/ctsTraffic) so the IO functors can hand completed buffers over
// unchanged.
//
//   PatternState     ctsTraffic/ctsIOPatternState.hpp:57-504 (ctsIoPatternState)
//   IoPattern        ctsTraffic/ctsIOPattern.cpp:133-743     (ctsIoPattern base)
//   Push/Pull/...    ctsTraffic/ctsIOPattern.cpp:796-1031    (concrete TCP patterns)
//   MediaStream      ctsTraffic/ctsIOPattern.cpp:1100-1175   (UDP server)
//                    ctsTraffic/ctsIOPatternMediaStream.cpp  (UDP client; frame accounting in cts_media_stream.cpp)
//
// The two hot-path pieces go to the GPU: the sender buffer is written by the
// fill kernel (cts_shared_buffer_init) and VerifyBuffer runs the verify kernel
// on the pattern's pinned, device-mapped recv buffers (zero copy) — per
// completion (CTS_VERIFY_SYNC) or batched (CTS_VERIFY_DEFERRED).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <deque>
#include <new>
#include <random>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "cts_engine.h"
#include "cts_media_stream_client.hpp"
#include "cts_pattern.h"
#include "cts_slices.hpp"

namespace {

constexpr uint32_t kPatternSize = CTS_PATTERN_PERIOD;  // c_bufferPatternSize, ctsIOPattern.cpp:35
constexpr uint32_t kStatusIoRunning = CTS_STATUS_IO_RUNNING;
constexpr uint32_t kNoError = 0;
constexpr char kCompletionMessage[CTS_COMPLETION_MESSAGE_SIZE + 1] = "DONE";  // ctsIOPatternState.hpp:24

// ---- process-wide state -------------------------------------------------------------------
// g_senderSharedBuffer / g_maximumBufferSize (ctsIOPattern.cpp:40-47): one per process.
struct SharedBuffer {
    std::mutex mu;
    char* host = nullptr;
    uint64_t bytes = 0;
    bool owned = false;       // pinned by cts_shared_buffer_init (hipHostFree on release)
    cts_engine* engine = nullptr;
    std::vector<char> receiver;  // g_receiverSharedBuffer (UseSharedBuffer, ctsIOPattern.cpp:138-152)
};
SharedBuffer g_shared;

// g_configSettings->rioFunctions: RIORegisterBuffer / RIODeregisterBuffer (cts_rio_functions_set)
struct RioFunctions {
    std::mutex mu;
    cts_rio_register_buffer_fn reg = nullptr;
    cts_rio_deregister_buffer_fn dereg = nullptr;
    void* ctx = nullptr;
};
RioFunctions g_rio;
constexpr uint64_t kRioInvalid = CTS_RIO_INVALID_BUFFERID;
constexpr uint64_t kMaxSupportedBytesInFlight = 0x1000000;  // c_maxSupportedBytesInFlight, ctsIOPattern.cpp:49

struct RioRegisterFailed {};

// ctTimer::snap_qpc_as_msec, replaceable by cts_pattern_clock_set (the unit-test hook)
struct Clock {
    std::mutex mu;
    cts_clock_ms_fn fn = nullptr;
    void* ctx = nullptr;
};
Clock g_clock;
int64_t NowMs()
{
    {
        std::lock_guard<std::mutex> lk(g_clock.mu);
        if (g_clock.fn != nullptr) return g_clock.fn(g_clock.ctx);
    }
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// TcpStatusDetails (ctsConfig.h:415) + a DataError tally
std::atomic<uint64_t> g_bytesSent{0};
std::atomic<uint64_t> g_bytesRecv{0};
std::atomic<uint64_t> g_dataErrors{0};

// ---- ctsIoPatternState ------------------------------------------------------------------------
enum class PatternType { NoIo, SendConnectionId, RecvConnectionId, MoreIo, SendCompletion, RecvCompletion,
                         GracefulShutdown, HardShutdown, RequestFin };
enum class PatternError { NoError, TooManyBytes, TooFewBytes, CorruptedBytes, ErrorIoFailed, SuccessfullyCompleted };

struct FailFast {
    std::string reason;
};
// Makes an engine's device current for the HIP calls a pattern makes itself (events, waits, copies, stream-ordered
// allocations) and gives the thread its own device back. IO threads and the MediaStream timer thread may have any
// device current, and an event must be created on the device of the stream it is recorded on.
struct EngineDevice {
    int prev = -1;
    bool switched = false;
    explicit EngineDevice(const cts_engine* e)
    {
        const int d = e != nullptr ? cts_engine_device(e) : -1;
        if (d < 0 || hipGetDevice(&prev) != hipSuccess) return;
        switched = prev != d && hipSetDevice(d) == hipSuccess;
    }
    ~EngineDevice()
    {
        if (switched) (void)hipSetDevice(prev);
    }
    EngineDevice(const EngineDevice&) = delete;
    EngineDevice& operator=(const EngineDevice&) = delete;
};

struct DeviceError {  // a verify call failed (HIP / engine status): CompleteIo returns it
    int rc;
};

class PatternState {
public:
    enum class Internal { Initialized, MoreIo, ServerSendConnectionId, ClientRecvConnectionId, ServerSendCompletion,
                          ClientRecvCompletion, CompletedTransfer, ErrorIoFailed, GracefulShutdown, HardShutdown,
                          RequestFin };

    PatternState(const cts_pattern_config& c, uint32_t max_buffer_size)  // ctsIOPatternState.hpp:108-114
        : m_maxTransfer(c.transfer_size),
          m_idealSendBacklog(c.pre_post_sends == 0 ? max_buffer_size : max_buffer_size * c.pre_post_sends),
          m_listening(c.listening != 0),
          m_graceful(c.tcp_shutdown != CTS_SHUTDOWN_HARD),
          m_udp(c.protocol == CTS_PROTOCOL_UDP)
    {
        if (m_udp) m_internal = Internal::MoreIo;
    }

    uint64_t GetRemainingTransfer() const  // ctsIOPatternState.hpp:123-141
    {
        const uint64_t already = m_confirmedBytes + m_inFlightBytes;
        if (already > m_maxTransfer) throw FailFast{"bytes already transferred exceed the total to transfer"};
        return m_maxTransfer - already;
    }
    uint64_t GetMaxTransfer() const { return m_maxTransfer; }
    // DEFERRED: completions accepted after a buffer that later failed verification are taken back
    // (the reference never saw them: it failed the connection at that buffer, ctsIOPattern.cpp:486-489)
    void RollbackConfirmed(uint64_t bytes) { m_confirmedBytes -= std::min(bytes, m_confirmedBytes); }
    void SetMaxTransfer(uint64_t v) { m_maxTransfer = v; }
    uint32_t GetIdealSendBacklog() const { return m_idealSendBacklog; }
    void SetIdealSendBacklog(uint32_t isb) { m_idealSendBacklog = isb; }  // ctsIOPatternState.hpp:155-158
    bool IsCompleted() const { return m_internal == Internal::CompletedTransfer || m_internal == Internal::ErrorIoFailed; }
    bool IsCurrentStateMoreIo() const { return m_internal == Internal::MoreIo; }

    PatternType GetNextPatternType()  // ctsIOPatternState.hpp:177-244
    {
        if (m_pended) return PatternType::NoIo;
        switch (m_internal) {
        case Internal::Initialized:
            m_pended = true;
            if (m_listening) {
                m_internal = Internal::ServerSendConnectionId;
                return PatternType::SendConnectionId;
            }
            m_internal = Internal::ClientRecvConnectionId;
            return PatternType::RecvConnectionId;
        case Internal::ServerSendConnectionId:
        case Internal::ClientRecvConnectionId:
            m_internal = Internal::MoreIo;
            return PatternType::MoreIo;
        case Internal::MoreIo:
            return (m_confirmedBytes + m_inFlightBytes) < m_maxTransfer ? PatternType::MoreIo : PatternType::NoIo;
        case Internal::ServerSendCompletion: m_pended = true; return PatternType::SendCompletion;
        case Internal::ClientRecvCompletion: m_pended = true; return PatternType::RecvCompletion;
        case Internal::GracefulShutdown: m_pended = true; return PatternType::GracefulShutdown;
        case Internal::HardShutdown: m_pended = true; return PatternType::HardShutdown;
        case Internal::RequestFin: m_pended = true; return PatternType::RequestFin;
        case Internal::CompletedTransfer:
        case Internal::ErrorIoFailed: return PatternType::NoIo;
        }
        throw FailFast{"GetNextPatternType called in an invalid state"};
    }

    void NotifyNextTask(const cts_task& t)  // ctsIOPatternState.hpp:246-252
    {
        if (t.track_io) m_inFlightBytes += t.buffer_length;
    }

    PatternError UpdateError(uint32_t error)  // ctsIOPatternState.hpp:254-293
    {
        if (m_internal == Internal::ErrorIoFailed) return PatternError::ErrorIoFailed;
        if (m_udp) {
            if (error != 0) {
                m_internal = Internal::ErrorIoFailed;
                return PatternError::ErrorIoFailed;
            }
            return PatternError::NoError;
        }
        if (error != 0 && !IsCompleted()) {
            // WSAETIMEDOUT / WSAECONNRESET / WSAECONNABORTED while a server waits for the FIN
            if (m_listening && m_internal == Internal::RequestFin && (error == 10060 || error == 10054 || error == 10053))
                return PatternError::NoError;
            m_internal = Internal::ErrorIoFailed;
            return PatternError::ErrorIoFailed;
        }
        return PatternError::NoError;
    }

    // True when CompletedTask(task, bytes) would return NoError and leave the
    // state in MoreIo without side effects beyond the byte accounting — the
    // completions a DEFERRED pattern may verify later (cts_io_pattern_flush).
    bool WouldStayMoreIo(const cts_task& t, uint32_t bytes) const
    {
        if (m_internal != Internal::MoreIo || !t.track_io) return false;
        if (bytes > t.buffer_length || t.buffer_length > m_inFlightBytes) return false;
        const uint64_t inflight = m_inFlightBytes - t.buffer_length;
        const uint64_t already = m_confirmedBytes + bytes + inflight;
        if (already < m_maxTransfer) return bytes != 0;
        if (already == m_maxTransfer) return inflight != 0;
        return false;
    }

    PatternError CompletedTask(const cts_task& t, uint32_t bytes)  // ctsIOPatternState.hpp:295-504
    {
        if (m_internal == Internal::ErrorIoFailed) return PatternError::ErrorIoFailed;
        if (m_internal == Internal::ServerSendConnectionId || m_internal == Internal::ClientRecvConnectionId) {
            if (bytes != CTS_CONNECTION_ID_LENGTH) {
                m_internal = Internal::ErrorIoFailed;
                return PatternError::TooFewBytes;
            }
            m_pended = false;
        }
        if (t.track_io) {
            if (bytes > m_inFlightBytes) throw FailFast{"task returned more bytes than were in flight"};
            if (t.buffer_length > m_inFlightBytes) throw FailFast{"task requested more bytes than were in flight"};
            if (bytes > t.buffer_length) throw FailFast{"task returned more bytes than were posted"};
            m_inFlightBytes -= t.buffer_length;
            m_confirmedBytes += bytes;
        }
        const uint64_t already = m_confirmedBytes + m_inFlightBytes;
        if (m_udp) return already == m_maxTransfer ? PatternError::SuccessfullyCompleted : PatternError::NoError;
        if (already < m_maxTransfer) {
            if (bytes == 0) {
                m_internal = Internal::ErrorIoFailed;
                return PatternError::TooFewBytes;
            }
        } else if (already == m_maxTransfer) {
            if (m_inFlightBytes == 0) {
                if (m_listening) {
                    switch (m_internal) {
                    case Internal::MoreIo:
                        m_internal = Internal::ServerSendCompletion;
                        m_pended = false;
                        break;
                    case Internal::ServerSendCompletion:
                        m_internal = Internal::RequestFin;
                        m_pended = false;
                        break;
                    case Internal::RequestFin:
                        if (bytes != 0) {
                            m_internal = Internal::ErrorIoFailed;
                            return PatternError::TooManyBytes;
                        }
                        m_internal = Internal::CompletedTransfer;
                        return PatternError::SuccessfullyCompleted;
                    default: throw FailFast{"CompletedTask: invalid server state"};
                    }
                } else {
                    switch (m_internal) {
                    case Internal::MoreIo:
                        m_internal = Internal::ClientRecvCompletion;
                        m_pended = false;
                        break;
                    case Internal::ClientRecvCompletion:
                        if (bytes != CTS_COMPLETION_MESSAGE_SIZE ||
                            std::memcmp(t.buffer, kCompletionMessage, CTS_COMPLETION_MESSAGE_SIZE) != 0) {
                            m_internal = Internal::ErrorIoFailed;
                            return PatternError::TooFewBytes;
                        }
                        m_internal = m_graceful ? Internal::GracefulShutdown : Internal::HardShutdown;
                        m_pended = false;
                        break;
                    case Internal::GracefulShutdown:
                        m_internal = Internal::RequestFin;
                        m_pended = false;
                        break;
                    case Internal::RequestFin:
                        if (bytes != 0) {
                            m_internal = Internal::ErrorIoFailed;
                            return PatternError::TooManyBytes;
                        }
                        m_internal = Internal::CompletedTransfer;
                        return PatternError::SuccessfullyCompleted;
                    case Internal::HardShutdown:
                        m_internal = Internal::CompletedTransfer;
                        return PatternError::SuccessfullyCompleted;
                    default: throw FailFast{"CompletedTask: invalid client state"};
                    }
                }
            }
        } else {
            m_internal = Internal::ErrorIoFailed;
            return PatternError::TooManyBytes;
        }
        return PatternError::NoError;
    }

private:
    uint64_t m_confirmedBytes = 0;
    uint64_t m_maxTransfer;
    uint64_t m_inFlightBytes = 0;
    uint32_t m_idealSendBacklog;
    Internal m_internal = Internal::Initialized;
    bool m_pended = false;
    bool m_listening;
    bool m_graceful;
    bool m_udp;
};

// ---- pinned host memory helpers -------------------------------------------------------------
struct Pinned {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;  // device view (hipHostGetDevicePointer)
    uint64_t bytes = 0;
    cts_engine* engine = nullptr;
    int alloc(cts_engine* e, uint64_t n)
    {
        void *h = nullptr, *d = nullptr;
        const int rc = cts_host_alloc(e, n, &h, &d);
        if (rc != CTS_OK) return rc;
        host = static_cast<uint8_t*>(h);
        dev = static_cast<uint8_t*>(d);
        bytes = n;
        engine = e;
        return CTS_OK;
    }
    void release()
    {
        if (host) (void)cts_host_free(engine, host);
        host = dev = nullptr;
        bytes = 0;
    }
    ~Pinned() { release(); }
};

struct Queued {
    uint32_t completion;        // recv completion index
    uint32_t transferred;
    uint64_t bytes_recv_after;  // m_bytesRecv after this completion (as the reference would count it)
    uint64_t bytes_sent_after;  // m_bytesSent at that point (sends completed later are rolled back on failure)
    uint32_t expected;          // the task's m_expectedPatternOffset
    uint64_t status_recv_after; // this pattern's TcpStatusDetails.m_bytesRecv contribution after this completion
    uint64_t status_sent_after; // ... and its m_bytesSent contribution at that point
};

}  // namespace

// ---- ctsIoPattern -----------------------------------------------------------------------------
struct cts_io_pattern {
    explicit cts_io_pattern(const cts_pattern_config& c, uint32_t maxbuf, uint32_t recv_count)
        : cfg(c), max_buffer_size(maxbuf), state(c, maxbuf), rng(c.random_seed), recvCount(recv_count),
          m_quantumPeriodMs(c.tcp_bytes_per_second_period > 0 ? c.tcp_bytes_per_second_period : 100),
          // (bytes/sec) * (1 sec/1000 ms) * (x ms/Quantum) == (bytes/quantum) (ctsIOPattern.cpp:219-224)
          m_bytesSendingPerQuantum(c.tcp_bytes_per_second * m_quantumPeriodMs / 1000),
          m_burstCount(c.burst_count), m_quantumStartTimeMs(NowMs())
    {
    }
    virtual ~cts_io_pattern()
    {
        EngineDevice on(engine);
        if (stream) {
            (void)hipStreamSynchronize(stream);  // kernels may still read the ring (cheap when idle)
            (void)cts_engine_stream_destroy(engine, stream);
        }
        for (Flight& f : flights) spare_events.push_back(f.done);
        for (hipEvent_t e : spare_events)
            if (e) (void)hipEventDestroy(e);
        if (sync_done) (void)hipEventDestroy(sync_done);
        // ~RioBufferId (ctsIOPattern.h:230-238) for every id this pattern registered
        if (!rio_owned.empty()) {
            std::lock_guard<std::mutex> lk(g_rio.mu);
            if (g_rio.dereg != nullptr)
                for (const uint64_t id : rio_owned) g_rio.dereg(g_rio.ctx, id);
        }
    }

    cts_pattern_config cfg;
    uint32_t max_buffer_size;
    // the pattern's critical section (ctsIoPattern::AcquireIoPatternLock, ctsIOPattern.h:405): every C-ABI call and
    // the MediaStream client's timer callbacks hold it; recursive, as a Windows critical section is, because a
    // callback may complete the task it hands out (ctsMediaStreamClient.cpp:317-331)
    mutable std::recursive_mutex mu;
    cts_task_callback m_callback = nullptr;  // RegisterCallback (ctsIOPattern.h:94-97)
    void* m_callback_ctx = nullptr;
    void SendTaskToCallback(const cts_task& t) const  // ctsIOPattern.h:333-339
    {
        if (m_callback != nullptr) m_callback(m_callback_ctx, &t);
    }
    PatternState state;
    std::mt19937_64 rng;
    uint32_t recvCount;
    cts_engine* engine = nullptr;
    cts_batch_verifier hook = nullptr;
    void* hook_ctx = nullptr;
    hipStream_t stream = nullptr;

    uint32_t m_sendPatternOffset = 0;
    uint32_t m_recvPatternOffset = 0;
    // send pacing (ctsIOPattern.h:204-205, 273-275); m_burstCount 0 with cfg.burst_count 0 = no burst
    int64_t m_quantumPeriodMs;
    int64_t m_bytesSendingPerQuantum;
    uint32_t m_burstCount;
    int64_t m_bytesSendingThisQuantum = 0;
    int64_t m_quantumStartTimeMs;
    uint32_t m_lastError = kStatusIoRunning;
    std::vector<char*> m_recvBufferFreeList;
    Pinned recv_pinned;                 // m_recvBufferContainer when a device verifies in place
    std::vector<char> recv_plain;       // m_recvBufferContainer otherwise
    std::array<char, CTS_COMPLETION_MESSAGE_SIZE> m_completionMessageBuffer{};
    char connection_id[CTS_CONNECTION_ID_LENGTH] = {};
    std::string fail_fast;

    // statistics + verify bookkeeping
    uint64_t bytes_sent = 0, bytes_recv = 0;
    // The reference's byte counters only ever Add (ctsStatistics.hpp:153-186; ctsIOPattern.cpp:505-521), and its
    // status timer prints their SnapValueDifference (ctsStatistics.hpp:363). A DEFERRED pattern therefore holds back
    // the bytes of every completion behind a recv whose verdict is not in yet: status_* is this pattern's running
    // contribution to TcpStatusDetails, published_* what it has added to g_bytesSent/g_bytesRecv so far. A batch that
    // verifies publishes up to its last buffer; a failing buffer publishes up to and including itself, and everything
    // after it is dropped unpublished (the reference never saw it). Nothing published is ever taken back.
    uint64_t status_sent = 0, status_recv = 0;
    uint64_t published_sent = 0, published_recv = 0;
    void Publish(uint64_t recv_to, uint64_t sent_to)
    {
        if (recv_to > published_recv) {
            g_bytesRecv.fetch_add(recv_to - published_recv);
            published_recv = recv_to;
        }
        if (sent_to > published_sent) {
            g_bytesSent.fetch_add(sent_to - published_sent);
            published_sent = sent_to;
        }
    }
    // held back: completed, counted by the pattern, not yet published (only while a DEFERRED verdict is pending; every
    // completion accepted meanwhile is a pattern-requested send/recv, so the per-connection counters hold back the same)
    uint64_t HeldRecv() const { return status_recv - published_recv; }
    uint64_t HeldSent() const { return status_sent - published_sent; }
    bool VerdictsPending() const { return !queue.empty() || !flights.empty(); }
    uint32_t InFlightCount() const
    {
        uint32_t n = 0;
        for (const Flight& f : flights) n += (uint32_t)f.q.size();
        return n;
    }
    void PublishIfSettled()
    {
        if (!VerdictsPending()) Publish(status_recv, status_sent);
    }
    uint64_t buffers_verified = 0, bytes_verified = 0, buffers_failed = 0;
    uint64_t bytes_recv_at_failure = 0;
    uint32_t recv_completions = 0;
    bool has_failure = false;
    uint32_t fail_length = 0, fail_offset = 0, fail_completion = 0;
    uint8_t fail_expected = 0, fail_actual = 0;

    // SYNC device verify: one descriptor + one result, pinned and device-mapped
    Pinned one;
    // DEFERRED queue
    Pinned stage, stage_desc, stage_res;
    std::vector<uint8_t> hstage;        // host staging when a hook verifies
    std::vector<cts_buf_desc> hdesc;
    std::vector<cts_verify_result> hres;
    std::vector<Queued> queue;
    uint64_t stage_used = 0;
    // pipelined batches (ring mode, device verify): a full batch is launched and left running while the next one
    // fills in another set of stage_desc/stage_res; up to Depth() batches run at once. The oldest one's verdicts are
    // applied when a launch would exceed Depth(), as soon as CompleteIo sees its kernel done, at any non-benign
    // completion and at Flush. A failing batch discards the ones launched after it.
    struct Flight {
        std::vector<Queued> q;
        hipEvent_t done = nullptr;  // recorded after the batch's launch, queried by CompleteIo
        uint32_t set = 0;           // its descriptor / result set
    };
    std::deque<Flight> flights;              // oldest first
    std::vector<hipEvent_t> spare_events;    // events of retired flights, for reuse
    std::vector<std::vector<Queued>> spare_queues;  // their entry vectors (capacity kept across batches)
    // Batches in flight per connection (CTS_DEFERRED_DEPTH, 1-4; default 2). Each launch holds
    // BatchCapacity() / (Depth() + 1) buffers, so a verdict is still known within BatchCapacity() completions.
    // Config 1 over loopback, four boxes, 40 alternated rounds: 2 beat 1 in 29.
    uint32_t depth_env = [] {
        const char* v = std::getenv("CTS_DEFERRED_DEPTH");
        if (v == nullptr || *v == 0) return 2u;
        const long n = std::atol(v);
        return n < 1 ? 1u : (n > 4 ? 4u : (uint32_t)n);
    }();
    // How Retire waits for the in-flight batch (CTS_DEFERRED_BLOCKING_SYNC): 0 = spin in hipStreamSynchronize,
    // 1 = hipEventSynchronize on a blocking-sync event, 2 (default) = sleep in 50 us steps between non-blocking
    // queries of the event. With 8 connections sharing the PCIe link, the first two burned ~2 ms of receive-thread
    // CPU per wait, 1 as much as 0 (tools/pattern_cpu_probe, profiles/r03/pattern_cpu/): the runtime's blocking wait
    // spins before it sleeps
    int retire_wait = [] {
        const char* v = std::getenv("CTS_DEFERRED_BLOCKING_SYNC");
        if (v == nullptr || *v == 0) return 2;
        const int n = std::atoi(v);
        return n < 0 || n > 2 ? 2 : n;
    }();
    // CompleteIo asks whether the in-flight batch is done every query_period-th completion (a power of two;
    // CTS_DEFERRED_QUERY_PERIOD, default 16; 0 = never: verdicts land at the next Rotate / Flush only)
    uint32_t query_period = [] {
        const char* v = std::getenv("CTS_DEFERRED_QUERY_PERIOD");
        if (v == nullptr || *v == 0) return 16u;
        const long n = std::atol(v);
        if (n <= 0) return 0u;
        uint32_t p = 1;
        while (p < (uint32_t)std::min<long>(n, 1L << 20)) p <<= 1;
        return p;
    }();
    uint32_t desc_set = 0;  // the set the filling batch uses
    // time the calls spent waiting for a DEFERRED batch's device verdicts (cts_pattern_stats.verify_wait_ns)
    uint64_t verify_wait_ns = 0;
    void AddVerifyWait(std::chrono::steady_clock::time_point t0)
    {
        verify_wait_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                              std::chrono::steady_clock::now() - t0).count();
    }
    // DEFERRED zero-copy ring: the recv container holds (1 or 2) x BatchCapacity() + recvCount + 1
    // buffer slots and a completed buffer's slot is not handed out again before its batch was
    // verified, so a batch is verified in place (no staging copy)
    bool ring = false, queue_in_ring = false;
    uint32_t ring_slots = 0, ring_next = 0;
    uint32_t slot_bytes = 0;  // one recv buffer (RecvSlotBytes)
    char* ring_base = nullptr;
    uint64_t ring_bytes = 0;

    // RIO buffer ids (ctsIOPattern.h:219-269). m_receivingRioBufferIds pairs with
    // m_recvBufferFreeList entry for entry; in ring mode every ring slot has its own id
    // (ring_rio_ids) and a recycled slot goes back with its id.
    std::vector<uint64_t> m_receivingRioBufferIds;
    std::vector<uint64_t> m_sendingRioBufferIds;
    std::vector<uint64_t> ring_rio_ids;
    std::vector<uint64_t> rio_owned;  // every id registered by this pattern (deregistered at destroy)
    uint64_t m_rioConnectionId = kRioInvalid;
    uint64_t m_rioCompletionMessage = kRioInvalid;

    bool Rio() const { return cfg.registered_io != 0; }
    uint64_t RioRegister(char* buffer, uint32_t length)  // RIORegisterBuffer, THROW_WIN32 on failure
    {
        uint64_t id = kRioInvalid;
        {
            std::lock_guard<std::mutex> lk(g_rio.mu);
            if (g_rio.reg != nullptr) id = g_rio.reg(g_rio.ctx, buffer, length);
        }
        if (id == kRioInvalid) throw RioRegisterFailed{};
        rio_owned.push_back(id);
        return id;
    }
    uint64_t RioBufferIdCount() const  // ctsIOPattern.h:114-123
    {
        if (!Rio()) return 0;
        return m_receivingRioBufferIds.size() + m_sendingRioBufferIds.size() + 2;
    }

    uint32_t GetBufferSize()  // ctsConfig.cpp:4679-4684
    {
        if (cfg.buffer_size_high == 0) return cfg.buffer_size_low;
        std::uniform_int_distribution<uint32_t> d(cfg.buffer_size_low, cfg.buffer_size_high);
        return d(rng);
    }

    // derived-pattern interface (ctsIOPattern.h:187-188)
    virtual cts_task GetNextTaskFromPattern() = 0;
    virtual PatternError CompleteTaskBackToPattern(const cts_task&, uint32_t) = 0;
    // a completion of t must be verified (and so needs an engine or a hook)
    virtual bool NeedsVerifier(const cts_task& t) const
    {
        return cfg.verify_buffers && t.io_action == CTS_TASK_RECV && t.track_io;
    }
    // The bytes of one recv buffer (m_recvBufferContainer holds GetMaxBufferSize() per recv, ctsIOPattern.cpp:156-175).
    // The MediaStream patterns never post a recv that large: their slots are sized to what they post.
    virtual uint32_t RecvSlotBytes() const { return max_buffer_size; }
    // Whether its recvs carry data to verify (a DEFERRED pattern that does gets the zero-copy recv ring)
    virtual bool VerifiesRecvs() const { return cfg.verify_buffers != 0; }
    // MediaStream surface (cts_io_pattern_media_stream_*): CTS_E_INVALID for the TCP patterns
    virtual int FireTimer(int) { return CTS_E_INVALID; }
    virtual int Timers(int64_t*, int64_t*) { return CTS_E_INVALID; }
    virtual int UdpStats(cts_media_stream_stats*) { return CTS_E_INVALID; }
    // cts_io_pattern_flush: the DEFERRED queue of this pattern
    virtual int FlushPending() { return Flush(); }
    // Stops and joins any thread of the pattern's own that calls into it (the MediaStream client's timers).
    virtual void StopTimers() {}

    uint64_t GetTotalTransfer() const { return state.GetMaxTransfer(); }
    void SetTotalTransfer(uint64_t v) { state.SetMaxTransfer(v); }
    uint32_t GetIdealSendBacklog() const { return state.GetIdealSendBacklog(); }

    uint32_t UpdateLastError(uint32_t error)  // ctsIOPattern.h:344-365
    {
        if (m_lastError == kStatusIoRunning) {
            const PatternError st = state.UpdateError(error);
            if (error == kNoError) {
                if (st != PatternError::ErrorIoFailed) m_lastError = kNoError;
            } else if (st == PatternError::ErrorIoFailed) {
                m_lastError = error;
                if (error == CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN) g_dataErrors.fetch_add(1);
            }
        }
        return m_lastError;
    }

    void UpdateLastPatternError(PatternError e)  // ctsIOPattern.h:367-392
    {
        switch (e) {
        case PatternError::CorruptedBytes: UpdateLastError(CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN); break;
        case PatternError::TooFewBytes: UpdateLastError(CTS_STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED); break;
        case PatternError::TooManyBytes: UpdateLastError(CTS_STATUS_ERROR_TOO_MUCH_DATA_TRANSFERRED); break;
        case PatternError::SuccessfullyCompleted: UpdateLastError(kNoError); break;
        case PatternError::NoError:
        case PatternError::ErrorIoFailed: break;
        }
    }

    int GetCurrentStatus() const  // ctsIOPattern.h:160-174
    {
        if (m_lastError == kStatusIoRunning) return CTS_IO_CONTINUE;
        if (m_lastError == kNoError) return CTS_IO_COMPLETED;
        return CTS_IO_FAILED;
    }

    int CreateRecvBuffers()  // ctsIOPattern.cpp:133-193
    {
        const int rc = CreateRecvSlots();
        if (rc != CTS_OK || !Rio()) return rc;
        // register the recv slots, then the connection id and the completion message (:141-192)
        if (ring) {
            ring_rio_ids.resize(ring_slots);
            for (uint32_t i = 0; i < ring_slots; ++i)
                ring_rio_ids[i] = RioRegister(ring_base + (size_t)i * slot_bytes, slot_bytes);
            for (const char* b : m_recvBufferFreeList) m_receivingRioBufferIds.push_back(ring_rio_ids[RingSlot(b)]);
        } else {
            const uint32_t len = cfg.use_shared_buffer ? (uint32_t)g_shared.bytes : slot_bytes;
            for (char* b : m_recvBufferFreeList) m_receivingRioBufferIds.push_back(RioRegister(b, len));
        }
        m_rioConnectionId = RioRegister(connection_id, CTS_CONNECTION_ID_LENGTH);
        m_rioCompletionMessage = RioRegister(m_completionMessageBuffer.data(), CTS_COMPLETION_MESSAGE_SIZE);
        return CTS_OK;
    }

    int CreateRecvSlots()
    {
        m_recvBufferFreeList.assign(recvCount, nullptr);
        if (recvCount == 0) return CTS_OK;
        if (cfg.use_shared_buffer) {
            std::lock_guard<std::mutex> lk(g_shared.mu);
            if (g_shared.receiver.size() < g_shared.bytes) g_shared.receiver.resize(g_shared.bytes);
            for (auto& b : m_recvBufferFreeList) b = g_shared.receiver.data();
            return CTS_OK;
        }
        ring = Deferred() && VerifiesRecvs();
        slot_bytes = RecvSlotBytes();
        // a slot is handed out again only after every batch that may hold it was verified: the filling batch and the
        // up to Depth() launches in flight hold (Depth() + 1) x BatchCapacity() / (Depth() + 1) = BatchCapacity()
        // unverified slots, and recvCount more are posted. The pipelined ring keeps a second BatchCapacity() of slots
        // beyond that bound (the depth-1 layout of round 3; config-1 throughput did not move with the ring's size
        // within the run-to-run spread)
        ring_slots = ring ? BatchCapacity() * (DoubleBuffered() ? 2u : 1u) + recvCount + 1 : recvCount;
        const uint64_t bytes = (uint64_t)slot_bytes * ring_slots;
        char* base = nullptr;
        if (engine != nullptr && hook == nullptr) {
            const int rc = recv_pinned.alloc(engine, bytes ? bytes : 16);
            if (rc != CTS_OK) return rc;
            base = reinterpret_cast<char*>(recv_pinned.host);
        } else {
            recv_plain.assign(bytes, 0);
            base = recv_plain.data();
        }
        for (uint32_t i = 0; i < recvCount; ++i) m_recvBufferFreeList[i] = base + (size_t)i * slot_bytes;
        ring_base = base;
        ring_bytes = bytes;
        ring_next = recvCount;
        return CTS_OK;
    }

    uint32_t RingSlot(const char* b) const { return (uint32_t)((size_t)(b - ring_base) / slot_bytes); }

    // the buffer (and its RIO id) to put back on the free lists after a completion
    // (ctsIOPattern.cpp:369-386): the completed one, or in ring mode the next ring slot (the
    // completed one waits for its batch)
    void RecycleRecvBuffer(const cts_task& t)
    {
        char* b = t.buffer;
        if (ring) {
            b = ring_base + (size_t)(ring_next % ring_slots) * slot_bytes;
            ++ring_next;
        }
        m_recvBufferFreeList.push_back(b);
        if (Rio()) m_receivingRioBufferIds.push_back(ring ? ring_rio_ids[RingSlot(b)] : t.rio_buffer_id);
    }

    void CreateSendBuffers()  // ctsIOPattern.cpp:195-217
    {
        std::memcpy(m_completionMessageBuffer.data(), kCompletionMessage, CTS_COMPLETION_MESSAGE_SIZE);
        if (Rio()) {
            // g_maxNumberOfRioSendBuffers = c_maxSupportedBytesInFlight / GetMinBufferSize() + 1 (:61)
            const uint64_t n = kMaxSupportedBytesInFlight / cfg.buffer_size_low + 1;
            m_sendingRioBufferIds.reserve(n);
            for (uint64_t i = 0; i < n; ++i)
                m_sendingRioBufferIds.push_back(RioRegister(g_shared.host, (uint32_t)g_shared.bytes));
        }
    }

    // When the next send of `size` bytes may go out (ctsIOPattern.cpp:593-674): with a rate limit, the
    // bytes of each TcpBytesPerSecondPeriod quantum are capped and a send past the cap is deferred to
    // the quantum it fills; otherwise every BurstCount-th send waits BurstDelay ms.
    int64_t SendTimeOffset(uint64_t size)
    {
        int64_t offset = 0;
        if (m_bytesSendingPerQuantum > 0) {
            const int64_t now = NowMs();
            if (m_bytesSendingThisQuantum < m_bytesSendingPerQuantum) {
                m_bytesSendingThisQuantum += (int64_t)size;
                if (now > m_quantumStartTimeMs + m_quantumPeriodMs) {
                    // now past this quantum: move to the one we are in, and take back the bytes the
                    // skipped quantums would have carried (never below zero)
                    const int64_t skipped = (now - m_quantumStartTimeMs) / m_quantumPeriodMs;
                    m_quantumStartTimeMs += skipped * m_quantumPeriodMs;
                    const int64_t adjust = m_bytesSendingPerQuantum * skipped;
                    m_bytesSendingThisQuantum = adjust > m_bytesSendingThisQuantum ? 0 : m_bytesSendingThisQuantum - adjust;
                }
            } else {
                // this quantum (and maybe more) is already full: carry the excess, defer this send to
                // the end of the quantums it fills
                const int64_t ahead = m_bytesSendingThisQuantum / m_bytesSendingPerQuantum;
                const int64_t skip_ms = (ahead - 1) * m_quantumPeriodMs;
                m_bytesSendingThisQuantum -= m_bytesSendingPerQuantum * ahead;
                m_bytesSendingThisQuantum += (int64_t)size;
                if (now < m_quantumStartTimeMs + m_quantumPeriodMs) offset = m_quantumStartTimeMs + m_quantumPeriodMs - now;
                offset += skip_ms;
                m_quantumStartTimeMs += skip_ms + m_quantumPeriodMs;
            }
        } else if (cfg.burst_count != 0) {
            if (m_burstCount == 0) m_burstCount = cfg.burst_count;
            m_burstCount -= 1;
            if (m_burstCount == 0) offset = (int64_t)cfg.burst_delay;
        }
        return offset;
    }

    cts_task CreateNewTask(uint8_t action, uint32_t maxTransfer)  // ctsIOPattern.cpp:550-743
    {
        const uint64_t remaining = state.GetRemainingTransfer();
        const uint64_t next = GetBufferSize();
        const uint64_t minBuf = std::min<uint64_t>(remaining, next);
        uint64_t newSize = minBuf;
        if (maxTransfer > 0 && maxTransfer < minBuf) newSize = maxTransfer;
        if (newSize > 0xFFFFFFFFull) throw FailFast{"next buffer size is greater than MAXDWORD"};
        const uint32_t size = (uint32_t)newSize;
        cts_task t{};
        t.rio_buffer_id = kRioInvalid;
        // with RIO only so many registered send buffers exist: once every one is in flight, no IO yet
        // (ctsIOPattern.cpp:580-587)
        if (action == CTS_TASK_SEND && Rio() && m_sendingRioBufferIds.empty()) return t;
        if (action == CTS_TASK_SEND) {
            t.time_offset_ms = SendTimeOffset(size);
            t.io_action = CTS_TASK_SEND;
            t.buffer_type = CTS_BUFFER_STATIC;
            t.buffer_length = size;
            t.buffer_offset = m_sendPatternOffset;
            t.expected_pattern_offset = 0;
            t.buffer = g_shared.host;
            // every RIOSend needs its own RIO_BUFFERID (ctsIOPattern.cpp:683-692)
            if (Rio()) {
                if (m_sendingRioBufferIds.empty()) throw FailFast{"m_sendingRioBufferIds is empty for a new Send task"};
                t.buffer_type = CTS_BUFFER_DYNAMIC;
                t.rio_buffer_id = m_sendingRioBufferIds.back();
                m_sendingRioBufferIds.pop_back();
            }
            m_sendPatternOffset += size;
            m_sendPatternOffset %= kPatternSize;
            if ((uint64_t)t.buffer_length + t.buffer_offset > g_shared.bytes)
                throw FailFast{"send task is larger than the shared sender buffer"};
        } else {
            t.io_action = CTS_TASK_RECV;
            t.buffer_type = CTS_BUFFER_DYNAMIC;
            t.buffer_length = size;
            t.buffer_offset = 0;
            t.expected_pattern_offset = m_recvPatternOffset;
            if (m_recvBufferFreeList.empty()) throw FailFast{"m_recvBufferFreeList is empty for a new Recv task"};
            t.buffer = m_recvBufferFreeList.back();
            m_recvBufferFreeList.pop_back();
            if (Rio()) {  // ctsIOPattern.cpp:716-725
                if (m_receivingRioBufferIds.empty()) throw FailFast{"m_receivingRioBufferIds is empty for a new Recv task"};
                t.rio_buffer_id = m_receivingRioBufferIds.back();
                m_receivingRioBufferIds.pop_back();
            }
            if (m_recvPatternOffset >= kPatternSize) throw FailFast{"recv pattern offset too large"};
        }
        return t;
    }
    cts_task CreateTrackedTask(uint8_t a, uint32_t maxTransfer = 0)
    {
        cts_task t = CreateNewTask(a, maxTransfer);
        t.track_io = 1;
        return t;
    }

    cts_task InitiateIo()  // ctsIOPattern.cpp:251-356
    {
        cts_task t{};
        t.rio_buffer_id = kRioInvalid;
        switch (state.GetNextPatternType()) {
        case PatternType::MoreIo:
            t = GetNextTaskFromPattern();
            if (t.io_action == CTS_TASK_NONE) t.rio_buffer_id = kRioInvalid;
            break;
        case PatternType::NoIo: break;
        case PatternType::SendConnectionId:
        case PatternType::RecvConnectionId:
            t.io_action = cfg.listening ? CTS_TASK_SEND : CTS_TASK_RECV;
            t.buffer = connection_id;
            t.rio_buffer_id = m_rioConnectionId;
            t.buffer_length = CTS_CONNECTION_ID_LENGTH;
            t.buffer_type = CTS_BUFFER_TCP_CONNECTION_ID;
            break;
        case PatternType::SendCompletion:
        case PatternType::RecvCompletion:
            t.io_action = cfg.listening ? CTS_TASK_SEND : CTS_TASK_RECV;
            t.buffer = m_completionMessageBuffer.data();
            t.rio_buffer_id = m_rioCompletionMessage;
            t.buffer_length = CTS_COMPLETION_MESSAGE_SIZE;
            t.buffer_type = CTS_BUFFER_COMPLETION_MESSAGE;
            break;
        case PatternType::HardShutdown: t.io_action = CTS_TASK_HARD_SHUTDOWN; break;
        case PatternType::GracefulShutdown: t.io_action = CTS_TASK_GRACEFUL_SHUTDOWN; break;
        case PatternType::RequestFin:
            t.io_action = CTS_TASK_RECV;
            t.buffer = m_completionMessageBuffer.data();
            t.rio_buffer_id = m_rioCompletionMessage;
            t.buffer_length = CTS_COMPLETION_MESSAGE_SIZE;
            t.buffer_type = CTS_BUFFER_STATIC;
            break;
        }
        state.NotifyNextTask(t);
        return t;
    }

    // ---- VerifyBuffer ------------------------------------------------------------------------
    void RecordFailure(uint32_t completion, uint32_t transferred, const cts_verify_result& r, uint64_t recv_after)
    {
        ++buffers_failed;
        if (has_failure) return;
        has_failure = true;
        fail_completion = completion;
        fail_length = transferred;
        fail_offset = r.first_mismatch;
        fail_expected = r.expected;
        fail_actual = r.actual;
        bytes_recv_at_failure = recv_after;
    }

    int EnsureStream()  // on the engine's device, not the calling thread's current one
    {
        if (stream != nullptr) return CTS_OK;
        void* s = nullptr;
        const int rc = cts_engine_stream_create(engine, &s);
        stream = static_cast<hipStream_t>(s);
        return rc;
    }

    // One buffer, now (ctsIOPattern.cpp:745-775). Returns CTS_OK and sets *pass.
    int VerifyNow(const cts_task& t, uint32_t transferred, cts_verify_result& r)
    {
        const char* src = t.buffer + t.buffer_offset;
        if (hook != nullptr) {
            cts_buf_desc d{0, transferred, t.expected_pattern_offset, 0, 0};
            return hook(hook_ctx, reinterpret_cast<const uint8_t*>(src), transferred, &d, 1, &r) == 0 ? CTS_OK
                                                                                                      : CTS_E_INVALID;
        }
        if (engine == nullptr) return CTS_E_INVALID;
        const uint8_t* rp = reinterpret_cast<const uint8_t*>(src);
        if (recv_pinned.host != nullptr && rp >= recv_pinned.host && rp + transferred <= recv_pinned.host + recv_pinned.bytes) {
            // zero copy: the kernel reads the pinned recv buffer in place over PCIe, as up to
            // cts::kSliceMax slices so the reads go out together (latency-bound; cts_slices.hpp)
            int mailbox = 0;
            if (cts_engine_get_attr(engine, CTS_ATTR_SYNC_MAILBOX, &mailbox) == CTS_OK && mailbox)
                return cts_verify_mapped(engine, recv_pinned.dev + (rp - recv_pinned.host), transferred,
                                         t.expected_pattern_offset, &r);
            int rc = EnsureStream();
            if (rc != CTS_OK) return rc;
            constexpr uint32_t kResAt = cts::kSliceMax * sizeof(cts_buf_desc);
            if (one.host == nullptr &&
                (rc = one.alloc(engine, kResAt + cts::kSliceMax * sizeof(cts_verify_result))) != CTS_OK)
                return rc;
            uint32_t slice_len = 0;
            const uint32_t ns = cts::slice_plan((uint64_t)(rp - recv_pinned.host), transferred,
                                                t.expected_pattern_offset, 0, reinterpret_cast<cts_buf_desc*>(one.host),
                                                &slice_len);
            rc = cts_verify(engine, recv_pinned.dev, recv_pinned.bytes, reinterpret_cast<cts_buf_desc*>(one.dev), ns,
                            slice_len, reinterpret_cast<cts_verify_result*>(one.dev + kResAt), nullptr, nullptr, 0,
                            stream);
            if (rc != CTS_OK) return rc;
            EngineDevice on(engine);
            if (hipStreamSynchronize(stream) != hipSuccess) return CTS_E_HIP;
            r = cts::slice_merge(reinterpret_cast<const cts_verify_result*>(one.host + kResAt), ns, slice_len,
                                 transferred);
            return CTS_OK;
        }
        return cts_verify_host(engine, src, transferred, t.expected_pattern_offset, &r);
    }

    uint64_t StageCapacity() const { return cfg.batch_bytes ? cfg.batch_bytes : (64ull << 20); }
    uint32_t BatchCapacity() const { return cfg.batch_buffers ? cfg.batch_buffers : 1024u; }
    bool DoubleBuffered() const { return engine != nullptr && hook == nullptr; }  // launches pipelined (Depth())
    // Batches in flight at once (pipelined: at least 1, and at most BatchCapacity() - 1 so that a launch holds a
    // buffer or more)
    uint32_t Depth() const
    {
        const uint32_t b = BatchCapacity();
        return b < 3u ? 1u : std::min(depth_env, b - 1u);
    }
    uint32_t Sets() const { return Depth() + 1u; }  // descriptor / result sets: the filling batch + those in flight
    // Completions queued before a batch goes to the device. Pipelined, each launch holds BatchCapacity() / Sets():
    // the oldest launch is retired at the latest when the filling one is full and Depth() are in flight, so every
    // verdict is known within BatchCapacity() completions of its own (fewer when a kernel is seen done earlier).
    uint32_t LaunchAt() const
    {
        const uint32_t b = BatchCapacity();
        return DoubleBuffered() && queue_in_ring ? std::max(1u, b / Sets()) : b;
    }

    // The oldest in-flight batch's kernel has finished (a non-blocking event query; CompleteIo asks every 16th
    // completion: a query costs about a microsecond, a completion of 64 KiB arrives every ~1.3 us at 50 GB/s).
    bool InflightDone() const
    {
        return !flights.empty() && flights.front().done && hipEventQuery(flights.front().done) == hipSuccess;
    }
    cts_buf_desc* StageDescs() const
    {
        return reinterpret_cast<cts_buf_desc*>(stage_desc.host) + (size_t)desc_set * BatchCapacity();
    }

    // Queue one buffer for the next batch (DEFERRED). Returns CTS_OK.
    bool InRing(const char* p, uint32_t n) const
    {
        return ring && p >= ring_base && p + n <= ring_base + ring_bytes;
    }

    int EnsureBatchDescs()
    {
        if (hook != nullptr) {
            if (hdesc.size() < BatchCapacity()) {
                hdesc.resize(BatchCapacity());
                hres.resize(BatchCapacity());
            }
            return CTS_OK;
        }
        if (engine == nullptr) return CTS_E_INVALID;
        return EnsureStageDescs();
    }

    int EnsureStageDescs()  // every set
    {
        if (stage_desc.host != nullptr) return CTS_OK;
        int rc;
        const uint64_t n = (uint64_t)Sets() * BatchCapacity();
        if ((rc = stage_desc.alloc(engine, sizeof(cts_buf_desc) * n)) != CTS_OK) return rc;
        return stage_res.alloc(engine, sizeof(cts_verify_result) * n);
    }

    int Enqueue(const cts_task& t, uint32_t transferred, uint64_t recv_after)
    {
        const char* src = t.buffer + t.buffer_offset;
        if (InRing(src, transferred) && (queue.empty() || queue_in_ring)) {
            // zero copy: the batch descriptor points at the recv buffer itself
            const int rc = EnsureBatchDescs();
            if (rc != CTS_OK) return rc;
            cts_buf_desc* descs = hook ? hdesc.data() : StageDescs();
            descs[queue.size()] = cts_buf_desc{(uint64_t)(src - ring_base), transferred, t.expected_pattern_offset, 0, 0};
            queue.push_back(Queued{recv_completions, transferred, recv_after, bytes_sent, t.expected_pattern_offset,
                                status_recv, status_sent});
            queue_in_ring = true;
            return CTS_OK;
        }
        if (!queue.empty() && queue_in_ring) {  // never mix ring and staged entries in one batch
            const int rc = Flush();
            if (rc < 0) return rc;
        }
        queue_in_ring = false;
        const uint64_t slot = ((uint64_t)transferred + 15u) & ~15ull;
        if (!queue.empty() && stage_used + slot > StageCapacity()) {
            const int rc = Flush();
            if (rc < 0) return rc;
        }
        const uint64_t cap = std::max<uint64_t>(StageCapacity(), slot);
        uint8_t* base = nullptr;
        if (hook != nullptr) {
            if (hstage.size() < cap) hstage.resize(cap);
            if (hdesc.size() < BatchCapacity()) {
                hdesc.resize(BatchCapacity());
                hres.resize(BatchCapacity());
            }
            base = hstage.data();
        } else {
            if (engine == nullptr) return CTS_E_INVALID;
            int rc;
            if (stage.bytes < cap) {
                stage.release();
                if ((rc = stage.alloc(engine, cap)) != CTS_OK) return rc;
            }
            if ((rc = EnsureStageDescs()) != CTS_OK) return rc;
            base = stage.host;
        }
        if (transferred) std::memcpy(base + stage_used, t.buffer + t.buffer_offset, transferred);
        cts_buf_desc* descs = hook ? hdesc.data() : StageDescs();
        descs[queue.size()] = cts_buf_desc{stage_used, transferred, t.expected_pattern_offset, 0, 0};
        queue.push_back(Queued{recv_completions, transferred, recv_after, bytes_sent, t.expected_pattern_offset,
                                status_recv, status_sent});
        stage_used += slot;
        return CTS_OK;
    }

    int LaunchBatch()  // verifies `queue` (descriptor set desc_set) on the pattern's stream, async
    {
        int rc = EnsureStream();
        if (rc != CTS_OK) return rc;
        uint32_t maxlen = 0;
        for (const auto& q : queue) maxlen = std::max(maxlen, q.transferred);
        const uint8_t* arena = queue_in_ring ? recv_pinned.dev : stage.dev;
        const uint64_t bytes = queue_in_ring ? recv_pinned.bytes : stage.bytes;
        const size_t set = (size_t)desc_set * BatchCapacity();
        return cts_verify(engine, arena, bytes, reinterpret_cast<cts_buf_desc*>(stage_desc.dev) + set,
                          (uint32_t)queue.size(), maxlen, reinterpret_cast<cts_verify_result*>(stage_res.dev) + set,
                          nullptr, nullptr, 0, stream);
    }

    // cts_io_pattern_destroy bounds its waits (a hung kernel must not hang teardown): while set, every wait below
    // polls its event and gives up with hipErrorNotReady once wait_deadline has passed.
    bool bounded_wait = false;
    std::chrono::steady_clock::time_point wait_deadline{};
    hipError_t PollEvent(hipEvent_t e, uint32_t step_us)
    {
        for (;;) {
            const hipError_t q = hipEventQuery(e);
            if (q != hipErrorNotReady) return q;
            if (bounded_wait && std::chrono::steady_clock::now() > wait_deadline) return hipErrorNotReady;
            std::this_thread::sleep_for(std::chrono::microseconds(step_us));
        }
    }

    // Waits for everything enqueued on the pattern's stream. With retire_wait 2 (or a bounded wait) it sleeps in
    // `step_us` steps between non-blocking queries of an event recorded behind the work (the runtime's own waits
    // spin first).
    hipEvent_t sync_done = nullptr;
    hipError_t SleepSync(uint32_t step_us)
    {
        const auto w0 = std::chrono::steady_clock::now();
        const hipError_t rc = SleepSyncImpl(step_us);
        AddVerifyWait(w0);
        return rc;
    }
    hipError_t SleepSyncImpl(uint32_t step_us)
    {
        EngineDevice on(engine);
        if (retire_wait != 2 && !bounded_wait) return hipStreamSynchronize(stream);
        if (sync_done == nullptr && hipEventCreateWithFlags(&sync_done, hipEventDisableTiming) != hipSuccess) {
            sync_done = nullptr;
            return bounded_wait ? hipErrorNotReady : hipStreamSynchronize(stream);
        }
        const hipError_t rc = hipEventRecord(sync_done, stream);
        if (rc != hipSuccess) return rc;
        return PollEvent(sync_done, step_us);
    }

    // A plain wait for the pattern's stream, bounded like the others while cts_io_pattern_destroy runs.
    hipError_t StreamWait(uint32_t step_us)
    {
        if (bounded_wait) return SleepSyncImpl(step_us);
        EngineDevice on(engine);
        return hipStreamSynchronize(stream);
    }

    hipError_t WaitInflight(hipEvent_t done)  // the kernel behind `done`
    {
        EngineDevice on(engine);
        if (bounded_wait) return done != nullptr ? PollEvent(done, 50) : SleepSyncImpl(50);
        if (done == nullptr || retire_wait == 0) return hipStreamSynchronize(stream);
        if (retire_wait == 1) return hipEventSynchronize(done);
        return PollEvent(done, 50);
    }

    // Waits for the oldest in-flight batch and applies its verdicts. A failure in it takes back everything completed
    // after the failing buffer: the batches launched after it and the filling batch are dropped.
    int RetireOldest()
    {
        if (flights.empty()) return CTS_OK;
        Flight& f = flights.front();
        const auto w0 = std::chrono::steady_clock::now();
        const hipError_t wr = WaitInflight(f.done);
        AddVerifyWait(w0);
        if (wr != hipSuccess) return CTS_E_HIP;
        const bool failed = ApplyVerdicts(
            f.q, reinterpret_cast<const cts_verify_result*>(stage_res.host) + (size_t)f.set * BatchCapacity());
        spare_events.push_back(f.done);
        f.q.clear();
        spare_queues.push_back(std::move(f.q));
        flights.pop_front();
        if (failed) {
            // the later kernels' verdicts are never applied; they finish before their sets are written again
            if (!flights.empty() && SleepSyncImpl(50) != hipSuccess) return CTS_E_HIP;
            for (Flight& g : flights) spare_events.push_back(g.done);
            flights.clear();
            queue.clear();
            stage_used = 0;
        }
        PublishIfSettled();
        return CTS_OK;
    }
    int Retire()  // every in-flight batch, oldest first, up to a failing one
    {
        const bool had_failure = has_failure;
        while (!flights.empty()) {
            const int rc = RetireOldest();
            if (rc != CTS_OK) return rc;
            if (has_failure && !had_failure) break;
        }
        return CTS_OK;
    }
    int RetireDone()  // the in-flight batches whose kernels have finished, oldest first
    {
        const bool had_failure = has_failure;
        while (InflightDone()) {
            const int rc = RetireOldest();
            if (rc != CTS_OK) return rc;
            if (has_failure && !had_failure) break;
        }
        return CTS_OK;
    }

    // The filling batch is full: retire the oldest in-flight one if Depth() are running, launch this one and keep
    // receiving.
    int Rotate()
    {
        if (!DoubleBuffered() || !queue_in_ring) return Flush();
        const bool had_failure = has_failure;
        while (flights.size() >= Depth()) {
            const int rc = RetireOldest();
            if (rc != CTS_OK) return rc;
            if (has_failure && !had_failure) return GetCurrentStatus();  // an in-flight batch failed
        }
        if (queue.empty()) return GetCurrentStatus();
        const int lr = LaunchBatch();
        if (lr != CTS_OK) return lr;
        EngineDevice on(engine);
        hipEvent_t e = nullptr;
        if (!spare_events.empty()) {
            e = spare_events.back();
            spare_events.pop_back();
        } else if (hipEventCreateWithFlags(&e, hipEventDisableTiming | (retire_wait == 1 ? hipEventBlockingSync : 0u)) !=
                   hipSuccess) {
            return CTS_E_HIP;
        }
        if (hipEventRecord(e, stream) != hipSuccess) {
            spare_events.push_back(e);
            return CTS_E_HIP;
        }
        flights.push_back(Flight{{}, e, desc_set});
        flights.back().q.swap(queue);
        if (!spare_queues.empty()) {
            queue.swap(spare_queues.back());
            spare_queues.pop_back();
        }
        queue.clear();
        desc_set = (desc_set + 1u) % Sets();
        return GetCurrentStatus();
    }

    int Flush()  // cts_io_pattern_flush
    {
        const int rr = Retire();
        if (rr != CTS_OK) return rr;
        if (queue.empty()) return GetCurrentStatus();
        const uint32_t n = (uint32_t)queue.size();
        const cts_verify_result* res = nullptr;
        if (hook != nullptr) {
            const uint8_t* arena = queue_in_ring ? reinterpret_cast<const uint8_t*>(ring_base) : hstage.data();
            const uint64_t bytes = queue_in_ring ? ring_bytes : stage_used;
            if (hook(hook_ctx, arena, bytes, hdesc.data(), n, hres.data()) != 0) return CTS_E_INVALID;
            res = hres.data();
        } else {
            const int rc = LaunchBatch();
            if (rc != CTS_OK) return rc;
            const auto w0 = std::chrono::steady_clock::now();
            const hipError_t wr = StreamWait(50);  // (destroy's flush of the filling batch: up to the deadline)
            AddVerifyWait(w0);
            if (wr != hipSuccess) return CTS_E_HIP;
            res = reinterpret_cast<const cts_verify_result*>(stage_res.host) + (size_t)desc_set * BatchCapacity();
        }
        ApplyVerdicts(queue, res);
        queue.clear();
        stage_used = 0;
        PublishIfSettled();
        return GetCurrentStatus();
    }

    // Counts the verdicts of batch q; returns true if one of its buffers failed.
    // The reference stops at the first failing buffer (its CompleteIo fails the connection on that
    // completion, ctsIOPattern.cpp:486-489, and TCP verify allows one posted recv,
    // ctsConfig.cpp:3440-3446). Buffers queued after it were never received there: they are neither
    // counted as verified nor as received, and the sends that completed after it are dropped too,
    // so every counter equals what the reference reports when it stops at that completion.
    bool ApplyVerdicts(const std::vector<Queued>& q, const cts_verify_result* res)
    {
        const uint32_t n = (uint32_t)q.size();
        uint32_t bad = n;
        for (uint32_t i = 0; i < n; ++i)
            if (!res[i].pass) {
                bad = i;
                break;
            }
        const uint32_t counted = bad < n ? bad + 1 : n;
        for (uint32_t i = 0; i < counted; ++i) {
            ++buffers_verified;
            bytes_verified += q[i].transferred;
        }
        if (n == 0) return false;
        if (bad == n) {
            // every buffer of the batch verified: the bytes up to its last completion are the reference's
            Publish(q[n - 1].status_recv_after, q[n - 1].status_sent_after);
            return false;
        }
        const Queued& f = q[bad];
        RecordFailure(f.completion, f.transferred, res[bad], f.bytes_recv_after);
        // the failing completion's own bytes are counted (the reference adds them after VerifyBuffer failed,
        // ctsIOPattern.cpp:505-516); nothing after it is
        Publish(f.status_recv_after, f.status_sent_after);
        RollbackAfter(f);
        UpdateLastError(CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN);
        return true;
    }

    // Drop the byte accounting (ctsStatistics, the pattern state and the recv pattern offset) of every
    // completion after the failing buffer f (DEFERRED; see Flush). Those bytes were held back, never
    // published to TcpStatusDetails, so the process-wide counters are not touched.
    void RollbackAfter(const Queued& f)
    {
        const uint64_t recv_undo = bytes_recv - f.bytes_recv_after;
        const uint64_t send_undo = bytes_sent - f.bytes_sent_after;
        bytes_recv = f.bytes_recv_after;
        bytes_sent = f.bytes_sent_after;
        status_recv = f.status_recv_after;
        status_sent = f.status_sent_after;
        state.RollbackConfirmed(recv_undo + send_undo);
        m_recvPatternOffset = (uint32_t)(((uint64_t)f.expected + f.transferred) % kPatternSize);
        recv_completions = f.completion + 1;
    }

    bool Deferred() const { return cfg.verify_mode == CTS_VERIFY_DEFERRED; }

    bool VerifyGate(const cts_task& t) const  // ctsIOPattern.cpp:475-479
    {
        return cfg.protocol == CTS_PROTOCOL_TCP && cfg.verify_buffers && t.io_action == CTS_TASK_RECV && t.track_io;
    }

    int CompleteIo(const cts_task& t, uint32_t transfer, uint32_t status)  // ctsIOPattern.cpp:364-534
    {
        // DEFERRED: anything but a plain in-transfer tracked send/recv sees the
        // queued verdicts first, so a pending data error latches before it.
        bool benign = status == kNoError && (t.io_action == CTS_TASK_SEND || t.io_action == CTS_TASK_RECV) &&
                      state.WouldStayMoreIo(t, transfer) && m_lastError == kStatusIoRunning;
        if (Deferred() && benign && query_period != 0 && (queue.size() & (query_period - 1u)) == 0 && InflightDone()) {
            // the in-flight batch's verdicts are in: apply them now, so a data error fails the connection at
            // this completion rather than at the next launch (ctsIOPattern.cpp:486-489 fails it at the
            // failing one; the completions in between are taken back by RollbackAfter)
            const bool had_failure = has_failure;
            const int rc = RetireDone();
            if (rc < 0) return rc;
            if (has_failure && !had_failure) return GetCurrentStatus();
        }
        if (Deferred() && (!queue.empty() || !flights.empty()) && !benign) {
            const bool had_failure = has_failure;
            const int rc = Flush();
            if (rc < 0) return rc;
            // a queued buffer failed: the reference failed the connection at that completion and never
            // saw this one, so it is not accounted (ctsIOPattern.cpp:486-489)
            if (has_failure && !had_failure) return GetCurrentStatus();
        }
        const bool wasIoRequestedFromPattern = state.IsCurrentStateMoreIo();
        if (t.buffer_type == CTS_BUFFER_DYNAMIC) {  // ctsIOPattern.cpp:369-386
            if (t.io_action == CTS_TASK_RECV) RecycleRecvBuffer(t);
            else if (Rio() && t.io_action == CTS_TASK_SEND) m_sendingRioBufferIds.push_back(t.rio_buffer_id);
        }

        bool verified_now = false, defer_this = false;
        cts_verify_result vr{};
        switch (t.io_action) {
        case CTS_TASK_NONE: break;
        case CTS_TASK_FATAL_ABORT: UpdateLastError(CTS_STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED); break;
        case CTS_TASK_ABORT: break;
        case CTS_TASK_GRACEFUL_SHUTDOWN:
        case CTS_TASK_HARD_SHUTDOWN:
        case CTS_TASK_RECV:
        case CTS_TASK_SEND: {
            bool verifyIo = true;
            if (t.buffer_type == CTS_BUFFER_TCP_CONNECTION_ID || t.buffer_type == CTS_BUFFER_COMPLETION_MESSAGE) {
                verifyIo = false;
                if (status != kNoError) {
                    UpdateLastError(status);
                } else {
                    UpdateLastPatternError(state.CompletedTask(t, transfer));
                }
            } else if (status != kNoError) {
                if (!(t.io_action == CTS_TASK_RECV && state.IsCompleted())) {
                    if (UpdateLastError(status) != kStatusIoRunning) verifyIo = false;
                }
            }
            if (verifyIo) {
                const PatternError ps = state.CompletedTask(t, transfer);
                UpdateLastPatternError(ps);
                if (VerifyGate(t) && (ps == PatternError::SuccessfullyCompleted || ps == PatternError::NoError)) {
                    if (t.expected_pattern_offset != m_recvPatternOffset)
                        throw FailFast{"task expected_pattern_offset does not match the current pattern offset"};
                    if (Deferred()) {
                        defer_this = true;
                    } else {
                        const int rc = VerifyNow(t, transfer, vr);
                        if (rc != CTS_OK) return rc;
                        verified_now = true;
                    }
                    m_recvPatternOffset += transfer;
                    m_recvPatternOffset %= kPatternSize;
                }
            }
            break;
        }
        default: throw FailFast{"CompleteIo: unknown task action"};
        }

        if (t.io_action != CTS_TASK_NONE && status == kNoError) {
            // TcpStatusDetails (ctsIOPattern.cpp:505-516): published below, or held back while a verdict is pending
            if (t.io_action == CTS_TASK_SEND) status_sent += transfer;
            else if (t.io_action == CTS_TASK_RECV) status_recv += transfer;
            if (wasIoRequestedFromPattern) UpdateLastPatternError(CompleteTaskBackToPattern(t, transfer));
        }
        if (verified_now) {
            ++buffers_verified;
            bytes_verified += transfer;
            if (!vr.pass) {
                RecordFailure(recv_completions, transfer, vr, bytes_recv);
                UpdateLastError(CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN);
            }
        }
        if (defer_this) {
            const int rc = Enqueue(t, transfer, bytes_recv);
            if (rc < 0) return rc;
            if (!benign || queue.size() >= LaunchAt()) {
                const int fr = benign ? Rotate() : Flush();
                if (fr < 0) return fr;
            }
        }
        if (t.io_action == CTS_TASK_RECV && t.track_io) ++recv_completions;
        PublishIfSettled();
        if (state.IsCompleted()) UpdateLastError(kNoError);
        return GetCurrentStatus();
    }
};

// The reference verifies inside CompleteIo *before* CompleteTaskBackToPattern
// adds the bytes to m_statistics; the data-error latch order is identical here
// (UpdateLastError keeps the first error), the verify call merely runs after the
// byte accounting so bytes_recv_at_failure includes the failing completion, as
// ctsIOPattern.cpp:505-521 counts it.

namespace {

// ---- concrete patterns (ctsIOPattern.cpp:796-1031) -------------------------------------------
struct PushOrPull : cts_io_pattern {
    // Push: the client sends, the server receives. Pull: the reverse.
    PushOrPull(const cts_pattern_config& c, uint32_t maxbuf, bool receiving)
        : cts_io_pattern(c, maxbuf, receiving ? c.pre_post_recvs : 0),
          m_ioAction(receiving ? CTS_TASK_RECV : CTS_TASK_SEND),
          m_recvNeeded(receiving ? c.pre_post_recvs : 0)
    {
    }
    uint8_t m_ioAction;
    uint32_t m_recvNeeded;
    uint32_t m_sendBytesInFlight = 0;
    cts_task GetNextTaskFromPattern() override  // :803-822 / :856-875
    {
        if (m_ioAction == CTS_TASK_RECV && m_recvNeeded > 0) {
            --m_recvNeeded;
            return CreateTrackedTask(m_ioAction);
        }
        if (m_ioAction == CTS_TASK_SEND && GetIdealSendBacklog() > m_sendBytesInFlight) {
            const cts_task t = CreateTrackedTask(m_ioAction);
            m_sendBytesInFlight += t.buffer_length;
            return t;
        }
        return cts_task{};
    }
    PatternError CompleteTaskBackToPattern(const cts_task& t, uint32_t bytes) override  // :824-838
    {
        if (t.io_action == CTS_TASK_SEND) {
            bytes_sent += bytes;
            m_sendBytesInFlight -= bytes;
        } else if (t.io_action == CTS_TASK_RECV) {
            bytes_recv += bytes;
            ++m_recvNeeded;
        }
        return PatternError::NoError;
    }
};

struct PushPull : cts_io_pattern {  // :888-966
    PushPull(const cts_pattern_config& c, uint32_t maxbuf)
        : cts_io_pattern(c, maxbuf, 1), m_push(c.push_bytes), m_pull(c.pull_bytes), m_listening(c.listening != 0),
          m_sending(c.listening == 0)
    {
    }
    uint32_t m_push, m_pull, m_intra = 0;
    bool m_listening, m_ioNeeded = true, m_sending;
    uint32_t Segment() const
    {
        return m_listening ? (m_sending ? m_pull : m_push) : (m_sending ? m_push : m_pull);
    }
    cts_task GetNextTaskFromPattern() override
    {
        const uint32_t seg = Segment();
        if (m_intra >= seg) throw FailFast{"invalid PushPull state: intra-segment transfer >= segment size"};
        if (m_ioNeeded) {
            m_ioNeeded = false;
            return CreateTrackedTask(m_sending ? CTS_TASK_SEND : CTS_TASK_RECV, seg - m_intra);
        }
        return cts_task{};
    }
    PatternError CompleteTaskBackToPattern(const cts_task& t, uint32_t bytes) override
    {
        if (t.io_action == CTS_TASK_SEND) bytes_sent += bytes;
        else if (t.io_action == CTS_TASK_RECV) bytes_recv += bytes;
        m_ioNeeded = true;
        m_intra += bytes;
        const uint32_t seg = Segment();
        if (m_intra > seg) throw FailFast{"invalid PushPull state: intra-segment transfer > segment size"};
        if (seg == m_intra) {
            m_sending = !m_sending;
            m_intra = 0;
        }
        return PatternError::NoError;
    }
};

struct Duplex : cts_io_pattern {  // :968-1031
    Duplex(const cts_pattern_config& c, uint32_t maxbuf)
        : cts_io_pattern(c, maxbuf, c.pre_post_recvs), m_recvNeeded(c.pre_post_recvs)
    {
        uint64_t total = GetTotalTransfer();
        if (total % 2 != 0) SetTotalTransfer(++total);
        m_remainingSend = total / 2;
        m_remainingRecv = m_remainingSend;
    }
    uint64_t m_remainingSend = 0, m_remainingRecv = 0;
    uint32_t m_recvNeeded;
    uint32_t m_sendBytesInFlight = 0;
    cts_task GetNextTaskFromPattern() override
    {
        constexpr uint64_t kMaxLong = 0x7FFFFFFF;
        cts_task t{};
        if (m_remainingRecv > 0 && m_recvNeeded > 0) {
            t = CreateTrackedTask(CTS_TASK_RECV, (uint32_t)std::min(m_remainingRecv, kMaxLong));
            m_remainingRecv -= t.buffer_length;
            --m_recvNeeded;
        } else if (m_remainingSend > 0 && GetIdealSendBacklog() > m_sendBytesInFlight) {
            t = CreateTrackedTask(CTS_TASK_SEND, (uint32_t)std::min(m_remainingSend, kMaxLong));
            m_remainingSend -= t.buffer_length;
            m_sendBytesInFlight += t.buffer_length;
        }
        return t;
    }
    PatternError CompleteTaskBackToPattern(const cts_task& t, uint32_t bytes) override
    {
        if (t.io_action == CTS_TASK_SEND) {
            bytes_sent += bytes;
            m_sendBytesInFlight -= bytes;
            m_remainingSend += t.buffer_length;
            m_remainingSend -= bytes;
        } else if (t.io_action == CTS_TASK_RECV) {
            bytes_recv += bytes;
            ++m_recvNeeded;
            m_remainingRecv += t.buffer_length;
            m_remainingRecv -= bytes;
        }
        return PatternError::NoError;
    }
};

// ---- MediaStream (UDP) patterns -----------------------------------------------------------------
uint16_t load_u16(const char* p)
{
    uint16_t v;
    std::memcpy(&v, p, sizeof v);
    return v;
}
int64_t load_i64(const char* p)
{
    int64_t v;
    std::memcpy(&v, p, sizeof v);
    return v;
}

// ctsIoPatternMediaStreamServer (ctsIOPattern.cpp:1100-1175): the connection-id datagram, then one tracked send
// of one frame per frame, timed to the frame rate.
struct MediaStreamServer : cts_io_pattern {
    MediaStreamServer(const cts_pattern_config& c, uint32_t maxbuf)
        : cts_io_pattern(c, maxbuf, 1),  // one recv buffer: the connection-id datagram is built in it
          m_frameSizeBytes(c.buffer_size_low), m_frameRateFps(c.ms_frames_per_second)
    {
    }
    enum class ServerState { NotStarted, IdSent, IoStarted } m_state = ServerState::NotStarted;
    // its one recv buffer only ever holds the connection-id datagram, and it receives nothing to verify (no ring)
    uint32_t RecvSlotBytes() const override { return (CTS_UDP_CONNECTION_ID_HEADER_LENGTH + 15u) & ~15u; }
    bool VerifiesRecvs() const override { return false; }
    int64_t m_baseTimeMilliseconds = 0;
    uint32_t m_frameSizeBytes;
    uint32_t m_currentFrameRequested = 0;
    uint32_t m_currentFrameCompleted = 0;
    uint32_t m_frameRateFps;
    uint32_t m_currentFrame = 1;
    int64_t m_bitsReceived = 0;  // m_statistics.m_bitsReceived (counts the bits sent)

    cts_task GetNextTaskFromPattern() override  // :1119-1154
    {
        cts_task t{};
        t.rio_buffer_id = kRioInvalid;
        switch (m_state) {
        case ServerState::NotStarted: {
            // ctsMediaStreamMessage::MakeConnectionIdTask (ctsMediaStreamProtocol.hpp:389-405) over a writable
            // (recv) buffer of c_udpDatagramConnectionIdHeaderLength bytes
            t = CreateNewTask(CTS_TASK_RECV, CTS_UDP_CONNECTION_ID_HEADER_LENGTH);
            if (t.buffer_length != CTS_CONNECTION_ID_LENGTH + CTS_UDP_FLAG_LENGTH)
                throw FailFast{"MakeConnectionIdTask: the task's buffer length is not the connection-id datagram length"};
            const uint16_t flag = CTS_UDP_FLAG_ID;
            std::memcpy(t.buffer, &flag, CTS_UDP_FLAG_LENGTH);
            std::memcpy(t.buffer + CTS_UDP_FLAG_LENGTH, connection_id, CTS_CONNECTION_ID_LENGTH);
            t.io_action = CTS_TASK_SEND;
            t.buffer_type = CTS_BUFFER_UDP_CONNECTION_ID;
            t.track_io = 0;
            m_state = ServerState::IdSent;
            break;
        }
        case ServerState::IdSent:
            m_baseTimeMilliseconds = NowMs();
            m_state = ServerState::IoStarted;
            [[fallthrough]];
        case ServerState::IoStarted:
            if (m_currentFrameRequested < m_frameSizeBytes) {
                t = CreateTrackedTask(CTS_TASK_SEND, m_frameSizeBytes);
                // the time of this frame relative to now
                t.time_offset_ms = m_baseTimeMilliseconds + ((int64_t)m_currentFrame * 1000LL / m_frameRateFps) - NowMs();
                m_currentFrameRequested += t.buffer_length;
            }
            break;
        }
        return t;
    }

    PatternError CompleteTaskBackToPattern(const cts_task& t, uint32_t currentTransfer) override  // :1156-1173
    {
        if (t.buffer_type != CTS_BUFFER_UDP_CONNECTION_ID) {
            const int64_t bits = (int64_t)currentTransfer * 8;
            cts::udp_status_add_bits(bits);
            m_bitsReceived += bits;
            m_currentFrameCompleted += currentTransfer;
            if (m_currentFrameCompleted == m_frameSizeBytes) {
                ++m_currentFrame;
                m_currentFrameRequested = 0;
                m_currentFrameCompleted = 0;
            }
        }
        return PatternError::NoError;
    }

    int UdpStats(cts_media_stream_stats* o) override
    {
        *o = cts_media_stream_stats{};
        o->bits_received = m_bitsReceived;
        o->last_error = m_lastError;
        return CTS_OK;
    }
};

// ctsIoPatternMediaStreamClient (ctsIOPatternMediaStream.cpp:46-530): untracked recvs of one datagram each;
// every data datagram's payload is verified (on the GPU) and booked to its frame in the jitter queue, which
// the renderer timer drains at the frame rate. The frame accounting is the one cts_media_stream_client_*
// exports (cts_media_stream.cpp); the pattern adds the recv tasks, the header checks, the verify and the timers.
struct MediaStreamClient : cts_io_pattern {
    MediaStreamClient(const cts_pattern_config& c, uint32_t maxbuf)
        : cts_io_pattern(c, maxbuf, c.pre_post_recvs),
          m_frameRateMsPerFrame(1000.0 / (double)c.ms_frames_per_second), m_frameSizeBytes(c.buffer_size_low),
          m_recvNeeded(c.pre_post_recvs), m_maxDatagramSize(c.ms_datagram_max_size), manual(c.ms_manual_timers != 0)
    {
    }
    void StopTimers() override
    {
        {
            std::lock_guard<std::recursive_mutex> lk(mu);
            stop = true;
            start_due = render_due = -1;
        }
        cv.notify_all();
        if (timer_thread.joinable()) timer_thread.join();
    }
    ~MediaStreamClient() override
    {
        StopTimers();
        if (ms != nullptr) (void)cts_media_stream_client_destroy(ms);
        EngineDevice on(engine);
        if (d_sums != nullptr) (void)hipFreeAsync(d_sums, stream);
        if (stream != nullptr) (void)hipStreamSynchronize(stream);
    }

    cts_media_stream_client* ms = nullptr;  // the jitter queue and frame accounting
    int64_t m_baseTimeMilliseconds = 0;
    const double m_frameRateMsPerFrame;
    const uint32_t m_frameSizeBytes;
    uint32_t m_recvNeeded;
    const uint32_t m_maxDatagramSize;
    uint64_t datagrams = 0;  // recv completions handed to CompleteTaskBackToPattern
    // the two timers (ctsIOPatternMediaStream.cpp:321-364): when each is due on the pattern clock, -1 = not armed
    const bool manual;
    int64_t start_due = -1, render_due = -1;
    bool stop = false;
    std::condition_variable_any cv;
    std::thread timer_thread;

    bool NeedsVerifier(const cts_task& t) const override  // every recv is a datagram to verify
    {
        return cfg.verify_buffers && t.io_action == CTS_TASK_RECV;
    }
    // every recv is one datagram of min(frame, DatagramMaxSize) bytes (GetNextTaskFromPattern): a slot of a frame's
    // size would leave 97 % of a README-sized (52083-B) slot unused, per slot of the DEFERRED ring
    uint32_t RecvSlotBytes() const override
    {
        return (std::max(std::min(m_frameSizeBytes, m_maxDatagramSize), 16u) + 15u) & ~15u;
    }

    // ---- DEFERRED: batched datagram verify (round 3) ---------------------------------------------------------
    // A data datagram whose header the CPU has checked (it is in host memory) stays in its recv-ring slot and is
    // queued; a batch goes to the GPU's frame-sum receive pass (cts_media_stream_verify_frames), whose sums are
    // applied as CompleteTaskBackToPattern would have applied each datagram (the jitter window moves only at a
    // render tick, and every tick flushes first). A batch holding a corrupt payload is replayed datagram by
    // datagram from the compact statuses (cts_media_stream_verify_status) up to that datagram, which fails the
    // stream with the first mismatch cts_verify finds in its payload. Anything else that completes (zero-byte,
    // short, unknown or ID datagram, Abort) flushes first, so the stream's status and counters are the reference's;
    // only the completion that reports a corrupt datagram comes later (at most one batch).
    struct MsQueued {
        uint64_t offset;     // of the datagram in the recv ring
        uint32_t completed;  // its bytes
        uint32_t index;      // its completion index
    };
    std::vector<MsQueued> msq, msq_spare;
    Pinned ms_desc, ms_sums, ms_status, ms_res;
    // the frame-sum pass adds into its totals and frame bytes with device-scope atomics: they live in device memory
    // (as cts_media_stream_verify_frames documents them), back to back in one allocation (the totals' shards, then one
    // u64 per window slot), so one memset clears them and one copy brings them to the pinned ms_sums: per render tick
    // a connection pays one launch, one memset and one copy (round 4; two of each before)
    static constexpr size_t kTotalsWords = CTS_FRAME_TOTAL_SHARDS * 4u;
    uint64_t* d_sums = nullptr;
    uint32_t d_sums_cap = 0;  // window slots
    // stream-ordered (hipMallocAsync / hipFreeAsync on the pattern's stream): a plain hipFree waits for the whole
    // device, and with other connections posting to the engine's resident SYNC mailbox grid that can be a long time
    int DeviceAlloc(void** p, size_t bytes)
    {
        return hipMallocAsync(p, bytes, stream) == hipSuccess ? CTS_OK : CTS_E_NOMEM;
    }

    void ApplyClean(const MsQueued& q)
    {
        const char* b = ring_base + q.offset;
        const cts::MsDatagram d{load_i64(b + CTS_UDP_FLAG_LENGTH), load_i64(b + 8), load_i64(b + 16), q.completed};
        cts::ms_client_apply_data(ms, d, ReceiverQpc(), 1000000000LL);
        ++buffers_verified;
        bytes_verified += q.completed - CTS_UDP_DATA_HEADER_LENGTH;
    }
    static int64_t ReceiverQpc()
    {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
            .count();
    }
    void FailQueued(const MsQueued& q, const cts_verify_result& r)
    {
        RecordFailure(q.index, q.completed - CTS_UDP_DATA_HEADER_LENGTH, r, 0);
        ++buffers_verified;
        bytes_verified += q.completed - CTS_UDP_DATA_HEADER_LENGTH;
        UpdateLastPatternError(Fail(q.index, PatternError::CorruptedBytes));
    }

    // Verifies and applies every queued datagram; true when one of them failed the stream.
    bool FlushMs()
    {
        if (msq.empty()) return false;
        const uint32_t n = (uint32_t)msq.size();
        // the batch moves to msq_spare and msq takes msq_spare's storage: both keep their capacity across ticks
        std::vector<MsQueued>& q = msq_spare;
        q.clear();
        q.swap(msq);
        if (hook != nullptr) {  // device-less harness: the batch verifier on the payload spans, then one by one
            std::vector<cts_buf_desc> d(n);
            std::vector<cts_verify_result> r(n);
            for (uint32_t i = 0; i < n; ++i)
                d[i] = cts_buf_desc{q[i].offset, q[i].completed, 0u, 0u, CTS_UDP_DATA_HEADER_LENGTH};
            if (hook(hook_ctx, reinterpret_cast<const uint8_t*>(ring_base), ring_bytes, d.data(), n, r.data()) != 0)
                throw DeviceError{CTS_E_INVALID};
            for (uint32_t i = 0; i < n; ++i) {
                if (!r[i].pass) {
                    FailQueued(q[i], r[i]);
                    return true;
                }
                ApplyClean(q[i]);
            }
            return false;
        }
        EngineDevice on(engine);
        int rc = EnsureStream();
        if (rc == CTS_OK && ms_desc.host == nullptr) {
            const uint32_t b = BatchCapacity();
            if ((rc = ms_desc.alloc(engine, sizeof(cts_buf_desc) * (uint64_t)b)) == CTS_OK &&
                (rc = ms_status.alloc(engine, sizeof(cts_datagram_status) * (uint64_t)b)) == CTS_OK)
                rc = ms_res.alloc(engine, sizeof(cts_verify_result) + sizeof(cts_buf_desc));
        }
        static_assert(kTotalsWords * sizeof(uint64_t) == (size_t)CTS_FRAME_TOTAL_SHARDS * 32u, "the totals block");
        cts_frame_window w{};
        if (rc == CTS_OK) rc = cts_media_stream_client_window(ms, &w);
        if (rc == CTS_OK && (d_sums == nullptr || d_sums_cap < std::max(w.frames, 1u))) {
            ms_sums.release();
            if (d_sums != nullptr) (void)hipFreeAsync(d_sums, stream);
            d_sums = nullptr;
            d_sums_cap = 0;
            const uint32_t cap = std::max(w.frames, 1u);
            const uint64_t bytes = sizeof(uint64_t) * (kTotalsWords + (uint64_t)cap);
            void* p = nullptr;
            if ((rc = DeviceAlloc(&p, bytes)) == CTS_OK && (rc = ms_sums.alloc(engine, bytes)) == CTS_OK) {
                d_sums = static_cast<uint64_t*>(p);
                d_sums_cap = cap;
            } else if (p != nullptr) {
                (void)hipFreeAsync(p, stream);
            }
        }
        if (rc != CTS_OK) throw DeviceError{rc};
        auto* descs = reinterpret_cast<cts_buf_desc*>(ms_desc.host);
        for (uint32_t i = 0; i < n; ++i) descs[i] = cts_buf_desc{q[i].offset, q[i].completed, 0u, 0u, 0u};
        rc = cts_media_stream_verify_frames(engine, recv_pinned.dev, recv_pinned.bytes,
                                            reinterpret_cast<const cts_buf_desc*>(ms_desc.dev), n, &w, d_sums,
                                            d_sums + kTotalsWords, nullptr, stream);
        if (rc == CTS_OK && hipMemcpyAsync(ms_sums.host, d_sums, sizeof(uint64_t) * (kTotalsWords + (uint64_t)w.frames),
                                           hipMemcpyDeviceToHost, stream) != hipSuccess)
            rc = CTS_E_HIP;
        // a short kernel (one render tick's datagrams) behind a launch: sleep rather than spin while it runs
        if (rc != CTS_OK || SleepSync(20) != hipSuccess) throw DeviceError{rc != CTS_OK ? rc : CTS_E_HIP};
        cts_frame_totals t{};
        (void)cts_frame_totals_fold(ms_sums.host, &t);
        if (t.exceptions == 0 && t.datagrams == n) {
            // every datagram clean: the sums are CompleteTaskBackToPattern over the batch (no sender timestamps)
            const int st = cts_media_stream_client_complete_frames(ms, &w, &t,
                                                                   reinterpret_cast<const uint64_t*>(ms_sums.host) +
                                                                       kTotalsWords,
                                                                   n, ReceiverQpc(), 1000000000LL);
            if (st < 0) throw DeviceError{st};
            buffers_verified += n;
            for (const MsQueued& e : q) bytes_verified += e.completed - CTS_UDP_DATA_HEADER_LENGTH;
            return false;
        }
        // a corrupt payload in the batch: replay from the statuses up to it
        rc = cts_media_stream_verify_status(engine, recv_pinned.dev, recv_pinned.bytes,
                                            reinterpret_cast<const cts_buf_desc*>(ms_desc.dev), n,
                                            reinterpret_cast<cts_datagram_status*>(ms_status.dev), nullptr, stream);
        if (rc != CTS_OK || StreamWait(20) != hipSuccess) throw DeviceError{rc != CTS_OK ? rc : CTS_E_HIP};
        const auto* st = reinterpret_cast<const cts_datagram_status*>(ms_status.host);
        for (uint32_t i = 0; i < n; ++i) {
            if (st[i].pass) {
                ApplyClean(q[i]);
                continue;
            }
            // the first mismatch of its payload (the reference prints it, ctsIOPattern.cpp:761-772)
            // (the descriptor first: the C ABI wants it 8-byte aligned, the result 4-byte aligned)
            *reinterpret_cast<cts_buf_desc*>(ms_res.host) =
                cts_buf_desc{q[i].offset, q[i].completed, 0u, 0u, CTS_UDP_DATA_HEADER_LENGTH};
            rc = cts_verify(engine, recv_pinned.dev, recv_pinned.bytes, reinterpret_cast<const cts_buf_desc*>(ms_res.dev),
                            1, q[i].completed, reinterpret_cast<cts_verify_result*>(ms_res.dev + sizeof(cts_buf_desc)),
                            nullptr, nullptr, 0, stream);
            if (rc != CTS_OK || StreamWait(20) != hipSuccess) throw DeviceError{rc != CTS_OK ? rc : CTS_E_HIP};
            FailQueued(q[i], *reinterpret_cast<const cts_verify_result*>(ms_res.host + sizeof(cts_buf_desc)));
            return true;
        }
        return false;
    }
    int FlushPending() override
    {
        (void)FlushMs();
        return GetCurrentStatus();
    }
    // FlushMs from a timer callback, which has no caller to return a device error to: the error fails the
    // pattern (a latched FAIL_FAST, as an inconsistency would)
    void TimerFlush()
    {
        try {
            (void)FlushMs();
        } catch (const DeviceError& d) {
            if (fail_fast.empty()) fail_fast = "the batched datagram verify failed in a timer callback (status " +
                                               std::to_string(d.rc) + ")";
            m_lastError = CTS_PATTERN_E_FAIL_FAST;
        }
    }

    bool FlushFailed() const { return m_lastError == CTS_PATTERN_E_FAIL_FAST; }

    // The batched verify failed on the device: the stream cannot be rendered further, so it ends here as a stream
    // that cannot continue does (ctsIOPatternMediaStream.cpp:490-508: a FatalAbort task). Sent once, by whichever
    // timer saw the failure first (the START timer can run before the renderer has been armed).
    bool device_abort_sent = false;
    void SendDeviceAbort()
    {
        if (device_abort_sent) return;
        device_abort_sent = true;
        cts_task t{};
        t.rio_buffer_id = kRioInvalid;
        t.io_action = CTS_TASK_FATAL_ABORT;
        SendTaskToCallback(t);
    }

    // SetNextTimer (:321-349): the renderer's next tick at base + offset frames; armed when more than 2 ms ahead
    // (always on the initial call)
    bool SetNextTimer(bool initial)
    {
        const int64_t due = m_baseTimeMilliseconds +
                            (int64_t)((double)cts::ms_client_timer_wheel_offset(ms) * m_frameRateMsPerFrame);
        if (!initial && due - NowMs() <= 2) return false;
        render_due = due;
        cv.notify_all();
        return true;
    }
    void SetNextStartTimer()  // :351-364
    {
        start_due = NowMs() + (int64_t)m_frameRateMsPerFrame + 500;
        cv.notify_all();
    }

    // StartCallback (:440-468): re-send START until the first datagram arrived
    void StartTimer()
    {
        static char kStart[] = "START";
        if (cts::ms_client_finished(ms)) return;
        TimerFlush();  // DEFERRED: the datagrams that arrived count
        if (FlushFailed()) {
            SendDeviceAbort();
            return;
        }
        if (!cts::ms_client_received_buffered_frames(ms)) {
            cts_task t{};
            t.rio_buffer_id = kRioInvalid;
            t.io_action = CTS_TASK_SEND;
            t.track_io = 0;
            t.buffer = kStart;
            t.buffer_offset = 0;
            t.buffer_length = sizeof(kStart) - 1;
            t.buffer_type = CTS_BUFFER_STATIC;
            SetNextStartTimer();
            SendTaskToCallback(t);
        }
    }
    // TimerCallback (:470-530): render frames until the next tick lies in the future
    void RenderTimer()
    {
        bool scheduled = false;
        while (!scheduled) {
            if (cts::ms_client_finished(ms)) return;
            TimerFlush();  // DEFERRED: a tick renders what arrived before it
            if (FlushFailed()) {
                SendDeviceAbort();
                return;
            }
            const int code = cts::ms_client_tick(ms);
            if (code != 0) {
                cts_task t{};
                t.rio_buffer_id = kRioInvalid;
                t.io_action = code == 2 ? CTS_TASK_FATAL_ABORT : CTS_TASK_ABORT;
                SendTaskToCallback(t);
                return;
            }
            scheduled = SetNextTimer(false);
        }
    }

    void TimerLoop()  // the threadpool timers: run each callback when it is due
    {
        std::unique_lock<std::recursive_mutex> lk(mu);
        while (!stop) {
            int64_t due = start_due;
            if (render_due >= 0 && (due < 0 || render_due < due)) due = render_due;
            if (due < 0) {
                cv.wait(lk);
                continue;
            }
            const int64_t now = NowMs();
            if (due > now) {
                // a bounded wait on the system clock: libstdc++ turns wait_for into pthread_cond_clockwait, which
                // ThreadSanitizer does not intercept (it then reports the pattern lock as double-locked); the
                // bound keeps a wall-clock step from stretching a wait
                cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(std::min<int64_t>(due - now, 50)));
                continue;
            }
            try {
                if (start_due >= 0 && start_due <= now) {
                    start_due = -1;
                    StartTimer();
                }
                if (!stop && render_due >= 0 && render_due <= now) {
                    render_due = -1;
                    RenderTimer();
                }
            } catch (const FailFast& f) {  // nothing may leave the timer thread
                if (fail_fast.empty()) fail_fast = f.reason;
                m_lastError = CTS_PATTERN_E_FAIL_FAST;
            } catch (const DeviceError& d) {
                if (fail_fast.empty()) fail_fast = "a timer callback failed (status " + std::to_string(d.rc) + ")";
                m_lastError = CTS_PATTERN_E_FAIL_FAST;
            } catch (const std::exception& e) {  // e.g. bad_alloc growing a queue: latched, never std::terminate
                if (fail_fast.empty()) fail_fast = std::string("a timer callback threw: ") + e.what();
                m_lastError = CTS_PATTERN_E_FAIL_FAST;
            }
        }
    }

    int FireTimer(int timer) override
    {
        if (timer == CTS_MS_TIMER_START) {
            start_due = -1;
            StartTimer();
        } else if (timer == CTS_MS_TIMER_RENDER) {
            render_due = -1;
            RenderTimer();
        } else {
            return CTS_E_INVALID;
        }
        return CTS_OK;
    }
    int Timers(int64_t* s, int64_t* r) override
    {
        if (s != nullptr) *s = start_due;
        if (r != nullptr) *r = render_due;
        return CTS_OK;
    }

    cts_task GetNextTaskFromPattern() override  // :115-138
    {
        if (m_baseTimeMilliseconds == 0) {
            // start the timers the first time the pattern is used: the thread first, so a thread that cannot start
            // leaves no armed timer behind and fails the pattern (a latched FAIL_FAST; nothing crosses the C ABI)
            if (!manual && !timer_thread.joinable()) {
                try {
                    timer_thread = std::thread([this] { TimerLoop(); });
                } catch (const std::system_error& e) {
                    throw FailFast{std::string("the MediaStream client's timer thread could not start: ") + e.what()};
                }
            }
            m_baseTimeMilliseconds = NowMs();
            SetNextStartTimer();
            (void)SetNextTimer(true);
        }
        cts_task t{};
        t.rio_buffer_id = kRioInvalid;
        if (m_recvNeeded > 0) {
            // one datagram per recv; a zero where the header's sequence number goes
            t = CreateNewTask(CTS_TASK_RECV, std::min(m_frameSizeBytes, m_maxDatagramSize));
            std::memset(t.buffer, 0, sizeof(int64_t));
            --m_recvNeeded;
        }
        return t;
    }

    PatternError CompleteTaskBackToPattern(const cts_task& t, uint32_t completedBytes) override  // :140-272
    {
        if (t.io_action == CTS_TASK_ABORT) {
            if (!cts::ms_client_finished(ms)) throw FailFast{"processed an Abort before the stream was finished"};
            if (FlushMs()) return PatternError::NoError;  // DEFERRED: a queued datagram failed the stream first
            return PatternError::SuccessfullyCompleted;
        }
        if (t.io_action != CTS_TASK_RECV) return PatternError::NoError;  // a START send
        const uint64_t index = datagrams++;
        const bool queue_data = Deferred() && cfg.verify_buffers && completedBytes >= CTS_UDP_DATA_HEADER_LENGTH &&
                                load_u16(t.buffer) == CTS_UDP_FLAG_DATA && InRing(t.buffer, completedBytes);
        if (queue_data) {
            // DEFERRED: verified and applied with its batch (FlushMs)
            msq.push_back(MsQueued{(uint64_t)(t.buffer - ring_base), completedBytes, (uint32_t)index});
            ++m_recvNeeded;
            if (msq.size() >= BatchCapacity()) (void)FlushMs();
            return PatternError::NoError;
        }
        if (FlushMs()) return PatternError::NoError;  // the datagrams before this one first
        if (completedBytes == 0) {
            // the final recv may complete with zero bytes once the sender closed
            return cts::ms_client_finished(ms) ? PatternError::NoError : Fail(index, PatternError::TooFewBytes);
        }
        // ValidateBufferLengthFromTask (ctsMediaStreamProtocol.hpp:284-329); GetProtocolHeaderFromTask reads the
        // flag at m_buffer itself (:331-334)
        if (completedBytes < CTS_UDP_FLAG_LENGTH) return Fail(index, PatternError::TooFewBytes);
        const uint16_t flag = load_u16(t.buffer);
        if (flag == CTS_UDP_FLAG_DATA) {
            if (completedBytes < CTS_UDP_DATA_HEADER_LENGTH) return Fail(index, PatternError::TooFewBytes);
        } else if (flag == CTS_UDP_FLAG_ID) {
            if (completedBytes < CTS_UDP_CONNECTION_ID_HEADER_LENGTH) return Fail(index, PatternError::TooFewBytes);
            // SetConnectionIdFromTask (:336-347)
            std::memcpy(connection_id, t.buffer + t.buffer_offset + CTS_UDP_FLAG_LENGTH, CTS_CONNECTION_ID_LENGTH);
            ++m_recvNeeded;
            return PatternError::NoError;
        } else {
            return Fail(index, PatternError::TooFewBytes);
        }
        // VerifyBuffer of the payload: skip the data header, pattern offset 0 (:185-192)
        if (cfg.verify_buffers) {
            const uint32_t payload = completedBytes - CTS_UDP_DATA_HEADER_LENGTH;
            cts_verify_result r{};
            r.first_mismatch = payload;
            r.pass = 1;
            if (payload > 0) {
                cts_task vt = t;
                vt.buffer_offset = CTS_UDP_DATA_HEADER_LENGTH;
                vt.buffer_length -= CTS_UDP_DATA_HEADER_LENGTH;
                const int rc = VerifyNow(vt, payload, r);
                if (rc != CTS_OK) throw DeviceError{rc};
            }
            ++buffers_verified;
            bytes_verified += payload;
            if (!r.pass) {
                RecordFailure((uint32_t)index, payload, r, 0);
                return Fail(index, PatternError::CorruptedBytes);
            }
        }
        // GetSequenceNumberFromTask (buffer + offset + 2) and the sender's QPC / QPF as the client reads them
        // (m_buffer + 8, + 16: ctsIOPatternMediaStream.cpp:218-219)
        const cts::MsDatagram d{load_i64(t.buffer + t.buffer_offset + CTS_UDP_FLAG_LENGTH), load_i64(t.buffer + 8),
                                load_i64(t.buffer + 16), completedBytes};
        const int64_t qpc = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now().time_since_epoch()).count();
        cts::ms_client_apply_data(ms, d, qpc, 1000000000LL);
        ++m_recvNeeded;
        return PatternError::NoError;
    }

    PatternError Fail(uint64_t index, PatternError e)
    {
        if (!udp_failed) {
            udp_failed = true;
            fail_datagram = (uint32_t)index;
        }
        return e;
    }
    bool udp_failed = false;
    uint32_t fail_datagram = 0;

    int UdpStats(cts_media_stream_stats* o) override
    {
        const int rc = cts_media_stream_client_stats(ms, o);
        if (rc != CTS_OK) return rc;
        o->datagrams = datagrams;
        o->last_error = m_lastError;
        o->fail_datagram = fail_datagram;
        o->has_failure = udp_failed ? 1u : 0u;
        return CTS_OK;
    }
};

void make_connection_id(char* out)  // ctsStatistics::GenerateConnectionId: a UUID string
{
    std::random_device rd;
    std::mt19937_64 g(((uint64_t)rd() << 32) ^ rd());
    uint8_t b[16];
    for (auto& x : b) x = (uint8_t)g();
    b[6] = (uint8_t)((b[6] & 0x0F) | 0x40);
    b[8] = (uint8_t)((b[8] & 0x3F) | 0x80);
    std::snprintf(out, CTS_CONNECTION_ID_LENGTH,
                  "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", b[0], b[1], b[2], b[3],
                  b[4], b[5], b[6], b[7], b[8], b[9], b[10], b[11], b[12], b[13], b[14], b[15]);
}

inline bool latch_fail_fast(cts_io_pattern* p, const FailFast& f)
{
    if (p->fail_fast.empty()) p->fail_fast = f.reason;
    p->m_lastError = CTS_PATTERN_E_FAIL_FAST;
    return true;
}

}  // namespace

extern "C" {

int cts_shared_buffer_init(cts_engine* engine, uint32_t max_buffer_size)
{
    if (engine == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::mutex> lk(g_shared.mu);
    const uint64_t need = cts_sender_buffer_size(max_buffer_size);
    if (g_shared.host != nullptr && g_shared.owned && g_shared.bytes >= need) return CTS_OK;
    void *h = nullptr, *d = nullptr;
    int rc = cts_host_alloc(engine, need, &h, &d);
    if (rc != CTS_OK) return rc;
    // the fill kernel writes the pinned sender buffer through its device view
    void* s = nullptr;
    if ((rc = cts_engine_stream_create(engine, &s)) != CTS_OK) {
        (void)cts_host_free(engine, h);
        return rc;
    }
    rc = cts_sender_buffer_fill(engine, d, max_buffer_size, s);
    if (rc == CTS_OK) {
        EngineDevice on(engine);
        if (hipStreamSynchronize(static_cast<hipStream_t>(s)) != hipSuccess) rc = CTS_E_HIP;
    }
    (void)cts_engine_stream_destroy(engine, s);
    if (rc != CTS_OK) {
        (void)cts_host_free(engine, h);
        return rc;
    }
    if (g_shared.owned && g_shared.host) (void)cts_host_free(g_shared.engine, g_shared.host);
    g_shared.host = static_cast<char*>(h);
    g_shared.bytes = need;
    g_shared.owned = true;
    g_shared.engine = engine;
    return CTS_OK;
}

int cts_shared_buffer_attach(const void* host, uint64_t bytes)
{
    if (host == nullptr || bytes < CTS_PATTERN_PERIOD) return CTS_E_INVALID;
    std::lock_guard<std::mutex> lk(g_shared.mu);
    if (g_shared.owned && g_shared.host) (void)cts_host_free(g_shared.engine, g_shared.host);
    g_shared.host = const_cast<char*>(static_cast<const char*>(host));
    g_shared.bytes = bytes;
    g_shared.owned = false;
    g_shared.engine = nullptr;
    return CTS_OK;
}

char* cts_shared_buffer(void) { return g_shared.host; }
uint64_t cts_shared_buffer_bytes(void) { return g_shared.bytes; }

void cts_shared_buffer_release(void)
{
    std::lock_guard<std::mutex> lk(g_shared.mu);
    if (g_shared.owned && g_shared.host) (void)cts_host_free(g_shared.engine, g_shared.host);
    g_shared.host = nullptr;
    g_shared.bytes = 0;
    g_shared.owned = false;
    g_shared.engine = nullptr;
}

int cts_io_pattern_create(const cts_pattern_config* c, cts_engine* engine, cts_io_pattern** out)
{
    if (c == nullptr || out == nullptr) return CTS_E_INVALID;
    *out = nullptr;
    const bool media = c->io_pattern == CTS_PATTERN_MEDIA_STREAM;
    if (c->protocol != (media ? CTS_PROTOCOL_UDP : CTS_PROTOCOL_TCP)) return CTS_E_INVALID;  // UDP is MediaStream only
    if (c->buffer_size_low == 0 || (c->buffer_size_high != 0 && c->buffer_size_high < c->buffer_size_low))
        return CTS_E_INVALID;
    if (c->pre_post_recvs == 0) return CTS_E_INVALID;                         // ctsConfig.cpp:2169-2171
    if (!media && c->verify_buffers && c->pre_post_recvs > 1) return CTS_E_INVALID;  // TCP: ctsConfig.cpp:3440-3446
    if (media) {
        // MediaStreamSettings::CalculateTransferSize and the buffer override (ctsConfig.h:297-364,
        // ctsConfig.cpp:3341-3350): the frame is the buffer, the stream is whole frames
        if (c->buffer_size_high != 0 || c->buffer_size_low < 40 || c->ms_frames_per_second == 0 ||
            c->ms_stream_length_frames <= 0 || c->ms_stream_length_frames > (int64_t)UINT32_MAX ||
            c->transfer_size != (uint64_t)c->buffer_size_low * (uint64_t)c->ms_stream_length_frames)
            return CTS_E_INVALID;
        if (!c->listening && (c->ms_buffered_frames == 0 || c->ms_datagram_max_size == 0)) return CTS_E_INVALID;
        // no RIO and no TCP pacing on the MediaStream path
        if (c->verify_mode > CTS_VERIFY_DEFERRED || c->registered_io || c->tcp_bytes_per_second != 0 || c->burst_count != 0)
            return CTS_E_INVALID;
    }
    if (c->use_shared_buffer && c->verify_buffers) return CTS_E_INVALID;      // ctsIOPattern.cpp:225-227
    if (c->verify_mode != CTS_VERIFY_SYNC && c->verify_mode != CTS_VERIFY_DEFERRED) return CTS_E_INVALID;
    const uint32_t maxbuf = c->buffer_size_high == 0 ? c->buffer_size_low : c->buffer_size_high;  // GetMaxBufferSize
    if (engine != nullptr) {
        const int rc = cts_shared_buffer_init(engine, maxbuf);  // InitOnceExecuteOnce(InitOnceIoPatternCallback)
        if (rc != CTS_OK) return rc;
    }
    if (g_shared.host == nullptr || g_shared.bytes < cts_sender_buffer_size(maxbuf)) return CTS_E_INVALID;
    cts_io_pattern* p = nullptr;
    try {
        switch (c->io_pattern) {
        case CTS_PATTERN_PUSH: p = new PushOrPull(*c, maxbuf, c->listening != 0); break;
        case CTS_PATTERN_PULL: p = new PushOrPull(*c, maxbuf, c->listening == 0); break;
        case CTS_PATTERN_PUSHPULL:
            if (c->push_bytes == 0 || c->pull_bytes == 0) return CTS_E_INVALID;
            p = new PushPull(*c, maxbuf);
            break;
        case CTS_PATTERN_DUPLEX: p = new Duplex(*c, maxbuf); break;
        case CTS_PATTERN_MEDIA_STREAM:
            if (c->listening) {
                p = new MediaStreamServer(*c, maxbuf);
            } else {
                auto* mc = new MediaStreamClient(*c, maxbuf);
                p = mc;
                const cts_media_stream_settings st{c->buffer_size_low, c->ms_datagram_max_size, c->ms_frames_per_second,
                                                   c->ms_buffered_frames, c->ms_stream_length_frames};
                const int mrc = cts_media_stream_client_create(&st, &mc->ms);
                if (mrc != CTS_OK) {
                    delete p;
                    return mrc;
                }
            }
            break;
        default: return CTS_E_INVALID;
        }
    } catch (const std::bad_alloc&) {
        return CTS_E_NOMEM;
    }
    p->engine = engine;
    if (c->listening) make_connection_id(p->connection_id);
    // ctsIoPatternStatistics ctor: CreateRecvBuffers + CreateSendBuffers (ctsIOPattern.h:420-432)
    int rc = CTS_OK;
    try {
        rc = p->CreateRecvBuffers();
        if (rc == CTS_OK) p->CreateSendBuffers();
    } catch (const std::bad_alloc&) {
        rc = CTS_E_NOMEM;
    } catch (const RioRegisterFailed&) {
        rc = CTS_E_INVALID;  // THROW_WIN32_MSG(WSAGetLastError(), "RIORegisterBuffer")
    }
    if (rc != CTS_OK) {
        delete p;
        return rc;
    }
    *out = p;
    return CTS_OK;
}

int cts_io_pattern_destroy(cts_io_pattern* p)
{
    if (p == nullptr) return CTS_E_INVALID;
    // a MediaStream client's timer thread is stopped and joined first (not under the pattern lock, which its
    // callbacks take): nothing calls into the engine from it once destroy has begun, whatever destroy returns
    p->StopTimers();
    int rc = CTS_OK;
    {
        // DEFERRED: completions still waiting for a verdict are verified now, so their bytes reach TcpStatusDetails
        // as the reference's (verified at completion) did. Every wait is bounded (CTS_PATTERN_DESTROY_WAIT_MS,
        // default 2000); nothing may leave the ABI.
        std::lock_guard<std::recursive_mutex> lk(p->mu);
        const char* env = std::getenv("CTS_PATTERN_DESTROY_WAIT_MS");
        const long ms = env != nullptr && *env != 0 ? std::atol(env) : 2000;
        p->bounded_wait = true;
        p->wait_deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms > 0 ? ms : 2000);
        if (p->fail_fast.empty() && p->VerdictsPending()) {
            try {
                const int fr = p->FlushPending();  // an io status (>= 0), or a negative CTS_E_* of the final verify
                if (fr < 0) rc = fr;
            } catch (const DeviceError& d) {
                rc = d.rc < 0 ? d.rc : CTS_E_HIP;
            } catch (...) {
                rc = CTS_E_HIP;
            }
        }
        // the pattern's buffers go with it: a kernel still reading them (it did not finish within the bound) keeps
        // them, and the pattern is left allocated rather than freed under the GPU's reads (CTS_E_TIMEOUT: call
        // destroy again later). Any other failure of that wait is the device's own (a sticky error): no kernel of
        // the pattern runs any more and a later call could not do better, so the pattern is freed (CTS_E_HIP).
        const hipError_t w = p->stream != nullptr ? p->SleepSyncImpl(50) : hipSuccess;
        if (w == hipErrorNotReady) {
            p->bounded_wait = false;
            return CTS_E_TIMEOUT;
        }
        if (w != hipSuccess) rc = CTS_E_HIP;
    }
    delete p;
    return rc;
}

int cts_io_pattern_set_verifier(cts_io_pattern* p, cts_batch_verifier fn, void* ctx)
{
    if (p == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    if (!p->queue.empty() || !p->flights.empty()) return CTS_E_INVALID;
    p->hook = fn;
    p->hook_ctx = ctx;
    return CTS_OK;
}

int cts_io_pattern_initiate_io(cts_io_pattern* p, cts_task* out)
{
    if (p == nullptr || out == nullptr) return CTS_E_INVALID;
    *out = cts_task{};
    out->rio_buffer_id = CTS_RIO_INVALID_BUFFERID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    if (!p->fail_fast.empty()) return CTS_OK;
    try {
        *out = p->InitiateIo();
    } catch (const FailFast& f) {
        latch_fail_fast(p, f);
        *out = cts_task{};
        out->rio_buffer_id = CTS_RIO_INVALID_BUFFERID;
    } catch (const std::bad_alloc&) {
        return CTS_E_NOMEM;
    } catch (const std::exception& e) {  // nothing may cross the C ABI
        latch_fail_fast(p, FailFast{std::string("InitiateIo threw: ") + e.what()});
        *out = cts_task{};
        out->rio_buffer_id = CTS_RIO_INVALID_BUFFERID;
    }
    return CTS_OK;
}

int cts_io_pattern_complete_io(cts_io_pattern* p, const cts_task* t, uint32_t current_transfer, uint32_t status)
{
    if (p == nullptr || t == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    if (!p->fail_fast.empty()) return CTS_IO_FAILED;
    if (p->hook == nullptr && p->engine == nullptr && p->NeedsVerifier(*t))
        return CTS_E_INVALID;  // no verifier: the product has no CPU verify path
    try {
        return p->CompleteIo(*t, current_transfer, status);
    } catch (const FailFast& f) {
        latch_fail_fast(p, f);
        return CTS_IO_FAILED;
    } catch (const DeviceError& d) {
        return d.rc;
    } catch (const std::bad_alloc&) {
        return CTS_E_NOMEM;
    } catch (const std::exception& e) {  // nothing may cross the C ABI
        latch_fail_fast(p, FailFast{std::string("CompleteIo threw: ") + e.what()});
        return CTS_IO_FAILED;
    }
}

uint32_t cts_io_pattern_last_error(const cts_io_pattern* p)
{
    if (p == nullptr) return CTS_STATUS_IO_RUNNING;
    std::lock_guard<std::recursive_mutex> lk(p->mu);  // a MediaStream client's timer thread may be completing a task
    return p->m_lastError;
}

uint64_t cts_io_pattern_rio_buffer_id_count(const cts_io_pattern* p)
{
    if (p == nullptr) return 0;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    return p->RioBufferIdCount();
}

int cts_pattern_clock_set(cts_clock_ms_fn fn, void* ctx)
{
    std::lock_guard<std::mutex> lk(g_clock.mu);
    g_clock.fn = fn;
    g_clock.ctx = fn != nullptr ? ctx : nullptr;
    return CTS_OK;
}

int cts_rio_functions_set(cts_rio_register_buffer_fn register_fn, cts_rio_deregister_buffer_fn deregister_fn,
                          void* ctx)
{
    if ((register_fn == nullptr) != (deregister_fn == nullptr)) return CTS_E_INVALID;
    std::lock_guard<std::mutex> lk(g_rio.mu);
    g_rio.reg = register_fn;
    g_rio.dereg = deregister_fn;
    g_rio.ctx = ctx;
    return CTS_OK;
}

int cts_io_pattern_set_ideal_send_backlog(cts_io_pattern* p, uint32_t bytes)
{
    if (p == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    p->state.SetIdealSendBacklog(bytes);
    return CTS_OK;
}

int cts_io_pattern_flush(cts_io_pattern* p)
{
    if (p == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    try {
        return p->FlushPending();
    } catch (const FailFast& f) {
        latch_fail_fast(p, f);
        return CTS_IO_FAILED;
    } catch (const DeviceError& d) {
        return d.rc;
    } catch (const std::bad_alloc&) {
        return CTS_E_NOMEM;
    } catch (const std::exception& e) {  // nothing may cross the C ABI
        latch_fail_fast(p, FailFast{std::string("Flush threw: ") + e.what()});
        return CTS_IO_FAILED;
    }
}

int cts_io_pattern_get_stats(const cts_io_pattern* p, cts_pattern_stats* o)
{
    if (p == nullptr || o == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    *o = cts_pattern_stats{};
    // m_statistics as published: a DEFERRED pattern's bytes behind a pending verdict are reported apart
    o->bytes_sent_held = std::min(p->HeldSent(), p->bytes_sent);
    o->bytes_recv_held = std::min(p->HeldRecv(), p->bytes_recv);
    o->bytes_sent = p->bytes_sent - o->bytes_sent_held;
    o->bytes_recv = p->bytes_recv - o->bytes_recv_held;
    o->buffers_verified = p->buffers_verified;
    o->bytes_verified = p->bytes_verified;
    o->buffers_failed = p->buffers_failed;
    o->bytes_recv_at_failure = p->has_failure ? p->bytes_recv_at_failure : o->bytes_recv;
    o->recv_pattern_offset = p->m_recvPatternOffset;
    o->send_pattern_offset = p->m_sendPatternOffset;
    o->last_error = p->m_lastError;
    o->queued = (uint32_t)p->queue.size() + p->InFlightCount();
    o->fail_length = p->fail_length;
    o->fail_offset = p->fail_offset;
    o->fail_expected = p->fail_expected;
    o->fail_actual = p->fail_actual;
    o->has_failure = p->has_failure ? 1 : 0;
    o->fail_completion = p->fail_completion;
    o->verify_wait_ns = p->verify_wait_ns;
    o->deferred_depth = p->Deferred() && p->DoubleBuffered() ? p->Depth() : 0u;
    return CTS_OK;
}

int cts_io_pattern_failure_message(const cts_io_pattern* p, char* buf, uint32_t buf_len)
{
    if (p == nullptr) return 0;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    if (!p->has_failure) return 0;
    // ctsIOPattern.cpp:761-772: the bytes are `char`, so values >= 0x80 print sign-extended
    // through %x (MSVC: 32-bit unsigned). Pointers are not part of the parity contract.
    char tmp[512];
    const int n = std::snprintf(tmp, sizeof(tmp),
                                "ctsIOPattern found data corruption: detected an invalid byte pattern in the returned "
                                "buffer (length %u): mismatch from expected pattern at offset (%u) [expected 32-bit "
                                "value '0x%x' didn't match '0x%x']",
                                p->fail_length, p->fail_offset, (unsigned)(int)(int8_t)p->fail_expected,
                                (unsigned)(int)(int8_t)p->fail_actual);
    if (buf != nullptr && buf_len > 0) {
        const size_t k = std::min<size_t>((size_t)n, buf_len - 1);
        std::memcpy(buf, tmp, k);
        buf[k] = 0;
    }
    return n;
}

const char* cts_io_pattern_fail_fast_reason(const cts_io_pattern* p)
{
    if (p == nullptr) return nullptr;
    std::lock_guard<std::recursive_mutex> lk(p->mu);  // the reason is written once and never changes after
    return p->fail_fast.empty() ? nullptr : p->fail_fast.c_str();
}

const char* cts_io_pattern_connection_id(cts_io_pattern* p) { return p ? p->connection_id : nullptr; }

int cts_io_pattern_register_callback(cts_io_pattern* p, cts_task_callback fn, void* ctx)
{
    if (p == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    p->m_callback = fn;
    p->m_callback_ctx = fn != nullptr ? ctx : nullptr;
    return CTS_OK;
}

int cts_io_pattern_media_stream_fire(cts_io_pattern* p, int timer)
{
    if (p == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    try {
        return p->FireTimer(timer);
    } catch (const FailFast& f) {
        latch_fail_fast(p, f);
        return CTS_OK;
    } catch (const DeviceError& d) {
        return d.rc;
    } catch (const std::bad_alloc&) {  // nothing may cross the C ABI
        return CTS_E_NOMEM;
    } catch (const std::exception& e) {
        latch_fail_fast(p, FailFast{std::string("a timer callback threw: ") + e.what()});
        return CTS_OK;
    }
}

int cts_io_pattern_media_stream_timers(cts_io_pattern* p, int64_t* start_due_ms, int64_t* render_due_ms)
{
    if (p == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    return p->Timers(start_due_ms, render_due_ms);
}

int cts_io_pattern_media_stream_stats(cts_io_pattern* p, cts_media_stream_stats* out)
{
    if (p == nullptr || out == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::recursive_mutex> lk(p->mu);
    return p->UdpStats(out);
}

}  // extern "C"

// ---- ctsIoPatternState on its own (ctsIOPatternState.hpp:51-504) ----------------------------
struct cts_io_pattern_state {
    PatternState st;
    std::string fail_fast;
    explicit cts_io_pattern_state(const cts_pattern_config& c)
        : st(c, c.buffer_size_high ? c.buffer_size_high : c.buffer_size_low)
    {
    }
};

namespace {
// an internal-consistency FAIL_FAST of the reference: latched, reported as CTS_E_INVALID
template <typename F>
int state_call(cts_io_pattern_state* s, F f)
{
    if (s == nullptr) return CTS_E_INVALID;
    if (!s->fail_fast.empty()) return CTS_E_INVALID;
    try {
        return f();
    } catch (const FailFast& e) {
        s->fail_fast = e.reason;
        return CTS_E_INVALID;
    }
}
}  // namespace

extern "C" {

int cts_io_pattern_state_create(const cts_pattern_config* c, cts_io_pattern_state** out)
{
    if (c == nullptr || out == nullptr) return CTS_E_INVALID;
    *out = nullptr;
    if (c->protocol != CTS_PROTOCOL_TCP && c->protocol != CTS_PROTOCOL_UDP) return CTS_E_INVALID;
    cts_io_pattern_state* s = new (std::nothrow) cts_io_pattern_state(*c);
    if (s == nullptr) return CTS_E_NOMEM;
    *out = s;
    return CTS_OK;
}

int cts_io_pattern_state_destroy(cts_io_pattern_state* s)
{
    if (s == nullptr) return CTS_E_INVALID;
    delete s;
    return CTS_OK;
}

uint64_t cts_io_pattern_state_get_remaining_transfer(cts_io_pattern_state* s)
{
    uint64_t v = 0;
    (void)state_call(s, [&] {
        v = s->st.GetRemainingTransfer();
        return CTS_OK;
    });
    return v;
}

uint64_t cts_io_pattern_state_get_max_transfer(const cts_io_pattern_state* s) { return s ? s->st.GetMaxTransfer() : 0; }

int cts_io_pattern_state_set_max_transfer(cts_io_pattern_state* s, uint64_t max_transfer)
{
    return state_call(s, [&] {
        s->st.SetMaxTransfer(max_transfer);
        return CTS_OK;
    });
}

uint32_t cts_io_pattern_state_get_ideal_send_backlog(const cts_io_pattern_state* s)
{
    return s ? s->st.GetIdealSendBacklog() : 0;
}

int cts_io_pattern_state_set_ideal_send_backlog(cts_io_pattern_state* s, uint32_t bytes)
{
    return state_call(s, [&] {
        s->st.SetIdealSendBacklog(bytes);
        return CTS_OK;
    });
}

int cts_io_pattern_state_is_completed(const cts_io_pattern_state* s) { return s ? (s->st.IsCompleted() ? 1 : 0) : CTS_E_INVALID; }

int cts_io_pattern_state_is_current_state_more_io(const cts_io_pattern_state* s)
{
    return s ? (s->st.IsCurrentStateMoreIo() ? 1 : 0) : CTS_E_INVALID;
}

int cts_io_pattern_state_get_next_pattern_type(cts_io_pattern_state* s)
{
    return state_call(s, [&] { return (int)s->st.GetNextPatternType(); });
}

int cts_io_pattern_state_notify_next_task(cts_io_pattern_state* s, const cts_task* t)
{
    if (t == nullptr) return CTS_E_INVALID;
    return state_call(s, [&] {
        s->st.NotifyNextTask(*t);
        return CTS_OK;
    });
}

int cts_io_pattern_state_completed_task(cts_io_pattern_state* s, const cts_task* t, uint32_t completed_bytes)
{
    if (t == nullptr) return CTS_E_INVALID;
    return state_call(s, [&] { return (int)s->st.CompletedTask(*t, completed_bytes); });
}

int cts_io_pattern_state_update_error(cts_io_pattern_state* s, uint32_t error)
{
    return state_call(s, [&] { return (int)s->st.UpdateError(error); });
}

const char* cts_io_pattern_state_fail_fast_reason(const cts_io_pattern_state* s)
{
    return (s == nullptr || s->fail_fast.empty()) ? nullptr : s->fail_fast.c_str();
}

int cts_status_details_read(cts_status_details* o)
{
    if (o == nullptr) return CTS_E_INVALID;
    o->bytes_sent = g_bytesSent.load();
    o->bytes_recv = g_bytesRecv.load();
    o->data_errors = g_dataErrors.load();
    return CTS_OK;
}

void cts_status_details_reset(void)
{
    g_bytesSent = 0;
    g_bytesRecv = 0;
    g_dataErrors = 0;
}

}  // extern "C"
