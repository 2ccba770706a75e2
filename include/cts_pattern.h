/*
 * cts_pattern.h — C ABI of the host-side ctsIoPattern mirror: the caller of the
 * GPU fill/verify engine (include/cts_engine.h).
 *
 * The IO functors of the reference (ctsSendRecvIocp.cpp:97,243,368;
 * ctsRioIocp.cpp:617,687,705,715,775; ctsReadWriteIocp.cpp:79,144,238) drive a
 * connection through exactly two calls on its pattern object:
 *
 *   ctsTask     ctsIoPattern::InitiateIo()                               ctsIOPattern.h:143
 *   ctsIoStatus ctsIoPattern::CompleteIo(task, currentTransfer, status)  ctsIOPattern.h:144
 *
 * (the MediaStream functors likewise: ctsMediaStreamClient.cpp:136-144,268,404,
 * ctsMediaStreamServerConnectedSocket.cpp:111-133),
 * plus the factory MakeIoPattern (ctsIOPattern.cpp:97-124), GetLastPatternError
 * (ctsIOPattern.h:126-129) and AccessSharedBuffer (ctsIOPattern.cpp:126-131,
 * which the reference's own tests use to simulate the wire). This header
 * exports those calls with the same argument meaning; the bodies restate
 * ctsIOPattern.cpp:219-743 and ctsIOPatternState.hpp:57-504 in C++ and route
 * the two hot-path pieces to the GPU:
 *
 *   g_senderSharedBuffer (InitOnceIoPatternCallback, ctsIOPattern.cpp:52-90)
 *       -> cts_shared_buffer_init: the gfx950 fill kernel writes it;
 *   VerifyBuffer (ctsIOPattern.cpp:745-775)
 *       -> the gfx950 verify kernel, on the pattern's pinned, device-mapped
 *          recv buffers (zero copy), either per completion (CTS_VERIFY_SYNC,
 *          the reference's timing) or batched (CTS_VERIFY_DEFERRED, §8f-1 of
 *          see cts_io_pattern_flush).
 *
 * Configuration that the reference reads from ctsConfig::g_configSettings and
 * the Get*Size() accessors (ctsConfig.h:370-462, ctsConfig.cpp:4679-4698) is
 * passed explicitly in cts_pattern_config.
 *
 * Error conventions: the reference's entry points are noexcept and FAIL_FAST
 * on internal inconsistency. Here every call returns normally; an internal
 * inconsistency latches CTS_PATTERN_E_FAIL_FAST on the pattern (readable with
 * cts_io_pattern_fail_fast_reason) and CompleteIo returns CTS_IO_FAILED.
 * Send pacing is restated: with cts_pattern_config.tcp_bytes_per_second (and
 * its period) or burst_count / burst_delay set, CreateNewTask gives send tasks
 * the reference's time_offset_ms (ctsIOPattern.cpp:593-674); with neither set
 * every time offset is 0.
 */
#ifndef CTS_PATTERN_H
#define CTS_PATTERN_H

#include <stddef.h>
#include <stdint.h>

#include "cts_engine.h"
#include "cts_media_stream.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ctsTaskAction (ctsIOTask.hpp:27-36) */
typedef enum cts_task_action {
    CTS_TASK_NONE = 0,
    CTS_TASK_SEND = 1,
    CTS_TASK_RECV = 2,
    CTS_TASK_GRACEFUL_SHUTDOWN = 3,
    CTS_TASK_HARD_SHUTDOWN = 4,
    CTS_TASK_ABORT = 5,
    CTS_TASK_FATAL_ABORT = 6
} cts_task_action;

/* ctsTask::BufferType (ctsIOTask.hpp:47-55) */
typedef enum cts_buffer_type {
    CTS_BUFFER_NULL = 0,
    CTS_BUFFER_TCP_CONNECTION_ID = 1,
    CTS_BUFFER_UDP_CONNECTION_ID = 2,
    CTS_BUFFER_COMPLETION_MESSAGE = 3,
    CTS_BUFFER_STATIC = 4,
    CTS_BUFFER_DYNAMIC = 5
} cts_buffer_type;

/* RIO_INVALID_BUFFERID (mswsock.h: (RIO_BUFFERID)(ULONG_PTR)0xFFFFFFFF), the ctsTask default
 * (ctsIOTask.hpp:40). Every task the pattern hands out carries it unless it carries a registered id. */
#define CTS_RIO_INVALID_BUFFERID 0xFFFFFFFFull

/* ctsTask (ctsIOTask.hpp:37-60), RIO_BUFFERID as a uint64. */
typedef struct cts_task {
    int64_t time_offset_ms;           /* m_timeOffsetMilliseconds */
    uint64_t rio_buffer_id;           /* m_rioBufferid */
    char* buffer;                     /* m_buffer */
    uint32_t buffer_length;           /* m_bufferLength */
    uint32_t buffer_offset;           /* m_bufferOffset */
    uint32_t expected_pattern_offset; /* m_expectedPatternOffset */
    uint8_t io_action;                /* m_ioAction (cts_task_action) */
    uint8_t buffer_type;              /* m_bufferType (cts_buffer_type) */
    uint8_t track_io;                 /* m_trackIo */
    uint8_t reserved;
} cts_task;                           /* 40 bytes */

/* ctsIoStatus (ctsIOPattern.h:38-43) */
typedef enum cts_io_status { CTS_IO_CONTINUE = 0, CTS_IO_COMPLETED = 1, CTS_IO_FAILED = 2 } cts_io_status;

/* Protocol error codes (ctsIOPattern.h:46-50) */
#define CTS_STATUS_IO_RUNNING 2147483647u                   /* c_statusIoRunning = MAXINT */
#define CTS_STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED 2147483646u /* MAXINT - 1 */
#define CTS_STATUS_ERROR_TOO_MUCH_DATA_TRANSFERRED 2147483645u /* MAXINT - 2 */
/* CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN (MAXINT - 3) is in cts_engine.h */
/* Not in the reference: the latched stand-in for a FAIL_FAST process abort. */
#define CTS_PATTERN_E_FAIL_FAST 2147483640u

/* ctsStatistics::ConnectionIdLength = 36 + 1 (ctsStatistics.hpp:36) */
#define CTS_CONNECTION_ID_LENGTH 37u
/* c_completionMessage "DONE" / c_completionMessageSize (ctsIOPatternState.hpp:24-25) */
#define CTS_COMPLETION_MESSAGE_SIZE 4u

typedef enum cts_io_pattern_type { /* ctsConfig::IoPatternType */
    CTS_PATTERN_PUSH = 1,
    CTS_PATTERN_PULL = 2,
    CTS_PATTERN_PUSHPULL = 3,
    CTS_PATTERN_DUPLEX = 4,
    /* UDP: listening = ctsIoPatternMediaStreamServer (ctsIOPattern.cpp:1100-1175), else
     * ctsIoPatternMediaStreamClient (ctsIOPatternMediaStream.cpp:46-530), MakeIoPattern :113-118 */
    CTS_PATTERN_MEDIA_STREAM = 5
} cts_io_pattern_type;

typedef enum cts_protocol { CTS_PROTOCOL_TCP = 1, CTS_PROTOCOL_UDP = 2 } cts_protocol;
typedef enum cts_tcp_shutdown { CTS_SHUTDOWN_GRACEFUL = 1, CTS_SHUTDOWN_HARD = 2 } cts_tcp_shutdown;

typedef enum cts_verify_mode {
    /* VerifyBuffer runs inside every CompleteIo, as in the reference. */
    CTS_VERIFY_SYNC = 0,
    /* Verified recv completions are queued and checked in batches (one kernel
     * launch per batch); see cts_io_pattern_flush for the exactness contract. */
    CTS_VERIFY_DEFERRED = 1
} cts_verify_mode;

typedef struct cts_pattern_config {
    uint32_t io_pattern;        /* cts_io_pattern_type      (g_configSettings->IoPattern) */
    uint32_t protocol;          /* cts_protocol             (->Protocol) */
    uint32_t listening;         /* ctsConfig::IsListening(): 1 = server */
    uint32_t verify_buffers;    /* ->ShouldVerifyBuffers (-verify:data) */
    uint32_t use_shared_buffer; /* ->UseSharedBuffer */
    uint32_t pre_post_recvs;    /* ->PrePostRecvs */
    uint32_t pre_post_sends;    /* ->PrePostSends (0 = rely on the ideal send backlog) */
    uint32_t buffer_size_low;   /* GetBufferSize(): fixed size, or the low end of -buffer:[lo,hi] */
    uint32_t buffer_size_high;  /* 0 = fixed; else GetBufferSize() draws uniformly in [lo, hi] */
    uint32_t push_bytes;        /* ->PushBytes (PushPull) */
    uint32_t pull_bytes;        /* ->PullBytes (PushPull) */
    uint32_t tcp_shutdown;      /* cts_tcp_shutdown (GetShutdownType()) */
    uint64_t transfer_size;     /* GetTransferSize() */
    uint64_t random_seed;       /* seed of the -buffer:[lo,hi] draw (reference: random_device) */
    uint32_t verify_mode;       /* cts_verify_mode */
    uint32_t batch_buffers;     /* DEFERRED: completions within which every verdict is known (0 = 1024); on a
                                   device the batch is launched in parts of batch_buffers / (depth + 1) with
                                   up to depth running while the next fills (CTS_DEFERRED_DEPTH, default 2), and
                                   the pinned recv ring holds 2 x batch_buffers + recvCount + 1 buffers */
    uint64_t batch_bytes;       /* DEFERRED: staging arena bytes (0 = 64 MiB) */
    uint32_t registered_io;     /* SocketFlags & WSA_FLAG_REGISTERED_IO (-io:rioiocp): register buffers with
                                 * the RIO functions of cts_rio_functions_set, hand their ids out in tasks */
    uint32_t reserved0;
    /* send pacing (ctsIOPattern.cpp:219-224, 593-674): sets ctsTask::m_timeOffsetMilliseconds of sends */
    int64_t tcp_bytes_per_second;        /* ctsConfig::GetTcpBytesPerSecond() of this connection (0 = no limit) */
    int64_t tcp_bytes_per_second_period; /* ->TcpBytesPerSecondPeriod, ms (0 = the reference default, 100) */
    uint32_t burst_count;                /* ->BurstCount (0 = not set); used only without a rate limit */
    uint32_t burst_delay;                /* ->BurstDelay, ms: the offset of every burst_count-th send */
    /* MediaStream (CTS_PATTERN_MEDIA_STREAM over CTS_PROTOCOL_UDP): ctsConfig::MediaStreamSettings
     * (ctsConfig.h:284-364). As CalculateTransferSize and the config parser set them (ctsConfig.cpp:1260,
     * 3341-3350), the frame size is buffer_size_low (buffer_size_high 0, at least 40 bytes) and transfer_size
     * must be buffer_size_low x ms_stream_length_frames. */
    uint32_t ms_frames_per_second;       /* FramesPerSecond */
    uint32_t ms_datagram_max_size;       /* DatagramMaxSize: the client posts recvs of min(frame, this) bytes */
    uint32_t ms_buffered_frames;         /* BufferedFrames (client) */
    uint32_t ms_manual_timers;           /* client: 0 = a timer thread fires the start and renderer timers at the
                                            reference's times; 1 = the caller fires them (cts_io_pattern_media_stream_fire) */
    int64_t ms_stream_length_frames;     /* StreamLengthFrames */
} cts_pattern_config;

/* The millisecond clock send pacing reads (ctTimer::snap_qpc_as_msec). NULL restores the default, a
 * monotonic clock. Process-wide, like the reference's unit-test hook ctTimer::g_unitTestQpcTimeMs. */
typedef int64_t (*cts_clock_ms_fn)(void* ctx);
int cts_pattern_clock_set(cts_clock_ms_fn fn, void* ctx);

/* Per-connection statistics (ctsTcpStatistics, ctsStatistics.hpp:316-373) and
 * the verify bookkeeping of this pattern. */
typedef struct cts_pattern_stats {
    uint64_t bytes_sent;          /* m_statistics.m_bytesSent (published: see bytes_sent_held) */
    uint64_t bytes_recv;          /* m_statistics.m_bytesRecv (published: see bytes_recv_held) */
    uint64_t buffers_verified;    /* VerifyBuffer calls that completed */
    uint64_t bytes_verified;      /* sum of their transferred bytes */
    uint64_t buffers_failed;      /* verify failures (0 or 1: the first fails the connection) */
    uint64_t bytes_recv_at_failure; /* DEFERRED: m_bytesRecv as it stood right after the failing completion */
    uint32_t recv_pattern_offset; /* m_recvPatternOffset */
    uint32_t send_pattern_offset; /* m_sendPatternOffset */
    uint32_t last_error;          /* GetLastPatternError() */
    uint32_t queued;              /* DEFERRED: buffers waiting for the next batch */
    /* first verify failure (ctsIOPattern.cpp:761-772 prints these) */
    uint32_t fail_length;         /* transferred bytes of the failing buffer */
    uint32_t fail_offset;         /* lengthMatched = RtlCompareMemory(...) */
    uint8_t fail_expected;        /* patternBuffer[lengthMatched] */
    uint8_t fail_actual;          /* received byte at lengthMatched */
    uint8_t has_failure;
    uint8_t reserved;
    uint32_t fail_completion;     /* index of the failing recv completion (0-based) */
    /* DEFERRED: bytes completed behind a recv whose batch verdict is still pending. They are held back from
     * bytes_sent / bytes_recv above and from the process-wide cts_status_details until that batch verifies, so
     * every counter only grows, as the reference's do (ctsStatistics.hpp:153-186). Bytes after a failing buffer
     * are dropped without ever being published. 0 in SYNC mode. */
    uint64_t bytes_sent_held;
    uint64_t bytes_recv_held;
    /* DEFERRED: wall time this pattern's calls spent waiting for batch verdicts from the device (retiring the oldest
     * in-flight launch, a flush's synchronize, a MediaStream client's batch): the receive thread is idle on the GPU
     * meanwhile. */
    uint64_t verify_wait_ns;
    /* DEFERRED: device launches this pattern keeps in flight at once (CTS_DEFERRED_DEPTH as clamped to the batch:
     * 1-4), 0 in SYNC mode or with a host batch verifier. */
    uint32_t deferred_depth;
    uint32_t reserved2;
} cts_pattern_stats;

/* Batch verifier hook: verify n buffers of a host arena (results[i] per
 * descs[i], RtlCompareMemory semantics). Return 0 on success. When a pattern has
 * a hook it is used instead of the engine (test harnesses: the reference's own
 * tests replace ctsConfig by link-time fakes in the same way). */
typedef int (*cts_batch_verifier)(void* ctx, const uint8_t* host_arena, uint64_t arena_bytes,
                                  const cts_buf_desc* descs, uint32_t n, cts_verify_result* results);

typedef struct cts_io_pattern cts_io_pattern;

/* ---- RIO buffer registration (g_configSettings->rioFunctions, ctsConfig.h) -------------------
 * RIORegisterBuffer / RIODeregisterBuffer as the pattern uses them (ctsIOPattern.cpp:133-217,
 * ctsIOPattern.h:219-269). A register function returns CTS_RIO_INVALID_BUFFERID on failure (the
 * reference then throws WSAGetLastError() out of the pattern's constructor: cts_io_pattern_create
 * returns CTS_E_INVALID). With registered_io set, a pattern registers
 *   - every recv buffer slot (or the shared receiver buffer once per slot with use_shared_buffer),
 *   - the sender buffer 16 MiB / buffer_size_low + 1 times (one id per concurrent send: RIO cannot
 *     use one RIO_BUFFERID in two sends at once, ctsIOPattern.cpp:49,61,198-210),
 *   - the connection id (37 B) and the completion message (4 B) buffers,
 * hands a recv / send task the id of its buffer (buffer type DYNAMIC, ctsIOPattern.cpp:683-692,
 * :716-725) and takes it back in CompleteIo (:369-386). The ids of a pattern are deregistered when
 * it is destroyed, including ids of tasks still in flight (the reference leaks those; its RIO
 * functor never destroys a pattern with IO outstanding). Process-wide; set before creating
 * patterns with registered_io. */
typedef uint64_t (*cts_rio_register_buffer_fn)(void* ctx, char* buffer, uint32_t length);
typedef void (*cts_rio_deregister_buffer_fn)(void* ctx, uint64_t buffer_id);
int cts_rio_functions_set(cts_rio_register_buffer_fn register_fn, cts_rio_deregister_buffer_fn deregister_fn,
                          void* ctx);

/* ---- g_senderSharedBuffer (process-wide, InitOnceIoPatternCallback) ------ */
/* Materialise the sender buffer (65536 + max_buffer_size bytes) in pinned,
 * device-mapped host memory with the gfx950 fill kernel. Idempotent for a
 * size <= the current one. */
int cts_shared_buffer_init(cts_engine* engine, uint32_t max_buffer_size);
/* Use caller-owned bytes as the sender buffer (harnesses without a device). */
int cts_shared_buffer_attach(const void* host, uint64_t bytes);
/* AccessSharedBuffer (ctsIOPattern.cpp:126-131): NULL until init/attach. */
char* cts_shared_buffer(void);
uint64_t cts_shared_buffer_bytes(void);
void cts_shared_buffer_release(void);

/* ---- pattern lifetime (MakeIoPattern, ctsIOPattern.cpp:97-124) ------------ */
/* engine may be NULL only when verify_buffers == 0 or a batch verifier is set
 * with cts_io_pattern_set_verifier before the first CompleteIo. */
int cts_io_pattern_create(const cts_pattern_config* config, cts_engine* engine, cts_io_pattern** out);
/* A DEFERRED pattern destroyed with completions still waiting for their batch verdict verifies them first, so their
 * bytes are published (cts_pattern_stats.bytes_*_held) as the reference counted them at completion. A data mismatch
 * found by that final verify reaches only the process-wide counters (cts_status_details_*): the caller has read this
 * pattern's stats before destroying it. A MediaStream client's timer thread is stopped and joined first, whatever
 * destroy then returns. Every wait of destroy is bounded (env CTS_PATTERN_DESTROY_WAIT_MS, default 2000), the flush
 * of the batch destroy itself launches included. Returns:
 *   CTS_OK        the pattern is freed;
 *   CTS_E_TIMEOUT a kernel still reads the pattern's buffers after the bound: nothing was freed, the handle stays
 *                 valid, and destroy should be called again (it flushes nothing more, only waits again);
 *   CTS_E_HIP / another negative status: the final verify failed, or the device reported an error (sticky: no later
 *                 call could wait better); the pattern is freed. */
int cts_io_pattern_destroy(cts_io_pattern* pattern);
int cts_io_pattern_set_verifier(cts_io_pattern* pattern, cts_batch_verifier fn, void* ctx);

/* ---- the boundary ---------------------------------------------------------- */
int cts_io_pattern_initiate_io(cts_io_pattern* pattern, cts_task* out_task);
/* Returns a cts_io_status (>= 0) or a negative cts_status on a bad argument /
 * device error. */
int cts_io_pattern_complete_io(cts_io_pattern* pattern, const cts_task* task, uint32_t current_transfer,
                               uint32_t status_code);
uint32_t cts_io_pattern_last_error(const cts_io_pattern* pattern);
/* ctsIoPattern::GetRioBufferIdCount (ctsIOPattern.h:114-123): 0 without registered_io, else the ids
 * on the pattern's free lists + 2 (connection id, completion message). ctsRioIocp sizes its request
 * queue and task table with it (ctsRioIocp.cpp:513-530). */
uint64_t cts_io_pattern_rio_buffer_id_count(const cts_io_pattern* pattern);
/* ctsIoPattern::SetIdealSendBacklog (ctsIOPattern.h:109-112): the socket's ideal send backlog
 * (SIO_IDEAL_SEND_BACKLOG_QUERY, ctsSocket.cpp:249) bounds the bytes of sends in flight when
 * pre_post_sends == 0. */
int cts_io_pattern_set_ideal_send_backlog(cts_io_pattern* pattern, uint32_t bytes);
/* DEFERRED mode: verify every queued buffer now (one kernel launch) and apply
 * the outcome as the reference would have at the first failing completion:
 * latch CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN and record its offset,
 * expected and actual bytes and the recv byte count at that completion.
 * Completions accepted after the failing buffer (the reference never saw them:
 * it failed the connection there, ctsIOPattern.cpp:486-489) are taken back:
 * they are not counted as verified, and their bytes leave the per-connection
 * statistics, TcpStatusDetails and the pattern state again, so every counter
 * equals the reference's after a data error. Sends that completed after the
 * failing recv are taken back the same way.
 * CompleteIo flushes by itself before any completion that is not a plain
 * in-transfer tracked send/recv (connection id, completion message, FIN,
 * a failed IO, the last bytes of the transfer) and when the batch is full; when
 * that flush fails a buffer, the completion that triggered it is not processed.
 * So the connection's final status and counters are exact; the one remaining
 * difference is timing: completions between a failing buffer and its flush
 * return CTS_IO_CONTINUE where the reference would have returned
 * CTS_IO_FAILED (the feeder keeps the socket open until then). Returns the
 * current cts_io_status. */
int cts_io_pattern_flush(cts_io_pattern* pattern);
int cts_io_pattern_get_stats(const cts_io_pattern* pattern, cts_pattern_stats* out);
/* The message ctsConfig::PrintErrorInfo receives on a verify failure
 * (ctsIOPattern.cpp:761-772, bytes printed as sign-extended char through %x).
 * Returns the length written (0 if no failure). */
int cts_io_pattern_failure_message(const cts_io_pattern* pattern, char* buf, uint32_t buf_len);
const char* cts_io_pattern_fail_fast_reason(const cts_io_pattern* pattern);
/* GetConnectionIdentifier(): the 36-char id + NUL (servers generate it). */
const char* cts_io_pattern_connection_id(cts_io_pattern* pattern);

/* ---- MediaStream patterns (CTS_PATTERN_MEDIA_STREAM) ---------------------------------------------
 * The server hands out its connection-id datagram (39 bytes: flag 0x1000 + the id, a UDP_CONNECTION_ID send
 * task) and then one tracked send task of one frame per frame, each with the time offset of its frame
 * (base + frame * 1000 / fps - now, ctsIOPattern.cpp:1119-1153); ctsMediaStreamServerConnectedSocket splits a
 * frame task into datagrams (cts_media_stream_split). The client posts untracked recvs of
 * min(frame, DatagramMaxSize) bytes, parses each completed datagram (ctsMediaStreamProtocol.hpp:284-366) and
 * verifies a data datagram's payload (offset 26, expected pattern offset 0) on the GPU, per completion,
 * before booking it to its frame (ctsIOPatternMediaStream.cpp:140-272). CTS_VERIFY_SYNC verifies each data
 * datagram in its CompleteIo (the reference's timing); CTS_VERIFY_DEFERRED queues data datagrams in the recv ring
 * (their headers checked on the CPU) and verifies batches of batch_buffers with the GPU frame-sum receive pass
 * (cts_media_stream_verify_frames), flushing before every render tick, every other completion and Abort, so the
 * frames, bits and the stream's status are the reference's; a corrupt payload fails the stream when its batch is
 * verified (at most one batch later), with the first mismatch cts_verify finds in it. registered_io is refused
 * (the MediaStream functors use WSARecvFrom / WSASendTo). Every call on a pattern holds the pattern's own
 * (recursive) lock, as the reference's functors and timer callbacks hold the pattern's critical section.
 *
 * RegisterCallback (ctsIOPattern.h:94-97): the client's timer callbacks hand tasks to the functor through it
 * (SendTaskToCallback, :333-339): a "START" send (5 bytes, untracked, STATIC) every 500 ms + one frame until
 * a frame arrived, Abort when the stream rendered its final frame, FatalAbort when nothing ever arrived. The
 * callback runs with the pattern's lock held and may call cts_io_pattern_complete_io on the task (the
 * reference functor completes Abort / FatalAbort from inside it, ctsMediaStreamClient.cpp:317-331). It must
 * not call cts_io_pattern_destroy: destroy joins the timer thread the callback runs on (as the reference's
 * destructor waits for its threadpool timer callbacks); destroy from another thread once it has returned. */
typedef void (*cts_task_callback)(void* ctx, const cts_task* task);
int cts_io_pattern_register_callback(cts_io_pattern* pattern, cts_task_callback fn, void* ctx);

/* The client's two threadpool timers (ctsIOPatternMediaStream.cpp:321-364, 440-530). With ms_manual_timers the
 * caller runs a timer's callback with cts_io_pattern_media_stream_fire (the renderer callback renders frames until
 * its next time lies more than 2 ms ahead of the pattern clock, cts_pattern_clock_set); otherwise a thread per
 * client pattern runs them when due. cts_io_pattern_media_stream_timers reads when each is due, on the pattern
 * clock (-1: not armed). CTS_E_INVALID on a server pattern or any other pattern. */
#define CTS_MS_TIMER_START 0
#define CTS_MS_TIMER_RENDER 1
int cts_io_pattern_media_stream_fire(cts_io_pattern* pattern, int timer);
int cts_io_pattern_media_stream_timers(cts_io_pattern* pattern, int64_t* start_due_ms, int64_t* render_due_ms);
/* ctsUdpStatistics of a MediaStream pattern: the client's frame accounting (as cts_media_stream_client_stats),
 * or for the server the bits it sent (bits_received, the reference's name, ctsIOPattern.cpp:1156-1172). */
int cts_io_pattern_media_stream_stats(cts_io_pattern* pattern, cts_media_stream_stats* out);

/* ---- ctsIoPatternState on its own (ctsIOPatternState.hpp:51-504) ----------------------------
 * The protocol state machine every pattern above runs on: connection id exchange, in-flight and
 * confirmed byte tracking against the transfer size, the completion message, the FIN / RST
 * shutdown, and the TCP error rules (a server waiting for the FIN accepts WSAETIMEDOUT,
 * WSAECONNRESET, WSAECONNABORTED). UDP (MediaStream) only tracks bytes. Exposed so its own MSTest
 * project (MSTest/ctsIOPatternStateUnitTest) replays against it; the config fields read are
 * protocol, listening, tcp_shutdown, transfer_size, pre_post_sends and the buffer size (the ideal
 * send backlog). A reference FAIL_FAST (an inconsistent completion) latches a reason and every
 * later call returns CTS_E_INVALID. */
typedef enum cts_pattern_type { /* ctsIoPatternType */
    CTS_PT_NO_IO = 0,
    CTS_PT_SEND_CONNECTION_ID = 1,
    CTS_PT_RECV_CONNECTION_ID = 2,
    CTS_PT_MORE_IO = 3,
    CTS_PT_SEND_COMPLETION = 4,
    CTS_PT_RECV_COMPLETION = 5,
    CTS_PT_GRACEFUL_SHUTDOWN = 6,
    CTS_PT_HARD_SHUTDOWN = 7,
    CTS_PT_REQUEST_FIN = 8
} cts_pattern_type;

typedef enum cts_pattern_error { /* ctsIoPatternError */
    CTS_PE_NO_ERROR = 0,
    CTS_PE_TOO_MANY_BYTES = 1,
    CTS_PE_TOO_FEW_BYTES = 2,
    CTS_PE_CORRUPTED_BYTES = 3,
    CTS_PE_ERROR_IO_FAILED = 4,
    CTS_PE_SUCCESSFULLY_COMPLETED = 5
} cts_pattern_error;

typedef struct cts_io_pattern_state cts_io_pattern_state;
int cts_io_pattern_state_create(const cts_pattern_config* config, cts_io_pattern_state** out);
int cts_io_pattern_state_destroy(cts_io_pattern_state* state);
uint64_t cts_io_pattern_state_get_remaining_transfer(cts_io_pattern_state* state);
uint64_t cts_io_pattern_state_get_max_transfer(const cts_io_pattern_state* state);
int cts_io_pattern_state_set_max_transfer(cts_io_pattern_state* state, uint64_t max_transfer);
uint32_t cts_io_pattern_state_get_ideal_send_backlog(const cts_io_pattern_state* state);
int cts_io_pattern_state_set_ideal_send_backlog(cts_io_pattern_state* state, uint32_t bytes);
int cts_io_pattern_state_is_completed(const cts_io_pattern_state* state);           /* 1 / 0 */
int cts_io_pattern_state_is_current_state_more_io(const cts_io_pattern_state* state); /* 1 / 0 */
int cts_io_pattern_state_get_next_pattern_type(cts_io_pattern_state* state);         /* cts_pattern_type */
int cts_io_pattern_state_notify_next_task(cts_io_pattern_state* state, const cts_task* task);
int cts_io_pattern_state_completed_task(cts_io_pattern_state* state, const cts_task* task,
                                        uint32_t completed_bytes);                   /* cts_pattern_error */
int cts_io_pattern_state_update_error(cts_io_pattern_state* state, uint32_t error); /* cts_pattern_error */
const char* cts_io_pattern_state_fail_fast_reason(const cts_io_pattern_state* state);

/* ---- process-wide status counters (TcpStatusDetails, ctsConfig.h:415-417) ---- */
typedef struct cts_status_details {
    uint64_t bytes_sent;        /* TcpStatusDetails.m_bytesSent */
    uint64_t bytes_recv;        /* TcpStatusDetails.m_bytesRecv */
    uint64_t data_errors;       /* patterns that latched DATA_DID_NOT_MATCH_BIT_PATTERN */
} cts_status_details;
int cts_status_details_read(cts_status_details* out);
void cts_status_details_reset(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* CTS_PATTERN_H */
