/*
 * cts_loopback.h — a Linux loopback-TCP feeder for the data-integrity path
 * (SURVEY.md §8f-3): the role of the reference's IOCP IO functor
 * (ctsTraffic/ctsSendRecvIocp.cpp:335-415, ctsSendRecvProcessTask :130-300)
 * played with blocking POSIX sockets over the ctsIoPattern mirror of
 * cts_pattern.h: one thread per connection side (Push, Pull, PushPull), or a
 * send and a recv thread per side (Duplex; see cts_loopback_functor). Senders
 * send g_senderSharedBuffer (written by the gfx950 fill kernel) and receivers
 * verify every received buffer on the GPU, so a push run is the reference's
 * config 1 end to end
 * ("-Pattern:push -Connections:8 -Buffer:65536 -Transfer:1GiB -Verify:data"
 * over loopback), host memory and the kernel stack included.
 */
#ifndef CTS_LOOPBACK_H
#define CTS_LOOPBACK_H

#include <stdint.h>

#include "cts_engine.h"
#include "cts_pattern.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cts_loopback_config {
    uint32_t connections;           /* -Connections (client/server pairs) */
    uint32_t io_pattern;            /* cts_io_pattern_type (0 = Push) */
    uint32_t buffer_size;           /* -Buffer */
    uint32_t verify_buffers;        /* -Verify:data */
    uint64_t transfer_size;         /* -Transfer, per connection */
    uint32_t verify_mode;           /* CTS_VERIFY_SYNC / CTS_VERIFY_DEFERRED */
    uint32_t batch_buffers;         /* DEFERRED batch (0 = default) */
    uint32_t corrupt_connection;    /* fault injection: connection whose data senders flip a byte, or ~0u */
    uint32_t corrupt_send_index;    /* ... in their n-th data send (0-based; each side counts its own) */
    uint32_t socket_buffer_bytes;   /* SO_SNDBUF / SO_RCVBUF (0 = system default) */
    uint32_t push_bytes;            /* -PushBytes (PushPull; 0 = buffer_size) */
    uint32_t pull_bytes;            /* -PullBytes (PushPull; 0 = buffer_size) */
    uint32_t functor;               /* cts_loopback_functor */
    uint32_t recv_whole;            /* 1 = data recvs complete with the whole posted length (MSG_WAITALL-like):
                                       deterministic completion sizes, so runs with different verifiers can be
                                       compared counter for counter; 0 = whatever arrived (partial completions) */
    int64_t tcp_bytes_per_second;   /* -RateLimit per connection (0 = none): senders wait the tasks' time offsets */
    uint32_t burst_count;           /* -BurstCount (0 = not set) */
    uint32_t burst_delay;           /* -BurstDelay, ms */
    uint32_t buffer_size_high;      /* -Buffer:[buffer_size,buffer_size_high]: every IO draws its size uniformly
                                       (GetBufferSize, ctsConfig.cpp:4679-4684); 0 = fixed buffer_size */
    uint32_t random_seed;           /* side i draws its sizes from random_seed + i */
    uint32_t recv_ring_buffers;     /* diagnostic, verify off and the sync functor only: every data recv lands in the
                                       next slot of a ring of this many max-buffer-size slots (round robin), as a
                                       DEFERRED pattern's recvs do, instead of the pattern's buffer (0 = off) */
    uint32_t recv_ring_pinned;      /* 1 = that ring in pinned host memory (cts_host_alloc on the first engine, as
                                       the DEFERRED ring), 0 = pageable */
} cts_loopback_config;

typedef enum cts_loopback_functor {
    CTS_LOOPBACK_FUNCTOR_AUTO = 0,  /* async for Duplex, sync otherwise */
    CTS_LOOPBACK_FUNCTOR_SYNC = 1,  /* one thread per side, one blocking IO at a time (Push, Pull, PushPull) */
    CTS_LOOPBACK_FUNCTOR_ASYNC = 2  /* a send and a recv thread per side; completions re-pump InitiateIo
                                       under the connection lock (ctsSendRecvIocp.cpp:47-127, 335-415) */
} cts_loopback_functor;

typedef struct cts_loopback_result {
    double seconds;                 /* wall time from the first connect to the last completed connection */
    uint64_t bytes_sent;            /* TcpStatusDetails.m_bytesSent delta */
    uint64_t bytes_recv;            /* TcpStatusDetails.m_bytesRecv delta */
    uint64_t buffers_verified;      /* sum over server patterns */
    uint32_t connections_ok;        /* both sides CompletedIo */
    uint32_t connections_failed;    /* any side FailedIo or a socket error */
    uint32_t data_errors;           /* patterns that latched DATA_DID_NOT_MATCH_BIT_PATTERN (README "DataError") */
    uint32_t reserved;
    double recv_cpu_seconds;        /* CPU time (user + sys, RUSAGE_THREAD) of the threads that ran the data recvs:
                                       the sync functor's side threads of the receiving sides (also their sends,
                                       PushPull), the async functor's recv workers -- recv() copies, CompleteIo
                                       and VerifyBuffer (ctsSendRecvIocp.cpp:60,97 run it on the IOCP thread) */
    double send_cpu_seconds;        /* the same for the threads that ran the data sends */
    double recv_io_cpu_seconds;     /* the part of recv_cpu_seconds spent inside the socket calls (recv() and, on a
                                       sync side thread, send()); the rest ran in the pattern: InitiateIo,
                                       CompleteIo, VerifyBuffer / the DEFERRED batch bookkeeping and launches
                                       (each socket call is bracketed by two CLOCK_THREAD_CPUTIME_ID reads, a few
                                       hundred ns that land in both shares alike in every arrangement) */
} cts_loopback_result;

/* Runs cfg->connections loopback connections to completion. engine may be NULL
 * only when verify_buffers == 0 or hook != NULL (hook: see cts_batch_verifier).
 * Returns CTS_OK when the run finished (connection outcomes are in *out). */
int cts_loopback_run(const cts_loopback_config* cfg, cts_engine* engine, cts_batch_verifier hook, void* hook_ctx,
                     cts_loopback_result* out);

/* The same over several engines (one per GPU): connection i's patterns verify on
 * engines[cts_shard_of(i, n_engines)], so a host's receive traffic spreads over its GPUs' PCIe
 * links with each connection on one GPU. n_engines == 0 runs on the hook alone. */
int cts_loopback_run_multi(const cts_loopback_config* cfg, cts_engine* const* engines, uint32_t n_engines,
                           cts_batch_verifier hook, void* hook_ctx, cts_loopback_result* out);

/* One connection side's outcome: its pattern's statistics (cts_io_pattern_get_stats), the final
 * cts_io_status its functor saw, and GetLastPatternError(). */
typedef struct cts_loopback_side {
    cts_pattern_stats stats;
    uint32_t status;
    uint32_t last_error;
} cts_loopback_side;

/* cts_loopback_run_multi, plus every side's outcome in sides[2 * connections] when sides != NULL:
 * sides[i] is connection i's client (connecting) side, sides[connections + i] its server side. */
int cts_loopback_run_detailed(const cts_loopback_config* cfg, cts_engine* const* engines, uint32_t n_engines,
                              cts_batch_verifier hook, void* hook_ctx, cts_loopback_result* out,
                              cts_loopback_side* sides);

/* ---- MediaStream over loopback UDP -----------------------------------------------------------------
 * The roles of ctsMediaStreamServer + ctsMediaStreamServerConnectedSocket (ctsMediaStreamServer.cpp:510-600,
 * ctsMediaStreamServerConnectedSocket.cpp:60-140) and ctsMediaStreamClient (ctsMediaStreamClient.cpp:60-420),
 * played with blocking POSIX UDP sockets over the MediaStream patterns of cts_pattern.h:
 *   - the client sends START, then its receive thread completes every datagram into the client pattern
 *     (header checks, payload verify on the GPU, frame accounting) while the pattern's own timer thread resends
 *     START until data arrives, renders frames at the frame rate and ends the stream with Abort, which the
 *     registered callback completes;
 *   - the server waits for START, sends the connection-id datagram, then sends each frame task when its time
 *     offset comes: the frame split into datagrams (cts_media_stream_split) of {flag 0, sequence number (one per
 *     frame, from 1), QPC, QPF} + the first bytes of g_senderSharedBuffer, and completes the task.
 * "-Protocol:UDP -Pattern:MediaStream -BitsPerSecond:.. -FrameRate:.. -StreamLength:.. -BufferDepth:.." over
 * loopback, host memory and the kernel's UDP stack included. */
typedef struct cts_media_stream_loopback_config {
    uint32_t connections;           /* client/server pairs, each on its own pair of UDP sockets */
    uint32_t frame_size_bytes;      /* FrameSizeBytes (BitsPerSecond / 8 / FramesPerSecond), >= 40 */
    uint32_t frames_per_second;     /* -FrameRate */
    uint32_t stream_length_frames;  /* StreamLengthFrames (-StreamLength seconds x FrameRate) */
    uint32_t buffered_frames;       /* BufferedFrames (-BufferDepth seconds x FrameRate) */
    uint32_t datagram_max_size;     /* -DatagramByteSize (0 = 1400, c_udpDatagramMaximumSizeBytes) */
    uint32_t pre_post_recvs;        /* -PrePostRecvs of the client (0 = 1) */
    uint32_t verify_buffers;        /* -Verify:data */
    uint32_t corrupt_connection;    /* fault injection: connection whose server flips one payload byte, or ~0u */
    uint32_t corrupt_datagram;      /* ... in its n-th data datagram (0-based) */
    uint32_t socket_buffer_bytes;   /* SO_SNDBUF / SO_RCVBUF (0 = 8 MiB) */
    uint32_t verify_mode;           /* the client's CTS_VERIFY_SYNC (per datagram) or CTS_VERIFY_DEFERRED (batches
                                       through the frame-sum receive pass, flushed at every render tick) */
    uint32_t batch_buffers;         /* the client's DEFERRED batch: datagrams queued before a flush between ticks,
                                       and half its recv ring (0 = the pattern's default, 1024) */
} cts_media_stream_loopback_config;

typedef struct cts_media_stream_loopback_result {
    double seconds;                 /* wall time from the first START to the last finished connection */
    uint32_t connections_ok;        /* the client completed its stream (Abort after the final frame) */
    uint32_t connections_failed;    /* a client failed (corrupt payload, invalid datagram, FatalAbort) or a socket error */
    uint32_t data_errors;           /* clients that latched DATA_DID_NOT_MATCH_BIT_PATTERN */
    uint32_t reserved;
    uint64_t datagrams_sent;        /* data datagrams the servers sent */
    uint64_t datagrams_received;    /* datagrams the clients completed */
    cts_media_stream_stats clients; /* the clients' ctsUdpStatistics, summed (frames, bits) */
    double recv_cpu_seconds;        /* CPU time of the clients' receive threads (recv, CompleteIo, VerifyBuffer) */
} cts_media_stream_loopback_result;

/* Runs cfg->connections MediaStream connections to completion. engine may be NULL only when verify_buffers == 0
 * or hook != NULL. Returns CTS_OK when the run finished (outcomes in *out). */
int cts_loopback_media_stream_run(const cts_media_stream_loopback_config* cfg, cts_engine* engine,
                                  cts_batch_verifier hook, void* hook_ctx, cts_media_stream_loopback_result* out);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* CTS_LOOPBACK_H */
