/*
 * cts_media_stream.h — C ABI of the MediaStream (UDP) datagram framing around
 * the verify path.
 *
 * A MediaStream server sends every frame of FrameSizeBytes as datagrams of at
 * most DatagramMaxSize bytes. Each datagram is a 26-byte data header
 * {u16 flag = 0, i64 sequence number (the frame), i64 QPC, i64 QPF} followed by
 * the first (length - 26) bytes of g_senderSharedBuffer
 * (ctsMediaStreamProtocol.hpp:43-52, 171-205, 242; ctsMediaStreamServer.cpp:559-563).
 * The client validates the header, verifies the payload against the pattern at
 * offset 0, and books the bytes to a frame of its jitter queue
 * (ctsIOPatternMediaStream.cpp:140-272), which a renderer timer drains
 * (:360-530).
 *
 * GPU side (batched, device-resident): cts_media_stream_fill writes whole data
 * datagrams; the receive pass parses + validates every received datagram and
 * verifies the data payloads in one pass. It comes in three output forms:
 *   - frame sums (cts_media_stream_verify_frames / _strided_frames): the product
 *     receive path (the DEFERRED MediaStream client pattern uses it); 2-3 % over
 *     the bare payload verify per 16 M datagrams;
 *   - compact statuses, 16 B per datagram (cts_media_stream_verify_status /
 *     _strided_status): per-datagram replay of a batch the sums cannot account
 *     for; 5-13 % over the bare verify;
 *   - records + results, 44 B per datagram (cts_media_stream_verify / _strided):
 *     DIAGNOSTIC, for a caller that keeps the jitter log's sender timestamps or
 *     wants every datagram's first mismatch. 16-24 % over the bare verify: a
 *     write stream of 3 % of the bytes read costs an HBM read stream that much
 *     whatever its shape ("Why the outputs cost 20 %").
 *     Not a throughput path; use the frame sums or the statuses.
 * Host side: cts_media_stream_split (frame -> datagram sizes) and the client's
 * frame accounting (cts_media_stream_client_*), fed with any of the three.
 * The ctsIoPattern form of both MediaStream roles (connection-id and START
 * datagrams, timed frame sends, the client's timers on a pattern thread) is
 * CTS_PATTERN_MEDIA_STREAM in cts_pattern.h, built on these calls.
 */
#ifndef CTS_MEDIA_STREAM_H
#define CTS_MEDIA_STREAM_H

#include <stddef.h>
#include <stdint.h>

#include "cts_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CTS_UDP_FLAG_DATA 0x0000u                 /* c_udpDatagramProtocolHeaderFlagData */
#define CTS_UDP_FLAG_ID 0x1000u                   /* c_udpDatagramProtocolHeaderFlagId */
#define CTS_UDP_FLAG_LENGTH 2u                    /* c_udpDatagramProtocolHeaderFlagLength */
#define CTS_UDP_CONNECTION_ID_HEADER_LENGTH 39u   /* flag + ctsStatistics::ConnectionIdLength */
/* CTS_UDP_DATA_HEADER_LENGTH (26) is in cts_engine.h */

/* kind of a received datagram (ctsMediaStreamMessage::ValidateBufferLengthFromTask,
 * ctsMediaStreamProtocol.hpp:284-329, plus the zero-byte case of
 * ctsIOPatternMediaStream.cpp:158-167) */
typedef enum cts_datagram_kind {
    CTS_DGRAM_DATA = 0,      /* flag 0, >= 26 bytes: payload verified */
    CTS_DGRAM_ID = 1,        /* flag 0x1000, >= 39 bytes: carries the connection id */
    CTS_DGRAM_ZERO = 2,      /* 0 bytes */
    CTS_DGRAM_SHORT = 3,     /* shorter than its header (rejected: TooFewBytes) */
    CTS_DGRAM_UNKNOWN = 4,   /* unknown flag (rejected: TooFewBytes) */
    CTS_DGRAM_BAD_DESC = 5   /* descriptor outside the arena */
} cts_datagram_kind;

/* Header values of one outgoing data datagram. */
typedef struct cts_datagram_header {
    int64_t sequence_number;
    int64_t qpc;
    int64_t qpf;
} cts_datagram_header;

/* What the client reads out of one received datagram. Field offsets follow the
 * reference's reads, including its two overlapping ones:
 *   sequence_number = *(int64*)(buf + 2)   GetSequenceNumberFromTask (ctsMediaStreamProtocol.hpp:352-366)
 *   sender_qpc      = *(int64*)(buf + 8)   ctsIOPatternMediaStream.cpp:218
 *   sender_qpf      = *(int64*)(buf + 16)  ctsIOPatternMediaStream.cpp:219
 * (the header itself carries qpc at +10 and qpf at +18). */
typedef struct cts_datagram_record {
    int64_t sequence_number;
    int64_t sender_qpc;
    int64_t sender_qpf;
    uint16_t flag;            /* GetProtocolHeaderFromTask: u16 at +0 (0 when < 2 bytes) */
    uint8_t kind;             /* cts_datagram_kind */
    uint8_t reserved;
    uint32_t completed_bytes;
} cts_datagram_record;        /* 32 bytes */

/* Set in cts_verify_result.flags for datagrams that carry no verified payload (not DATA). */
#define CTS_RESULT_FLAG_NOT_DATA 0x2u

/* ctsMediaStreamSendRequests iteration (ctsMediaStreamProtocol.hpp:151-205):
 * the total lengths (header included) of the datagrams one frame of
 * frame_bytes is sent as. Writes min(count, cap) lengths and returns count,
 * or 0 when frame_bytes <= 26 (the reference FAIL_FASTs) or max_datagram <= 26. */
uint64_t cts_media_stream_split(uint64_t frame_bytes, uint32_t max_datagram, uint32_t* out_lengths, uint64_t cap);

/* Sender: for every descriptor d (one data datagram of d.length bytes at
 * d.byte_offset; skip_head/expected ignored), write the 26-byte header
 * {0, headers[i]} and the payload P[0 .. d.length - 26). dev_descs and
 * dev_headers must be 8-byte aligned (CTS_E_INVALID otherwise). Descriptors and
 * headers are staged in LDS 256 at a time; a datagram on a 16-byte boundary is
 * written as whole 16-byte chunks. */
int cts_media_stream_fill(cts_engine* engine, void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs,
                          const cts_datagram_header* dev_headers, uint32_t n, void* stream);

/* Sender over a ring (the layout cts_media_stream_verify_strided reads): datagram i occupies
 * [i * stride, i * stride + dev_lengths[i]) of the arena and gets the header {0, dev_headers[i]} and the payload
 * P[0 .. dev_lengths[i] - 26), as cts_media_stream_fill writes it. A length below 26, above the stride or past
 * the arena leaves its slot unwritten; the bytes between a datagram's end and the next slot are never written.
 * stride must be a multiple of 16 in [32, 1 MiB], dev_arena 16-byte aligned, dev_lengths 4-byte and dev_headers
 * 8-byte aligned (CTS_E_INVALID otherwise). The ring is written as whole 16-byte chunks, one contiguous run per
 * wave (16 M x 1472 B: 4.6-4.9 ms against 5.1-5.4 ms through descriptors). */
int cts_media_stream_fill_strided(cts_engine* engine, void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                                  const uint32_t* dev_lengths, const cts_datagram_header* dev_headers, uint32_t n,
                                  void* stream);

/* Receiver, records + results form (DIAGNOSTIC: see the top of this header; the throughput paths are
 * cts_media_stream_verify_frames and cts_media_stream_verify_status).
 * d.length = completed bytes of datagram i at d.byte_offset
 * (skip_head/expected ignored). records[i] gets the parsed header; for DATA
 * datagrams results[i] is the payload verify (skip 26, expected offset 0,
 * RtlCompareMemory semantics, ctsIOPatternMediaStream.cpp:185-192) and the
 * counters (cts_counters_device_bytes block, accumulated) count it; for other
 * kinds results[i].flags = CTS_RESULT_FLAG_NOT_DATA and nothing is counted.
 * Any output may be NULL. */
int cts_media_stream_verify(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes,
                            const cts_buf_desc* dev_descs, uint32_t n, cts_datagram_record* dev_records,
                            cts_verify_result* dev_results, void* dev_counters, void* stream);

/* The same receive pass (records + results: DIAGNOSTIC) over a uniformly strided receive ring: datagram i occupies
 * [i * stride, i * stride + dev_lengths[i]) of the arena (the completed byte count of the recv
 * posted into that slot, ctsMediaStreamClient.cpp:268,404), so the kernel reads 4 bytes of
 * metadata per datagram instead of a 24-byte descriptor. A length above the stride or past the
 * arena is CTS_DGRAM_BAD_DESC. Outputs and counters as cts_media_stream_verify. dev_lengths must be
 * 4-byte aligned, dev_arena 16-byte aligned with arena_bytes >= 16. */
int cts_media_stream_verify_strided(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                                    const uint32_t* dev_lengths, uint32_t n, cts_datagram_record* dev_records,
                                    cts_verify_result* dev_results, void* dev_counters, void* stream);

/* Compact receive output: what the client's frame accounting reads of one datagram when no jitter log is
 * written. The sender timestamps of cts_datagram_record feed only the jitter log and its time-in-flight
 * estimate (ctsIOPatternMediaStream.cpp:218-223, 366-393; ctsConfig.cpp:3910-3930), and a failing payload
 * ends the stream whatever its first mismatch was (:185-190), so 16 bytes per datagram replace the 32-byte
 * record and the 12-byte result. (Per 16 M datagrams the receive pass takes 3.99-4.39 ms with statuses against
 * 4.31-4.89 ms with records + results and 3.67 ms with no outputs, by box: DESIGN.md section 3.) */
typedef struct cts_datagram_status {
    int64_t sequence_number;  /* DATA datagrams: header bytes 2..9 (GetSequenceNumberFromTask); otherwise 0 */
    uint32_t completed_bytes;
    uint16_t flag;            /* as cts_datagram_record.flag */
    uint8_t kind;             /* cts_datagram_kind */
    uint8_t pass;             /* DATA: 1 = payload verified clean, 0 = corrupt; other kinds: 0 */
} cts_datagram_status;        /* 16 bytes */

/* The receive pass of cts_media_stream_verify / cts_media_stream_verify_strided writing one
 * cts_datagram_status per datagram (dev_status may be NULL: counters only). Counters as there; the first
 * mismatch of a failing datagram is cts_verify of its payload span (skip 26, expected offset 0) when wanted. */
int cts_media_stream_verify_status(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes,
                                   const cts_buf_desc* dev_descs, uint32_t n, cts_datagram_status* dev_status,
                                   void* dev_counters, void* stream);
int cts_media_stream_verify_strided_status(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes,
                                           uint32_t stride, const uint32_t* dev_lengths, uint32_t n,
                                           cts_datagram_status* dev_status, void* dev_counters, void* stream);

/* ---- the receive pass with the client's frame accounting summed on the GPU -------------------------
 * Between two render ticks the client's jitter window does not move, so CompleteTaskBackToPattern
 * (ctsIOPatternMediaStream.cpp:150-272) over a batch of received datagrams is a sum over its DATA datagrams whose
 * payload verified clean: their bits, the bytes of each frame of the window, and one error frame for each datagram
 * whose sequence number is past the final frame or outside the window. cts_media_stream_verify_frames verifies the
 * batch and writes exactly those sums (no per-datagram output). Every other datagram -- an ID datagram, a zero-byte
 * one (unless the stream finished), a short or unknown one, a corrupt payload -- is an exception: the sums then do not
 * apply, cts_media_stream_client_complete_frames says so (CTS_MS_FRAMES_REPLAY) and the caller replays the batch datagram
 * by datagram (cts_media_stream_verify_status + cts_media_stream_client_complete_status). */
typedef struct cts_frame_window {
    int64_t head_sequence_number;  /* the jitter queue's head frame */
    int64_t final_frame;           /* m_finalFrame */
    uint32_t frames;               /* the queue's size: sequence numbers head .. head + frames - 1 */
    uint32_t finished;             /* the stream finished: a zero-byte datagram is not an exception */
} cts_frame_window;

#define CTS_FRAME_TOTAL_SHARDS 64
/* The batch's sums, folded from the device block (cts_frame_totals_fold). */
typedef struct cts_frame_totals {
    uint64_t bits_received;        /* clean DATA datagrams: completed bytes x 8 */
    uint64_t error_frames;         /* ... of them outside the window or past the final frame */
    uint64_t datagrams;            /* clean DATA datagrams */
    uint32_t first_exception;      /* lowest index of an exception (0xFFFFFFFF: none) */
    uint32_t exceptions;
} cts_frame_totals;

/* Bytes of the device block of totals: CTS_FRAME_TOTAL_SHARDS shards of 32 bytes (workgroups add into shard
 * blockIdx mod 64, as the counter block). */
size_t cts_frame_totals_device_bytes(void);
/* Fold a host copy of the device block. */
int cts_frame_totals_fold(const void* host_block, cts_frame_totals* out);

/* The receive pass of cts_media_stream_verify (descriptors) / _strided (a receive ring) summing the batch's frame
 * accounting for `window` into dev_totals (cts_frame_totals_device_bytes(), 8-byte aligned) and
 * dev_frame_bytes[window->frames] (bytes of sequence number head + k). Both are zeroed on the stream first. The
 * counter block (may be NULL) accumulates as in cts_media_stream_verify. */
int cts_media_stream_verify_frames(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes,
                                   const cts_buf_desc* dev_descs, uint32_t n, const cts_frame_window* window,
                                   void* dev_totals, uint64_t* dev_frame_bytes, void* dev_counters, void* stream);
int cts_media_stream_verify_strided_frames(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes,
                                           uint32_t stride, const uint32_t* dev_lengths, uint32_t n,
                                           const cts_frame_window* window, void* dev_totals,
                                           uint64_t* dev_frame_bytes, void* dev_counters, void* stream);

/* ---- client frame accounting (ctsIoPatternMediaStreamClient) ---------------- */
typedef struct cts_media_stream_settings { /* ctsConfig::MediaStreamSettings */
    uint32_t frame_size_bytes;
    uint32_t datagram_max_size;
    uint32_t frames_per_second;
    uint32_t buffered_frames;
    int64_t stream_length_frames;
} cts_media_stream_settings;

/* ctsUdpStatistics (ctsStatistics.hpp:249-314) + the first failure */
typedef struct cts_media_stream_stats {
    int64_t bits_received;
    int64_t successful_frames;
    int64_t dropped_frames;
    int64_t duplicate_frames;
    int64_t error_frames;
    uint64_t datagrams;          /* datagrams completed into the pattern */
    uint32_t last_error;         /* GetLastPatternError(): 0 / running / protocol error */
    uint32_t finished;           /* 1 = stream rendered to its final frame (Abort), 2 = FatalAbort */
    int64_t head_sequence_number;
    uint32_t fail_datagram;      /* index (in completion order) of the datagram that failed the stream */
    uint32_t has_failure;
} cts_media_stream_stats;

typedef struct cts_media_stream_client cts_media_stream_client;

int cts_media_stream_client_create(const cts_media_stream_settings* settings, cts_media_stream_client** out);
int cts_media_stream_client_destroy(cts_media_stream_client* client);
/* CompleteIo of n received datagrams in completion order (records/results from
 * cts_media_stream_verify, copied to host). Stops at the first datagram that
 * fails the stream (zero bytes before the end, a rejected header, a corrupted
 * payload), as the reference's FailedIo would. *consumed = datagrams applied.
 * Returns a cts_io_status (cts_pattern.h) or a negative cts_status.
 * An ID datagram's connection id must be handed over with
 * cts_media_stream_client_set_connection_id (the record does not carry it). */
int cts_media_stream_client_complete(cts_media_stream_client* client, const cts_datagram_record* records,
                                     const cts_verify_result* results, uint32_t n, int64_t receiver_qpc,
                                     int64_t receiver_qpf, uint32_t* consumed);
/* The same CompleteIo over compact statuses (cts_media_stream_verify_status): frames keep sender
 * timestamps of 0, everything else (bits, successful / dropped / duplicate / error frames, the failure) is
 * identical to cts_media_stream_client_complete. */
int cts_media_stream_client_complete_status(cts_media_stream_client* client, const cts_datagram_status* status,
                                            uint32_t n, int64_t receiver_qpc, int64_t receiver_qpf, uint32_t* consumed);
/* The client's current window for cts_media_stream_verify_frames (it moves only at a render tick). */
int cts_media_stream_client_window(const cts_media_stream_client* client, cts_frame_window* out);
/* CompleteIo of a batch of n datagrams from its GPU sums (cts_media_stream_verify_frames over `window`, folded;
 * frame_bytes[window->frames] copied to host). Returns a cts_io_status as cts_media_stream_client_complete does
 * (every datagram consumed), CTS_MS_FRAMES_REPLAY when the batch holds an exception (nothing applied: replay it with
 * cts_media_stream_client_complete_status), or CTS_E_INVALID when `window` is not the client's current one.
 * Frames booked from sums (as from statuses) carry no sender timestamps (0): the jitter log's time-in-flight estimate
 * (ctsIOPatternMediaStream.cpp:366-393) is left at 0 for them rather than computed from a zero frequency; a caller
 * that logs jitter uses the records form. */
#define CTS_MS_FRAMES_REPLAY 16
int cts_media_stream_client_complete_frames(cts_media_stream_client* client, const cts_frame_window* window,
                                            const cts_frame_totals* totals, const uint64_t* frame_bytes, uint32_t n,
                                            int64_t receiver_qpc, int64_t receiver_qpf);
int cts_media_stream_client_set_connection_id(cts_media_stream_client* client, const char* datagram, uint32_t len);
/* One renderer-timer tick (TimerCallback, ctsIOPatternMediaStream.cpp:470-530,
 * without the wall-clock scheduling, which CTS_PATTERN_MEDIA_STREAM adds): returns 0 = keep rendering, 1 = the stream
 * finished (Abort), 2 = nothing was ever received (FatalAbort). */
int cts_media_stream_client_render(cts_media_stream_client* client);
int cts_media_stream_client_stats(const cts_media_stream_client* client, cts_media_stream_stats* out);
/* The client's connection id (37 bytes incl. NUL) once an ID datagram was applied. */
const char* cts_media_stream_client_connection_id(const cts_media_stream_client* client);

/* ---- process-wide UDP status counters (UdpStatusDetails, ctsConfig.h:417) ----
 * Every client adds to these where it adds to its own cts_media_stream_stats, as
 * ctsIOPatternMediaStream.cpp:195-202, 245-246, 385-386, 405-406, 420-421, 501-502 feed
 * g_configSettings->UdpStatusDetails; the UDP status line and exit summary (cts_status.h) print them.
 * A corrupt payload is not an error frame: it fails the stream (CorruptedBytes, :185-190), which the
 * connection outcome (ProtocolErrors) counts. */
typedef struct cts_udp_status_details {
    int64_t bits_received;
    int64_t successful_frames;
    int64_t dropped_frames;
    int64_t duplicate_frames;
    int64_t error_frames;
} cts_udp_status_details;
int cts_udp_status_details_read(cts_udp_status_details* out);
void cts_udp_status_details_reset(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* CTS_MEDIA_STREAM_H */
