// cts_media_stream.cpp — host side of the MediaStream (UDP) framing around the
// verify path (include/cts_media_stream.h):
//
//   cts_media_stream_split    ctsMediaStreamSendRequests::iterator
//                             (ctsTraffic/ctsMediaStreamProtocol.hpp:151-205)
//   cts_media_stream_client_* the frame accounting of ctsIoPatternMediaStreamClient
//                             (ctsTraffic/ctsIOPatternMediaStream.cpp:46-300, 302-414,
//                             470-530) driven by explicit render ticks instead of
//                             threadpool timers, fed with the records and verify
//                             results cts_media_stream_verify produces on the GPU.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <new>
#include <vector>

#include "cts_media_stream.h"
#include "cts_media_stream_client.hpp"
#include "cts_pattern.h"

namespace {

constexpr uint32_t kHeader = CTS_UDP_DATA_HEADER_LENGTH;

// ctsMediaStreamSendRequests::iterator::UpdateBufferLength (ctsMediaStreamProtocol.hpp:171-205):
// the total length (header included) of the next datagram with bytes_to_send left.
uint32_t update_buffer_length(int64_t bytes_to_send, uint32_t max_datagram)
{
    uint32_t payload = bytes_to_send > (int64_t)max_datagram ? max_datagram - kHeader
                                                             : (uint32_t)(bytes_to_send - kHeader);
    uint32_t total = kHeader + payload;  // WSABUF[0..3] = 2 + 8 + 8 + 8
    const int64_t remaining = bytes_to_send - (int64_t)total;
    if (remaining > 0 && remaining <= (int64_t)kHeader) {
        // leave enough for the next datagram's header plus one byte of data
        const uint32_t delta = kHeader + 1 - (uint32_t)remaining;
        payload -= delta;
        total -= delta;
    }
    return total;
}

// the process-wide UdpStatusDetails (ctsConfig.h:417): every client adds to it exactly where it adds to its own
// ctsUdpStatistics (ctsIOPatternMediaStream.cpp:195-202, 245-246, 385-386, 405-406, 420-421, 501-502)
struct UdpStatusDetails {
    std::atomic<int64_t> bits_received{0}, successful_frames{0}, dropped_frames{0}, duplicate_frames{0},
        error_frames{0};
} g_udp;

struct Frame {  // ctsConfig::JitterFrameEntry (ctsConfig.h:188-197)
    int64_t bytes_received = 0;
    int64_t sequence_number = 0;
    int64_t sender_qpc = 0;
    int64_t sender_qpf = 0;
    int64_t receiver_qpc = 0;
    int64_t receiver_qpf = 0;
    double estimated_time_in_flight_ms = 0;
};

}  // namespace

struct cts_media_stream_client {
    cts_media_stream_settings cfg{};
    int64_t final_frame = 0;
    uint32_t initial_buffer_frames = 0;
    uint32_t timer_wheel_offset_frames = 0;
    std::vector<Frame> frames;
    size_t head = 0;
    Frame first_frame, previous_frame;
    bool finished = false;
    uint32_t finished_code = 0;
    uint32_t last_error = CTS_STATUS_IO_RUNNING;
    bool has_failure = false;
    uint32_t fail_datagram = 0;
    uint64_t datagrams = 0;
    int64_t bits_received = 0, successful = 0, dropped = 0, duplicate = 0, error_frames = 0;
    char connection_id[CTS_CONNECTION_ID_LENGTH] = {};

    // FindSequenceNumber (ctsIOPatternMediaStream.cpp:280-300); -1 = end(m_frameEntries)
    ptrdiff_t find(int64_t seq) const
    {
        const int64_t head_seq = frames[head].sequence_number;
        const int64_t tail_seq = head_seq + (int64_t)frames.size() - 1;
        const int64_t vector_end_seq = frames.back().sequence_number;
        if (seq > tail_seq || seq < head_seq) return -1;
        if (seq <= vector_end_seq) return (ptrdiff_t)head + (ptrdiff_t)(seq - head_seq);
        return (ptrdiff_t)(seq - vector_end_seq - 1);
    }

    // ReceivedBufferedFrames (:302-318)
    bool received_buffered_frames() const
    {
        if (frames[0].sequence_number > 1) return true;
        if (head != 0) return true;
        return std::any_of(frames.begin(), frames.end(), [](const Frame& f) { return f.bytes_received > 0; });
    }

    // UpdateLastError for UDP (ctsIOPattern.h:344-365 + ctsIOPatternState.hpp:254-270): first error wins
    void latch(uint32_t error)
    {
        if (last_error == CTS_STATUS_IO_RUNNING) last_error = error;
    }

    // RenderFrame (:360-414)
    void render_frame()
    {
        Frame& h = frames[head];
        // frames booked from GPU batch sums (statuses, frame sums) carry no sender timestamps (qpf 0): no estimate
        if (h.receiver_qpf != 0 && first_frame.receiver_qpf != 0 && h.sender_qpf != 0 && first_frame.sender_qpf != 0) {
            const double ms_since_first_receive = (double)h.receiver_qpc * 1000.0 / (double)h.receiver_qpf -
                                                  (double)first_frame.receiver_qpc * 1000.0 / (double)first_frame.receiver_qpf;
            const double ms_since_first_send = (double)h.sender_qpc * 1000.0 / (double)h.sender_qpf -
                                               (double)first_frame.sender_qpc * 1000.0 / (double)first_frame.sender_qpf;
            h.estimated_time_in_flight_ms = ms_since_first_receive - ms_since_first_send;
        }
        if (h.bytes_received == (int64_t)cfg.frame_size_bytes) {
            ++successful;
            g_udp.successful_frames.fetch_add(1, std::memory_order_relaxed);  // :385-386
            if (first_frame.receiver_qpc == 0) first_frame = h;
            previous_frame = h;
        } else if (h.bytes_received < (int64_t)cfg.frame_size_bytes) {
            ++dropped;
            g_udp.dropped_frames.fetch_add(1, std::memory_order_relaxed);  // :405-406
        } else {
            ++duplicate;
            g_udp.duplicate_frames.fetch_add(1, std::memory_order_relaxed);  // :420-421
        }
        h.sequence_number += (int64_t)frames.size();
        h.bytes_received = 0;
        if (++head == frames.size()) head = 0;
    }
};

extern "C" {

uint64_t cts_media_stream_split(uint64_t frame_bytes, uint32_t max_datagram, uint32_t* out_lengths, uint64_t cap)
{
    // the ctor FAIL_FASTs on bytesToSend <= c_udpDatagramDataHeaderLength (:214-216)
    if (frame_bytes <= kHeader || max_datagram <= kHeader) return 0;
    int64_t bytes = (int64_t)frame_bytes;
    uint64_t count = 0;
    // begin(): the first length is taken in the iterator's constructor; operator++
    // takes the next one while bytes remain (:139-149, :164-169)
    while (bytes > 0) {
        const uint32_t len = update_buffer_length(bytes, max_datagram);
        if (out_lengths != nullptr && count < cap) out_lengths[count] = len;
        ++count;
        bytes -= len;
    }
    return count;
}

int cts_media_stream_client_create(const cts_media_stream_settings* s, cts_media_stream_client** out)
{
    if (s == nullptr || out == nullptr) return CTS_E_INVALID;
    *out = nullptr;
    if (s->frame_size_bytes == 0 || s->frames_per_second == 0 || s->stream_length_frames <= 0 ||
        s->stream_length_frames > (int64_t)UINT32_MAX)
        return CTS_E_INVALID;  // FAIL_FAST_IF(m_finalFrame > UINT32_MAX), :53
    cts_media_stream_client* c = new (std::nothrow) cts_media_stream_client();
    if (c == nullptr) return CTS_E_NOMEM;
    c->cfg = *s;
    c->final_frame = s->stream_length_frames;
    c->initial_buffer_frames = std::min<uint32_t>((uint32_t)c->final_frame, s->buffered_frames);
    c->timer_wheel_offset_frames = c->initial_buffer_frames;
    const int64_t queue_size = 2 * (int64_t)c->initial_buffer_frames;  // extraBufferDepthFactor
    if (queue_size < 2) {  // "BufferDepth & FrameSize don't allow for enough buffered stream"
        delete c;
        return CTS_E_INVALID;
    }
    try {
        c->frames.resize((size_t)queue_size);
    } catch (const std::bad_alloc&) {
        delete c;
        return CTS_E_NOMEM;
    }
    int64_t seq = 1;
    for (auto& f : c->frames) f.sequence_number = seq++;
    *out = c;
    return CTS_OK;
}

int cts_media_stream_client_destroy(cts_media_stream_client* c)
{
    if (c == nullptr) return CTS_E_INVALID;
    delete c;
    return CTS_OK;
}

}  // extern "C"

namespace {
// CompleteTaskBackToPattern (ctsIOPatternMediaStream.cpp:150-272) over n datagrams in completion order; at(j)
// gives datagram j's {kind, pass, completed bytes, sequence number, sender qpc, sender qpf}.
struct DgramView {
    uint32_t kind, pass, completed;
    int64_t seq, qpc, qpf;
};

template <typename At>
int complete_datagrams(cts_media_stream_client* c, uint32_t n, At at, int64_t receiver_qpc, int64_t receiver_qpf,
                       uint32_t* consumed)
{
    uint32_t j = 0;
    for (; j < n && c->last_error == CTS_STATUS_IO_RUNNING; ++j) {
        const DgramView r = at(j);
        ++c->datagrams;
        uint32_t err = 0;
        switch (r.kind) {
        case CTS_DGRAM_ZERO:
            if (!c->finished) err = CTS_STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED;  // zero-byte datagram: TooFewBytes
            break;
        case CTS_DGRAM_SHORT:
        case CTS_DGRAM_UNKNOWN:
        case CTS_DGRAM_BAD_DESC: err = CTS_STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED; break;  // invalid header
        case CTS_DGRAM_ID: break;  // SetConnectionIdFromTask: see cts_media_stream_client_set_connection_id
        case CTS_DGRAM_DATA:
            if (!r.pass) {  // VerifyBuffer failed: CorruptedBytes
                err = CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN;
                break;
            }
            cts::ms_client_apply_data(c, cts::MsDatagram{r.seq, r.qpc, r.qpf, r.completed}, receiver_qpc,
                                      receiver_qpf);
            break;
        default: err = CTS_STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED; break;
        }
        if (err != 0) {
            c->latch(err);
            c->has_failure = true;
            c->fail_datagram = (uint32_t)(c->datagrams - 1);
        }
    }
    if (consumed != nullptr) *consumed = j;
    if (c->last_error == CTS_STATUS_IO_RUNNING) return CTS_IO_CONTINUE;
    return c->last_error == 0 ? CTS_IO_COMPLETED : CTS_IO_FAILED;
}
}  // namespace

extern "C" {

int cts_media_stream_client_complete(cts_media_stream_client* c, const cts_datagram_record* recs,
                                     const cts_verify_result* res, uint32_t n, int64_t receiver_qpc,
                                     int64_t receiver_qpf, uint32_t* consumed)
{
    if (c == nullptr || (n != 0 && (recs == nullptr || res == nullptr))) return CTS_E_INVALID;
    return complete_datagrams(
        c, n,
        [&](uint32_t j) {
            const cts_datagram_record& r = recs[j];
            return DgramView{r.kind, res[j].pass, r.completed_bytes, r.sequence_number, r.sender_qpc, r.sender_qpf};
        },
        receiver_qpc, receiver_qpf, consumed);
}

int cts_media_stream_client_complete_status(cts_media_stream_client* c, const cts_datagram_status* st, uint32_t n,
                                            int64_t receiver_qpc, int64_t receiver_qpf, uint32_t* consumed)
{
    if (c == nullptr || (n != 0 && st == nullptr)) return CTS_E_INVALID;
    return complete_datagrams(
        c, n,
        [&](uint32_t j) {
            const cts_datagram_status& r = st[j];
            return DgramView{r.kind, r.pass, r.completed_bytes, r.sequence_number, 0, 0};
        },
        receiver_qpc, receiver_qpf, consumed);
}

int cts_media_stream_client_set_connection_id(cts_media_stream_client* c, const char* dgram, uint32_t len)
{
    if (c == nullptr || dgram == nullptr || len < CTS_UDP_CONNECTION_ID_HEADER_LENGTH) return CTS_E_INVALID;
    const uint16_t flag = (uint16_t)((uint8_t)dgram[0] | ((uint16_t)(uint8_t)dgram[1] << 8));
    if (flag != CTS_UDP_FLAG_ID) return CTS_E_INVALID;
    std::memcpy(c->connection_id, dgram + CTS_UDP_FLAG_LENGTH, CTS_CONNECTION_ID_LENGTH);  // :337-348
    c->connection_id[CTS_CONNECTION_ID_LENGTH - 1] = 0;
    return CTS_OK;
}

int cts_media_stream_client_render(cts_media_stream_client* c)
{
    if (c == nullptr) return CTS_E_INVALID;
    if (c->finished) return (int)c->finished_code;
    const int code = cts::ms_client_tick(c);
    if (code == 2) c->latch(CTS_STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED);  // CompleteIo(FatalAbort), ctsIOPattern.cpp:385-388
    if (code == 1) c->latch(0);  // CompleteIo(Abort) -> SuccessfullyCompleted (:143-150)
    return code;
}

int cts_media_stream_client_stats(const cts_media_stream_client* c, cts_media_stream_stats* o)
{
    if (c == nullptr || o == nullptr) return CTS_E_INVALID;
    *o = cts_media_stream_stats{};
    o->bits_received = c->bits_received;
    o->successful_frames = c->successful;
    o->dropped_frames = c->dropped;
    o->duplicate_frames = c->duplicate;
    o->error_frames = c->error_frames;
    o->datagrams = c->datagrams;
    o->last_error = c->last_error;
    o->finished = c->finished_code;
    o->head_sequence_number = c->frames[c->head].sequence_number;
    o->fail_datagram = c->fail_datagram;
    o->has_failure = c->has_failure ? 1u : 0u;
    return CTS_OK;
}

const char* cts_media_stream_client_connection_id(const cts_media_stream_client* c)
{
    return c == nullptr ? nullptr : c->connection_id;
}

size_t cts_frame_totals_device_bytes(void) { return (size_t)CTS_FRAME_TOTAL_SHARDS * 4u * sizeof(uint64_t); }

int cts_frame_totals_fold(const void* host_block, cts_frame_totals* o)
{
    if (host_block == nullptr || o == nullptr) return CTS_E_INVALID;
    // shard: {bits, error frames, datagrams, u32 ~first exception | u32 exceptions << 32} (media_stream_verify_quad_kernel)
    const uint64_t* b = static_cast<const uint64_t*>(host_block);
    *o = cts_frame_totals{};
    uint32_t inv_first = 0;
    for (uint32_t sh = 0; sh < CTS_FRAME_TOTAL_SHARDS; ++sh, b += 4) {
        o->bits_received += b[0];
        o->error_frames += b[1];
        o->datagrams += b[2];
        inv_first = std::max(inv_first, (uint32_t)b[3]);
        o->exceptions += (uint32_t)(b[3] >> 32);
    }
    o->first_exception = inv_first != 0 ? ~inv_first : 0xFFFFFFFFu;
    return CTS_OK;
}

int cts_media_stream_client_window(const cts_media_stream_client* c, cts_frame_window* o)
{
    if (c == nullptr || o == nullptr) return CTS_E_INVALID;
    *o = cts_frame_window{c->frames[c->head].sequence_number, c->final_frame, (uint32_t)c->frames.size(),
                          c->finished ? 1u : 0u};
    return CTS_OK;
}

int cts_media_stream_client_complete_frames(cts_media_stream_client* c, const cts_frame_window* w,
                                            const cts_frame_totals* t, const uint64_t* frame_bytes, uint32_t n,
                                            int64_t receiver_qpc, int64_t receiver_qpf)
{
    if (c == nullptr || w == nullptr || t == nullptr || (w->frames != 0 && frame_bytes == nullptr))
        return CTS_E_INVALID;
    cts_frame_window now{};
    (void)cts_media_stream_client_window(c, &now);
    if (w->head_sequence_number != now.head_sequence_number || w->final_frame != now.final_frame ||
        w->frames != now.frames || w->finished != now.finished)
        return CTS_E_INVALID;  // a render tick moved the window since the batch was summed
    if (c->last_error != CTS_STATUS_IO_RUNNING) return c->last_error == 0 ? CTS_IO_COMPLETED : CTS_IO_FAILED;
    if (t->datagrams > n || t->error_frames > t->datagrams) return CTS_E_INVALID;  // not the sums of these n
    if (t->first_exception != 0xFFFFFFFFu || t->exceptions != 0) return CTS_MS_FRAMES_REPLAY;
    // the per-datagram accounting of complete_datagrams, summed (ctsIOPatternMediaStream.cpp:195-265)
    c->datagrams += n;
    c->bits_received += (int64_t)t->bits_received;
    g_udp.bits_received.fetch_add((int64_t)t->bits_received, std::memory_order_relaxed);
    c->error_frames += (int64_t)t->error_frames;
    g_udp.error_frames.fetch_add((int64_t)t->error_frames, std::memory_order_relaxed);
    for (uint32_t k = 0; k < w->frames; ++k) {
        if (frame_bytes[k] == 0) continue;
        Frame& f = c->frames[(c->head + k) % c->frames.size()];
        f.sender_qpc = 0;  // (the sums carry no sender timestamps: no jitter log, as the compact statuses)
        f.sender_qpf = 0;
        f.receiver_qpc = receiver_qpc;
        f.receiver_qpf = receiver_qpf;
        f.bytes_received += (int64_t)frame_bytes[k];
    }
    return CTS_IO_CONTINUE;
}

int cts_udp_status_details_read(cts_udp_status_details* o)
{
    if (o == nullptr) return CTS_E_INVALID;
    o->bits_received = g_udp.bits_received.load();
    o->successful_frames = g_udp.successful_frames.load();
    o->dropped_frames = g_udp.dropped_frames.load();
    o->duplicate_frames = g_udp.duplicate_frames.load();
    o->error_frames = g_udp.error_frames.load();
    return CTS_OK;
}

void cts_udp_status_details_reset(void)
{
    g_udp.bits_received = 0;
    g_udp.successful_frames = 0;
    g_udp.dropped_frames = 0;
    g_udp.duplicate_frames = 0;
    g_udp.error_frames = 0;
}

}  // extern "C"

namespace cts {

void ms_client_apply_data(cts_media_stream_client* c, const MsDatagram& d, int64_t receiver_qpc, int64_t receiver_qpf)
{
    c->bits_received += (int64_t)d.completed_bytes * 8;
    g_udp.bits_received.fetch_add((int64_t)d.completed_bytes * 8, std::memory_order_relaxed);  // :195-196
    if (d.sequence_number > c->final_frame) {
        ++c->error_frames;  // an unknown seq number past the final frame
        g_udp.error_frames.fetch_add(1, std::memory_order_relaxed);  // :201-202
        return;
    }
    const ptrdiff_t slot = c->find(d.sequence_number);
    if (slot < 0) {
        ++c->error_frames;  // a stale or a future seq number
        g_udp.error_frames.fetch_add(1, std::memory_order_relaxed);  // :245-246
        return;
    }
    Frame& f = c->frames[(size_t)slot];
    f.sender_qpc = d.sender_qpc;
    f.sender_qpf = d.sender_qpf;
    f.receiver_qpc = receiver_qpc;
    f.receiver_qpf = receiver_qpf;
    f.bytes_received += d.completed_bytes;
}

int ms_client_tick(cts_media_stream_client* c)
{
    ++c->timer_wheel_offset_frames;  // TimerCallback (:470-530)
    if (c->timer_wheel_offset_frames >= c->initial_buffer_frames && c->frames[c->head].sequence_number <= c->final_frame) {
        if (!c->received_buffered_frames()) {
            // "have received nothing from the server": every frame counts as dropped, FatalAbort
            c->dropped += c->final_frame;
            g_udp.dropped_frames.fetch_add(c->final_frame, std::memory_order_relaxed);  // :501-502
            c->finished = true;
            c->finished_code = 2;
            return 2;
        }
        c->render_frame();
    }
    if (c->frames[c->head].sequence_number <= c->final_frame) return 0;
    c->finished = true;
    c->finished_code = 1;
    return 1;
}

uint32_t ms_client_timer_wheel_offset(const cts_media_stream_client* c) { return c->timer_wheel_offset_frames; }
bool ms_client_received_buffered_frames(const cts_media_stream_client* c) { return c->received_buffered_frames(); }
bool ms_client_finished(const cts_media_stream_client* c) { return c->finished; }
void udp_status_add_bits(int64_t bits) { g_udp.bits_received.fetch_add(bits, std::memory_order_relaxed); }

}  // namespace cts
