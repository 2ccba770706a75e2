// cts_media_stream_client.hpp — the MediaStream client's frame accounting (cts_media_stream.cpp) as the
// MediaStream client pattern of the ctsIoPattern mirror (cts_pattern.cpp) drives it: one datagram and one
// renderer-timer tick at a time, with the pattern (not the accounting object) owning the connection's status.
// Host-only (no HIP types): the sanitizer builds compile it with g++.
#pragma once

#include <stdint.h>

#include "cts_media_stream.h"

namespace cts {

// the header fields CompleteTaskBackToPattern reads of a clean DATA datagram (ctsIOPatternMediaStream.cpp:198-223)
struct MsDatagram {
    int64_t sequence_number;  // GetSequenceNumberFromTask: buffer + 2
    int64_t sender_qpc;       // buffer + 8
    int64_t sender_qpf;       // buffer + 16
    uint32_t completed_bytes;
};

// ctsIOPatternMediaStream.cpp:195-263 for one DATA datagram whose payload verified clean: its bits, then its
// frame slot or an error frame (the process-wide UdpStatusDetails too).
void ms_client_apply_data(cts_media_stream_client* c, const MsDatagram& d, int64_t receiver_qpc,
                          int64_t receiver_qpf);
// One pass of TimerCallback's loop body (:477-520): 0 = keep rendering, 1 = the stream is done (the caller sends
// Abort), 2 = nothing was received (every frame dropped, the caller sends FatalAbort). Marks the stream finished
// for 1 and 2; latches nothing (the pattern's CompleteIo of the Abort / FatalAbort task sets the status).
int ms_client_tick(cts_media_stream_client* c);
uint32_t ms_client_timer_wheel_offset(const cts_media_stream_client* c);  // m_timerWheelOffsetFrames
bool ms_client_received_buffered_frames(const cts_media_stream_client* c); // ReceivedBufferedFrames (:302-318)
bool ms_client_finished(const cts_media_stream_client* c);                // m_finishedStream
// UdpStatusDetails.m_bitsReceived.Add (the server pattern's sends, ctsIOPattern.cpp:1160-1163)
void udp_status_add_bits(int64_t bits);

}  // namespace cts
