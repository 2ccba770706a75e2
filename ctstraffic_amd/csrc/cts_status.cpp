// cts_status.cpp — status output (include/cts_status.h), restating
// ctsTcpStatusInformation (ctsTraffic/ctsPrintStatus.hpp:452-600),
// ctsUdpStatusInformation (:314-446), the exit summary (ctsTraffic.cpp:155-200)
// and the helpers of their base class (RightJustifyOutput :166-229, AppendCsvOutput
// :245-320): a 1024-column space-filled line, each value right-justified to
// end at its column offset, falling back to x^6 / x^9 / x^12 notation and then
// "9+++T" when it does not fit its width.
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <string>

#include "cts_status.h"

namespace {

constexpr uint32_t kOutputBufferSize = 1024;  // c_outputBufferSize

// column layout of ctsTcpStatusInformation (ctsPrintStatus.hpp:582-597)
constexpr uint32_t kTimeSliceOffset = 10, kTimeSliceLength = 10;
constexpr uint32_t kSendOffset = 23, kSendLength = 11;
constexpr uint32_t kRecvOffset = 36, kRecvLength = 11;
constexpr uint32_t kInFlightOffset = 47, kInFlightLength = 7;
constexpr uint32_t kCompletedOffset = 58, kCompletedLength = 7;
constexpr uint32_t kNetErrorOffset = 68, kNetErrorLength = 7;
constexpr uint32_t kDataErrorOffset = 79, kDataErrorLength = 7;

// column layout of ctsUdpStatusInformation (ctsPrintStatus.hpp:426-445)
constexpr uint32_t kUdpTimeSliceOffset = 10, kUdpTimeSliceLength = 10;
constexpr uint32_t kBitsPerSecondOffset = 25, kBitsPerSecondLength = 12;
constexpr uint32_t kStreamsOffset = 36, kStreamsLength = 8;
constexpr uint32_t kCompletedFramesOffset = 48, kCompletedFramesLength = 9;
constexpr uint32_t kDroppedFramesOffset = 58, kDroppedFramesLength = 7;
constexpr uint32_t kRepeatedFramesOffset = 69, kRepeatedFramesLength = 7;
constexpr uint32_t kErrorFramesOffset = 79, kErrorFramesLength = 7;

struct Line {
    char buf[kOutputBufferSize + 1];
    Line()
    {
        std::memset(buf, ' ', kOutputBufferSize);  // ResetBuffer
        buf[kOutputBufferSize] = 0;
    }
    template <typename T>
    void right_justify(uint32_t offset, uint32_t max_length, T value)  // RightJustifyOutput
    {
        char conv[32];
        int n = format(conv, value);
        if (n < 0) return;
        if ((uint32_t)n > max_length) n = std::snprintf(conv, sizeof(conv), "%.1fx^6", (double)value / 1000000.0);
        if ((uint32_t)n > max_length) n = std::snprintf(conv, sizeof(conv), "%.1fx^9", (double)value / 1000000000.0);
        if ((uint32_t)n > max_length) n = std::snprintf(conv, sizeof(conv), "%.1fx^12", (double)value / 1000000000000.0);
        if ((uint32_t)n > max_length) n = std::snprintf(conv, sizeof(conv), "9+++T");
        std::memcpy(buf + (offset - (uint32_t)n), conv, (size_t)n);
    }
    static int format(char* c, int64_t v) { return std::snprintf(c, 32, "%" PRId64, v); }
    static int format(char* c, float v) { return std::snprintf(c, 32, "%.3f", (double)v); }
};

int emit(const char* s, size_t n, char* out, uint32_t cap)
{
    if (out == nullptr || n + 1 > cap) return -1;
    std::memcpy(out, s, n);
    out[n] = 0;
    return (int)n;
}

template <typename Slice>
int64_t rate(int64_t units, const Slice& s)  // units * 1000 / timeElapsed
{
    const int64_t elapsed = s.end_time_ms - s.start_time_ms;
    return elapsed > 0 ? units * 1000 / elapsed : 0;
}

// the CSV form of both lines: the time slice as %.3f, then the values, comma separated, "\r\n" at the end
// (AppendCsvOutput / TerminateFileString)
int csv_line(float seconds, std::initializer_list<int64_t> values, char* out, uint32_t cap)
{
    char b[512];
    int n = std::snprintf(b, sizeof(b), "%.3f", (double)seconds);
    for (int64_t v : values) n += std::snprintf(b + n, sizeof(b) - (size_t)n, ",%" PRIu64, (uint64_t)v);  // _ui64tow_s
    n += std::snprintf(b + n, sizeof(b) - (size_t)n, "\r\n");
    return emit(b, (size_t)n, out, cap);
}

int legend(int format, std::initializer_list<const char*> lines, char* out, uint32_t cap)
{
    if (format == CTS_STATUS_CSV) return emit("", 0, out, cap);  // no legend for CSV (:66-70)
    const char* eol = format == CTS_STATUS_CONSOLE ? "\n" : "\r\n";
    std::string s;
    for (const char* l : lines) {
        s += l;
        s += eol;
    }
    return emit(s.data(), s.size(), out, cap);
}

int finish(const Line& l, uint32_t end, int format, char* out, uint32_t cap)  // TerminateString / TerminateFileString
{
    std::string s(l.buf, end);
    s += format == CTS_STATUS_CONSOLE ? "\n" : "\r\n";
    return emit(s.data(), s.size(), out, cap);
}

constexpr const char* kHistoric = "\n\n"
                                  "  Historic Connection Statistics (all connections over the complete lifetime)  \n"
                                  "-------------------------------------------------------------------------------\n"
                                  "  SuccessfulConnections [%" PRId64 "]   NetworkErrors [%" PRId64
                                  "]   ProtocolErrors [%" PRId64 "]\n";

}  // namespace

extern "C" {

int cts_status_tcp_header(int format, char* out, uint32_t cap)  // FormatHeader (:552-569)
{
    const char* s = format == CTS_STATUS_CSV ? "TimeSlice,SendBps,RecvBps,In-Flight,Completed,NetError,DataError\r\n"
                    : format == CTS_STATUS_CONSOLE
                        ? " TimeSlice      SendBps      RecvBps  In-Flight  Completed  NetError  DataError \n"
                        : " TimeSlice      SendBps      RecvBps  In-Flight  Completed  NetError  DataError \r\n";
    return emit(s, std::strlen(s), out, cap);
}

int cts_status_tcp_legend(int format, char* out, uint32_t cap)  // FormatLegend (:524-550)
{
    return legend(format,
                  {"Legend:", "* TimeSlice - (seconds) cumulative runtime",
                   "* Send & Recv Rates - bytes/sec that were transferred within the TimeSlice period",
                   "* In-Flight - count of established connections transmitting IO pattern data",
                   "* Completed - cumulative count of successfully completed IO patterns",
                   "* Network Errors - cumulative count of failed IO patterns due to Winsock errors",
                   "* Data Errors - cumulative count of failed IO patterns due to data errors", ""},
                  out, cap);
}

int cts_status_tcp_line(int format, const cts_tcp_status* st, char* out, uint32_t cap)  // FormatData (:467-521)
{
    if (st == nullptr) return -1;
    const float seconds = (float)st->current_time_ms / 1000.0f;
    if (format == CTS_STATUS_CSV)
        return csv_line(seconds, {rate(st->bytes_sent, *st), rate(st->bytes_recv, *st), st->active_connections,
                                  st->successful, st->connection_errors, st->protocol_errors},
                        out, cap);
    Line l;
    l.right_justify(kTimeSliceOffset, kTimeSliceLength, seconds);
    l.right_justify(kSendOffset, kSendLength, rate(st->bytes_sent, *st));
    l.right_justify(kRecvOffset, kRecvLength, rate(st->bytes_recv, *st));
    l.right_justify(kInFlightOffset, kInFlightLength, st->active_connections);
    l.right_justify(kCompletedOffset, kCompletedLength, st->successful);
    l.right_justify(kNetErrorOffset, kNetErrorLength, st->connection_errors);
    l.right_justify(kDataErrorOffset, kDataErrorLength, st->protocol_errors);
    return finish(l, kDataErrorOffset, format, out, cap);
}

int cts_status_summary(int64_t successful, int64_t network_errors, int64_t protocol_errors, int64_t bytes_recv,
                       int64_t bytes_sent, char* out, uint32_t cap)  // ctsTraffic.cpp:155-171
{
    char b[1024];
    int n = std::snprintf(b, sizeof(b), kHistoric, successful, network_errors, protocol_errors);
    n += std::snprintf(b + n, sizeof(b) - (size_t)n,
                       "\n"
                       "  Total Bytes Recv : %" PRId64 "\n"
                       "  Total Bytes Sent : %" PRId64 "\n",
                       bytes_recv, bytes_sent);
    return emit(b, (size_t)n, out, cap);
}

int cts_status_udp_header(int format, char* out, uint32_t cap)  // FormatHeader (:349-368)
{
    const char* s = format == CTS_STATUS_CSV ? "TimeSlice,Bits/Sec,Streams,Completed,Dropped,Repeated,Errors\r\n"
                    : format == CTS_STATUS_CONSOLE
                        ? " TimeSlice       Bits/Sec    Streams   Completed   Dropped   Repeated    Errors \n"
                        : " TimeSlice       Bits/Sec    Streams   Completed   Dropped   Repeated    Errors \r\n";
    return emit(s, std::strlen(s), out, cap);
}

int cts_status_udp_legend(int format, char* out, uint32_t cap)  // FormatLegend (:324-347)
{
    return legend(format,
                  {"Legend:", "* TimeSlice - (seconds) cumulative runtime",
                   "* Streams - count of current number of UDP streams",
                   "* Bits/Sec - bits streamed within the TimeSlice period",
                   "* Completed Frames - count of frames successfully processed within the TimeSlice",
                   "* Dropped Frames - count of frames that were never seen within the TimeSlice",
                   "* Repeated Frames - count of frames received multiple times within the TimeSlice",
                   "* Stream Errors - count of invalid frames or buffers within the TimeSlice", ""},
                  out, cap);
}

int cts_status_udp_line(int format, const cts_udp_status* st, char* out, uint32_t cap)  // FormatData (:370-423)
{
    if (st == nullptr) return -1;
    const float seconds = (float)st->current_time_ms / 1000.0f;
    if (format == CTS_STATUS_CSV)
        return csv_line(seconds, {rate(st->bits_received, *st), st->active_streams, st->successful_frames,
                                  st->dropped_frames, st->duplicate_frames, st->error_frames},
                        out, cap);
    Line l;
    l.right_justify(kUdpTimeSliceOffset, kUdpTimeSliceLength, seconds);
    l.right_justify(kBitsPerSecondOffset, kBitsPerSecondLength, rate(st->bits_received, *st));
    l.right_justify(kStreamsOffset, kStreamsLength, st->active_streams);
    l.right_justify(kCompletedFramesOffset, kCompletedFramesLength, st->successful_frames);
    l.right_justify(kDroppedFramesOffset, kDroppedFramesLength, st->dropped_frames);
    l.right_justify(kRepeatedFramesOffset, kRepeatedFramesLength, st->duplicate_frames);
    l.right_justify(kErrorFramesOffset, kErrorFramesLength, st->error_frames);
    return finish(l, kErrorFramesOffset, format, out, cap);
}

int cts_status_udp_summary(int64_t successful, int64_t network_errors, int64_t protocol_errors,
                           int64_t bits_received, int64_t successful_frames, int64_t dropped_frames,
                           int64_t duplicate_frames, int64_t error_frames, char* out, uint32_t cap)
{
    // ctsTraffic.cpp:155-162 + the UDP client branch :173-200
    const int64_t total = successful_frames + dropped_frames + duplicate_frames + error_frames;
    auto pct = [total](int64_t v) { return total > 0 ? (double)v / (double)total * 100.0 : 0.0; };
    char b[1536];
    int n = std::snprintf(b, sizeof(b), kHistoric, successful, network_errors, protocol_errors);
    n += std::snprintf(b + n, sizeof(b) - (size_t)n,
                       "\n"
                       "  Total Bytes Recv : %" PRId64 "\n"
                       "  Total Successful Frames : %" PRId64 " (%f)\n"
                       "  Total Dropped Frames : %" PRId64 " (%f)\n"
                       "  Total Duplicate Frames : %" PRId64 " (%f)\n"
                       "  Total Error Frames : %" PRId64 " (%f)\n",
                       bits_received / 8, successful_frames, pct(successful_frames), dropped_frames,
                       pct(dropped_frames), duplicate_frames, pct(duplicate_frames), error_frames, pct(error_frames));
    return emit(b, (size_t)n, out, cap);
}

}  // extern "C"
