// cts_status.cpp — TCP status output (include/cts_status.h), restating
// ctsTcpStatusInformation (ctsTraffic/ctsPrintStatus.hpp:452-600) and the
// helpers of its base class (RightJustifyOutput :166-229, AppendCsvOutput
// :245-320): a 1024-column space-filled line, each value right-justified to
// end at its column offset, falling back to x^6 / x^9 / x^12 notation and then
// "9+++T" when it does not fit its width.
#include <cinttypes>
#include <cstdio>
#include <cstring>
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

int64_t rate(int64_t bytes, const cts_tcp_status& s)  // bytes * 1000 / timeElapsed
{
    const int64_t elapsed = s.end_time_ms - s.start_time_ms;
    return elapsed > 0 ? bytes * 1000 / elapsed : 0;
}

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

int cts_status_tcp_legend(int format, char* out, uint32_t cap)  // FormatLegend (:524-550); none for CSV (:66-70)
{
    if (format == CTS_STATUS_CSV) return emit("", 0, out, cap);
    const char* eol = format == CTS_STATUS_CONSOLE ? "\n" : "\r\n";
    std::string s;
    for (const char* l : {"Legend:", "* TimeSlice - (seconds) cumulative runtime",
                          "* Send & Recv Rates - bytes/sec that were transferred within the TimeSlice period",
                          "* In-Flight - count of established connections transmitting IO pattern data",
                          "* Completed - cumulative count of successfully completed IO patterns",
                          "* Network Errors - cumulative count of failed IO patterns due to Winsock errors",
                          "* Data Errors - cumulative count of failed IO patterns due to data errors", ""}) {
        s += l;
        s += eol;
    }
    return emit(s.data(), s.size(), out, cap);
}

int cts_status_tcp_line(int format, const cts_tcp_status* st, char* out, uint32_t cap)  // FormatData (:467-521)
{
    if (st == nullptr) return -1;
    const float seconds = (float)st->current_time_ms / 1000.0f;
    if (format == CTS_STATUS_CSV) {
        char b[512];
        int n = std::snprintf(b, sizeof(b), "%.3f,", (double)seconds);
        for (int64_t v : {rate(st->bytes_sent, *st), rate(st->bytes_recv, *st), st->active_connections,
                          st->successful, st->connection_errors})
            n += std::snprintf(b + n, sizeof(b) - (size_t)n, "%" PRIu64 ",", (uint64_t)v);  // _ui64tow_s
        n += std::snprintf(b + n, sizeof(b) - (size_t)n, "%" PRIu64 "\r\n", (uint64_t)st->protocol_errors);
        return emit(b, (size_t)n, out, cap);
    }
    Line l;
    l.right_justify(kTimeSliceOffset, kTimeSliceLength, seconds);
    l.right_justify(kSendOffset, kSendLength, rate(st->bytes_sent, *st));
    l.right_justify(kRecvOffset, kRecvLength, rate(st->bytes_recv, *st));
    l.right_justify(kInFlightOffset, kInFlightLength, st->active_connections);
    l.right_justify(kCompletedOffset, kCompletedLength, st->successful);
    l.right_justify(kNetErrorOffset, kNetErrorLength, st->connection_errors);
    l.right_justify(kDataErrorOffset, kDataErrorLength, st->protocol_errors);
    const char* eol = format == CTS_STATUS_CONSOLE ? "\n" : "\r\n";  // TerminateString / TerminateFileString
    std::string s(l.buf, kDataErrorOffset);
    s += eol;
    return emit(s.data(), s.size(), out, cap);
}

int cts_status_summary(int64_t successful, int64_t network_errors, int64_t protocol_errors, int64_t bytes_recv,
                       int64_t bytes_sent, char* out, uint32_t cap)
{
    char b[1024];
    const int n = std::snprintf(b, sizeof(b),
                                "\n\n"
                                "  Historic Connection Statistics (all connections over the complete lifetime)  \n"
                                "-------------------------------------------------------------------------------\n"
                                "  SuccessfulConnections [%" PRId64 "]   NetworkErrors [%" PRId64
                                "]   ProtocolErrors [%" PRId64 "]\n"
                                "\n"
                                "  Total Bytes Recv : %" PRId64 "\n"
                                "  Total Bytes Sent : %" PRId64 "\n",
                                successful, network_errors, protocol_errors, bytes_recv, bytes_sent);
    return emit(b, (size_t)n, out, cap);
}

}  // extern "C"
