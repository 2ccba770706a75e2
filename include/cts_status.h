/*
 * cts_status.h — status output of the data-integrity counters:
 * the TCP status line, header and legend of ctsTcpStatusInformation
 * (ctsTraffic/ctsPrintStatus.hpp:452-600), the UDP (MediaStream) ones of
 * ctsUdpStatusInformation (:314-446), console and CSV formats, and the historic
 * summary ctsTraffic prints at exit (ctsTraffic.cpp:155-200, TCP and UDP-client
 * branches), fed by the counters the GPU engine, the pattern mirror and the
 * MediaStream client maintain (cts_status_details, cts_udp_status_details,
 * cts_counters, per-connection outcomes). Output is ASCII (the reference writes
 * wchar_t).
 */
#ifndef CTS_STATUS_H
#define CTS_STATUS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum cts_status_format { /* ctsConfig::StatusFormatting */
    CTS_STATUS_CONSOLE = 1,
    CTS_STATUS_CSV = 2,
    CTS_STATUS_CLEAR_TEXT = 3    /* console layout with \r\n line ends (status file) */
} cts_status_format;

/* One status time slice: the ctsTcpStatistics + ctsConnectionStatistics values
 * FormatData reads (ctsStatistics.hpp:201-247, 316-373). */
typedef struct cts_tcp_status {
    int64_t current_time_ms;     /* TimeSlice (cumulative runtime) */
    int64_t start_time_ms;       /* m_startTime of the slice */
    int64_t end_time_ms;         /* m_endTime of the slice */
    int64_t bytes_sent;          /* m_bytesSent within the slice */
    int64_t bytes_recv;          /* m_bytesRecv within the slice */
    int64_t active_connections;  /* In-Flight */
    int64_t successful;          /* Completed */
    int64_t connection_errors;   /* NetError */
    int64_t protocol_errors;     /* DataError */
} cts_tcp_status;

/* One UDP status time slice: the ctsUdpStatistics + ctsConnectionStatistics values
 * ctsUdpStatusInformation::FormatData reads (ctsStatistics.hpp:249-314). */
typedef struct cts_udp_status {
    int64_t current_time_ms;     /* TimeSlice (cumulative runtime) */
    int64_t start_time_ms;       /* m_startTime of the slice */
    int64_t end_time_ms;         /* m_endTime of the slice */
    int64_t bits_received;       /* m_bitsReceived within the slice (Bits/Sec = bits * 1000 / elapsed ms) */
    int64_t active_streams;      /* Streams (m_activeConnectionCount) */
    int64_t successful_frames;   /* Completed */
    int64_t dropped_frames;      /* Dropped */
    int64_t duplicate_frames;    /* Repeated */
    int64_t error_frames;        /* Errors */
} cts_udp_status;

/* Each returns the number of characters written (excluding the NUL), or -1
 * if `cap` is too small. */
int cts_status_tcp_header(int format, char* out, uint32_t cap);
int cts_status_tcp_legend(int format, char* out, uint32_t cap);
int cts_status_tcp_line(int format, const cts_tcp_status* s, char* out, uint32_t cap);
/* The exit summary (ctsTraffic.cpp:155-171, TCP branch). */
int cts_status_summary(int64_t successful, int64_t network_errors, int64_t protocol_errors, int64_t bytes_recv,
                       int64_t bytes_sent, char* out, uint32_t cap);
int cts_status_udp_header(int format, char* out, uint32_t cap);
int cts_status_udp_legend(int format, char* out, uint32_t cap);
int cts_status_udp_line(int format, const cts_udp_status* s, char* out, uint32_t cap);
/* The exit summary of a UDP client (ctsTraffic.cpp:155-162, 173-200): Total Bytes Recv = bits / 8 and each
 * frame count with its percentage of all frames. */
int cts_status_udp_summary(int64_t successful, int64_t network_errors, int64_t protocol_errors,
                           int64_t bits_received, int64_t successful_frames, int64_t dropped_frames,
                           int64_t duplicate_frames, int64_t error_frames, char* out, uint32_t cap);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* CTS_STATUS_H */
