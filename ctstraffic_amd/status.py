"""Status output of the data-integrity counters (include/cts_status.h): the
ctsTcpStatusInformation header / legend / line (ctsPrintStatus.hpp:452-600), the
ctsUdpStatusInformation ones (:314-446) and the exit summary (ctsTraffic.cpp:155-200)."""
from __future__ import annotations

import ctypes

from ._lib import lib

CONSOLE, CSV, CLEAR_TEXT = 1, 2, 3


class TcpStatus(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int64) for f in ("current_time_ms", "start_time_ms", "end_time_ms", "bytes_sent",
                                               "bytes_recv", "active_connections", "successful", "connection_errors",
                                               "protocol_errors")]


class UdpStatus(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int64) for f in ("current_time_ms", "start_time_ms", "end_time_ms", "bits_received",
                                               "active_streams", "successful_frames", "dropped_frames",
                                               "duplicate_frames", "error_frames")]


def declare(L: ctypes.CDLL) -> None:
    P, u32, i32, i64 = ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_int64
    for name, args in (("cts_status_tcp_header", [i32, P, u32]), ("cts_status_tcp_legend", [i32, P, u32]),
                       ("cts_status_tcp_line", [i32, ctypes.POINTER(TcpStatus), P, u32]),
                       ("cts_status_summary", [i64, i64, i64, i64, i64, P, u32]),
                       ("cts_status_udp_header", [i32, P, u32]), ("cts_status_udp_legend", [i32, P, u32]),
                       ("cts_status_udp_line", [i32, ctypes.POINTER(UdpStatus), P, u32]),
                       ("cts_status_udp_summary", [i64] * 8 + [P, u32])):
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = i32


def _call(fn, *args) -> str:
    buf = ctypes.create_string_buffer(4096)
    n = fn(*args, buf, 4096)
    if n < 0:
        raise ValueError("status output did not fit")
    return buf.value.decode()


def header(fmt: int = CONSOLE) -> str:
    return _call(lib().cts_status_tcp_header, fmt)


def legend(fmt: int = CONSOLE) -> str:
    return _call(lib().cts_status_tcp_legend, fmt)


def line(fmt: int = CONSOLE, **values) -> str:
    s = TcpStatus(**values)
    return _call(lib().cts_status_tcp_line, fmt, ctypes.byref(s))


def summary(successful: int, network_errors: int, protocol_errors: int, bytes_recv: int, bytes_sent: int) -> str:
    return _call(lib().cts_status_summary, successful, network_errors, protocol_errors, bytes_recv, bytes_sent)


def udp_header(fmt: int = CONSOLE) -> str:
    return _call(lib().cts_status_udp_header, fmt)


def udp_legend(fmt: int = CONSOLE) -> str:
    return _call(lib().cts_status_udp_legend, fmt)


def udp_line(fmt: int = CONSOLE, **values) -> str:
    s = UdpStatus(**values)
    return _call(lib().cts_status_udp_line, fmt, ctypes.byref(s))


def udp_summary(successful: int, network_errors: int, protocol_errors: int, bits_received: int,
                successful_frames: int, dropped_frames: int, duplicate_frames: int, error_frames: int) -> str:
    return _call(lib().cts_status_udp_summary, successful, network_errors, protocol_errors, bits_received,
                 successful_frames, dropped_frames, duplicate_frames, error_frames)
