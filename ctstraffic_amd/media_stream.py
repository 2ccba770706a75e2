"""MediaStream (UDP) framing around the verify path — Python handle over
include/cts_media_stream.h.

* :func:`split` — ctsMediaStreamSendRequests' datagram sizes for one frame
  (ctsMediaStreamProtocol.hpp:151-205);
* :func:`fill` / :func:`verify` — the gfx950 datagram kernels (sender
  materialisation; receiver header parse + validate + payload verify);
* :class:`MediaStreamClient` — ctsIoPatternMediaStreamClient's frame accounting
  (ctsIOPatternMediaStream.cpp), driven by explicit render ticks.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import CtsError, check, lib
from .types import DESC_DTYPE, DGRAM_HEADER_DTYPE, DGRAM_RECORD_DTYPE, DGRAM_STATUS_DTYPE, RESULT_DTYPE

DGRAM_DATA, DGRAM_ID, DGRAM_ZERO, DGRAM_SHORT, DGRAM_UNKNOWN, DGRAM_BAD_DESC = range(6)
FLAG_DATA, FLAG_ID = 0x0000, 0x1000
DATA_HEADER_LENGTH = 26
CONNECTION_ID_HEADER_LENGTH = 39


class Settings(ctypes.Structure):
    """ctsConfig::MediaStreamSettings (the fields the client reads)."""

    _fields_ = [("frame_size_bytes", ctypes.c_uint32), ("datagram_max_size", ctypes.c_uint32),
                ("frames_per_second", ctypes.c_uint32), ("buffered_frames", ctypes.c_uint32),
                ("stream_length_frames", ctypes.c_int64)]


class Stats(ctypes.Structure):
    _fields_ = [("bits_received", ctypes.c_int64), ("successful_frames", ctypes.c_int64),
                ("dropped_frames", ctypes.c_int64), ("duplicate_frames", ctypes.c_int64),
                ("error_frames", ctypes.c_int64), ("datagrams", ctypes.c_uint64), ("last_error", ctypes.c_uint32),
                ("finished", ctypes.c_uint32), ("head_sequence_number", ctypes.c_int64),
                ("fail_datagram", ctypes.c_uint32), ("has_failure", ctypes.c_uint32)]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class FrameWindow(ctypes.Structure):
    """cts_frame_window: the client's jitter window a batch is summed for."""

    _fields_ = [("head_sequence_number", ctypes.c_int64), ("final_frame", ctypes.c_int64),
                ("frames", ctypes.c_uint32), ("finished", ctypes.c_uint32)]


class FrameTotals(ctypes.Structure):
    """cts_frame_totals: a batch's sums, folded from the device block."""

    _fields_ = [("bits_received", ctypes.c_uint64), ("error_frames", ctypes.c_uint64), ("datagrams", ctypes.c_uint64),
                ("first_exception", ctypes.c_uint32), ("exceptions", ctypes.c_uint32)]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


FRAMES_REPLAY = 16  # CTS_MS_FRAMES_REPLAY
NO_EXCEPTION = 0xFFFFFFFF


class UdpStatusDetails(ctypes.Structure):
    """cts_udp_status_details: the process-wide UdpStatusDetails (ctsConfig.h:417)."""

    _fields_ = [(f, ctypes.c_int64) for f in ("bits_received", "successful_frames", "dropped_frames",
                                               "duplicate_frames", "error_frames")]


def declare(L: ctypes.CDLL) -> None:
    P = ctypes.c_void_p
    u32, u64, i32, i64 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64
    sigs = {
        "cts_media_stream_split": ([u64, u32, P, u64], u64),
        "cts_media_stream_fill": ([P, P, u64, P, P, u32, P], i32),
        "cts_media_stream_fill_strided": ([P, P, u64, u32, P, P, u32, P], i32),
        "cts_media_stream_verify": ([P, P, u64, P, u32, P, P, P, P], i32),
        "cts_media_stream_verify_strided": ([P, P, u64, u32, P, u32, P, P, P, P], i32),
        "cts_media_stream_verify_status": ([P, P, u64, P, u32, P, P, P], i32),
        "cts_media_stream_verify_strided_status": ([P, P, u64, u32, P, u32, P, P, P], i32),
        "cts_media_stream_client_complete_status": ([P, P, u32, i64, i64, ctypes.POINTER(u32)], i32),
        "cts_media_stream_client_create": ([ctypes.POINTER(Settings), ctypes.POINTER(P)], i32),
        "cts_media_stream_client_destroy": ([P], i32),
        "cts_media_stream_client_complete": ([P, P, P, u32, i64, i64, ctypes.POINTER(u32)], i32),
        "cts_media_stream_client_set_connection_id": ([P, ctypes.c_char_p, u32], i32),
        "cts_media_stream_client_render": ([P], i32),
        "cts_media_stream_client_stats": ([P, ctypes.POINTER(Stats)], i32),
        "cts_media_stream_client_connection_id": ([P], ctypes.c_char_p),
        "cts_frame_totals_device_bytes": ([], ctypes.c_size_t),
        "cts_frame_totals_fold": ([P, ctypes.POINTER(FrameTotals)], i32),
        "cts_media_stream_verify_frames": ([P, P, u64, P, u32, ctypes.POINTER(FrameWindow), P, P, P, P], i32),
        "cts_media_stream_verify_strided_frames": ([P, P, u64, u32, P, u32, ctypes.POINTER(FrameWindow), P, P, P, P],
                                                   i32),
        "cts_media_stream_client_window": ([P, ctypes.POINTER(FrameWindow)], i32),
        "cts_media_stream_client_complete_frames": ([P, ctypes.POINTER(FrameWindow), ctypes.POINTER(FrameTotals), P,
                                                     u32, i64, i64], i32),
        "cts_udp_status_details_read": ([ctypes.POINTER(UdpStatusDetails)], i32),
        "cts_udp_status_details_reset": ([], None),
    }
    for name, (argtypes, restype) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = restype


def udp_status_details() -> dict:
    """The process-wide UDP counters every MediaStreamClient feeds (cts_udp_status_details_read)."""
    s = UdpStatusDetails()
    check("cts_udp_status_details_read", lib().cts_udp_status_details_read(ctypes.byref(s)))
    return {f: int(getattr(s, f)) for f, _ in s._fields_}


def udp_status_details_reset() -> None:
    lib().cts_udp_status_details_reset()


def split(frame_bytes: int, max_datagram: int) -> np.ndarray:
    """Total lengths (26-byte header included) of the datagrams one frame is sent as."""
    n = int(lib().cts_media_stream_split(frame_bytes, max_datagram, None, 0))
    out = np.zeros(n, dtype=np.uint32)
    if n:
        lib().cts_media_stream_split(frame_bytes, max_datagram, out.ctypes.data, n)
    return out


def _ptr(x):
    from .engine import _ptr as p

    return p(x)


def fill(engine, arena, descs, headers, stream=None) -> None:
    """cts_media_stream_fill: descs (uint8 device tensor of DESC_DTYPE), headers (uint8 device tensor of
    DGRAM_HEADER_DTYPE)."""
    from .engine import _nbytes, _stream

    n = _nbytes(descs) // DESC_DTYPE.itemsize
    if _nbytes(headers) < n * DGRAM_HEADER_DTYPE.itemsize:
        raise ValueError("headers holds %d bytes, %d datagrams need %d" % (_nbytes(headers), n,
                                                                          n * DGRAM_HEADER_DTYPE.itemsize))
    check("cts_media_stream_fill", engine._L.cts_media_stream_fill(engine._h, _ptr(arena), _nbytes(arena), _ptr(descs),
                                                               _ptr(headers), n, _stream(stream)))


def fill_strided(engine, arena, stride: int, lengths, headers, stream=None) -> None:
    """cts_media_stream_fill_strided: datagram i at arena + i * stride, lengths (uint32 device tensor) its bytes,
    headers (uint8 device tensor of DGRAM_HEADER_DTYPE) its header values."""
    from .engine import _nbytes, _stream

    n = _nbytes(lengths) // 4
    if _nbytes(headers) < n * DGRAM_HEADER_DTYPE.itemsize:
        raise ValueError("headers holds %d bytes, %d datagrams need %d" % (_nbytes(headers), n,
                                                                          n * DGRAM_HEADER_DTYPE.itemsize))
    check("cts_media_stream_fill_strided",
          engine._L.cts_media_stream_fill_strided(engine._h, _ptr(arena), _nbytes(arena), stride, _ptr(lengths),
                                                  _ptr(headers), n, _stream(stream)))


def verify(engine, arena, descs, records=None, results=None, counters=None, stream=None) -> None:
    from .engine import _check_outputs, _nbytes, _stream

    n = _nbytes(descs) // DESC_DTYPE.itemsize
    _check_outputs(n, results, counters)
    if records is not None and _nbytes(records) < n * DGRAM_RECORD_DTYPE.itemsize:
        raise ValueError("records holds %d bytes, %d datagrams need %d" % (_nbytes(records), n,
                                                                          n * DGRAM_RECORD_DTYPE.itemsize))
    check("cts_media_stream_verify",
          engine._L.cts_media_stream_verify(engine._h, _ptr(arena), _nbytes(arena), _ptr(descs), n, _ptr(records),
                                        _ptr(results), _ptr(counters), _stream(stream)))


def verify_strided(engine, arena, stride: int, lengths, records=None, results=None, counters=None,
                   stream=None) -> None:
    """cts_media_stream_verify_strided: datagram i at arena + i * stride, lengths (uint32 device tensor) its
    completed bytes."""
    from .engine import _check_outputs, _nbytes, _stream

    n = _nbytes(lengths) // 4
    _check_outputs(n, results, counters)
    if records is not None and _nbytes(records) < n * DGRAM_RECORD_DTYPE.itemsize:
        raise ValueError("records holds %d bytes, %d datagrams need %d" % (_nbytes(records), n,
                                                                          n * DGRAM_RECORD_DTYPE.itemsize))
    check("cts_media_stream_verify_strided",
          engine._L.cts_media_stream_verify_strided(engine._h, _ptr(arena), _nbytes(arena), stride, _ptr(lengths), n,
                                                _ptr(records), _ptr(results), _ptr(counters), _stream(stream)))


def _check_status(n, status):
    from .engine import _nbytes

    if status is not None and _nbytes(status) < n * DGRAM_STATUS_DTYPE.itemsize:
        raise ValueError("status holds %d bytes, %d datagrams need %d" % (_nbytes(status), n,
                                                                         n * DGRAM_STATUS_DTYPE.itemsize))


def verify_status(engine, arena, descs, status=None, counters=None, stream=None) -> None:
    """cts_media_stream_verify_status: the receive pass writing one 16-byte cts_datagram_status per datagram."""
    from .engine import _check_outputs, _nbytes, _stream

    n = _nbytes(descs) // DESC_DTYPE.itemsize
    _check_outputs(n, None, counters)
    _check_status(n, status)
    check("cts_media_stream_verify_status",
          engine._L.cts_media_stream_verify_status(engine._h, _ptr(arena), _nbytes(arena), _ptr(descs), n, _ptr(status),
                                                   _ptr(counters), _stream(stream)))


def verify_strided_status(engine, arena, stride: int, lengths, status=None, counters=None, stream=None) -> None:
    """cts_media_stream_verify_strided_status: the strided receive ring, 16-byte statuses."""
    from .engine import _check_outputs, _nbytes, _stream

    n = _nbytes(lengths) // 4
    _check_outputs(n, None, counters)
    _check_status(n, status)
    check("cts_media_stream_verify_strided_status",
          engine._L.cts_media_stream_verify_strided_status(engine._h, _ptr(arena), _nbytes(arena), stride,
                                                           _ptr(lengths), n, _ptr(status), _ptr(counters),
                                                           _stream(stream)))


class FrameSums:
    """Device outputs of one cts_media_stream_verify_frames launch: the totals block and bytes per window slot."""

    def __init__(self, window_frames: int, device="cuda"):
        import torch

        self.totals = torch.zeros(int(lib().cts_frame_totals_device_bytes()), dtype=torch.uint8, device=device)
        self.frame_bytes = torch.zeros(max(1, window_frames), dtype=torch.int64, device=device)

    def read(self):
        """(FrameTotals folded on the host, frame_bytes as uint64 numpy)."""
        t = FrameTotals()
        host = np.ascontiguousarray(self.totals.cpu().numpy())
        check("cts_frame_totals_fold", lib().cts_frame_totals_fold(host.ctypes.data, ctypes.byref(t)))
        return t, self.frame_bytes.cpu().numpy().view(np.uint64)


def verify_frames(engine, arena, descs, window: FrameWindow, sums: FrameSums, counters=None, stream=None) -> None:
    """cts_media_stream_verify_frames: the receive pass summing the client's frame accounting for `window`."""
    from .engine import _check_outputs, _nbytes, _stream

    n = _nbytes(descs) // DESC_DTYPE.itemsize
    _check_outputs(n, None, counters)
    if sums.frame_bytes.numel() < window.frames:
        raise ValueError("frame_bytes holds %d slots, the window %d" % (sums.frame_bytes.numel(), window.frames))
    check("cts_media_stream_verify_frames",
          engine._L.cts_media_stream_verify_frames(engine._h, _ptr(arena), _nbytes(arena), _ptr(descs), n,
                                                   ctypes.byref(window), _ptr(sums.totals), _ptr(sums.frame_bytes),
                                                   _ptr(counters), _stream(stream)))


def verify_strided_frames(engine, arena, stride: int, lengths, window: FrameWindow, sums: FrameSums, counters=None,
                          stream=None) -> None:
    """cts_media_stream_verify_strided_frames: the same over a strided receive ring."""
    from .engine import _check_outputs, _nbytes, _stream

    n = _nbytes(lengths) // 4
    _check_outputs(n, None, counters)
    if sums.frame_bytes.numel() < window.frames:
        raise ValueError("frame_bytes holds %d slots, the window %d" % (sums.frame_bytes.numel(), window.frames))
    check("cts_media_stream_verify_strided_frames",
          engine._L.cts_media_stream_verify_strided_frames(engine._h, _ptr(arena), _nbytes(arena), stride,
                                                           _ptr(lengths), n, ctypes.byref(window), _ptr(sums.totals),
                                                           _ptr(sums.frame_bytes), _ptr(counters), _stream(stream)))


class MediaStreamClient:
    """ctsIoPatternMediaStreamClient's frame accounting (ctsIOPatternMediaStream.cpp:46-530)."""

    def __init__(self, frame_size_bytes: int, buffered_frames: int, stream_length_frames: int,
                 datagram_max_size: int = 1400, frames_per_second: int = 60):
        self._s = Settings(frame_size_bytes, datagram_max_size, frames_per_second, buffered_frames,
                           stream_length_frames)
        h = ctypes.c_void_p()
        check("cts_media_stream_client_create", lib().cts_media_stream_client_create(ctypes.byref(self._s),
                                                                                       ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().cts_media_stream_client_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def complete(self, records: np.ndarray, results: np.ndarray, receiver_qpc: int = 0, receiver_qpf: int = 0):
        """Returns (cts_io_status, consumed)."""
        records = np.ascontiguousarray(records, dtype=DGRAM_RECORD_DTYPE)
        results = np.ascontiguousarray(results, dtype=RESULT_DTYPE)
        if len(records) != len(results):
            raise ValueError("%d records but %d results" % (len(records), len(results)))
        consumed = ctypes.c_uint32()
        rc = lib().cts_media_stream_client_complete(self._h, records.ctypes.data, results.ctypes.data, len(records),
                                                    receiver_qpc, receiver_qpf, ctypes.byref(consumed))
        if rc < 0:
            raise CtsError("cts_media_stream_client_complete", rc)
        return rc, consumed.value

    def complete_status(self, status: np.ndarray, receiver_qpc: int = 0, receiver_qpf: int = 0):
        """CompleteIo over compact statuses (cts_media_stream_client_complete_status). Returns (cts_io_status,
        consumed)."""
        status = np.ascontiguousarray(status, dtype=DGRAM_STATUS_DTYPE)
        consumed = ctypes.c_uint32()
        rc = lib().cts_media_stream_client_complete_status(self._h, status.ctypes.data, len(status), receiver_qpc,
                                                           receiver_qpf, ctypes.byref(consumed))
        if rc < 0:
            raise CtsError("cts_media_stream_client_complete_status", rc)
        return rc, consumed.value

    def window(self) -> FrameWindow:
        w = FrameWindow()
        check("cts_media_stream_client_window", lib().cts_media_stream_client_window(self._h, ctypes.byref(w)))
        return w

    def complete_frames(self, window: FrameWindow, totals: FrameTotals, frame_bytes: np.ndarray, n: int,
                        receiver_qpc: int = 0, receiver_qpf: int = 0) -> int:
        """CompleteIo of a batch of n datagrams from its GPU sums. Returns a cts_io_status, or FRAMES_REPLAY when
        the batch holds an exception (nothing applied)."""
        fb = np.ascontiguousarray(frame_bytes, dtype=np.uint64)
        rc = lib().cts_media_stream_client_complete_frames(self._h, ctypes.byref(window), ctypes.byref(totals),
                                                           fb.ctypes.data, n, receiver_qpc, receiver_qpf)
        if rc < 0:
            raise CtsError("cts_media_stream_client_complete_frames", rc)
        return rc

    def complete_batch_on_gpu(self, engine, arena, descs, sums: "FrameSums" = None, status=None, receiver_qpc: int = 0,
                              receiver_qpf: int = 0):
        """One batch through the GPU sums, replayed datagram by datagram from compact statuses when it holds an
        exception. Returns (cts_io_status, replayed)."""
        import torch

        from .engine import _nbytes

        n = _nbytes(descs) // DESC_DTYPE.itemsize
        w = self.window()
        sums = sums or FrameSums(w.frames, device=arena.device)
        verify_frames(engine, arena, descs, w, sums)
        torch.cuda.synchronize(arena.device)
        t, fb = sums.read()
        rc = self.complete_frames(w, t, fb, n, receiver_qpc, receiver_qpf)
        if rc != FRAMES_REPLAY:
            return rc, False
        st = status if status is not None else torch.empty(n * DGRAM_STATUS_DTYPE.itemsize, dtype=torch.uint8,
                                                           device=arena.device)
        verify_status(engine, arena, descs, status=st)
        torch.cuda.synchronize(arena.device)
        rc, _ = self.complete_status(st[: n * DGRAM_STATUS_DTYPE.itemsize].cpu().numpy().view(DGRAM_STATUS_DTYPE),
                                     receiver_qpc, receiver_qpf)
        return rc, True

    def set_connection_id(self, datagram: bytes) -> None:
        check("cts_media_stream_client_set_connection_id",
              lib().cts_media_stream_client_set_connection_id(self._h, datagram, len(datagram)))

    def render(self) -> int:
        rc = lib().cts_media_stream_client_render(self._h)
        if rc < 0:
            raise CtsError("cts_media_stream_client_render", rc)
        return rc

    def stats(self) -> dict:
        s = Stats()
        check("cts_media_stream_client_stats", lib().cts_media_stream_client_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    def connection_id(self) -> str:
        return lib().cts_media_stream_client_connection_id(self._h).decode()
