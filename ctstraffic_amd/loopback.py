"""Loopback-TCP feeder (include/cts_loopback.h): the reference's config 1 end to end
("-Pattern:push -Connections:8 -Buffer:65536 -Transfer:1GiB -Verify:data" over
loopback) with the sender buffer written by the fill kernel and every received
buffer verified by the verify kernel."""
from __future__ import annotations

import ctypes

from . import _pattern_abi as A
from ._lib import check, lib


class LoopbackConfig(ctypes.Structure):
    _fields_ = [("connections", ctypes.c_uint32), ("io_pattern", ctypes.c_uint32), ("buffer_size", ctypes.c_uint32),
                ("verify_buffers", ctypes.c_uint32), ("transfer_size", ctypes.c_uint64),
                ("verify_mode", ctypes.c_uint32), ("batch_buffers", ctypes.c_uint32),
                ("corrupt_connection", ctypes.c_uint32), ("corrupt_send_index", ctypes.c_uint32),
                ("socket_buffer_bytes", ctypes.c_uint32), ("push_bytes", ctypes.c_uint32),
                ("pull_bytes", ctypes.c_uint32), ("functor", ctypes.c_uint32), ("recv_whole", ctypes.c_uint32),
                ("tcp_bytes_per_second", ctypes.c_int64), ("burst_count", ctypes.c_uint32),
                ("burst_delay", ctypes.c_uint32), ("buffer_size_high", ctypes.c_uint32),
                ("random_seed", ctypes.c_uint32), ("recv_ring_buffers", ctypes.c_uint32),
                ("recv_ring_pinned", ctypes.c_uint32)]


FUNCTOR_AUTO, FUNCTOR_SYNC, FUNCTOR_ASYNC = 0, 1, 2


class LoopbackResult(ctypes.Structure):
    _fields_ = [("seconds", ctypes.c_double), ("bytes_sent", ctypes.c_uint64), ("bytes_recv", ctypes.c_uint64),
                ("buffers_verified", ctypes.c_uint64), ("connections_ok", ctypes.c_uint32),
                ("connections_failed", ctypes.c_uint32), ("data_errors", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("recv_cpu_seconds", ctypes.c_double),
                ("send_cpu_seconds", ctypes.c_double), ("recv_io_cpu_seconds", ctypes.c_double)]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved"}
        d["GBps_recv"] = self.bytes_recv / self.seconds / 1e9 if self.seconds > 0 else 0.0
        # receive-thread CPU per GiB received: what verifying on the GPU saves (or costs) the host
        gib = self.bytes_recv / (1 << 30)
        d["recv_cpu_s_per_GiB"] = self.recv_cpu_seconds / gib if self.bytes_recv else 0.0
        # ... split into the socket calls and the rest (the pattern: CompleteIo, verify, batch bookkeeping)
        d["recv_io_cpu_s_per_GiB"] = self.recv_io_cpu_seconds / gib if self.bytes_recv else 0.0
        d["recv_pattern_cpu_s_per_GiB"] = d["recv_cpu_s_per_GiB"] - d["recv_io_cpu_s_per_GiB"]
        return d


class LoopbackSide(ctypes.Structure):
    _fields_ = [("stats", A.CtsPatternStats), ("status", ctypes.c_uint32), ("last_error", ctypes.c_uint32)]

    def as_dict(self) -> dict:
        d = self.stats.as_dict()
        d["status"] = int(self.status)
        d["final_error"] = int(self.last_error)
        return d


def declare(L: ctypes.CDLL) -> None:
    fn = L.cts_loopback_run
    fn.argtypes = [ctypes.POINTER(LoopbackConfig), ctypes.c_void_p, A.BATCH_VERIFIER, ctypes.c_void_p,
                   ctypes.POINTER(LoopbackResult)]
    fn.restype = ctypes.c_int
    fn = L.cts_loopback_run_multi
    fn.argtypes = [ctypes.POINTER(LoopbackConfig), ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                   A.BATCH_VERIFIER, ctypes.c_void_p, ctypes.POINTER(LoopbackResult)]
    fn.restype = ctypes.c_int
    fn = L.cts_loopback_run_detailed
    fn.argtypes = [ctypes.POINTER(LoopbackConfig), ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                   A.BATCH_VERIFIER, ctypes.c_void_p, ctypes.POINTER(LoopbackResult), ctypes.POINTER(LoopbackSide)]
    fn.restype = ctypes.c_int


def run(connections=8, buffer_size=65536, transfer_size=1 << 30, engine=None, verifier=None,
        io_pattern=A.PATTERN_PUSH, verify=True, verify_mode=A.VERIFY_DEFERRED, batch_buffers=0,
        corrupt_connection=None, corrupt_send_index=0, socket_buffer_bytes=0, push_bytes=0, pull_bytes=0,
        functor=FUNCTOR_AUTO, recv_whole=False, sides=False, tcp_bytes_per_second=0, burst_count=0,
        burst_delay=0, buffer_size_high=0, random_seed=0, recv_ring_buffers=0, recv_ring_pinned=False) -> dict:
    """One loopback run. ``engine`` is one Engine or a list of them (one per GPU: connection i verifies on
    engine[cts_shard_of(i, len)]). ``verifier`` (a cts_batch_verifier or a python fn(arena, descs) -> results)
    replaces the engines' kernel (test harnesses / the CPU baseline). ``recv_whole``: data recvs complete
    with the whole posted length (deterministic completions). ``sides``: add every side's pattern statistics,
    status and last error under "sides" (clients [0, connections), servers [connections, 2 connections)).
    ``tcp_bytes_per_second`` / ``burst_count`` / ``burst_delay``: send pacing of every side (the senders wait the
    tasks' time offsets). ``buffer_size_high``: -Buffer:[buffer_size, buffer_size_high], every IO's size drawn
    uniformly (side i seeded with ``random_seed`` + i). ``recv_ring_buffers`` (diagnostic, ``verify=False``, sync
    functor): data recvs land round robin in a ring of that many buffers (pinned with ``recv_ring_pinned``, on the
    first engine), as a DEFERRED pattern's do."""
    from .pattern import batch_verifier

    cfg = LoopbackConfig(connections, io_pattern, buffer_size, int(verify), transfer_size, verify_mode, batch_buffers,
                         0xFFFFFFFF if corrupt_connection is None else corrupt_connection, corrupt_send_index,
                         socket_buffer_bytes, push_bytes, pull_bytes, functor, int(recv_whole), tcp_bytes_per_second,
                         burst_count, burst_delay, buffer_size_high, random_seed, recv_ring_buffers,
                         int(recv_ring_pinned))
    hook = None
    if verifier is not None:
        hook = verifier if isinstance(verifier, A.BATCH_VERIFIER) else batch_verifier(verifier)
    res = LoopbackResult()
    engines = engine if isinstance(engine, (list, tuple)) else ([] if engine is None else [engine])
    arr = (ctypes.c_void_p * max(1, len(engines)))(*[e._h.value for e in engines])
    side_arr = (LoopbackSide * (2 * connections))() if sides else None
    check("cts_loopback_run_detailed",
          lib().cts_loopback_run_detailed(ctypes.byref(cfg), arr if engines else None, len(engines),
                                          hook if hook is not None else A.BATCH_VERIFIER(), None, ctypes.byref(res),
                                          side_arr))
    out = res.as_dict()
    if sides:
        out["sides"] = [s.as_dict() for s in side_arr]
    return out


# ---- MediaStream over loopback UDP (cts_loopback_media_stream_run) --------------------------------------------
class MediaStreamLoopbackConfig(ctypes.Structure):
    _fields_ = [("connections", ctypes.c_uint32), ("frame_size_bytes", ctypes.c_uint32),
                ("frames_per_second", ctypes.c_uint32), ("stream_length_frames", ctypes.c_uint32),
                ("buffered_frames", ctypes.c_uint32), ("datagram_max_size", ctypes.c_uint32),
                ("pre_post_recvs", ctypes.c_uint32), ("verify_buffers", ctypes.c_uint32),
                ("corrupt_connection", ctypes.c_uint32), ("corrupt_datagram", ctypes.c_uint32),
                ("socket_buffer_bytes", ctypes.c_uint32), ("verify_mode", ctypes.c_uint32),
                ("batch_buffers", ctypes.c_uint32)]


def _media_stream_result_type():
    from .media_stream import Stats

    class MediaStreamLoopbackResult(ctypes.Structure):
        _fields_ = [("seconds", ctypes.c_double), ("connections_ok", ctypes.c_uint32),
                    ("connections_failed", ctypes.c_uint32), ("data_errors", ctypes.c_uint32),
                    ("reserved", ctypes.c_uint32), ("datagrams_sent", ctypes.c_uint64),
                    ("datagrams_received", ctypes.c_uint64), ("clients", Stats),
                    ("recv_cpu_seconds", ctypes.c_double)]

    return MediaStreamLoopbackResult


def media_stream_run(connections=2, frame_size=52083, frames_per_second=60, stream_length_frames=60,
                     buffered_frames=10, datagram_max_size=1400, pre_post_recvs=2, engine=None, verifier=None,
                     verify=True, corrupt_connection=None, corrupt_datagram=0, socket_buffer_bytes=0,
                     verify_mode=A.VERIFY_SYNC, batch_buffers=0) -> dict:
    """MediaStream over loopback UDP ("-Protocol:UDP -Pattern:MediaStream", README sizing by default: FrameSize
    52083 B at 60 frames/s): every connection's server streams its frames at the frame rate and its client verifies
    every datagram's payload (on ``engine`` or through ``verifier``) and renders the frames."""
    from .pattern import batch_verifier

    R = _media_stream_result_type()
    L = lib()
    fn = L.cts_loopback_media_stream_run
    fn.argtypes = [ctypes.POINTER(MediaStreamLoopbackConfig), ctypes.c_void_p, A.BATCH_VERIFIER, ctypes.c_void_p,
                   ctypes.POINTER(R)]
    fn.restype = ctypes.c_int
    cfg = MediaStreamLoopbackConfig(connections, frame_size, frames_per_second, stream_length_frames,
                                    buffered_frames, datagram_max_size, pre_post_recvs, int(verify),
                                    0xFFFFFFFF if corrupt_connection is None else corrupt_connection,
                                    corrupt_datagram, socket_buffer_bytes, verify_mode, batch_buffers)
    hook = None
    if verifier is not None:
        hook = verifier if isinstance(verifier, A.BATCH_VERIFIER) else batch_verifier(verifier)
    res = R()
    check("cts_loopback_media_stream_run",
          fn(ctypes.byref(cfg), None if engine is None else engine._h.value,
             hook if hook is not None else A.BATCH_VERIFIER(), None, ctypes.byref(res)))
    d = {f: getattr(res, f) for f, _ in R._fields_ if f not in ("reserved", "clients")}
    d["clients"] = res.clients.as_dict()
    d["payload_MBps"] = (res.clients.bits_received / 8 / 1e6 / res.seconds) if res.seconds > 0 else 0.0
    return d
