"""Python handle over the ctsIoPattern mirror (include/cts_pattern.h).

Keeps the reference's names (ctsTraffic/ctsIOPattern.h:80-144):
``IoPattern.MakeIoPattern(config, engine)``, ``InitiateIo()``,
``CompleteIo(task, currentTransfer, statusCode)``, ``GetLastPatternError()``,
``AccessSharedBuffer()``, so tests replaying the reference's MSTest scenarios
read like the originals.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np

from . import _pattern_abi as A
from . import _lib
from ._lib import CtsError, check, lib
from .types import DESC_DTYPE, RESULT_DTYPE

ctsTask = A.CtsTask


@dataclass
class PatternConfig:
    """The ctsConfig settings the pattern reads (ctsConfig.h:370-462), explicit."""

    io_pattern: int = A.PATTERN_PUSH
    listening: bool = False
    verify_buffers: bool = True
    use_shared_buffer: bool = False
    pre_post_recvs: int = 1
    pre_post_sends: int = 1
    buffer_size: int = 65536
    buffer_size_high: int = 0
    push_bytes: int = 0
    pull_bytes: int = 0
    tcp_shutdown: int = A.SHUTDOWN_GRACEFUL
    transfer_size: int = 1 << 30
    random_seed: int = 0
    verify_mode: int = A.VERIFY_SYNC
    batch_buffers: int = 0
    batch_bytes: int = 0
    registered_io: bool = False  # -io:rioiocp (WSA_FLAG_REGISTERED_IO): see rio_functions_set
    tcp_bytes_per_second: int = 0  # send pacing (ctsIOPattern.cpp:593-655); 0 = no limit
    tcp_bytes_per_second_period: int = 100  # ms per quantum
    burst_count: int = 0  # -burstcount (0 = not set); only without a rate limit (:657-674)
    burst_delay: int = 0  # -burstdelay, ms
    # MediaStream (io_pattern PATTERN_MEDIA_STREAM, UDP): buffer_size is the frame size and transfer_size must be
    # buffer_size * ms_stream_length_frames (MediaStreamSettings::CalculateTransferSize, ctsConfig.h:297-364)
    ms_frames_per_second: int = 0
    ms_datagram_max_size: int = 1400  # c_udpDatagramMaximumSizeBytes (ctsConfig.cpp:106)
    ms_buffered_frames: int = 0
    ms_stream_length_frames: int = 0
    ms_manual_timers: bool = False  # the caller fires the client's timers (IoPattern.media_stream_fire)

    @classmethod
    def media_stream(cls, *, listening: bool, frame_size: int, frames_per_second: int, stream_length_frames: int,
                     buffered_frames: int = 0, datagram_max_size: int = 1400, pre_post_recvs: int = 1, **kw):
        """A MediaStream server (listening) or client config as ctsConfig derives it for -Protocol:UDP."""
        return cls(io_pattern=A.PATTERN_MEDIA_STREAM, listening=listening, buffer_size=frame_size,
                   transfer_size=frame_size * stream_length_frames, ms_frames_per_second=frames_per_second,
                   ms_stream_length_frames=stream_length_frames, ms_buffered_frames=buffered_frames,
                   ms_datagram_max_size=datagram_max_size, pre_post_recvs=pre_post_recvs, **kw)

    @property
    def protocol(self) -> int:
        return A.PROTOCOL_UDP if self.io_pattern == A.PATTERN_MEDIA_STREAM else A.PROTOCOL_TCP

    def to_c(self) -> A.CtsPatternConfig:
        c = A.CtsPatternConfig()
        c.io_pattern = self.io_pattern
        c.protocol = self.protocol
        c.listening = int(bool(self.listening))
        c.verify_buffers = int(bool(self.verify_buffers))
        c.use_shared_buffer = int(bool(self.use_shared_buffer))
        c.pre_post_recvs = self.pre_post_recvs
        c.pre_post_sends = self.pre_post_sends
        c.buffer_size_low = self.buffer_size
        c.buffer_size_high = self.buffer_size_high
        c.push_bytes = self.push_bytes
        c.pull_bytes = self.pull_bytes
        c.tcp_shutdown = self.tcp_shutdown
        c.transfer_size = self.transfer_size
        c.random_seed = self.random_seed
        c.verify_mode = self.verify_mode
        c.batch_buffers = self.batch_buffers
        c.batch_bytes = self.batch_bytes
        c.registered_io = int(bool(self.registered_io))
        c.tcp_bytes_per_second = self.tcp_bytes_per_second
        c.tcp_bytes_per_second_period = self.tcp_bytes_per_second_period
        c.burst_count = self.burst_count
        c.burst_delay = self.burst_delay
        c.ms_frames_per_second = self.ms_frames_per_second
        c.ms_datagram_max_size = self.ms_datagram_max_size
        c.ms_buffered_frames = self.ms_buffered_frames
        c.ms_manual_timers = int(bool(self.ms_manual_timers))
        c.ms_stream_length_frames = self.ms_stream_length_frames
        return c

    @property
    def max_buffer_size(self) -> int:
        return self.buffer_size_high or self.buffer_size


def batch_verifier(fn: Callable[[np.ndarray, np.ndarray], np.ndarray]):
    """Wrap ``fn(arena_u8, descs) -> results(RESULT_DTYPE)`` as a cts_batch_verifier hook."""

    def _cb(ctx, arena, arena_bytes, descs, n, results):
        try:
            a = np.ctypeslib.as_array((ctypes.c_uint8 * max(int(arena_bytes), 1)).from_address(arena))[:arena_bytes]
            d = np.frombuffer((ctypes.c_uint8 * (24 * n)).from_address(descs), dtype=DESC_DTYPE, count=n).copy()
            r = fn(np.ascontiguousarray(a), d)
            ctypes.memmove(ctypes.cast(results, ctypes.c_void_p).value, r.astype(RESULT_DTYPE).tobytes(), 12 * n)
            return 0
        except Exception:  # pragma: no cover - reported as a failed verify call
            return -1

    return A.BATCH_VERIFIER(_cb)


class IoPattern:
    """One connection's ctsIoPattern (MakeIoPattern, ctsIOPattern.cpp:97-124)."""

    def __init__(self, config: PatternConfig, engine=None, verifier=None):
        self.config = config
        self._cfg = config.to_c()
        h = ctypes.c_void_p()
        check("cts_io_pattern_create",
              lib().cts_io_pattern_create(ctypes.byref(self._cfg), None if engine is None else _product(engine),
                                          ctypes.byref(h)))
        self._h = h
        self._hook = None
        if verifier is not None:
            self._hook = verifier if isinstance(verifier, A.BATCH_VERIFIER) else batch_verifier(verifier)
            check("cts_io_pattern_set_verifier", lib().cts_io_pattern_set_verifier(self._h, self._hook, None))

    MakeIoPattern = classmethod(lambda cls, config, engine=None, verifier=None: cls(config, engine, verifier))

    def close(self) -> None:
        """cts_io_pattern_destroy. On CTS_E_TIMEOUT (a kernel still reads the pattern's buffers) the handle is kept
        and CtsError raised: call close() again. Any other failure frees the pattern and raises."""
        if getattr(self, "_h", None) is not None and self._h.value:
            rc = lib().cts_io_pattern_destroy(self._h)
            if rc != _lib.CTS_E_TIMEOUT:
                self._h = None
            check("cts_io_pattern_destroy", rc)

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---- the boundary (ctsIOPattern.h:143-144) -------------------------------
    def InitiateIo(self) -> A.CtsTask:
        t = A.CtsTask()
        check("cts_io_pattern_initiate_io", lib().cts_io_pattern_initiate_io(self._h, ctypes.byref(t)))
        return t

    def CompleteIo(self, task: A.CtsTask, current_transfer: int, status_code: int = 0) -> int:
        rc = lib().cts_io_pattern_complete_io(self._h, ctypes.byref(task), current_transfer, status_code)
        if rc < 0:
            raise CtsError("cts_io_pattern_complete_io", rc)
        return rc

    def GetLastPatternError(self) -> int:
        return int(lib().cts_io_pattern_last_error(self._h))

    def GetRioBufferIdCount(self) -> int:
        return int(lib().cts_io_pattern_rio_buffer_id_count(self._h))

    def SetIdealSendBacklog(self, isb: int) -> None:
        check("cts_io_pattern_set_ideal_send_backlog", lib().cts_io_pattern_set_ideal_send_backlog(self._h, isb))

    def Flush(self) -> int:
        rc = lib().cts_io_pattern_flush(self._h)
        if rc < 0:
            raise CtsError("cts_io_pattern_flush", rc)
        return rc

    def stats(self) -> dict:
        s = A.CtsPatternStats()
        check("cts_io_pattern_get_stats", lib().cts_io_pattern_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    def failure_message(self) -> str:
        buf = ctypes.create_string_buffer(512)
        n = lib().cts_io_pattern_failure_message(self._h, buf, 512)
        return buf.value.decode() if n else ""

    def fail_fast_reason(self) -> Optional[str]:
        r = lib().cts_io_pattern_fail_fast_reason(self._h)
        return r.decode() if r else None

    def connection_id(self) -> str:
        return lib().cts_io_pattern_connection_id(self._h).decode()

    # ---- MediaStream (PATTERN_MEDIA_STREAM) ------------------------------------------------
    def RegisterCallback(self, fn) -> None:
        """ctsIoPattern::RegisterCallback (ctsIOPattern.h:94-97): fn(task) receives the tasks the client's timers
        hand out (START sends, Abort, FatalAbort); it runs with the pattern's lock held and may CompleteIo them."""
        if fn is None:
            self._callback = None
            check("cts_io_pattern_register_callback", lib().cts_io_pattern_register_callback(self._h, A.TASK_CALLBACK(), None))
            return
        self._callback = A.TASK_CALLBACK(lambda _ctx, t: fn(A.CtsTask.from_buffer_copy(t.contents)))
        check("cts_io_pattern_register_callback", lib().cts_io_pattern_register_callback(self._h, self._callback, None))

    def media_stream_fire(self, timer: int) -> None:
        """Run the client's StartCallback (MS_TIMER_START) or TimerCallback (MS_TIMER_RENDER) now."""
        check("cts_io_pattern_media_stream_fire", lib().cts_io_pattern_media_stream_fire(self._h, timer))

    def media_stream_timers(self) -> tuple:
        """(start_due_ms, render_due_ms) on the pattern clock; -1 = not armed."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        check("cts_io_pattern_media_stream_timers",
              lib().cts_io_pattern_media_stream_timers(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def media_stream_stats(self) -> dict:
        from .media_stream import Stats

        s = Stats()
        check("cts_io_pattern_media_stream_stats", lib().cts_io_pattern_media_stream_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    # ---- helpers the tests use to "simulate the wire" ---------------------------
    @staticmethod
    def AccessSharedBuffer() -> int:
        """g_senderSharedBuffer address (ctsIOPattern.cpp:126-131)."""
        return int(lib().cts_shared_buffer() or 0)

    @staticmethod
    def write_task_buffer(task: A.CtsTask, data: bytes, offset: int = 0) -> None:
        ctypes.memmove(task.buffer + task.buffer_offset + offset, data, len(data))

    @staticmethod
    def read_task_buffer(task: A.CtsTask, n: int, offset: int = 0) -> bytes:
        return ctypes.string_at(task.buffer + task.buffer_offset + offset, n)

    @staticmethod
    def recv_from_wire(task: A.CtsTask, nbytes: int) -> None:
        """memcpy(task.m_buffer, AccessSharedBuffer() + task.m_expectedPatternOffset, n)
        — the MSTest convention (ctsIOPatternUnitTest_Server.cpp:295)."""
        ctypes.memmove(task.buffer + task.buffer_offset, IoPattern.AccessSharedBuffer() + task.expected_pattern_offset,
                       nbytes)


def shared_buffer_init(engine, max_buffer_size: int) -> None:
    check("cts_shared_buffer_init", lib().cts_shared_buffer_init(_product(engine), max_buffer_size))


_shared_keepalive = None


def shared_buffer_attach(buf: np.ndarray) -> None:
    """Harnesses without a device: use caller-owned bytes as g_senderSharedBuffer. The library keeps only the
    pointer, so the array is held here until the next attach or release."""
    global _shared_keepalive
    check("cts_shared_buffer_attach", lib().cts_shared_buffer_attach(buf.ctypes.data, buf.nbytes))
    _shared_keepalive = buf


def shared_buffer_release() -> None:
    global _shared_keepalive
    lib().cts_shared_buffer_release()
    _shared_keepalive = None


def rio_functions_set(register_fn, deregister_fn, ctx=None) -> None:
    """g_configSettings->rioFunctions: RIORegisterBuffer / RIODeregisterBuffer for patterns created with
    registered_io. Takes C function pointers (ints) or Python callables (kept alive here); None clears."""
    global _rio_keepalive
    if register_fn is None:
        check("cts_rio_functions_set", lib().cts_rio_functions_set(None, None, None))
        _rio_keepalive = None
        return
    reg = register_fn if isinstance(register_fn, int) else A.RIO_REGISTER(register_fn)
    dereg = deregister_fn if isinstance(deregister_fn, int) else A.RIO_DEREGISTER(deregister_fn)
    _rio_keepalive = (reg, dereg)
    as_ptr = lambda f: f if isinstance(f, int) else ctypes.cast(f, ctypes.c_void_p).value
    check("cts_rio_functions_set", lib().cts_rio_functions_set(as_ptr(reg), as_ptr(dereg), ctx))


_rio_keepalive = None


def clock_set(now_ms) -> None:
    """The millisecond clock send pacing reads (ctTimer::snap_qpc_as_msec; the reference's unit tests drive
    ctTimer::g_unitTestQpcTimeMs). A Python callable returning ms, a C function pointer (int), or None for the
    default monotonic clock."""
    global _clock_keepalive
    if now_ms is None:
        check("cts_pattern_clock_set", lib().cts_pattern_clock_set(None, None))
        _clock_keepalive = None
        return
    fn = now_ms if isinstance(now_ms, int) else A.CLOCK_MS(lambda _ctx: int(now_ms()))
    _clock_keepalive = fn
    ptr = fn if isinstance(fn, int) else ctypes.cast(fn, ctypes.c_void_p).value
    check("cts_pattern_clock_set", lib().cts_pattern_clock_set(ptr, None))


_clock_keepalive = None


def status_details() -> dict:
    s = A.CtsStatusDetails()
    check("cts_status_details_read", lib().cts_status_details_read(ctypes.byref(s)))
    return {"bytes_sent": s.bytes_sent, "bytes_recv": s.bytes_recv, "data_errors": s.data_errors}


def status_details_reset() -> None:
    lib().cts_status_details_reset()


def _product(engine):
    """The engine handle the pattern mirror passes to the C ABI."""
    return engine._h
