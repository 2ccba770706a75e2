"""Python handle over the C ABI (``include/cts_engine.h``).

torch tensors are used only as device-memory/stream plumbing: their
``data_ptr()`` and the current HIP stream are passed straight through the
C ABI, which never sees a torch type.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import CtsAllreduceSetup, CtsCounters, CtsCountersEx, CtsVerifyResult, check, lib
from .types import DESC_DTYPE, RESULT_DTYPE

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def _ptr(x) -> Optional[int]:
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if torch is not None and isinstance(x, torch.Tensor):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError("unsupported buffer type %r" % type(x))


def _nbytes(x) -> int:
    if torch is not None and isinstance(x, torch.Tensor):
        return x.numel() * x.element_size()
    if isinstance(x, np.ndarray):
        return x.nbytes
    raise TypeError("unsupported buffer type %r" % type(x))


def _stream(stream) -> Optional[int]:
    if stream is None:
        if torch is not None and torch.cuda.is_available():
            return torch.cuda.current_stream().cuda_stream
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def pattern_byte(stream_offset: int) -> int:
    """Byte of g_senderSharedBuffer at a stream offset (ctsIOPattern.cpp:55-80)."""
    return int(lib().cts_pattern_byte(stream_offset))


def sender_buffer_size(max_buffer_size: int) -> int:
    return int(lib().cts_sender_buffer_size(max_buffer_size))


def descs_to_device(descs: np.ndarray, device="cuda"):
    """Structured DESC_DTYPE array -> uint8 device tensor (24 bytes per descriptor)."""
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    return torch.from_numpy(descs.view(np.uint8).copy()).to(device)


def results_from_device(t) -> np.ndarray:
    return t.cpu().numpy().view(RESULT_DTYPE)


def _check_outputs(n: int, results, counters) -> None:
    """The C ABI takes raw device pointers and cannot see their sizes: a results tensor shorter than n records or
    a counter block shorter than cts_counters_device_bytes() would be written past its end, so refuse them here."""
    if results is not None and _nbytes(results) < n * RESULT_DTYPE.itemsize:
        raise ValueError("results holds %d bytes, %d buffers need %d" % (_nbytes(results), n,
                                                                        n * RESULT_DTYPE.itemsize))
    if counters is not None and _nbytes(counters) < int(lib().cts_counters_device_bytes()):
        raise ValueError("counters holds %d bytes, the device block is %d" % (_nbytes(counters),
                                                                             int(lib().cts_counters_device_bytes())))


def _multi_args(engines, blocks, streams):
    n = len(engines)
    E = (ctypes.c_void_p * max(1, n))(*[e._h.value for e in engines])
    C = (ctypes.c_void_p * max(1, n))(*[_ptr(b) for b in blocks])
    S = None
    if streams is not None:
        S = (ctypes.c_void_p * max(1, n))(*[_stream(s) for s in streams])
    return E, C, S, n


def counters_read_multi(engines: Sequence["Engine"], blocks, streams=None) -> dict:
    """cts_counters_read_multi: the node-wide counters of one process's engines (one per GPU), folded on the host."""
    E, C, S, n = _multi_args(engines, blocks, streams)
    out = CtsCounters()
    check("cts_counters_read_multi", lib().cts_counters_read_multi(E, C, S, n, ctypes.byref(out)))
    return out.as_dict()


def counters_read_multi_ex(engines: Sequence["Engine"], blocks, streams=None) -> dict:
    """cts_counters_read_multi_ex: counters_read_multi plus connections_failed (the node's DataError count)."""
    E, C, S, n = _multi_args(engines, blocks, streams)
    out = CtsCountersEx()
    check("cts_counters_read_multi_ex", lib().cts_counters_read_multi_ex(E, C, S, n, ctypes.byref(out)))
    return out.as_dict()


def counters_allreduce(engines: Sequence["Engine"], blocks, streams=None) -> dict:
    """cts_counters_allreduce: the same node-wide counters reduced on the GPUs: each block folded on its engine's
    device, then one RCCL all-reduce (sum, u64) per device over xGMI (one process drives every GPU)."""
    E, C, S, n = _multi_args(engines, blocks, streams)
    out = CtsCounters()
    check("cts_counters_allreduce", lib().cts_counters_allreduce(E, C, S, n, ctypes.byref(out)))
    return out.as_dict()


def counters_allreduce_ex(engines: Sequence["Engine"], blocks, streams=None) -> dict:
    """cts_counters_allreduce_ex: counters_allreduce plus connections_failed (u64 x 6 over RCCL)."""
    E, C, S, n = _multi_args(engines, blocks, streams)
    out = CtsCountersEx()
    check("cts_counters_allreduce_ex", lib().cts_counters_allreduce_ex(E, C, S, n, ctypes.byref(out)))
    return out.as_dict()


def counters_allreduce_prepare(engines: Sequence["Engine"]) -> None:
    """cts_counters_allreduce_prepare: build the RCCL clique of these engines' devices (and run its first
    all-reduce) now, so the status timer's first counter read (t = 0, ctsTraffic.cpp:107-113) does not pay it."""
    n = len(engines)
    E = (ctypes.c_void_p * max(1, n))(*[e._h.value for e in engines])
    check("cts_counters_allreduce_prepare", lib().cts_counters_allreduce_prepare(E, n))


def counters_allreduce_setup_times() -> dict:
    """cts_counters_allreduce_setup_times: the newest clique's set-up breakdown (ms)."""
    out = CtsAllreduceSetup()
    check("cts_counters_allreduce_setup_times", lib().cts_counters_allreduce_setup_times(ctypes.byref(out)))
    return out.as_dict()


def counters_allreduce_release() -> None:
    """cts_counters_allreduce_release: destroy the cached RCCL communicators (before the devices go away)."""
    check("cts_counters_allreduce_release", lib().cts_counters_allreduce_release())


class Engine:
    """One engine per GPU (cts_engine_create). Thread-safe across streams."""

    def __init__(self, device: int = 0):
        self._L = lib()
        h = ctypes.c_void_p()
        check("cts_engine_create", self._L.cts_engine_create(device, ctypes.byref(h)))
        self._h = h
        self.device = device

    # ---- lifetime ----------------------------------------------------------
    def device_ordinal(self) -> int:
        """cts_engine_device: the GPU this engine launches on (as the library sees it)."""
        return int(self._L.cts_engine_device(self._h))

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.cts_engine_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ---- launch attributes ----------------------------------------------------
    def set_attr(self, attr: int, value: int) -> None:
        check("cts_engine_set_attr", self._L.cts_engine_set_attr(self._h, attr, value))

    def get_attr(self, attr: int) -> int:
        v = ctypes.c_int()
        check("cts_engine_get_attr", self._L.cts_engine_get_attr(self._h, attr, ctypes.byref(v)))
        return v.value

    # ---- streams ---------------------------------------------------------------
    def stream_create(self) -> int:
        """A non-blocking HIP stream on the engine's device (cts_engine_stream_create); raw handle."""
        p = ctypes.c_void_p()
        check("cts_engine_stream_create", self._L.cts_engine_stream_create(self._h, ctypes.byref(p)))
        return p.value

    def stream_destroy(self, stream: int) -> None:
        check("cts_engine_stream_destroy", self._L.cts_engine_stream_destroy(self._h, stream))

    def stream_synchronize(self, stream: int) -> None:
        """Wait for a stream of this engine (the GIL is released while waiting)."""
        torch.cuda.ExternalStream(stream, device="cuda:%d" % self.device).synchronize()

    # ---- fill ----------------------------------------------------------------
    def sender_buffer(self, max_buffer_size: int, stream=None):
        """Device copy of g_senderSharedBuffer (InitOnceIoPatternCallback, ctsIOPattern.cpp:52-90)."""
        n = sender_buffer_size(max_buffer_size)
        out = torch.empty(n + 16, dtype=torch.uint8, device="cuda:%d" % self.device)[:n]
        check("cts_sender_buffer_fill",
              self._L.cts_sender_buffer_fill(self._h, _ptr(out), max_buffer_size, _stream(stream)))
        return out

    def numa_node(self) -> int:
        """The host NUMA node of the engine's GPU (-1 if unknown): pin SYNC-verify threads there."""
        return int(self._L.cts_engine_numa_node(self._h))

    def cpus_near(self) -> list:
        """The CPUs of numa_node() (empty if unknown), for os.sched_setaffinity."""
        node = self.numa_node()
        if node < 0:
            return []
        try:
            spec = open("/sys/devices/system/node/node%d/cpulist" % node).read().strip()
        except OSError:
            return []
        cpus = []
        for part in spec.split(","):
            lo, _, hi = part.partition("-")
            cpus.extend(range(int(lo), int(hi or lo) + 1))
        return cpus

    def fill(self, arena, descs, max_length_hint: int = 0, stream=None) -> None:
        n = _nbytes(descs) // DESC_DTYPE.itemsize
        check("cts_fill", self._L.cts_fill(self._h, _ptr(arena), _nbytes(arena), _ptr(descs), n, max_length_hint,
                                         _stream(stream)))

    # ---- verify --------------------------------------------------------------
    def verify(self, arena, descs, *, max_length_hint: int = 0, results=None, counters=None,
               conn_first_fail=None, stream=None) -> None:
        n = _nbytes(descs) // DESC_DTYPE.itemsize
        n_conns = 0 if conn_first_fail is None else _nbytes(conn_first_fail) // 4
        _check_outputs(n, results, counters)
        check("cts_verify", self._L.cts_verify(self._h, _ptr(arena), _nbytes(arena), _ptr(descs), n, max_length_hint,
                                             _ptr(results), _ptr(counters), _ptr(conn_first_fail), n_conns,
                                             _stream(stream)))

    def verify_strided(self, arena, stride: int, lengths, *, skip_head: int = 0, expected_offset: int = 0,
                       conn_index: int = 0, results=None, counters=None, conn_first_fail=None, stream=None) -> None:
        """cts_verify_strided: buffer i at arena + i * stride, lengths (uint32 device tensor) its completed bytes,
        one skip / expected offset / connection for the whole ring."""
        n = _nbytes(lengths) // 4
        n_conns = 0 if conn_first_fail is None else _nbytes(conn_first_fail) // 4
        _check_outputs(n, results, counters)
        check("cts_verify_strided", self._L.cts_verify_strided(self._h, _ptr(arena), _nbytes(arena), stride,
                                                             _ptr(lengths), n, skip_head, expected_offset, conn_index,
                                                             _ptr(results), _ptr(counters), _ptr(conn_first_fail),
                                                             n_conns, _stream(stream)))

    def new_results(self, n: int):
        return torch.zeros(n * RESULT_DTYPE.itemsize, dtype=torch.uint8, device="cuda:%d" % self.device)

    # ---- counters --------------------------------------------------------------
    def new_counters(self):
        nbytes = int(self._L.cts_counters_device_bytes())
        return torch.zeros(nbytes // 8, dtype=torch.int64, device="cuda:%d" % self.device)

    def reset_counters(self, counters, stream=None) -> None:
        check("cts_counters_reset", self._L.cts_counters_reset(self._h, _ptr(counters), _stream(stream)))

    def read_counters(self, counters, stream=None) -> dict:
        c = CtsCounters()
        check("cts_counters_read", self._L.cts_counters_read(self._h, _ptr(counters), ctypes.byref(c),
                                                           _stream(stream)))
        return c.as_dict()

    def read_counters_ex(self, counters, stream=None) -> dict:
        """cts_counters_read_ex: read_counters plus connections_failed (the DataError count, ctsSocketState.cpp:
        221-228), counted by the verifies given a conn_first_fail array."""
        c = CtsCountersEx()
        check("cts_counters_read_ex", self._L.cts_counters_read_ex(self._h, _ptr(counters), ctypes.byref(c),
                                                                 _stream(stream)))
        return c.as_dict()

    # ---- pinned host arenas ---------------------------------------------------------
    def host_alloc(self, nbytes: int):
        """Pinned, device-mapped host arena. Returns (numpy uint8 view, host ptr, device-view ptr)."""
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        check("cts_host_alloc", self._L.cts_host_alloc(self._h, nbytes, ctypes.byref(h), ctypes.byref(d)))
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(h.value))
        return arr, h.value, d.value

    def host_free(self, host_ptr: int) -> None:
        check("cts_host_free", self._L.cts_host_free(self._h, host_ptr))

    def verify_ptr(self, arena_ptr: int, arena_bytes: int, descs, *, max_length_hint: int = 0, results=None,
                   counters=None, stream=None) -> None:
        """cts_verify on a raw device address (e.g. the device view of a pinned host arena)."""
        n = _nbytes(descs) // DESC_DTYPE.itemsize
        _check_outputs(n, results, counters)
        check("cts_verify", self._L.cts_verify(self._h, arena_ptr, arena_bytes, _ptr(descs), n, max_length_hint,
                                             _ptr(results), _ptr(counters), None, 0, _stream(stream)))

    # ---- host buffers (drop-in VerifyBuffer) ------------------------------------
    def verify_host(self, buf, expected_offset: int) -> dict:
        a = np.frombuffer(bytes(buf), dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
        a = np.ascontiguousarray(a, dtype=np.uint8)
        r = CtsVerifyResult()
        check("cts_verify_host", self._L.cts_verify_host(self._h, a.ctypes.data if a.size else None, a.size,
                                                       expected_offset, ctypes.byref(r)))
        return {"pass": bool(r.pass_), "first_mismatch": r.first_mismatch, "mismatch_bytes": r.mismatch_bytes,
                "expected": r.expected, "actual": r.actual, "flags": r.flags}

    def verify_mapped(self, dev_ptr: int, length: int, expected_offset: int) -> dict:
        """cts_verify_mapped: one GPU-addressable buffer verified in place and waited for, through the
        engine's resident mailbox grid (no launch per call); concurrent callers' jobs run side by side."""
        r = CtsVerifyResult()
        check("cts_verify_mapped", self._L.cts_verify_mapped(self._h, dev_ptr, length, expected_offset,
                                                           ctypes.byref(r)))
        return {"pass": bool(r.pass_), "first_mismatch": r.first_mismatch, "mismatch_bytes": r.mismatch_bytes,
                "expected": r.expected, "actual": r.actual, "flags": r.flags}

    def mailbox_launches(self) -> int:
        """How often the mailbox grid behind verify_mapped was (re)started."""
        return int(self._L.cts_mailbox_launches(self._h))

    def verify_host_batch(self, bufs: Sequence[np.ndarray], expected: Sequence[int],
                          skip_heads: Optional[Sequence[int]] = None):
        n = len(bufs)
        arrs = [np.ascontiguousarray(b, dtype=np.uint8) for b in bufs]
        ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data if a.size else None for a in arrs])
        lens = np.array([a.size for a in arrs], dtype=np.uint32)
        exp = np.array(expected, dtype=np.uint32)
        skips = None if skip_heads is None else np.array(skip_heads, dtype=np.uint32)
        results = np.zeros(n, dtype=RESULT_DTYPE)
        c = CtsCounters()
        check("cts_verify_host_batch",
              self._L.cts_verify_host_batch(self._h, ptrs, lens.ctypes.data, exp.ctypes.data,
                                          None if skips is None else skips.ctypes.data, n, results.ctypes.data,
                                          ctypes.byref(c)))
        return results, c.as_dict()


__all__ = ["Engine", "pattern_byte", "sender_buffer_size", "descs_to_device", "results_from_device", "_lib"]
