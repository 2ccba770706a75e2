"""CPU oracle for ctsTraffic's pattern fill + verify — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` may import this module, and only as the checker (or as the timed
CPU baseline). The product package ``ctstraffic_amd`` never imports it.

ctypes bindings over ``oracle/libcts_oracle.so`` (built from ``cts_oracle.c``
by ``oracle/Makefile``), which restates:

* ``ctsTraffic/ctsIOPattern.cpp:35-36,52-90``  pattern table + sender buffer
* ``ctsTraffic/ctsIOPattern.cpp:745-775``      VerifyBuffer / RtlCompareMemory
* ``ctsTraffic/ctsIOPattern.cpp:491-492,695-697`` offset advance mod 65536
* ``ctsTraffic/ctsIOPatternMediaStream.cpp:185-192`` UDP verify (skip 26, offset 0)

Parity pinning: see ``cts_oracle.h`` (reference unbuildable; byte values
pinned by source through ``tests/golden/pattern_kat.json``; behaviour pinned
by the reference's MSTest scenarios replayed in ``tests/``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libcts_oracle.so")

PATTERN_SIZE = 65536

DESC_DTYPE = np.dtype(
    [
        ("byte_offset", "<u8"),
        ("length", "<u4"),
        ("expected_pattern_offset", "<u4"),
        ("conn_index", "<u4"),
        ("skip_head", "<u4"),
    ]
)
RESULT_DTYPE = np.dtype(
    [
        ("first_mismatch", "<u4"),
        ("mismatch_bytes", "<u4"),
        ("expected", "u1"),
        ("actual", "u1"),
        ("pass", "u1"),
        ("flags", "u1"),
    ]
)
DGRAM_RECORD_DTYPE = np.dtype(
    [
        ("sequence_number", "<i8"),
        ("sender_qpc", "<i8"),
        ("sender_qpf", "<i8"),
        ("flag", "<u2"),
        ("kind", "u1"),
        ("reserved", "u1"),
        ("completed_bytes", "<u4"),
    ]
)
COUNTER_FIELDS = ("bytes_checked", "bytes_ok", "buffers_checked", "buffers_failed", "mismatched_bytes")
assert DESC_DTYPE.itemsize == 24 and RESULT_DTYPE.itemsize == 12


class OraCounters(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in COUNTER_FIELDS]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f in COUNTER_FIELDS}


class OraResult(ctypes.Structure):
    _fields_ = [
        ("first_mismatch", ctypes.c_uint32),
        ("mismatch_bytes", ctypes.c_uint32),
        ("expected", ctypes.c_uint8),
        ("actual", ctypes.c_uint8),
        ("pass_", ctypes.c_uint8),
        ("flags", ctypes.c_uint8),
    ]


_lib = None


def build() -> str:
    """Compile the oracle with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.ora_build_pattern_table.argtypes = [P]
        L.ora_sender_buffer_size.argtypes = [ctypes.c_uint32]
        L.ora_sender_buffer_size.restype = ctypes.c_uint64
        L.ora_build_sender_buffer.argtypes = [P, ctypes.c_uint32]
        L.ora_compare_memory.argtypes = [P, P, ctypes.c_size_t]
        L.ora_compare_memory.restype = ctypes.c_size_t
        L.ora_verify_buffer.argtypes = [P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.POINTER(OraResult)]
        L.ora_verify_buffer.restype = ctypes.c_int
        L.ora_advance_offset.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.ora_advance_offset.restype = ctypes.c_uint32
        L.ora_pattern_byte.argtypes = [ctypes.c_uint64]
        L.ora_pattern_byte.restype = ctypes.c_uint8
        L.ora_fill.argtypes = [P, ctypes.c_uint64, P, ctypes.c_uint32]
        L.ora_verify_batch.argtypes = [P, ctypes.c_uint64, P, ctypes.c_uint32, P,
                                       ctypes.POINTER(OraCounters), P, ctypes.c_uint32, ctypes.c_int]
        L.ora_verify_batch.restype = ctypes.c_int
        L.ora_media_stream_verify.argtypes = [P, ctypes.c_uint64, P, ctypes.c_uint32, P, P,
                                              ctypes.POINTER(OraCounters)]
        L.ora_media_stream_verify.restype = None
        L.ora_fnv1a64.argtypes = [P, ctypes.c_size_t]
        L.ora_fnv1a64.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def pattern_table() -> np.ndarray:
    out = np.zeros(2 * PATTERN_SIZE, dtype=np.uint8)
    lib().ora_build_pattern_table(_ptr(out))
    return out


def sender_buffer(max_buffer_size: int) -> np.ndarray:
    n = int(lib().ora_sender_buffer_size(max_buffer_size))
    out = np.zeros(n, dtype=np.uint8)
    lib().ora_build_sender_buffer(_ptr(out), max_buffer_size)
    return out


def compare_memory(a: np.ndarray, b: np.ndarray, n: int) -> int:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    assert a.size >= n and b.size >= n
    return int(lib().ora_compare_memory(_ptr(a), _ptr(b), n))


def verify_buffer(buf: np.ndarray, buffer_offset: int, expected: int, transferred: int) -> dict:
    """VerifyBuffer(task{m_buffer=buf, m_bufferOffset, m_expectedPatternOffset}, transferred)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    assert buf.size >= buffer_offset + transferred and expected < PATTERN_SIZE
    S = sender_buffer(max(transferred, 1))
    r = OraResult()
    ok = lib().ora_verify_buffer(_ptr(S), _ptr(buf), buffer_offset, expected, transferred, ctypes.byref(r))
    return {
        "pass": bool(ok),
        "first_mismatch": r.first_mismatch,
        "mismatch_bytes": r.mismatch_bytes,
        "expected": r.expected,
        "actual": r.actual,
    }


def advance_offset(offset: int, nbytes: int) -> int:
    return int(lib().ora_advance_offset(offset, nbytes))


def pattern_byte(pos: int) -> int:
    return int(lib().ora_pattern_byte(pos))


def fill(arena: np.ndarray, descs: np.ndarray) -> None:
    assert arena.dtype == np.uint8 and arena.flags.c_contiguous
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    lib().ora_fill(_ptr(arena), arena.size, _ptr(descs), len(descs))


def verify_batch(arena: np.ndarray, descs: np.ndarray, n_conns: int = 0, nthreads: int = 1,
                 want_results: bool = True):
    """Returns (results[n] RESULT_DTYPE or None, counters dict, conn_first_fail u32[n_conns])."""
    assert arena.dtype == np.uint8 and arena.flags.c_contiguous
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    n = len(descs)
    results = np.zeros(n, dtype=RESULT_DTYPE) if want_results else None
    cff = np.full(n_conns, 0xFFFFFFFF, dtype=np.uint32) if n_conns else None
    c = OraCounters()
    rc = lib().ora_verify_batch(_ptr(arena), arena.size, _ptr(descs), n, _ptr(results), ctypes.byref(c),
                                _ptr(cff), n_conns, nthreads)
    if rc != 0:
        raise ValueError("ora_verify_batch: bad argument")
    return results, c.as_dict(), (cff if cff is not None else np.zeros(0, np.uint32))


def fnv1a64(data: np.ndarray) -> int:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    return int(lib().ora_fnv1a64(_ptr(data), data.size))


def media_stream_verify(arena: np.ndarray, descs: np.ndarray):
    """MediaStream client receive path per datagram: (records DGRAM_RECORD_DTYPE, results, counters)."""
    assert arena.dtype == np.uint8 and arena.flags.c_contiguous
    descs = np.ascontiguousarray(descs, dtype=DESC_DTYPE)
    n = len(descs)
    recs = np.zeros(n, dtype=DGRAM_RECORD_DTYPE)
    results = np.zeros(n, dtype=RESULT_DTYPE)
    c = OraCounters()
    lib().ora_media_stream_verify(_ptr(arena), arena.size, _ptr(descs), n, _ptr(recs), _ptr(results), ctypes.byref(c))
    return recs, results, c.as_dict()


def batch_verifier_address() -> int:
    """Address of ora_batch_verifier (a cts_batch_verifier): the CPU VerifyBuffer for C callers."""
    return ctypes.cast(lib().ora_batch_verifier, ctypes.c_void_p).value
