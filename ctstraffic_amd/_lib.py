"""ctypes binding of ``libcts_engine.so`` (the C ABI declared in ``include/cts_engine.h``).

The shared library is built in-tree by ``make`` / ``__graft_entry__.build()``
(hipcc --offload-arch=gfx950). There is NO fallback: if the library is missing
or fails to load, :func:`lib` raises, so a GPU run can never silently take a
CPU path.

torch (when installed) is imported *before* the library is loaded: torch ships
its own ``libamdhip64.so.7``, and loading ours first would put two HIP runtimes
in one process. With torch already loaded the dynamic loader resolves our
``libamdhip64.so.7`` dependency to torch's copy (same SONAME), so device
pointers and streams are shared.
"""
from __future__ import annotations

import ctypes
import os

try:  # plumbing only: device memory / streams / torch.distributed
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# CTS_ENGINE_LIB: an alternative in-tree build of the same library (tools/ A/B runs)
LIB_PATH = os.environ.get("CTS_ENGINE_LIB") or os.path.join(_HERE, "libcts_engine.so")

CTS_OK = 0
CTS_E_INVALID = -1
CTS_E_HIP = -2
CTS_E_NOMEM = -3
CTS_E_NO_DEVICE = -4
CTS_E_UNAVAILABLE = -5
CTS_E_TIMEOUT = -6

PATTERN_PERIOD = 65536
UDP_DATA_HEADER_LENGTH = 26
STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN = 2147483644  # MAXINT - 3, ctsIOPattern.h:49
COUNTER_SHARDS = 64
ATTR_BLOCKS_PER_CU = 1
ATTR_NT_LOADS = 2
ATTR_SMALL_THRESHOLD = 3
ATTR_VERIFY_VARIANT = 4
ATTR_SMALL_BLOCKS_PER_CU = 5
ATTR_SMALL_VARIANT = 6
ATTR_FILL_BLOCKS_PER_CU = 7
ATTR_MS_VARIANT = 8
ATTR_SMALL_CHUNK = 9
ATTR_FILL_NT = 10
ATTR_SYNC_MAILBOX = 11


# the large-buffer verify kernel (CTS_ATTR_VERIFY_VARIANT reports its id, 25), demangled as rocprofv3 prints it;
# the nontemporal-load form is the default (CTS_ATTR_NT_LOADS)
VERIFY_KERNEL_ID = 25


def verify_kernel_name(nontemporal: bool = True) -> str:
    return ("void cts::verify_wg_kernel<%s>(unsigned char const*, unsigned long, cts_buf_desc const*, unsigned int, "
            "cts_verify_result*, unsigned long*, unsigned int*, unsigned int)" % ("true" if nontemporal else "false"))


class CtsError(RuntimeError):
    def __init__(self, fn: str, status: int):
        super().__init__("%s failed: %s (%d)" % (fn, _status_string(status), status))
        self.status = status


class CtsCounters(ctypes.Structure):
    _fields_ = [
        ("bytes_checked", ctypes.c_uint64),
        ("bytes_ok", ctypes.c_uint64),
        ("buffers_checked", ctypes.c_uint64),
        ("buffers_failed", ctypes.c_uint64),
        ("mismatched_bytes", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class CtsCountersEx(ctypes.Structure):
    """cts_counters_ex: cts_counters plus the DataError count (connections with a failing buffer)."""
    _fields_ = CtsCounters._fields_ + [("connections_failed", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class CtsAllreduceSetup(ctypes.Structure):
    """cts_allreduce_setup: where the newest RCCL clique's set-up time went (ms)."""
    _fields_ = [
        ("rccl_load_ms", ctypes.c_double),
        ("slots_ms", ctypes.c_double),
        ("comm_init_ms", ctypes.c_double),
        ("first_allreduce_ms", ctypes.c_double),
        ("devices", ctypes.c_uint32),
        ("prepared", ctypes.c_uint32),
        ("last_fold_us", ctypes.c_double),
        ("last_allreduce_us", ctypes.c_double),
        ("last_readback_us", ctypes.c_double),
        ("last_total_us", ctypes.c_double),
    ]

    def as_dict(self) -> dict:
        return {f: (float if t is ctypes.c_double else int)(getattr(self, f)) for f, t in self._fields_}


class CtsVerifyResult(ctypes.Structure):
    _fields_ = [
        ("first_mismatch", ctypes.c_uint32),
        ("mismatch_bytes", ctypes.c_uint32),
        ("expected", ctypes.c_uint8),
        ("actual", ctypes.c_uint8),
        ("pass_", ctypes.c_uint8),
        ("flags", ctypes.c_uint8),
    ]


assert ctypes.sizeof(CtsVerifyResult) == 12

_lib = None


def _status_string(status: int) -> str:
    try:
        return lib().cts_status_string(status).decode()
    except Exception:
        return "status"


def _declare(L: ctypes.CDLL) -> None:
    P = ctypes.c_void_p
    u32, u64, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sigs = {
        "cts_version": ([], ctypes.c_char_p),
        "cts_status_string": ([i32], ctypes.c_char_p),
        "cts_pattern_byte": ([u64], ctypes.c_uint8),
        "cts_sender_buffer_size": ([u32], u64),
        "cts_shard_of": ([u32, u32], u32),
        "cts_engine_create": ([i32, ctypes.POINTER(P)], i32),
        "cts_engine_destroy": ([P], i32),
        "cts_engine_device": ([P], i32),
        "cts_engine_numa_node": ([P], i32),
        "cts_sender_buffer_fill": ([P, P, u32, P], i32),
        "cts_fill": ([P, P, u64, P, u32, u32, P], i32),
        "cts_verify": ([P, P, u64, P, u32, u32, P, P, P, u32, P], i32),
        "cts_verify_strided": ([P, P, u64, u32, P, u32, u32, u32, u32, P, P, P, u32, P], i32),
        "cts_counters_device_bytes": ([], ctypes.c_size_t),
        "cts_counters_reset": ([P, P, P], i32),
        "cts_counters_read": ([P, P, ctypes.POINTER(CtsCounters), P], i32),
        "cts_counters_read_multi": ([ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), u32,
                                     ctypes.POINTER(CtsCounters)], i32),
        "cts_counters_allreduce": ([ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), u32,
                                    ctypes.POINTER(CtsCounters)], i32),
        "cts_counters_allreduce_release": ([], i32),
        "cts_counters_read_ex": ([P, P, ctypes.POINTER(CtsCountersEx), P], i32),
        "cts_counters_read_multi_ex": ([ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), u32,
                                        ctypes.POINTER(CtsCountersEx)], i32),
        "cts_counters_allreduce_ex": ([ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P), u32,
                                       ctypes.POINTER(CtsCountersEx)], i32),
        "cts_counters_allreduce_prepare": ([ctypes.POINTER(P), u32], i32),
        "cts_counters_allreduce_setup_times": ([ctypes.POINTER(CtsAllreduceSetup)], i32),
        "cts_verify_host": ([P, P, u32, u32, ctypes.POINTER(CtsVerifyResult)], i32),
        "cts_verify_mapped": ([P, P, u32, u32, ctypes.POINTER(CtsVerifyResult)], i32),
        "cts_mailbox_launches": ([P], u64),
        "cts_verify_host_batch": ([P, P, P, P, P, u32, P, ctypes.POINTER(CtsCounters)], i32),
        "cts_host_alloc": ([P, u64, ctypes.POINTER(P), ctypes.POINTER(P)], i32),
        "cts_host_free": ([P, P], i32),
        "cts_engine_set_attr": ([P, i32, i32], i32),
        "cts_engine_get_attr": ([P, i32, ctypes.POINTER(i32)], i32),
        "cts_engine_stream_create": ([P, ctypes.POINTER(P)], i32),
        "cts_engine_stream_destroy": ([P, P], i32),
        "cts_host_device_pointer": ([P, ctypes.POINTER(P)], i32),
    }
    for name, (argtypes, restype) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = restype
    from . import _pattern_abi, loopback, media_stream, status

    _pattern_abi.declare(L)
    media_stream.declare(L)
    loopback.declare(L)
    status.declare(L)


def lib() -> ctypes.CDLL:
    """Load the engine library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                "ctstraffic_amd: %s not built — run `make` or __graft_entry__.build() "
                "(the HIP engine has no CPU fallback)" % LIB_PATH
            )
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _declare(L)
        _lib = L
    return _lib


def check(fn: str, status: int) -> None:
    if status != CTS_OK:
        raise CtsError(fn, status)
