"""ctypes declarations of the ctsIoPattern mirror's C ABI (include/cts_pattern.h)."""
from __future__ import annotations

import ctypes

from ._lib import CtsVerifyResult

TASK_NONE, TASK_SEND, TASK_RECV, TASK_GRACEFUL_SHUTDOWN, TASK_HARD_SHUTDOWN, TASK_ABORT, TASK_FATAL_ABORT = range(7)
(BUFFER_NULL, BUFFER_TCP_CONNECTION_ID, BUFFER_UDP_CONNECTION_ID, BUFFER_COMPLETION_MESSAGE, BUFFER_STATIC,
 BUFFER_DYNAMIC) = range(6)
IO_CONTINUE, IO_COMPLETED, IO_FAILED = 0, 1, 2
PATTERN_PUSH, PATTERN_PULL, PATTERN_PUSHPULL, PATTERN_DUPLEX, PATTERN_MEDIA_STREAM = 1, 2, 3, 4, 5
MS_TIMER_START, MS_TIMER_RENDER = 0, 1  # CTS_MS_TIMER_*
PROTOCOL_TCP, PROTOCOL_UDP = 1, 2
SHUTDOWN_GRACEFUL, SHUTDOWN_HARD = 1, 2
VERIFY_SYNC, VERIFY_DEFERRED = 0, 1

# ctsIoPatternType / ctsIoPatternError (ctsIOPatternState.hpp:27-48)
(PT_NO_IO, PT_SEND_CONNECTION_ID, PT_RECV_CONNECTION_ID, PT_MORE_IO, PT_SEND_COMPLETION, PT_RECV_COMPLETION,
 PT_GRACEFUL_SHUTDOWN, PT_HARD_SHUTDOWN, PT_REQUEST_FIN) = range(9)
(PE_NO_ERROR, PE_TOO_MANY_BYTES, PE_TOO_FEW_BYTES, PE_CORRUPTED_BYTES, PE_ERROR_IO_FAILED,
 PE_SUCCESSFULLY_COMPLETED) = range(6)

STATUS_IO_RUNNING = 2147483647
STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED = 2147483646
STATUS_ERROR_TOO_MUCH_DATA_TRANSFERRED = 2147483645
STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN = 2147483644
PATTERN_E_FAIL_FAST = 2147483640
CONNECTION_ID_LENGTH = 37
RIO_INVALID_BUFFERID = 0xFFFFFFFF
COMPLETION_MESSAGE_SIZE = 4


class CtsTask(ctypes.Structure):
    """ctsTask (ctsIOTask.hpp:37-60)."""

    _fields_ = [
        ("time_offset_ms", ctypes.c_int64),
        ("rio_buffer_id", ctypes.c_uint64),
        ("buffer", ctypes.c_void_p),
        ("buffer_length", ctypes.c_uint32),
        ("buffer_offset", ctypes.c_uint32),
        ("expected_pattern_offset", ctypes.c_uint32),
        ("io_action", ctypes.c_uint8),
        ("buffer_type", ctypes.c_uint8),
        ("track_io", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
    ]


class CtsPatternConfig(ctypes.Structure):
    _fields_ = [
        ("io_pattern", ctypes.c_uint32),
        ("protocol", ctypes.c_uint32),
        ("listening", ctypes.c_uint32),
        ("verify_buffers", ctypes.c_uint32),
        ("use_shared_buffer", ctypes.c_uint32),
        ("pre_post_recvs", ctypes.c_uint32),
        ("pre_post_sends", ctypes.c_uint32),
        ("buffer_size_low", ctypes.c_uint32),
        ("buffer_size_high", ctypes.c_uint32),
        ("push_bytes", ctypes.c_uint32),
        ("pull_bytes", ctypes.c_uint32),
        ("tcp_shutdown", ctypes.c_uint32),
        ("transfer_size", ctypes.c_uint64),
        ("random_seed", ctypes.c_uint64),
        ("verify_mode", ctypes.c_uint32),
        ("batch_buffers", ctypes.c_uint32),
        ("batch_bytes", ctypes.c_uint64),
        ("registered_io", ctypes.c_uint32),
        ("reserved0", ctypes.c_uint32),
        ("tcp_bytes_per_second", ctypes.c_int64),
        ("tcp_bytes_per_second_period", ctypes.c_int64),
        ("burst_count", ctypes.c_uint32),
        ("burst_delay", ctypes.c_uint32),
        ("ms_frames_per_second", ctypes.c_uint32),
        ("ms_datagram_max_size", ctypes.c_uint32),
        ("ms_buffered_frames", ctypes.c_uint32),
        ("ms_manual_timers", ctypes.c_uint32),
        ("ms_stream_length_frames", ctypes.c_int64),
    ]


class CtsPatternStats(ctypes.Structure):
    _fields_ = [
        ("bytes_sent", ctypes.c_uint64),
        ("bytes_recv", ctypes.c_uint64),
        ("buffers_verified", ctypes.c_uint64),
        ("bytes_verified", ctypes.c_uint64),
        ("buffers_failed", ctypes.c_uint64),
        ("bytes_recv_at_failure", ctypes.c_uint64),
        ("recv_pattern_offset", ctypes.c_uint32),
        ("send_pattern_offset", ctypes.c_uint32),
        ("last_error", ctypes.c_uint32),
        ("queued", ctypes.c_uint32),
        ("fail_length", ctypes.c_uint32),
        ("fail_offset", ctypes.c_uint32),
        ("fail_expected", ctypes.c_uint8),
        ("fail_actual", ctypes.c_uint8),
        ("has_failure", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8),
        ("fail_completion", ctypes.c_uint32),
        ("bytes_sent_held", ctypes.c_uint64),
        ("bytes_recv_held", ctypes.c_uint64),
        ("verify_wait_ns", ctypes.c_uint64),
        ("deferred_depth", ctypes.c_uint32),
        ("reserved2", ctypes.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_ if f not in ("reserved", "reserved2")}


class CtsStatusDetails(ctypes.Structure):
    _fields_ = [("bytes_sent", ctypes.c_uint64), ("bytes_recv", ctypes.c_uint64), ("data_errors", ctypes.c_uint64)]


assert ctypes.sizeof(CtsTask) == 40
assert ctypes.sizeof(CtsPatternConfig) == 136

# int (*)(void* ctx, const uint8_t* host_arena, uint64_t arena_bytes, const cts_buf_desc* descs,
#         uint32_t n, cts_verify_result* results)
BATCH_VERIFIER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                  ctypes.c_uint32, ctypes.POINTER(CtsVerifyResult))


# uint64_t (*)(void* ctx, char* buffer, uint32_t length) / void (*)(void* ctx, uint64_t buffer_id)
RIO_REGISTER = ctypes.CFUNCTYPE(ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32)
RIO_DEREGISTER = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64)
# int64_t (*)(void* ctx): the millisecond clock of send pacing (cts_pattern_clock_set)
CLOCK_MS = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p)
# void (*)(void* ctx, const cts_task* task): RegisterCallback (cts_io_pattern_register_callback)
TASK_CALLBACK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(CtsTask))


def declare(L: ctypes.CDLL) -> None:
    P = ctypes.c_void_p
    u32, u64, i32 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sigs = {
        "cts_shared_buffer_init": ([P, u32], i32),
        "cts_shared_buffer_attach": ([P, u64], i32),
        "cts_shared_buffer": ([], P),
        "cts_shared_buffer_bytes": ([], u64),
        "cts_shared_buffer_release": ([], None),
        "cts_io_pattern_create": ([ctypes.POINTER(CtsPatternConfig), P, ctypes.POINTER(P)], i32),
        "cts_io_pattern_destroy": ([P], i32),
        "cts_io_pattern_set_verifier": ([P, BATCH_VERIFIER, P], i32),
        "cts_io_pattern_initiate_io": ([P, ctypes.POINTER(CtsTask)], i32),
        "cts_io_pattern_complete_io": ([P, ctypes.POINTER(CtsTask), u32, u32], i32),
        "cts_io_pattern_last_error": ([P], u32),
        "cts_io_pattern_rio_buffer_id_count": ([P], u64),
        "cts_rio_functions_set": ([P, P, P], i32),
        "cts_pattern_clock_set": ([P, P], i32),
        "cts_io_pattern_set_ideal_send_backlog": ([P, u32], i32),
        "cts_io_pattern_flush": ([P], i32),
        "cts_io_pattern_get_stats": ([P, ctypes.POINTER(CtsPatternStats)], i32),
        "cts_io_pattern_failure_message": ([P, ctypes.c_char_p, u32], i32),
        "cts_io_pattern_fail_fast_reason": ([P], ctypes.c_char_p),
        "cts_io_pattern_connection_id": ([P], ctypes.c_char_p),
        "cts_io_pattern_register_callback": ([P, TASK_CALLBACK, P], i32),
        "cts_io_pattern_media_stream_fire": ([P, ctypes.c_int], i32),
        "cts_io_pattern_media_stream_timers": ([P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)],
                                               i32),
        "cts_io_pattern_media_stream_stats": ([P, P], i32),
        "cts_io_pattern_state_create": ([ctypes.POINTER(CtsPatternConfig), ctypes.POINTER(P)], i32),
        "cts_io_pattern_state_destroy": ([P], i32),
        "cts_io_pattern_state_get_remaining_transfer": ([P], u64),
        "cts_io_pattern_state_get_max_transfer": ([P], u64),
        "cts_io_pattern_state_set_max_transfer": ([P, u64], i32),
        "cts_io_pattern_state_get_ideal_send_backlog": ([P], u32),
        "cts_io_pattern_state_set_ideal_send_backlog": ([P, u32], i32),
        "cts_io_pattern_state_is_completed": ([P], i32),
        "cts_io_pattern_state_is_current_state_more_io": ([P], i32),
        "cts_io_pattern_state_get_next_pattern_type": ([P], i32),
        "cts_io_pattern_state_notify_next_task": ([P, ctypes.POINTER(CtsTask)], i32),
        "cts_io_pattern_state_completed_task": ([P, ctypes.POINTER(CtsTask), u32], i32),
        "cts_io_pattern_state_update_error": ([P, u32], i32),
        "cts_io_pattern_state_fail_fast_reason": ([P], ctypes.c_char_p),
        "cts_status_details_read": ([ctypes.POINTER(CtsStatusDetails)], i32),
        "cts_status_details_reset": ([], None),
    }
    for name, (argtypes, restype) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = restype
