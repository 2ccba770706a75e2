"""numpy mirrors of the C ABI structs (include/cts_engine.h)."""
import numpy as np

# cts_buf_desc: the ctsTask fields the hot path reads (ctsIOTask.hpp:37-60)
DESC_DTYPE = np.dtype(
    [
        ("byte_offset", "<u8"),
        ("length", "<u4"),
        ("expected_pattern_offset", "<u4"),
        ("conn_index", "<u4"),
        ("skip_head", "<u4"),
    ]
)
# cts_verify_result
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
COUNTER_FIELDS = ("bytes_checked", "bytes_ok", "buffers_checked", "buffers_failed", "mismatched_bytes")
# cts_counters_ex: plus the DataError count (ctsSocketState.cpp:221-228), slot 5 of a device counter shard
COUNTER_FIELDS_EX = COUNTER_FIELDS + ("connections_failed",)
RESULT_FLAG_BAD_DESC = 0x1

assert DESC_DTYPE.itemsize == 24 and RESULT_DTYPE.itemsize == 12
# cts_datagram_record (include/cts_media_stream.h)
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
# cts_datagram_status (compact receive output)
DGRAM_STATUS_DTYPE = np.dtype(
    [
        ("sequence_number", "<i8"),
        ("completed_bytes", "<u4"),
        ("flag", "<u2"),
        ("kind", "u1"),
        ("pass", "u1"),
    ]
)
assert DGRAM_STATUS_DTYPE.itemsize == 16
# cts_datagram_header
DGRAM_HEADER_DTYPE = np.dtype([("sequence_number", "<i8"), ("qpc", "<i8"), ("qpf", "<i8")])
RESULT_FLAG_NOT_DATA = 0x2
assert DGRAM_RECORD_DTYPE.itemsize == 32 and DGRAM_HEADER_DTYPE.itemsize == 24
