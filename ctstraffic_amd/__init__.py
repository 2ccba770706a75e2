"""ctstraffic_amd — MI355X-native engine for ctsTraffic's data-integrity path.

The path (microsoft/ctsTraffic, ctsTraffic/ctsIOPattern.cpp): the deterministic
bit-pattern fill of outgoing IO buffers (InitOnceIoPatternCallback, :52-90) and
the per-byte verify of every received buffer against that pattern
(ctsIoPattern::VerifyBuffer, :745-775), as hand-written gfx950 HIP kernels
behind the C ABI in include/cts_engine.h (libcts_engine.so).

There is no CPU fallback: importing the engine requires the built library.
"""
from ._lib import CtsError, lib  # noqa: F401
from .engine import Engine, descs_to_device, pattern_byte, results_from_device, sender_buffer_size  # noqa: F401
from .types import COUNTER_FIELDS, DESC_DTYPE, RESULT_DTYPE, RESULT_FLAG_BAD_DESC  # noqa: F401

__version__ = "0.1.0"
