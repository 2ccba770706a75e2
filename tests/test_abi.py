"""CPU: the C-ABI library loads, exports every symbol include/*.h declares, and
its struct layouts match the Python mirrors. No device compute is issued."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_functions():
    names = []
    for h in sorted(os.listdir(INCLUDE)):
        if not h.endswith(".h"):
            continue
        src = open(os.path.join(INCLUDE, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(cts_\w+)\s*\(", src, flags=re.M):
            names.append(m.group(1))
    return sorted(set(names))


def test_header_declares_functions():
    names = declared_functions()
    assert "cts_verify" in names and "cts_fill" in names and "cts_engine_create" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from ctstraffic_amd import _lib

    L = _lib.lib()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {line.split()[-1] for line in out.stdout.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    for n in declared_functions():
        assert hasattr(L, n)


def test_library_is_gfx950_code_object():
    from ctstraffic_amd import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_struct_layouts_match_c():
    """Compile a probe against include/cts_engine.h and compare sizeof/offsetof."""
    probe = r"""
#include <stdio.h>
#include <stddef.h>
#include "cts_engine.h"
int main(void){
 printf("%zu %zu %zu %zu %zu %zu\n", sizeof(cts_buf_desc), offsetof(cts_buf_desc,length),
   offsetof(cts_buf_desc,expected_pattern_offset), offsetof(cts_buf_desc,conn_index), offsetof(cts_buf_desc,skip_head),
   sizeof(cts_verify_result));
 printf("%zu %zu %zu %zu %zu\n", offsetof(cts_verify_result,mismatch_bytes), offsetof(cts_verify_result,expected),
   offsetof(cts_verify_result,actual), offsetof(cts_verify_result,pass), offsetof(cts_verify_result,flags));
 printf("%zu\n", sizeof(cts_counters));
 return 0; }
"""
    import tempfile

    from ctstraffic_amd.types import DESC_DTYPE, RESULT_DTYPE

    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(probe)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-std=c11", "-I", INCLUDE, c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    a = list(map(int, lines[0].split()))
    b = list(map(int, lines[1].split()))
    assert a[0] == DESC_DTYPE.itemsize == oracle.DESC_DTYPE.itemsize == 24
    assert a[1:5] == [DESC_DTYPE.fields[f][1] for f in ("length", "expected_pattern_offset", "conn_index", "skip_head")]
    assert a[5] == RESULT_DTYPE.itemsize == 12
    assert b == [RESULT_DTYPE.fields[f][1] for f in ("mismatch_bytes", "expected", "actual", "pass", "flags")]
    assert int(lines[2]) == 40


def test_pattern_byte_helper_matches_oracle():
    # cts_pattern_byte is the ABI's pure-arithmetic helper (no device involved)
    from ctstraffic_amd import pattern_byte

    S = oracle.sender_buffer(65536)
    for p in list(range(0, 64)) + list(range(65500, 65600)) + [131071, 2**33 + 5]:
        assert pattern_byte(p) == S[p % 65536]
    from ctstraffic_amd import sender_buffer_size

    assert sender_buffer_size(65536) == 131072


def test_status_strings_and_invalid_args_without_device():
    from ctstraffic_amd import _lib

    L = _lib.lib()
    assert L.cts_status_string(0) == b"ok"
    assert L.cts_status_string(-4) == b"no such HIP device"
    # null engine -> CTS_E_INVALID, never a crash and never a compute call
    assert L.cts_verify(None, None, 0, None, 1, 0, None, None, None, 0, None) == _lib.CTS_E_INVALID
    assert L.cts_fill(None, None, 0, None, 1, 0, None) == _lib.CTS_E_INVALID
    assert L.cts_engine_destroy(None) == _lib.CTS_E_INVALID
    assert L.cts_counters_device_bytes() == _lib.COUNTER_SHARDS * 64


def test_engine_create_without_device_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from ctstraffic_amd import CtsError, Engine

    with pytest.raises(CtsError):
        Engine(0)


def test_pattern_struct_layouts_match_c():
    """cts_task / cts_pattern_config / cts_pattern_stats (include/cts_pattern.h) vs the ctypes mirrors."""
    import ctypes
    import tempfile

    from ctstraffic_amd import _pattern_abi as A

    probe = r"""
#include <stdio.h>
#include <stddef.h>
#include "cts_pattern.h"
#define O(T,f) printf("%s %zu\n", #f, offsetof(T,f))
int main(void){
 printf("sizeof %zu %zu %zu %zu\n", sizeof(cts_task), sizeof(cts_pattern_config), sizeof(cts_pattern_stats),
        sizeof(cts_status_details));
 O(cts_task,buffer); O(cts_task,buffer_length); O(cts_task,expected_pattern_offset); O(cts_task,io_action);
 O(cts_task,track_io);
 O(cts_pattern_config,transfer_size); O(cts_pattern_config,random_seed); O(cts_pattern_config,verify_mode);
 O(cts_pattern_config,batch_bytes);
 O(cts_pattern_stats,recv_pattern_offset); O(cts_pattern_stats,fail_expected); O(cts_pattern_stats,fail_completion);
 O(cts_pattern_stats,bytes_recv_held); O(cts_pattern_stats,verify_wait_ns); O(cts_pattern_stats,deferred_depth);
 return 0; }
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(probe)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-std=c11", "-I", INCLUDE, c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = list(map(int, lines[0].split()[1:]))
    assert sizes == [ctypes.sizeof(A.CtsTask), ctypes.sizeof(A.CtsPatternConfig), ctypes.sizeof(A.CtsPatternStats),
                     ctypes.sizeof(A.CtsStatusDetails)]
    structs = {"buffer": A.CtsTask, "buffer_length": A.CtsTask, "expected_pattern_offset": A.CtsTask,
               "io_action": A.CtsTask, "track_io": A.CtsTask, "transfer_size": A.CtsPatternConfig,
               "random_seed": A.CtsPatternConfig, "verify_mode": A.CtsPatternConfig,
               "batch_bytes": A.CtsPatternConfig, "recv_pattern_offset": A.CtsPatternStats,
               "fail_expected": A.CtsPatternStats, "fail_completion": A.CtsPatternStats,
               "bytes_recv_held": A.CtsPatternStats, "verify_wait_ns": A.CtsPatternStats,
               "deferred_depth": A.CtsPatternStats}
    for line in lines[1:]:
        if not line.strip():
            continue
        f, off = line.split()
        assert getattr(structs[f], f).offset == int(off), f


def test_media_stream_struct_layouts_match_c():
    import ctypes
    import tempfile

    from ctstraffic_amd import media_stream as M
    from ctstraffic_amd.types import DGRAM_HEADER_DTYPE, DGRAM_RECORD_DTYPE

    probe = r"""
#include <stdio.h>
#include <stddef.h>
#include "cts_media_stream.h"
int main(void){
 printf("%zu %zu %zu %zu\n", sizeof(cts_datagram_record), sizeof(cts_datagram_header),
        sizeof(cts_media_stream_settings), sizeof(cts_media_stream_stats));
 printf("%zu %zu %zu %zu\n", offsetof(cts_datagram_record,flag), offsetof(cts_datagram_record,kind),
        offsetof(cts_datagram_record,completed_bytes), offsetof(cts_media_stream_stats,head_sequence_number));
 return 0; }
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(probe)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-std=c11", "-I", INCLUDE, c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    a = list(map(int, lines[0].split()))
    b = list(map(int, lines[1].split()))
    assert a == [DGRAM_RECORD_DTYPE.itemsize, DGRAM_HEADER_DTYPE.itemsize, ctypes.sizeof(M.Settings),
                 ctypes.sizeof(M.Stats)]
    assert b == [DGRAM_RECORD_DTYPE.fields["flag"][1], DGRAM_RECORD_DTYPE.fields["kind"][1],
                 DGRAM_RECORD_DTYPE.fields["completed_bytes"][1], M.Stats.head_sequence_number.offset]
    assert DGRAM_RECORD_DTYPE == oracle.DGRAM_RECORD_DTYPE


def test_shard_of_matches_workload_sharding():
    """cts_shard_of (the C ABI's connection -> GPU map) is workload.shard_of: fmix32(conn) mod G."""
    import numpy as np

    from ctstraffic_amd import _lib
    from ctstraffic_amd import workload as W

    conns = np.concatenate([np.arange(5000), np.array([2**31 - 1, 2**31, 2**32 - 1])]).astype(np.uint32)
    for g in (1, 2, 3, 4, 8):
        want = W.shard_of(conns, g)
        got = np.array([_lib.lib().cts_shard_of(int(c), g) for c in conns])
        assert np.array_equal(got, want), g
    assert _lib.lib().cts_shard_of(12345, 0) == 0


def test_engine_stream_create_rejects_null():
    import ctypes

    from ctstraffic_amd import _lib

    s = ctypes.c_void_p()
    assert _lib.lib().cts_engine_stream_create(None, ctypes.byref(s)) == _lib.CTS_E_INVALID
    assert _lib.lib().cts_engine_stream_destroy(None, None) == _lib.CTS_E_INVALID


def test_python_handle_refuses_short_output_buffers():
    """The ABI cannot see buffer sizes; the Python handle checks them before any launch (no device needed)."""
    import numpy as np
    import pytest

    from ctstraffic_amd import engine as E
    from ctstraffic_amd.types import RESULT_DTYPE

    with pytest.raises(ValueError):
        E._check_outputs(10, np.zeros(9 * RESULT_DTYPE.itemsize, np.uint8), None)
    with pytest.raises(ValueError):
        E._check_outputs(1, None, np.zeros(8, np.uint8))
    E._check_outputs(10, np.zeros(10 * RESULT_DTYPE.itemsize, np.uint8), np.zeros(64 * 64, np.uint8))


def _kernels(path):
    import re

    blob = open(path, "rb").read()
    return set(m.decode() for m in re.findall(rb"_ZN3cts\d+[a-z_]+kernel[A-Za-z0-9_]*\.kd", blob))


def test_product_library_carries_only_the_default_kernels():
    """The .so compiles one kernel per path (verify 25, small-buffer 15, MediaStream 3, the fills: the 64 KiB fill in
    piece order when a length hint is given, one workgroup or wave per buffer otherwise), each for
    nontemporal and plain loads, the small-buffer and MediaStream kernels' strided-ring forms, the MediaStream
    compact-status and frame-sum forms (descriptors and strided ring), the MediaStream fills (descriptors, and the ring
    for strides from 1024 and below it) for plain and nontemporal stores, the SYNC mailbox grid and the counter fold of
    cts_counters_allreduce; the alternatives measured on the way are not in the source."""
    from ctstraffic_amd import _lib

    prod = _kernels(_lib.LIB_PATH)
    wg = sorted(k for k in prod if "verify_wg_kernel" in k)
    assert wg == ["_ZN3cts16verify_wg_kernelILb%dEEEvPKhmPK12cts_buf_descjP17cts_verify_resultPmPjj.kd" % nt
                  for nt in (0, 1)]
    assert not any("verify_wave" in k or "_nb_" in k for k in prod)
    assert len(prod) == 33, sorted(prod)
    assert sorted(k for k in prod if "fill_pieces_kernel" in k) == [
        "_ZN3cts18fill_pieces_kernelILb%dELj8192ELi16EEEvPhmPK12cts_buf_descjj.kd" % nts for nts in (0, 1)]
    assert any("mailbox_kernel" in k for k in prod) and any("counters_fold_kernel" in k for k in prod)
