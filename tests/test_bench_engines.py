"""bench.py's single-process leg (`--engines N`): one process, one engine per GPU, the timed launches issued from one
native thread per GPU through the C ABI (tools/bench_multi.cpp), counters folded by cts_counters_read_multi.

CPU: the helper library loads next to the engine library and refuses malformed work lists before any GPU call.
GPU: the leg runs with 1 engine and with 2 / 4 engines sharing the one GPU of a test box (--engines-same-gpu), and
its records, first-failure slots and folded counters equal the corruption plan's.
"""
import ctypes
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
_RANK_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")


def test_bench_multi_library_refuses_bad_work_lists():
    sys.path.insert(0, ROOT)
    import bench
    from ctstraffic_amd import lib

    lib()  # the engine library first: the helper binds its cts_verify
    L = bench._bench_multi_lib()
    t0, t1, ts = (ctypes.c_double * 1)(), (ctypes.c_double * 1)(), ctypes.c_double()
    assert L.cts_bench_run_multi(None, 1, 1, t0, t1, ctypes.byref(ts), 1) == -1
    work = (bench._BenchGpu * 1)()
    assert L.cts_bench_run_multi(work, 0, 1, t0, t1, ctypes.byref(ts), 1) == -1
    assert L.cts_bench_run_multi(work, 1, 1, t0, t1, ctypes.byref(ts), 1) == -1  # no arenas / streams


def _run(*argv):
    env = {k: v for k, v in os.environ.items() if k not in _RANK_ENV}
    r = subprocess.run([sys.executable, BENCH, *argv], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("engines", [1, 2, 4])
def test_engines_leg_native_threads(engines):
    # 2048 buffers: two corrupt ones per batch (1/1024), so DataErrors are counted
    argv = ["--engines", str(engines), "--steps", "3", "--warmup", "1", "--arenas", "2", "--buffers", "2048"]
    if engines > 1:
        argv.append("--engines-same-gpu")
    j = _run(*argv)
    p = j["parity"]
    assert p["folded_counters_match_expected"] and p["fold_equals_sum_of_reads"] and p["records_and_first_fail_match"]
    assert j["config"]["engines"] == engines and len(j["per_gpu_GiBps"]) == engines
    assert sum(j["config"]["connections_per_gpu"]) == 2048 * engines
    assert p["counters"]["buffers_checked"] == 2048 * engines * 3 * 2
    assert j["value"] > 0
    # the node's counters over RCCL from the C ABI (every engine on this GPU: one device, one rank) = the host fold
    nc = j["node_counters"]
    assert "allreduce_error" not in nc, nc
    assert p["allreduce_equals_fold"] and nc["allreduce_counters_us"] > 0 and nc["devices"] == [0] * engines
    # the DataError count: the timed launches claim each failed connection once per arena (slots emptied before)
    assert p["counters"]["connections_failed"] > 0
    # the clique was built by cts_counters_allreduce_prepare at start-up, so the first counter read pays no set-up
    st = nc["allreduce_setup_breakdown_ms"]
    assert st["prepared"] == 1 and st["devices"] == 1 and nc["prepare_ms"] > 0
    # the first read after prepare: inside the C ABI (fold, all-reduce, copy back) it is tens of us, as later ones
    ph = nc["allreduce_first_call_phases_us"]
    assert ph["fold_us"] + ph["allreduce_us"] + ph["readback_us"] < 1000, nc
    assert nc["allreduce_first_call_us"] < 50e3, nc
    # the whole first call inside the C ABI (entry to return) holds its three phases
    assert ph["total_us"] == nc["allreduce_first_call_c_abi_us"] >= ph["fold_us"] + ph["allreduce_us"] + ph["readback_us"]
    assert nc["allreduce_first_call_c_abi_us"] < 1000, nc


@pytest.mark.gpu
@pytest.mark.parametrize("launcher", ["native", "python"])
def test_headline_launchers(launcher):
    j = _run("--launcher", launcher, "--steps", "3", "--warmup", "1", "--arenas", "2", "--buffers", "2048",
             "--no-cpu-baseline", "--no-extras", "--no-engines-leg")
    assert j["parity"]["counters_match_expected"] and j["parity"]["records_and_first_fail_match"]
    assert j["config"]["launcher"].startswith(launcher)
    assert j["parity"]["counters"]["buffers_checked"] == 2048 * 3 * 2
    assert j["parity"]["counters"]["connections_failed"] == j["parity"]["connections_failed_expected"] > 0
