"""The C ABI from C++ (no Python in the loop): tests/cpp/pattern_replay.cpp replays the reference's
MSTest server scenarios against libcts_engine.so with the oracle's C verifier as the pattern's
hook — the way a maintainer would bind the reference's ctsIoPattern to the engine — and, on the
GPU, the device-resident headline path driven from C++ (tests/cpp/device_verify.cpp)."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_pattern_replay():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "pattern_replay")
        subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tests", "cpp", "pattern_replay.cpp"), "-o", exe,
                        "-L", os.path.join(ROOT, "ctstraffic_amd"), "-lcts_engine",
                        "-L", os.path.join(ROOT, "oracle"), "-lcts_oracle",
                        "-Wl,-rpath," + os.path.join(ROOT, "ctstraffic_amd") + ":" + os.path.join(ROOT, "oracle")],
                       check=True)
        out = subprocess.run([exe], capture_output=True, text=True, timeout=60)
        assert out.returncode == 0, out.stderr
        assert "pattern_replay: ok" in out.stdout


@pytest.mark.gpu
def test_cpp_device_verify():
    """The headline path from C++ (tests/cpp/device_verify.cpp, built by `make`): hipMalloc'd arena, cts_fill,
    corruptions, cts_verify with results + counters + per-connection first failure, all checked in C++."""
    exe = os.path.join(ROOT, "ctstraffic_amd", "build", "device_verify")
    assert os.path.exists(exe), "run `make` (or __graft_entry__.build()) first"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "device_verify: ok" in out.stdout
