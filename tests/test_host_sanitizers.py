"""Host C++ under sanitizers (the reference has none; "ASan/UBSan on host code").

The host half of the engine — the ctsIoPattern mirror (cts_pattern.cpp), MediaStream framing and
client accounting (cts_media_stream.cpp), status output (cts_status.cpp) and the loopback feeder
with its sync and async functors (cts_loopback.cpp) — is built from source with g++ against
link-time fakes of the device entry points (tests/cpp/engine_stub.cpp), with the oracle's C
verifier as every pattern's hook. Two builds run the MSTest replay (tests/cpp/pattern_replay.cpp),
whole loopback connections of every TCP pattern (tests/cpp/loopback_stress.cpp) and the MediaStream
client fed per datagram, by statuses and by GPU-style frame sums over random streams, several clients
on threads at once feeding the process-wide UDP counters (tests/cpp/media_stream_client.cpp):
AddressSanitizer + UndefinedBehaviorSanitizer, and ThreadSanitizer (the async functor's send and
recv threads share one pattern under the connection lock). Any report fails the test.
"""
import concurrent.futures
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_SRCS = ["cts_pattern.cpp", "cts_media_stream.cpp", "cts_status.cpp", "cts_loopback.cpp", "cts_loopback_udp.cpp",
             "cts_host_util.cpp", "cts_collective.cpp"]
SAN = {
    "plain": [],
    "asan-ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
    "tsan": ["-fsanitize=thread"],
}
ENV = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:exitcode=23",
       "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1:exitcode=24",
       "TSAN_OPTIONS": "halt_on_error=1:exitcode=25"}


def _build(d, san, driver, extra_link=()):
    flags = ["-g", "-O1", "-fno-omit-frame-pointer", "-pthread"] + SAN[san]
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "ctstraffic_amd", "csrc"),
           "-I", os.path.join(ROOT, "oracle"), "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
    objs = []
    for src in [os.path.join(ROOT, "ctstraffic_amd", "csrc", s) for s in HOST_SRCS] + [
            os.path.join(ROOT, "tests", "cpp", "engine_stub.cpp"), os.path.join(ROOT, "tests", "cpp", driver)]:
        o = os.path.join(d, os.path.basename(src) + ".o")
        subprocess.run(["g++", "-std=c++17", *flags, *inc, "-c", src, "-o", o], check=True)
        objs.append(o)
    o = os.path.join(d, "cts_oracle.o")
    subprocess.run(["gcc", "-std=c11", *flags, "-I", os.path.join(ROOT, "oracle"), "-c",
                    os.path.join(ROOT, "oracle", "cts_oracle.c"), "-o", o], check=True)
    objs.append(o)
    exe = os.path.join(d, driver[:-4])
    subprocess.run(["g++", *flags, *objs, "-o", exe, *extra_link, "-ldl"], check=True)
    return exe


def _build_rccl_stub(d, san):
    """tests/cpp/rccl_stub.cpp as the shared library cts_counters_allreduce loads ($CTS_RCCL_LIBRARY)."""
    so = os.path.join(d, "librccl_stub.so")
    subprocess.run(["g++", "-std=c++17", "-g", "-O1", "-fPIC", "-shared", "-pthread", *SAN[san], "-I", "/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "tests", "cpp", "rccl_stub.cpp"), "-o", so], check=True)
    return so


@pytest.mark.parametrize("san", sorted(set(SAN) - {"plain"}))
@pytest.mark.parametrize("driver", ["pattern_replay.cpp", "loopback_stress.cpp", "slices_check.cpp",
                                    "counters_fold.cpp", "media_stream_client.cpp",
                                    "media_stream_pattern.cpp"])
def test_host_code_under_sanitizer(san, driver):
    with tempfile.TemporaryDirectory() as d:
        exe = _build(d, san, driver)
        # counters_fold also drives cts_counters_allreduce against a stub RCCL (tests/cpp/rccl_stub.cpp)
        args = [_build_rccl_stub(d, san)] if driver == "counters_fold.cpp" else []
        out = subprocess.run([exe, *args], capture_output=True, text=True, timeout=300, env={**os.environ, **ENV})
        assert out.returncode == 0, (out.returncode, out.stderr[-4000:])
        assert ": ok" in out.stdout
        assert "runtime error" not in out.stderr and "WARNING: ThreadSanitizer" not in out.stderr, out.stderr[-4000:]


@pytest.mark.parametrize("san", sorted(set(SAN) - {"plain"}))
def test_engine_abi_on_eight_fake_devices(san):
    """The engine's C ABI (cts_engine.cpp) and the host half above it on a fake eight-device HIP runtime
    (tests/cpp/engine_devices.cpp): engines on devices 0-7 plus a second one on device 5, driven from threads whose own
    device differs, one after the other and all at once; then whole loopback TCP connections (Push, Pull, PushPull,
    Duplex on the async functor; SYNC and DEFERRED; clean and corrupt) spread over the eight engines from feeder
    threads that start on device 0; then MediaStream connections (SYNC, and DEFERRED through an emulated frame-sum
    pass) on device 6 with the client timer thread on device 0; then cts_counters_allreduce_prepare and
    cts_counters_allreduce_ex over the nine engines (a stub RCCL, tests/cpp/rccl_stub.cpp) against the host fold and
    the oracle's sums, the DataError count (connections_failed) included; then bench.py's
    single-process leg at eight GPUs (tools/bench_multi.cpp: one native launch thread per engine); then a DEFERRED
    pattern destroyed under a launch that has not finished, and one whose own final flush is late (bounded:
    CTS_E_TIMEOUT, the pattern kept until a second destroy). Every stream-ordered HIP call and launch must run with
    its engine's device current, every event must be recorded on a stream of its own device, the caller's device must
    be current again afterwards, and no pinned free may run while a SYNC mailbox grid (emulated by a host thread that
    polls the slot rings as mailbox_kernel does) is resident on the current device: hipHostFree is an implicit
    hipDeviceSynchronize. Launches compute with the oracle, so verdicts are checked too. The one-GPU test box never
    runs an engine on a device other than 0."""
    flags = ["-g", "-O1", "-fno-omit-frame-pointer", "-pthread"] + SAN[san]
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "ctstraffic_amd", "csrc"),
           "-I", os.path.join(ROOT, "oracle"), "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"]
    srcs = [os.path.join(ROOT, "ctstraffic_amd", "csrc", x) for x in (
        "cts_engine.cpp", "cts_host_util.cpp", "cts_pattern.cpp", "cts_media_stream.cpp", "cts_status.cpp",
        "cts_loopback.cpp", "cts_loopback_udp.cpp", "cts_collective.cpp")] + [
        os.path.join(ROOT, "tests", "cpp", "engine_devices.cpp"), os.path.join(ROOT, "tools", "bench_multi.cpp")]
    with tempfile.TemporaryDirectory() as d:
        objs = [os.path.join(d, os.path.basename(src) + ".o") for src in srcs]
        with concurrent.futures.ThreadPoolExecutor(4) as pool:  # (the pattern mirror alone takes ~30 s under a sanitizer)
            for f in [pool.submit(subprocess.run, ["g++", "-std=c++17", *flags, *inc, "-c", src, "-o", o], check=True)
                      for src, o in zip(srcs, objs)]:
                f.result()
        o = os.path.join(d, "cts_oracle.o")
        subprocess.run(["gcc", "-std=c11", *flags, "-I", os.path.join(ROOT, "oracle"), "-c",
                        os.path.join(ROOT, "oracle", "cts_oracle.c"), "-o", o], check=True)
        objs.append(o)
        exe = os.path.join(d, "engine_devices")
        subprocess.run(["g++", *flags, *objs, "-o", exe, "-ldl"], check=True)
        out = subprocess.run([exe, _build_rccl_stub(d, san)], capture_output=True, text=True, timeout=300,
                             env={**os.environ, **ENV})
        assert out.returncode == 0, (out.returncode, out.stdout[-2000:], out.stderr[-4000:])
        assert "engine_devices: ok" in out.stdout and "violation" not in out.stderr
        assert "equal to the host fold and the oracle" in out.stdout and "bench_multi: 8 GPUs" in out.stdout
        assert "destroy under a hung launch: CTS_E_TIMEOUT" in out.stdout
        assert "destroy whose own flush is late: CTS_E_TIMEOUT" in out.stdout
        assert "runtime error" not in out.stderr and "WARNING: ThreadSanitizer" not in out.stderr, out.stderr[-4000:]


def test_thread_start_failure_never_crosses_the_abi():
    """Every host thread start (the MediaStream client's timer thread, the TCP and UDP feeders' side threads) fails
    on demand through a pthread_create interposer (tests/cpp/thread_start_failure.cpp): the client latches a
    FAIL_FAST with no timer left armed, the feeders fail those connections and return, and no std::system_error
    reaches std::terminate. Built without a sanitizer (they intercept pthread_create themselves)."""
    with tempfile.TemporaryDirectory() as d:
        exe = _build(d, "plain", "thread_start_failure.cpp", extra_link=("-rdynamic", "-ldl"))
        out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, (out.returncode, out.stderr[-4000:])
        assert ": ok" in out.stdout
