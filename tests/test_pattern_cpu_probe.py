"""tools/pattern_cpu_probe: Push server patterns driven from C++ through the C ABI (no sockets), several connections at
once, one thread each. On the GPU every 64 KiB completion is verified (SYNC through the mailbox, DEFERRED in
double-buffered half batches whose retire sleeps between event queries), and each connection must complete with all
of its buffers verified."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "pattern_cpu_probe")


def test_probe_is_built():
    assert os.access(PROBE, os.X_OK), "make tools/pattern_cpu_probe"


@pytest.mark.gpu
@pytest.mark.parametrize("mode,batch,wait", [("sync", 0, "2"), ("deferred", 64, "2"), ("deferred", 1024, "2"),
                                             ("deferred", 1024, "1"), ("deferred", 1024, "0"), ("off", 0, "2")])
def test_probe_connections_complete(mode, batch, wait):
    threads = 4
    env = dict(os.environ, CTS_DEFERRED_BLOCKING_SYNC=wait)
    out = subprocess.run([PROBE, mode, "1", str(batch), str(threads)], capture_output=True, text=True, timeout=100,
                         env=env)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["status"] == 1 and d["last_error"] == 0  # CTS_IO_COMPLETED on every connection
    assert d["recvs"] == threads * 16384
    assert d["buffers_verified"] == (0 if mode == "off" else threads * 16384)
    assert d["complete_cpu_s_per_GiB"] > 0
