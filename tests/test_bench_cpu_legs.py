"""bench.py's CPU legs beside the datagram numbers (run here on the CPU: they use the oracle only, no GPU):
- cpu_baseline.config3: the oracle's VerifyBuffer (skip 26, expected 0; ctsIOPatternMediaStream.cpp:185-192) over a
  slice of the config-3 ring built in host memory, counters equal to the corruption plan's;
- cpu_baseline.loopback_media_stream_oracle: the MediaStream loopback run with the oracle as every client's
  VerifyBuffer, per datagram on the receive thread (the reference's arrangement)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from ctstraffic_amd import workload as W  # noqa: E402


def test_cpu_baseline_config3_slice_matches_plan():
    r = bench.cpu_baseline_config3(W, 0.05, n_datagrams=1 << 14, ring=1 << 18)
    assert r["counters_match_expected"] is True
    assert r["unit"] == "GiB/s of payload" and r["kind"] == "port"
    assert set(r["threads_GiBps"]) >= {"1"} and r["value"] > 0


def test_loopback_media_stream_oracle_leg():
    r = bench.loopback_media_stream_oracle()
    assert "error" not in r, r
    assert r["connections_ok"] == 16 and r["data_errors"] == 0
    assert r["successful_frames"] + r["dropped_frames"] == 16 * 240
    assert r["recv_cpu_us_per_datagram"] > 0


def test_cpu_baseline_labels_the_configs_it_times():
    """BASELINE.md promises the full config set or a labelled subset: the line names what the CPU legs time."""
    import torch

    w = W.tcp_resident(n_buffers=64)
    arena = torch.zeros(w.arena_bytes, dtype=torch.uint8)
    r = bench.cpu_baseline(arena, w, 0.02, loopback=False)
    assert r["configs_timed"] == ["config1-loopback", "config2", "config3-slice(1/16)"]
    assert "configs 4 and 5" in r["configs_note"]
    assert r["kind"] == "port" and r["value"] > 0
