#!/usr/bin/env python3
"""Where does cts_fill's time go on config-2 descriptors? A/B in one process: the config-2 descriptor
list (75 % even phase, 25 % random), the same list with every phase 0, and with every phase odd; one
JSON line per case (us per 256 MiB launch, 4 arenas rotated)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ctstraffic_amd import Engine, workload as W  # noqa: E402
from ctstraffic_amd.engine import descs_to_device  # noqa: E402


def main():
    eng = Engine(0)
    w = W.tcp_resident()
    arenas = [torch.zeros(w.arena_bytes, dtype=torch.uint8, device="cuda") for _ in range(4)]
    cases = {"config2": w.descs.copy()}
    d0 = w.descs.copy()
    d0["expected_pattern_offset"] = 0
    cases["all_phase0"] = d0
    d1 = w.descs.copy()
    d1["expected_pattern_offset"] = 1
    cases["all_odd"] = d1
    d2 = w.descs.copy()
    d2["expected_pattern_offset"] = 2
    cases["all_phase2"] = d2
    dev = {k: descs_to_device(v, "cuda") for k, v in cases.items()}
    s = torch.cuda.current_stream()
    for rnd in range(3):
        for name, dd in dev.items():
            eng.fill(arenas[0], dd, max_length_hint=65536)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for i in range(40):
                eng.fill(arenas[i % 4], dd, max_length_hint=65536)
            b.record(s)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / 40
            print(json.dumps({"round": rnd, "case": name, "us": round(us, 2),
                              "GBps": round(w.arena_bytes / us / 1e3, 1)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
