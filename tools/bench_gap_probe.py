#!/usr/bin/env python3
"""How much of a config-2 step is launch gap? Times K verify launches over rotated
arenas three ways in ONE process, interleaved over rounds:
  events   : an event pair around every launch (what bench.py r01 did)
  plain    : back-to-back launches, events only around the region
  graph    : a HIP graph (torch.cuda.graph capture) of R launches, replayed K/R times
Prints one JSON line per (mode, round) plus a summary.
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ctstraffic_amd import Engine, workload as W  # noqa: E402


def main():
    K, R, rounds = 200, 8, 3
    torch.cuda.set_device(0)
    eng = Engine(0)
    w = W.tcp_resident(n_buffers=4096)
    arenas, descs = [], None
    for _ in range(R):
        a, descs = W.materialize(eng, w)
        arenas.append(a)
    ctr = eng.new_counters()
    s = torch.cuda.Stream()
    nbytes = w.verified_bytes()

    def launch(i):
        eng.verify(arenas[i % R], descs, max_length_hint=w.max_length, counters=ctr, stream=s)

    with torch.cuda.stream(s):
        for i in range(2 * R):
            launch(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(R):
            launch(i)
    torch.cuda.synchronize()

    res = {"events": [], "plain": [], "graph": []}
    for rnd in range(rounds):
        for mode in res:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            per = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            a.record(s)
            if mode == "events":
                for i in range(K):
                    per[i][0].record(s)
                    launch(i)
                    per[i][1].record(s)
            elif mode == "plain":
                for i in range(K):
                    launch(i)
            else:
                for _ in range(K // R):
                    g.replay()
            b.record(s)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            region_us = a.elapsed_time(b) * 1e3 / K
            line = {"mode": mode, "round": rnd, "region_us_per_step": round(region_us, 2),
                    "wall_us_per_step": round(wall / K * 1e6, 2), "GBps_region": round(nbytes / region_us / 1e3, 1)}
            if mode == "events":
                line["per_launch_us"] = round(float(np.mean([x.elapsed_time(y) for x, y in per])) * 1e3, 2)
            res[mode].append(line)
            print(json.dumps(line), flush=True)
    print(json.dumps({m: float(np.median([x["region_us_per_step"] for x in v])) for m, v in res.items()}))


if __name__ == "__main__":
    main()
