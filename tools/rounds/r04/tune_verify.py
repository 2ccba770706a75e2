#!/usr/bin/env python3
"""Interleaved A/B of verify launch variants in ONE process (methodology rule 24).

For each round, every (variant, blocks_per_cu, nt) configuration runs `--launches`
back-to-back verify launches over rotated arenas; the per-launch kernel time comes
from HIP events on the launch stream. Prints a JSON table (median over rounds).
"""
import argparse
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ctstraffic_amd import Engine, _lib, workload as W  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--launches", type=int, default=40)
    p.add_argument("--arenas", type=int, default=8)
    p.add_argument("--variants", default="0,1,2,3,4,5")
    p.add_argument("--bpc", default="4,8,16")
    p.add_argument("--nt", default="1,0")
    p.add_argument("--workload", default="config2")
    p.add_argument("--buffers", type=int, default=4096)
    p.add_argument("--corrupt-rate", type=int, default=1024, help="1 in N buffers corrupted (0 = none)")
    p.add_argument("--results", action="store_true", help="also write the per-buffer result records")
    p.add_argument("--op", default="verify", choices=["verify", "fill"],
                   help="fill: time cts_fill over the same descriptors (write-bound twin)")
    args = p.parse_args()
    torch.cuda.set_device(0)
    eng = Engine(0, tuning=True)  # every launch variant (libcts_engine_tuning.so)
    if args.workload == "config2":
        w = W.tcp_resident(n_buffers=args.buffers, corrupt_rate=args.corrupt_rate)
    else:
        w = W.udp_datagrams(n_datagrams=4 * 1024 * 1024, corrupt_rate=args.corrupt_rate)
    arenas, descs = [], None
    for _ in range(args.arenas):
        a, descs = W.materialize(eng, w)
        arenas.append(a)
    _, _, exp, _ = W.expected_results(w)
    ctr = eng.new_counters()
    res = eng.new_results(w.n) if args.results else None
    s = torch.cuda.current_stream()
    combos = list(itertools.product([int(x) for x in args.variants.split(",")],
                                    [int(x) for x in args.bpc.split(",")],
                                    [int(x) for x in args.nt.split(",")]))
    times = {c: [] for c in combos}
    for r in range(args.rounds):
        for c in combos:
            v, bpc, nt = c
            # the variant list names small-path kernels for config3 (datagrams), else large-path ones
            eng.set_attr(_lib.ATTR_SMALL_VARIANT if args.workload == "config3" else _lib.ATTR_VERIFY_VARIANT, v)
            eng.set_attr(_lib.ATTR_BLOCKS_PER_CU, bpc)
            eng.set_attr(_lib.ATTR_FILL_BLOCKS_PER_CU, bpc)
            eng.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, bpc)
            # (--op fill: the nt dimension is the fill's store policy)
            eng.set_attr(_lib.ATTR_FILL_NT if args.op == "fill" else _lib.ATTR_NT_LOADS, nt)
            eng.reset_counters(ctr)
            # region timing: per-launch event pairs add ~2.5 us to every launch on this stack
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if args.op == "fill":
                eng.fill(arenas[0], descs, max_length_hint=w.max_length)
                ea.record(s)
                for i in range(args.launches - 1):
                    eng.fill(arenas[(i + 1) % len(arenas)], descs, max_length_hint=w.max_length)
                eb.record(s)
                torch.cuda.synchronize()
            else:
                eng.verify(arenas[0], descs, max_length_hint=w.max_length, counters=ctr, results=res)
                ea.record(s)
                for i in range(args.launches - 1):
                    eng.verify(arenas[(i + 1) % len(arenas)], descs, max_length_hint=w.max_length, counters=ctr,
                               results=res)
                eb.record(s)
                torch.cuda.synchronize()
                got = eng.read_counters(ctr)
                assert got == {k: v_ * args.launches for k, v_ in exp.items()}, (c, got)
            times[c].append(ea.elapsed_time(eb) / (args.launches - 1))
    nbytes = w.verified_bytes()
    rows = []
    for c in combos:
        t = float(np.median(times[c])) / 1e3
        rows.append({"variant": c[0], "blocks_per_cu": c[1], "nt": c[2], "us": round(t * 1e6, 2),
                     "GBps": round(nbytes / t / 1e9, 1), "spread_us": round((max(times[c]) - min(times[c])) * 1e3, 2)})
    rows.sort(key=lambda x: x["us"])
    print(json.dumps({"workload": w.name, "op": args.op, "bytes": nbytes, "results": bool(args.results), "rows": rows}, indent=0))


if __name__ == "__main__":
    main()
