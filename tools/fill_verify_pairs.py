#!/usr/bin/env python3
"""Config 2's "fill+verify" pairs alone, for rocprofv3 PMC passes (profiles/r06/fill_verify/).

bench.py's extras time the pair as: fill arena i, then verify arena i + R/2 (filled R/2 pairs earlier, so its
lines have left the 256 MB Infinity Cache), beside the same-arena pair whose verify reads what the fill just wrote.
This runs only those launches (no headline leg), so a `--pmc FETCH_SIZE` or `--pmc WRITE_SIZE` pass over it gives
each kernel's HBM bytes per launch in each arrangement: the first `--pairs` dispatches of each kernel are the
rotated pairs, the next `--pairs` the same-arena ones. Prints one JSON line with the HIP-event times.

usage: python tools/fill_verify_pairs.py [--pairs 64] [--arenas 8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--arenas", type=int, default=8)
    a = ap.parse_args()
    import torch

    from ctstraffic_amd import Engine, workload as W

    R, P = a.arenas, a.pairs
    with Engine(0) as e:
        w = W.tcp_resident()
        arenas, descs = [], None
        for _ in range(R):
            ar, descs = W.materialize(e, w)
            arenas.append(ar)
        ctr = e.new_counters()
        nbytes = w.verified_bytes()

        def pairs(shift):
            s = torch.cuda.current_stream()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record(s)
            for i in range(P):
                e.fill(arenas[i % R], descs, max_length_hint=w.max_length)
                e.verify(arenas[(i + shift) % R], descs, max_length_hint=w.max_length, counters=ctr)
            t1.record(s)
            torch.cuda.synchronize()
            return t0.elapsed_time(t1) / 1e3 / P

        torch.cuda.synchronize()
        t_rot = pairs(R // 2)
        t_same = pairs(0)
        print(json.dumps({"pairs": P, "arenas": R, "arena_bytes": nbytes,
                          "rotated_us_per_pair": round(t_rot * 1e6, 2),
                          "rotated_GiBps_verified": round(nbytes / t_rot / 2 ** 30, 1),
                          "same_arena_us_per_pair": round(t_same * 1e6, 2),
                          "same_arena_GiBps_verified": round(nbytes / t_same / 2 ** 30, 1)}), flush=True)


if __name__ == "__main__":
    main()
