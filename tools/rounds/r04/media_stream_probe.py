#!/usr/bin/env python3
"""Where does MediaStream receive time go? Interleaved A/B in one process over config-3-shaped
datagrams (4 M x 1472 B by default): plain datagram verify with/without per-datagram results,
and cts_media_stream_verify with/without records and results, for each small-path variant
given. Prints one JSON line per (case, round).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ctstraffic_amd import Engine, _lib, media_stream as MS, workload as W  # noqa: E402
from ctstraffic_amd.types import DGRAM_HEADER_DTYPE  # noqa: E402


def _with_attr(eng, attr, value, fn):
    old = eng.get_attr(attr)
    eng.set_attr(attr, value)
    try:
        fn()
    finally:
        eng.set_attr(attr, old)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--datagrams", type=int, default=4 * 1024 * 1024)
    p.add_argument("--launches", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--ms-variants", default="", help="comma list of ATTR_MS_VARIANT values to A/B")
    p.add_argument("--small-variants", default="", help="comma list of ATTR_SMALL_VARIANT values to A/B")
    p.add_argument("--chunks", default="", help="comma list of ATTR_SMALL_CHUNK values (chunked walks)")
    p.add_argument("--arenas", type=int, default=4)
    p.add_argument("--only", default="", help="comma list of case names to run (default: all)")
    args = p.parse_args()
    torch.cuda.set_device(0)
    eng = Engine(0, tuning=True)  # every launch variant (libcts_engine_tuning.so)
    w = W.udp_datagrams(n_datagrams=args.datagrams)
    arenas = []
    for _ in range(args.arenas):
        a, d = W.materialize(eng, w)
        arenas.append(a)
    lens = torch.from_numpy(w.descs["length"].astype("uint32")).cuda()
    recs = torch.empty(w.n * 32, dtype=torch.uint8, device="cuda")
    st = torch.empty(w.n * 16, dtype=torch.uint8, device="cuda")
    res = eng.new_results(w.n)
    ctr = eng.new_counters()
    s = torch.cuda.current_stream()
    msv = [int(x) for x in args.ms_variants.split(",") if x] or [None]
    svs = [int(x) for x in args.small_variants.split(",") if x] or [None]
    chunks = [int(x) for x in args.chunks.split(",") if x] or [None]
    only = set(x for x in args.only.split(",") if x)
    cases = []
    for ch in chunks:
        for sv in svs:
            cases += [("verify", ("small", sv, ch),
                       lambda a: eng.verify(a, d, max_length_hint=w.max_length, counters=ctr)),
                      ("verify+results", ("small", sv, ch),
                       lambda a: eng.verify(a, d, max_length_hint=w.max_length, counters=ctr, results=res))]
        for v in msv:
            cases += [("ms", ("ms", v, ch), lambda a: MS.verify(eng, a, d)),
                      ("ms+results", ("ms", v, ch), lambda a: MS.verify(eng, a, d, results=res)),
                      ("ms+records", ("ms", v, ch), lambda a: MS.verify(eng, a, d, records=recs)),
                      ("ms+records+results", ("ms", v, ch),
                       lambda a: MS.verify(eng, a, d, records=recs, results=res))]
        # the receive ring's descriptor-free form (datagram i at i * 1472, lengths only; windowed kernel)
        cases += [("ms_strided+records+results", ("ms", 3, ch),
                   lambda a: MS.verify_strided(eng, a, w.max_length, lens, records=recs, results=res))]
        # the compact receive pass (16-byte statuses), descriptors and strided ring
        # the bare datagram verify over the strided ring (the small path's product kernel)
        cases += [("verify_strided", ("small", None, ch),
                   lambda a: eng.verify_strided(a, w.max_length, lens, skip_head=26, expected_offset=0,
                                                counters=ctr))]
        # the compact receive over the strided ring for every MediaStream variant asked for (3 = product;
        # 12 = its header / edge loads nontemporal, round 2)
        for v in msv:
            if v is not None:
                cases += [("ms_strided+status_v%d" % v, ("ms", v, ch),
                           lambda a: MS.verify_strided_status(eng, a, w.max_length, lens, status=st))]
        # the receive pass with the frame accounting summed on the GPU (a 10-frame window from sequence number 1)
        win = MS.FrameWindow(1, w.n, 10, 0)
        sums = MS.FrameSums(win.frames)
        cases += [("ms+frames", ("ms", 3, ch), lambda a: MS.verify_frames(eng, a, d, win, sums)),
                  ("ms_strided+frames", ("ms", 3, ch),
                   lambda a: MS.verify_strided_frames(eng, a, w.max_length, lens, win, sums))]
        cases += [("ms+status", ("ms", 3, ch), lambda a: MS.verify_status(eng, a, d, status=st)),
                  ("ms+status_two_pass", ("ms", 7, ch), lambda a: MS.verify_status(eng, a, d, status=st)),
                  ("ms+status_every_round", ("ms", 8, ch), lambda a: MS.verify_status(eng, a, d, status=st)),
                  ("ms+status_ring16", ("ms", 9, ch), lambda a: MS.verify_status(eng, a, d, status=st)),
                  ("ms+status_ring32", ("ms", 10, ch), lambda a: MS.verify_status(eng, a, d, status=st)),
                  ("ms_strided+status", ("ms", 3, ch),
                   lambda a: MS.verify_strided_status(eng, a, w.max_length, lens, status=st))]
    # the sender side: the payload fill of the same descriptors (skip 26: header bytes untouched) and the whole-
    # datagram fill (header + payload, cts_media_stream_fill); "GBps_written" counts the bytes each writes
    hdr = np.zeros(w.n, dtype=DGRAM_HEADER_DTYPE)
    hdr["sequence_number"] = np.arange(1, w.n + 1)
    hdr_d = torch.from_numpy(hdr.view(np.uint8)).cuda()
    cases += [("fill_payload", ("small", None, None), lambda a: eng.fill(a, d, max_length_hint=w.max_length)),
              ("ms_fill", ("ms", None, None), lambda a: MS.fill(eng, a, d, hdr_d)),
              ("ms_fill_strided", ("ms", None, None), lambda a: MS.fill_strided(eng, a, w.max_length, lens, hdr_d)),
              ("ms_fill_plain", ("ms", None, None), lambda a: _with_attr(eng, _lib.ATTR_FILL_NT, 0,
                                                                         lambda: MS.fill(eng, a, d, hdr_d))),
              ("fill_payload_plain", ("small", None, None), lambda a: _with_attr(
                  eng, _lib.ATTR_FILL_NT, 0, lambda: eng.fill(a, d, max_length_hint=w.max_length)))]
    written = {"fill_payload": w.verified_bytes(), "ms_fill": w.arena_bytes, "ms_fill_strided": w.arena_bytes, "ms_fill_plain": w.arena_bytes,
               "fill_payload_plain": w.verified_bytes()}
    cases = [c for c in cases if not only or c[0] in only]
    for r in range(args.rounds):
        for name, v, fn in cases:
            kind, var, ch = v
            if var is not None:
                eng.set_attr(_lib.ATTR_SMALL_VARIANT if kind == "small" else _lib.ATTR_MS_VARIANT, var)
            if ch is not None:
                eng.set_attr(_lib.ATTR_SMALL_CHUNK, ch)
            fn(arenas[0])
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ea.record(s)
            for i in range(args.launches):
                fn(arenas[(i + 1) % len(arenas)])
            eb.record(s)
            torch.cuda.synchronize()
            us = ea.elapsed_time(eb) * 1e3 / args.launches
            print(json.dumps({"round": r, "case": name, "variant": v, "us": round(us, 1),
                              "GBps_payload": round(w.verified_bytes() / us / 1e3, 1),
                              "Mdgram_per_s": round(w.n / us, 1),
                              **({"GBps_written": round(written[name] / us / 1e3, 1)} if name in written else {})}),
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
