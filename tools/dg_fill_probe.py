#!/usr/bin/env python3
"""Is config 3's payload-only fill (cts_fill on 16 M x 1472 B slots, skip 26: 4.26 TB/s of payload) bound by its
partially written first line? One process, the datagram path (hint 1472, a wave per buffer), the same 1472-B slots
with the payload starting at byte 0 / 26 / 32 / 64 of the slot, and the skip-26 bytes described as a 1446-B buffer
at slot + 26 (the same bytes, no skip). HBM3E has no byte-write mask, so a store that leaves part of a 64-B sector
unwritten costs the memory controller a read-modify-write of that sector. One JSON line per case and round: us per
launch and GB/s of bytes written. Diagnostic only.
    usage: python tools/dg_fill_probe.py [datagrams]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ctstraffic_amd import Engine  # noqa: E402
from ctstraffic_amd.engine import descs_to_device  # noqa: E402
from ctstraffic_amd.types import DESC_DTYPE  # noqa: E402

STRIDE = 1472


def descs(n, skip, at=0):
    d = np.zeros(n, dtype=DESC_DTYPE)
    d["byte_offset"] = np.arange(n, dtype=np.uint64) * STRIDE + at
    d["length"] = STRIDE - at
    d["skip_head"] = skip
    d["conn_index"] = np.arange(n, dtype=np.uint32)
    return d


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16 << 20
    eng = Engine(0)
    arena = torch.zeros(n * STRIDE, dtype=torch.uint8, device="cuda")
    cases = {"skip0_whole_slot": descs(n, 0), "skip26_payload": descs(n, 26), "skip32": descs(n, 32),
             "skip64_sector_aligned": descs(n, 64), "at26_len1446_noskip": descs(n, 0, at=26)}
    dev = {k: descs_to_device(v, "cuda") for k, v in cases.items()}
    written = {k: int((v["length"].astype(np.int64) - v["skip_head"]).sum()) for k, v in cases.items()}
    s = torch.cuda.current_stream()
    for rnd in range(3):
        for name, dd in dev.items():
            eng.fill(arena, dd, max_length_hint=STRIDE)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(5):
                eng.fill(arena, dd, max_length_hint=STRIDE)
            b.record(s)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / 5
            print(json.dumps({"round": rnd, "case": name, "datagrams": n, "bytes_written": written[name],
                              "us": round(us, 1), "GBps_written": round(written[name] / us / 1e3, 1)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
