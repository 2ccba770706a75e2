#!/usr/bin/env python3
"""Config 1 (loopback TCP push, 8 connections x 1 GiB, 64 KiB IO) with GPU DEFERRED verify at 1, 2 and 3 batches in
flight per connection (CTS_DEFERRED_DEPTH, read when a pattern is made), beside verify off, legs rotated over rounds in
one process. Each launch holds batch / (depth + 1) buffers, so the ring and the verdict bound stay the
same. One JSON line per leg and round: GB/s received, receive-thread CPU per GiB, and the verdict waits
(cts_pattern_stats.verify_wait_ns summed over the receiving sides) per GiB.
usage: python tools/deferred_depth_ab.py [rounds] [batch_buffers] [legs, e.g. off,1,2 or 2@512,2@1024]
(a leg "d@b" runs depth d at batch b; "ring" / "ringpinned" run verify off with every data recv landing round robin in
a ring the size of a DEFERRED pattern's at that batch, 2 x batch + 2 buffers, pageable / pinned: the feeder's
diagnostic recv ring)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ctstraffic_amd import Engine, _pattern_abi as PA, loopback as LB  # noqa: E402
from ctstraffic_amd.pattern import shared_buffer_init  # noqa: E402

GIB = float(1 << 30)


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    eng = Engine(0)
    shared_buffer_init(eng, 65536)
    legs = sys.argv[3].split(",") if len(sys.argv) > 3 else ["off", "1", "2", "3"]
    for r in range(rounds):
        for leg in legs[r % len(legs):] + legs[:r % len(legs)]:
            if leg == "off":
                res = LB.run(connections=8, buffer_size=65536, transfer_size=1 << 30, verify=False)
                wait = 0.0
            elif leg in ("ring", "ringpinned"):
                slots = 2 * (batch or 512) + 2  # the DEFERRED ring: 2 x batch + PrePostRecvs + 1
                res = LB.run(connections=8, buffer_size=65536, transfer_size=1 << 30, verify=False, engine=eng,
                             recv_ring_buffers=slots, recv_ring_pinned=leg == "ringpinned")
                wait = 0.0
            else:
                depth, _, b = leg.partition("@")
                os.environ["CTS_DEFERRED_DEPTH"] = depth
                try:
                    res = LB.run(connections=8, buffer_size=65536, transfer_size=1 << 30, engine=eng,
                                 verify_mode=PA.VERIFY_DEFERRED, batch_buffers=int(b) if b else batch, sides=True)
                finally:
                    os.environ.pop("CTS_DEFERRED_DEPTH", None)
                wait = sum(sd["verify_wait_ns"] for sd in res["sides"]) * 1e-9
            name = {"off": "verify_off", "ring": "verify_off_ring", "ringpinned": "verify_off_pinned_ring"}.get(
                leg, "deferred_depth_" + leg)
            print(json.dumps({"round": r, "leg": name,
                              "batch_buffers": batch if "@" not in leg else int(leg.partition("@")[2]), "GBps_recv": round(res["GBps_recv"], 3),
                              "connections_ok": res["connections_ok"], "data_errors": res.get("data_errors", 0),
                              "recv_cpu_s_per_GiB": round(res["recv_cpu_s_per_GiB"], 4),
                              "verdict_wait_s_per_GiB": round(wait / max(res["bytes_recv"] / GIB, 1e-9), 4)}),
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
