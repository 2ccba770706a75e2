#!/usr/bin/env python3
"""MediaStream over loopback UDP (bench sizing: 16 connections, 52083-byte frames at 240 frames/s, 240 frames): the
receive-thread CPU per datagram with GPU DEFERRED at client batches of 1024 (the default: a 2 x 1024-slot recv ring,
2.9 MB per connection), 256 and 64 datagrams, beside verify off. Does the ring's footprint cost the receive thread?
(The oracle's figure is bench.py's cpu_baseline.loopback_media_stream_oracle.) Legs rotated over rounds; one JSON
line per leg.
usage: python tools/ms_ring_probe.py [rounds]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ctstraffic_amd import Engine, _pattern_abi as PA, loopback as LB  # noqa: E402
from ctstraffic_amd.pattern import shared_buffer_init  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    eng = Engine(0)
    shared_buffer_init(eng, 65536)
    legs = ["off", "1024", "256", "64"]
    for r in range(rounds):
        for leg in legs[r % len(legs):] + legs[:r % len(legs)]:
            kw = dict(connections=16, frame_size=52083, frames_per_second=240, stream_length_frames=240,
                      buffered_frames=60)
            if leg == "off":
                res = LB.media_stream_run(verify=False, **kw)
            else:
                res = LB.media_stream_run(engine=eng, verify_mode=PA.VERIFY_DEFERRED, batch_buffers=int(leg), **kw)
            c = res["clients"]
            print(json.dumps({"round": r, "leg": "verify_off" if leg == "off" else "deferred_batch_" + leg,
                              "connections_ok": res["connections_ok"], "data_errors": res["data_errors"],
                              "successful_frames": c["successful_frames"], "dropped_frames": c["dropped_frames"],
                              "recv_cpu_us_per_datagram": round(1e6 * res["recv_cpu_seconds"] /
                                                                max(1, res["datagrams_received"]), 3)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
