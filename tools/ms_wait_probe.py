#!/usr/bin/env python3
"""MediaStream over loopback UDP, DEFERRED: receive-thread CPU per datagram with the batch flush waiting by sleeping
between event queries (CTS_DEFERRED_BLOCKING_SYNC=2, the default) or spinning in hipStreamSynchronize (=0). The
bench's sizing: 16 connections, 52083-byte frames at 240 frames/s, 240 frames. One JSON line per (case, round)."""
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
    for r in range(rounds):
        for name, wait in (("deferred_spin", "0"), ("deferred_sleep_poll", "2")):
            os.environ["CTS_DEFERRED_BLOCKING_SYNC"] = wait
            res = LB.media_stream_run(connections=16, frame_size=52083, frames_per_second=240,
                                      stream_length_frames=240, buffered_frames=60, engine=eng,
                                      verify_mode=PA.VERIFY_DEFERRED)
            c = res["clients"]
            print(json.dumps({"round": r, "case": name, "connections_ok": res["connections_ok"],
                              "data_errors": res["data_errors"], "successful_frames": c["successful_frames"],
                              "dropped_frames": c["dropped_frames"],
                              "recv_cpu_us_per_datagram": round(1e6 * res["recv_cpu_seconds"] /
                                                                max(1, res["datagrams_received"]), 3)}), flush=True)
    os.environ.pop("CTS_DEFERRED_BLOCKING_SYNC", None)
    eng.close()


if __name__ == "__main__":
    main()
