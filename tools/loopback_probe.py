#!/usr/bin/env python3
"""Config-1 loopback (8 connections x 1 GiB push, 64 KiB) under different verify arrangements, to see
what bounds each: no verification (the socket path alone), the C oracle on each receive thread (the
reference's arrangement), GPU DEFERRED at several batch sizes, GPU SYNC (mailbox). One JSON line per
(case, round)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from ctstraffic_amd import Engine, _pattern_abi as PA, loopback as LB  # noqa: E402
from ctstraffic_amd.pattern import shared_buffer_attach, shared_buffer_init  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--gib", type=int, default=1)
    p.add_argument("--cases", default="all", choices=["all", "deferred_sync_ab", "cpu_split", "query_period"])
    args = p.parse_args()
    eng = Engine(0)
    S = oracle.sender_buffer(65536)
    hook = PA.BATCH_VERIFIER(oracle.batch_verifier_address())
    if args.cases == "deferred_sync_ab":
        # round 3: DEFERRED's Retire sleeping on a blocking-sync event vs spinning in hipStreamSynchronize, and
        # the receive threads' CPU time per GiB next to the socket path alone and the CPU oracle
        cases = [("no_verify", dict(verify=False)),
                 ("cpu_oracle_sync", dict(verifier=hook, verify_mode=PA.VERIFY_SYNC)),
                 ("gpu_deferred_spin", dict(engine=eng, _env={"CTS_DEFERRED_BLOCKING_SYNC": "0"})),
                 ("gpu_deferred_blocking", dict(engine=eng, _env={"CTS_DEFERRED_BLOCKING_SYNC": "1"})),
                 ("gpu_deferred_sleep_poll", dict(engine=eng, _env={"CTS_DEFERRED_BLOCKING_SYNC": "2"})),
                 ("gpu_sync_mailbox", dict(engine=eng, verify_mode=PA.VERIFY_SYNC))]
    elif args.cases == "cpu_split":
        # where a receive thread's CPU goes (socket calls vs the pattern), per arrangement
        cases = [("no_verify", dict(verify=False)),
                 ("cpu_oracle_sync", dict(verifier=hook, verify_mode=PA.VERIFY_SYNC)),
                 ("cpu_oracle_deferred_b1024", dict(verifier=hook, verify_mode=PA.VERIFY_DEFERRED, batch_buffers=1024)),
                 ("gpu_deferred_b1024", dict(engine=eng, batch_buffers=1024)),
                 ("gpu_deferred_b4096", dict(engine=eng, batch_buffers=4096)),
                 ("gpu_sync_mailbox", dict(engine=eng, verify_mode=PA.VERIFY_SYNC))]
    elif args.cases == "query_period":
        # the DEFERRED early retire's hipEventQuery: how much receive-thread CPU it costs per GiB
        cases = [("no_verify", dict(verify=False)),
                 ("cpu_oracle_sync", dict(verifier=hook, verify_mode=PA.VERIFY_SYNC))]
        cases += [("gpu_deferred_b1024_q%s" % q, dict(engine=eng, batch_buffers=1024,
                                                     _env={"CTS_DEFERRED_QUERY_PERIOD": q}))
                  for q in ("16", "0", "256")]
    else:
        cases = None
    cases = cases or [("no_verify", dict(verify=False)),
             ("cpu_oracle_sync", dict(verifier=hook, verify_mode=PA.VERIFY_SYNC)),
             ("gpu_deferred_b256", dict(engine=eng, batch_buffers=256)),
             ("gpu_deferred_b1024", dict(engine=eng, batch_buffers=1024)),
             ("gpu_deferred_b4096", dict(engine=eng, batch_buffers=4096)),
             ("gpu_sync_mailbox", dict(engine=eng, verify_mode=PA.VERIFY_SYNC)),
             ("duplex_no_verify", dict(verify=False, io_pattern=PA.PATTERN_DUPLEX)),
             ("duplex_cpu_oracle_sync", dict(verifier=hook, verify_mode=PA.VERIFY_SYNC, io_pattern=PA.PATTERN_DUPLEX)),
             ("duplex_gpu_deferred_b1024", dict(engine=eng, batch_buffers=1024, io_pattern=PA.PATTERN_DUPLEX))]
    for r in range(args.rounds):
        for name, kw in cases:
            kw = dict(kw)
            env = kw.pop("_env", {})
            os.environ.update(env)  # read by each pattern at creation
            if "engine" in kw:
                shared_buffer_init(eng, 65536)
            else:
                shared_buffer_attach(S)
            res = LB.run(connections=8, buffer_size=65536, transfer_size=args.gib << 30, **kw)
            for k in env:
                os.environ.pop(k)
            print(json.dumps({"round": r, "case": name, "GBps_recv": round(res["GBps_recv"], 2),
                              "recv_cpu_s_per_GiB": round(res["recv_cpu_s_per_GiB"], 4),
                              "recv_pattern_cpu_s_per_GiB": round(res["recv_pattern_cpu_s_per_GiB"], 4),
                              "connections_ok": res["connections_ok"], "data_errors": res["data_errors"]}),
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
