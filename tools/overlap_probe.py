#!/usr/bin/env python3
"""Do config-2 verify launches over independent arenas gain from overlapping on several streams?

One stream serialises launches: each launch's ramp-up and tail (the ~2.6 us a 256 MiB read loses
to a 1 GiB read) leave CUs idle. With S streams taking the rotated arenas round
robin, the next batch's workgroups can fill the previous batch's tail. Prints one JSON line per S:
wall time per step (K steps, synchronize on both sides) and the verified rate; counters are checked.
  usage (GPU box): python tools/overlap_probe.py [K]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ctstraffic_amd import Engine, workload as W  # noqa: E402

GIB = 1 << 30


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    engine = Engine(0)
    w = W.tcp_resident(n_buffers=4096, conn_base=0)
    R = 8
    arenas = []
    descs = None
    for _ in range(R):
        a, d = W.materialize(engine, w, device="cuda:0")
        arenas.append(a)
        descs = d
    _, _, exp_ctr, _ = W.expected_results(w)
    counters = engine.new_counters()
    torch.cuda.synchronize()
    import ctypes
    from ctstraffic_amd._lib import lib

    def engine_stream():
        p = ctypes.c_void_p()
        assert lib().cts_engine_stream_create(engine._h, ctypes.byref(p)) == 0
        return p.value

    from ctstraffic_amd.engine import _ptr, _nbytes

    n = _nbytes(descs) // 24
    L = lib()
    pa = [(_ptr(a), _nbytes(a)) for a in arenas]
    pd, pc = _ptr(descs), _ptr(counters)

    def launch(i, s, direct):
        if direct:
            L.cts_verify(engine._h, pa[i % R][0], pa[i % R][1], pd, n, w.max_length, None, pc, None, 0, s)
        else:
            engine.verify(arenas[i % R], descs, max_length_hint=w.max_length, counters=counters, stream=s)

    mode = sys.argv[2] if len(sys.argv) > 2 else "sweep"
    if mode == "bpc":  # workgroup-per-buffer grid cap x streams
        from ctstraffic_amd import _lib
        default_bpc = engine.get_attr(_lib.ATTR_BLOCKS_PER_CU)
        for trial in range(2):
            for bpc in (2, 3, 4, 6, 8):
                engine.set_attr(_lib.ATTR_BLOCKS_PER_CU, bpc)
                for S in (1, 2, 3):
                    streams = [engine_stream() for _ in range(S)]
                    for i in range(2 * R):
                        launch(i, streams[i % S], True)
                    torch.cuda.synchronize()
                    engine.reset_counters(counters)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(K):
                        launch(i, streams[i % S], True)
                    torch.cuda.synchronize()
                    t = time.perf_counter() - t0
                    ok = engine.read_counters(counters) == {k: v * K for k, v in exp_ctr.items()}
                    print(json.dumps({"trial": trial, "blocks_per_cu": bpc, "streams": S, "steps": K,
                                      "us_per_step": round(t / K * 1e6, 2),
                                      "TBps": round(w.verified_bytes() * K / t / 1e12, 3), "counters_ok": ok}),
                          flush=True)
        engine.set_attr(_lib.ATTR_BLOCKS_PER_CU, default_bpc)
        return
    kinds = ("torch", "engine") if mode == "sweep" else ("engine",)
    sweep = (1, 2, 3, 4, 6, 8) if mode == "sweep" else (1, 2, 3)
    for trial in range(3):
        for kind in kinds:
            for direct in ((False,) if mode == "sweep" else (False, True)):
                for S in sweep:
                    if kind == "torch":
                        streams = [torch.cuda.Stream().cuda_stream for _ in range(S)]
                    else:
                        streams = [engine_stream() for _ in range(S)]
                    for i in range(2 * R):
                        launch(i, streams[i % S], direct)
                    torch.cuda.synchronize()
                    engine.reset_counters(counters)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(K):
                        launch(i, streams[i % S], direct)
                    t_host = time.perf_counter() - t0
                    torch.cuda.synchronize()
                    t = time.perf_counter() - t0
                    ok = engine.read_counters(counters) == {k: v * K for k, v in exp_ctr.items()}
                    print(json.dumps({"trial": trial, "kind": kind, "direct": direct, "streams": S, "steps": K,
                                      "us_per_step": round(t / K * 1e6, 2),
                                      "host_us_per_launch": round(t_host / K * 1e6, 2),
                                      "TBps": round(w.verified_bytes() * K / t / 1e12, 3), "counters_ok": ok}),
                          flush=True)

if __name__ == "__main__":
    main()
