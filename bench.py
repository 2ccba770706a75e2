#!/usr/bin/env python3
"""bench.py — headline benchmark for the ctsTraffic data-integrity path on MI355X.

Metric (BASELINE.json): "GiB/s verified, 64 KiB buffers device-resident; % MI355X
HBM roofline". Workload (BASELINE configs[1]): per GPU,
4096 x 64 KiB received buffers resident in HBM (expected offsets 75 % phase 0,
25 % random, seed 0xC75; 1 in 1024 buffers carries a one-byte corruption,
seed 0xBAD). A step = one cts_verify pass over one such batch. The batch
rotates over R >= 8 identical arenas (2 GiB) so every pass streams from HBM
rather than the 256 MiB Infinity Cache. The fill kernel (the sender's
materialisation, InitOnceIoPatternCallback's role) builds the arenas untimed.
Batches are independent, so the headline leg issues step i on engine stream
i mod S (S = 3): one launch's tail overlaps the next one's ramp-up, as a receiver
verifying a stream of batches would run. roofline.achieved comes from a separate
serialized leg (one stream, HIP events), the per-kernel time rocprof reports.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Each rank verifies its own shard (no data-path collective: "scaling": "weak");
one RCCL all-reduce of the 5 ctsStatistics-style counters closes the timed region.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)
METRIC = "GiB/s verified, 64 KiB buffers device-resident; % MI355X HBM roofline"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--arenas", type=int, default=8, help="rotated copies of the batch (defeat the 256 MiB MALL)")
    p.add_argument("--buffers", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="budget per CPU-baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip fill / datagram / host-path extras")
    p.add_argument("--extras-only", default="", help="comma list: fill,datagram,host")
    p.add_argument("--stream", choices=["new", "default"], default="default",
                   help="launch stream: a new HIP stream or the device's default stream")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    p.add_argument("--graph", action="store_true", help="replay the timed steps from a HIP graph (measured: no gain; "
                   "implies --pipeline-streams 1)")
    p.add_argument("--pipeline-streams", type=int, default=3,
                   help="headline leg: steps round-robin over S engine streams, so one batch's tail overlaps the "
                        "next batch's ramp-up (1 = serialized launches; tools/overlap_probe.py)")
    p.add_argument("--verify-variant", type=int, default=-1,
                   help="CTS_ATTR_VERIFY_VARIANT for both legs (-1 = engine default; tools/tune_verify.py)")
    p.add_argument("--pipeline-blocks-per-cu", type=int, default=0,
                   help="verify grid cap (CTS_ATTR_BLOCKS_PER_CU) for the pipelined leg; 0 = engine default (4). "
                        "In bench.py A/B on one box 4 beat 3 (39.3-40.0 vs 39.8-40.3 us per step) and 2 (42.9-43.5)")
    return p.parse_args()


def main():
    args = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch

    from ctstraffic_amd.distributed import dist_env

    world, rank, local = dist_env()
    import torch.distributed as dist

    if not torch.cuda.is_available():
        print("bench.py: no HIP device visible", file=sys.stderr)
        sys.exit(2)
    gpu = local % torch.cuda.device_count()  # one rank per GPU; ranks share a GPU only in rehearsals
    torch.cuda.set_device(gpu)
    dev = "cuda:%d" % gpu
    from ctstraffic_amd import Engine, workload as W
    from ctstraffic_amd import distributed as D

    if world > 1:
        D.init(args.dist_backend, device=torch.device(dev) if args.dist_backend == "nccl" else None)

    engine = Engine(gpu)
    if args.verify_variant >= 0:
        from ctstraffic_amd import _lib as L

        engine.set_attr(L.ATTR_VERIFY_VARIANT, args.verify_variant)
    stream = torch.cuda.Stream() if args.stream == "new" else torch.cuda.current_stream()

    # ---- workload (per rank: weak scaling) --------------------------------------------------
    # weak scaling: every rank verifies a config-2 batch of its own connections (rank-disjoint
    # connection ids, so the per-connection DataError decisions never span GPUs)
    w = W.tcp_resident(n_buffers=args.buffers, conn_base=rank * args.buffers)
    R = max(1, args.arenas)
    arenas = []
    descs = None
    for _ in range(R):
        a, d = W.materialize(engine, w, device=dev)
        arenas.append(a)
        descs = d
    first, count, exp_ctr, _ = W.expected_results(w)
    bytes_per_step = w.verified_bytes()
    counters = engine.new_counters()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    # ---- HIP graph of one rotation (R launches), replayed in the timed region ----------------
    graph = None
    if args.graph:
        for i in range(R):  # first launches outside capture (module load, allocator)
            engine.verify(arenas[i], descs, max_length_hint=w.max_length, counters=counters, stream=stream)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for i in range(R):
                engine.verify(arenas[i], descs, max_length_hint=w.max_length, counters=counters, stream=stream)
        torch.cuda.synchronize()

    def run_steps(k0, k):
        """k verify steps starting at rotation index k0 on `stream` (graph replays for whole rotations)."""
        done = 0
        with torch.cuda.stream(stream):
            if graph is not None and k0 % R == 0:
                for _ in range(k // R):
                    graph.replay()
                done = (k // R) * R
            for i in range(done, k):
                engine.verify(arenas[(k0 + i) % R], descs, max_length_hint=w.max_length, counters=counters,
                              stream=stream)

    # pipelined steps: batch i on engine stream i mod S (independent arenas; the counter block takes
    # device atomics from every stream), then `stream` waits for all S before anything reads it
    S = 1 if graph is not None else max(1, args.pipeline_streams)
    pipe = [torch.cuda.ExternalStream(engine.stream_create(), device=dev) for _ in range(S)] if S > 1 else []

    from ctstraffic_amd import _lib

    default_bpc = engine.get_attr(_lib.ATTR_BLOCKS_PER_CU)
    pipe_bpc = args.pipeline_blocks_per_cu if pipe and args.pipeline_blocks_per_cu > 0 else default_bpc

    def run_pipelined(k0, k):
        if not pipe:
            run_steps(k0, k)
            return
        engine.set_attr(_lib.ATTR_BLOCKS_PER_CU, pipe_bpc)  # read at launch time; launches below are queued
        start = torch.cuda.Event()
        start.record(stream)
        for ps in pipe:
            ps.wait_event(start)
        for i in range(k):
            engine.verify(arenas[(k0 + i) % R], descs, max_length_hint=w.max_length, counters=counters,
                          stream=pipe[i % S].cuda_stream)
        for ps in pipe:
            ev = torch.cuda.Event()
            ev.record(ps)
            stream.wait_event(ev)
        engine.set_attr(_lib.ATTR_BLOCKS_PER_CU, default_bpc)

    # ---- warmup -------------------------------------------------------------------------------
    run_steps(0, max(args.warmup, 1))
    run_pipelined(0, max(args.warmup, 1))
    torch.cuda.synchronize()
    K = args.steps

    # ---- roofline leg: serialized launches on one stream, HIP events around exactly the K launches.
    # This is the per-kernel duration rocprof reports (run with --pipeline-streams 1 for the trace).
    avg_kernel_s = None
    ser_ok = True
    if pipe:
        engine.reset_counters(counters, stream=stream)
        ev_a = torch.cuda.Event(enable_timing=True)
        ev_b = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev_a.record(stream)
        run_steps(0, K)
        ev_b.record(stream)
        torch.cuda.synchronize()
        avg_kernel_s = ev_a.elapsed_time(ev_b) / 1e3 / K
        ser_ok = engine.read_counters(counters) == {k: v * K for k, v in exp_ctr.items()}

    engine.reset_counters(counters, stream=stream)
    if world > 1:
        # the counter all-reduce once before the clock starts (communicator and kernel set-up)
        with torch.cuda.stream(stream):
            D.allreduce_counters(D.fold_counters(counters))
    torch.cuda.synchronize()

    # ---- timed region (headline) --------------------------------------------------------------
    ev_a = torch.cuda.Event(enable_timing=True)
    ev_b = torch.cuda.Event(enable_timing=True)
    ctr_reduced = None
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_a.record(stream)
    run_pipelined(0, K)
    ev_b.record(stream)
    if world > 1:
        # fold the shards on-device and all-reduce the 5 counters over RCCL/xGMI
        with torch.cuda.stream(stream):
            ctr_reduced = D.allreduce_counters(D.fold_counters(counters))
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = D.max_over_ranks(t1 - t0, device=dev)
    pipe_step_s = ev_a.elapsed_time(ev_b) / 1e3 / K

    # S = 1: the events on the launch stream bracket exactly the K launches of the headline leg, and
    # the average launch duration includes the (graph) dispatch gaps, so it is an upper bound of the
    # kernel time rocprof reports
    if avg_kernel_s is None:
        avg_kernel_s = pipe_step_s
    local_ctr = engine.read_counters(counters)
    parity_ok = ser_ok and local_ctr == {k: v * K for k, v in exp_ctr.items()}
    if world > 1:
        glob = D.counters_dict(ctr_reduced)
        exp_glob = {f: exp_ctr[f] * K * world for f in exp_ctr}
        parity_ok = parity_ok and glob == exp_glob
        ok_t = torch.tensor([1 if parity_ok else 0], device=dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        parity_ok = bool(ok_t.item())

    total_bytes = bytes_per_step * K * world
    value = total_bytes / elapsed / GIB
    achieved_gbps = bytes_per_step / avg_kernel_s / 1e9

    # allreduce latency (separately, outside the headline)
    allreduce_us = None
    if world > 1:
        torch.cuda.synchronize()
        ta = time.perf_counter()
        for _ in range(20):
            D.allreduce_counters(ctr_reduced)
        torch.cuda.synchronize()
        allreduce_us = (time.perf_counter() - ta) / 20 * 1e6

    extras = {}
    cpu = None
    if rank == 0 and world == 1:
        want = set(x for x in args.extras_only.split(",") if x) or {"fill", "datagram", "host", "loopback"}
        if not args.no_extras:
            extras = run_extras(engine, torch, W, w, arenas, descs, dev, want)
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(arenas[0], w, args.cpu_seconds)

    traffic, traffic_src = pmc_traffic(w.name, args.buffers)
    from ctstraffic_amd import _lib

    variant = engine.get_attr(_lib.ATTR_VERIFY_VARIANT)
    kernel = VERIFY_KERNELS.get(variant, "variant %d" % variant)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded pattern fill + 1/1024 one-byte corruptions, seeds 0xC75/0xBAD)",
            "config": {
                "workload": "config2: %d x 64 KiB received buffers resident in HBM per GPU, cts_verify "
                            "(RtlCompareMemory semantics), %d rotated arenas" % (args.buffers, R),
                "buffers_per_gpu": args.buffers,
                "buffer_bytes": 65536,
                "verified_bytes_per_step_per_gpu": bytes_per_step,
                "arenas_rotated": R,
                "pipeline_streams": S,
                "parallelism": "%d rank(s), one config-2 batch of its own connections each, no data-path "
                               "collective; RCCL all-reduce of the 5 counters closes the timed region" % world,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved_gbps, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved_gbps / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": kernel,
                "avg_kernel_us": round(avg_kernel_s * 1e6, 2),
                "timing": ("HIP events on the launch stream around the K timed launches (%s), / K"
                           % ("HIP-graph replays" if graph is not None else "host launches")) if not pipe else
                          ("separate serialized leg of K launches on one stream, HIP events around them, / K "
                           "(the per-kernel duration rocprof reports); the headline value is the pipelined leg"),
                "algorithmic_bytes_per_launch": bytes_per_step,
                "pipelined": {
                    "streams": S,
                    "blocks_per_cu": pipe_bpc,
                    "us_per_step": round(pipe_step_s * 1e6, 2),
                    "effective_GBps": round(bytes_per_step / pipe_step_s / 1e9, 1),
                    "frac": round(bytes_per_step / pipe_step_s / 1e9 / HBM_PEAK_GBPS, 4),
                    "timing": "HIP events around the headline leg's K steps, / K: batch i on engine stream i mod S, "
                              "so one launch's tail overlaps the next launch's ramp-up",
                },
            },
            "cpu_baseline": cpu,
            "parity": {"counters_match_expected": bool(parity_ok), "counters": local_ctr},
        }
        if allreduce_us is not None:
            line["allreduce_counters_us"] = round(allreduce_us, 1)
        if extras:
            line["extras"] = extras
        print(json.dumps(line), flush=True)
    torch.cuda.synchronize()
    for ps in pipe:
        engine.stream_destroy(ps.cuda_stream)
    engine.close()
    if world > 1:
        dist.destroy_process_group()


def _time_kernel(torch, fn, steps):
    """Average time per launch: events around `steps` back-to-back launches (per-launch event pairs
    would add ~2.5 us to every launch)."""
    s = torch.cuda.current_stream()
    fn(0)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for i in range(steps):
        fn(i)
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / 1e3 / steps


VERIFY_KERNELS = {0: "cts::verify_wg_kernel<8,true>", 1: "cts::verify_wg_kernel<4,true>",
                  2: "cts::verify_wg_kernel<16,true>", 3: "cts::verify_wave_kernel<8,true>",
                  4: "cts::verify_wg_nb_kernel<8,true>", 5: "cts::verify_wg_nb_kernel<4,true>",
                  6: "cts::verify_wg_kernel<8,true,true>", 7: "cts::verify_wg_kernel<4,true,true>",
                  8: "cts::verify_wg_kernel<8,true,true,true>", 9: "cts::verify_wg_kernel<8,true,true,false,true>",
                  10: "cts::verify_wg_kernel<4,true,true,false,true>",
                  11: "cts::verify_wg_kernel<4,true,true,false,true,true>",
                  12: "cts::verify_wg_kernel<8,true,true,false,true,true>",
                  13: "cts::verify_wg_kernel<2,true,true,false,true,true>",
                  14: "cts::verify_wg_kernel<1,true,true,false,true,true>"}


def pmc_traffic(workload, buffers):
    """HBM bytes per verify launch from the newest profiles/<round>/pmc_traffic.json (rocprofv3 PMC,
    corrected per MI355X_MICROARCH.md; written by tools/prof_summary.py), or None."""
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
    try:
        rounds = sorted(d for d in os.listdir(root) if os.path.exists(os.path.join(root, d, "pmc_traffic.json")))
    except OSError:
        return None, None
    for d in reversed(rounds):
        try:
            tj = json.load(open(os.path.join(root, d, "pmc_traffic.json")))
        except Exception:
            continue
        if tj.get("workload") == workload and tj.get("buffers") == buffers and tj.get("hbm_bytes_per_launch"):
            return int(tj["hbm_bytes_per_launch"]), "profiles/%s/pmc_traffic.json" % d
    return None, None


def run_extras(engine, torch, W, w, arenas, descs, dev, want):
    out = {}
    R = len(arenas)
    nbytes = w.verified_bytes()
    if "fill" in want:
        # fill kernel over the same batch (write-bound twin); re-materialise corruptions afterwards
        t = _time_kernel(torch, lambda i: engine.fill(arenas[i % R], descs, max_length_hint=w.max_length), 100)
        out["fill_GiBps"] = round(nbytes / t / GIB, 1)
        out["fill_GBps"] = round(nbytes / t / 1e9, 1)
        # fused view: fill + verify of the same batch back to back
        ctr = engine.new_counters()

        def fv(i):
            engine.fill(arenas[i % R], descs, max_length_hint=w.max_length)
            engine.verify(arenas[i % R], descs, max_length_hint=w.max_length, counters=ctr)

        t = _time_kernel(torch, fv, 50)
        out["fill_then_verify_GiBps_verified"] = round(nbytes / t / GIB, 1)
        for a in arenas:  # restore the corruption plan
            pos = torch.from_numpy(w.corrupt_abs_offsets()).to(dev)
            a[pos] = a[pos] ^ torch.from_numpy(w.corrupt_xor).to(dev)
    if "datagram" in want:
        try:
            # config 3 in full: 16 M x 1472-byte MediaStream datagrams (23 GiB resident)
            from ctstraffic_amd import media_stream as MS

            wd = W.udp_datagrams(n_datagrams=16 * 1024 * 1024)
            ad, dd = W.materialize(engine, wd, device=dev)
            ctr = engine.new_counters()
            t = _time_kernel(torch, lambda i: engine.verify(ad, dd, max_length_hint=wd.max_length, counters=ctr), 10)
            out["datagram_1472_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            out["datagram_1472_verify_GBps_payload"] = round(wd.verified_bytes() / t / 1e9, 1)
            out["datagram_1472_verify_Mdgram_per_s"] = round(wd.n / t / 1e6, 1)
            out["datagram_config"] = "config3: 16M x 1472 B (26 B header skipped; payload bytes counted)"
            ok = engine.read_counters(ctr)["buffers_failed"] == 11 * len(np.unique(wd.corrupt_buf))
            out["datagram_parity"] = bool(ok)
            # the MediaStream client path: header parse + validate + payload verify + 32-byte record
            recs = torch.empty(wd.n * 32, dtype=torch.uint8, device=dev)
            res = engine.new_results(wd.n)
            t = _time_kernel(torch, lambda i: MS.verify(engine, ad, dd, records=recs, results=res), 10)
            out["media_stream_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            out["media_stream_verify_Mdgram_per_s"] = round(wd.n / t / 1e6, 1)
            del recs, res
            del ad, dd
        except Exception as e:  # pragma: no cover
            out["datagram_error"] = repr(e)
    if "loopback" in want:
        try:
            # config 1 end to end: loopback TCP push, 8 conns, 64 KiB IO, 1 GiB/conn, -verify:data; the
            # sender buffer comes from the fill kernel, every received buffer is verified on the GPU
            from ctstraffic_amd import _pattern_abi as PA
            from ctstraffic_amd import loopback as LB

            for name, mode, pat in (("deferred", PA.VERIFY_DEFERRED, PA.PATTERN_PUSH),
                                    ("sync", PA.VERIFY_SYNC, PA.PATTERN_PUSH),
                                    ("duplex_deferred", PA.VERIFY_DEFERRED, PA.PATTERN_DUPLEX)):
                # (duplex: each side sends and receives half of the 1 GiB at once, both directions verified)
                r = LB.run(connections=8, buffer_size=65536, transfer_size=1 << 30, engine=engine, verify_mode=mode,
                           io_pattern=pat)
                out["loopback_config1_%s" % name] = {
                    "GBps_recv": round(r["GBps_recv"], 3), "seconds": round(r["seconds"], 3),
                    "connections_ok": r["connections_ok"], "data_errors": r["data_errors"],
                    "buffers_verified": r["buffers_verified"]}
        except Exception as e:  # pragma: no cover
            out["loopback_error"] = repr(e)
    if "host" in want:
        try:
            # pinned, device-mapped host arena = the recv-buffer container of a GPU-verified ctsIoPattern
            hview, hptr, dptr = engine.host_alloc(arenas[0].numel())
            hview[:] = arenas[0].cpu().numpy()
            ctr = engine.new_counters()
            # (a) zero-copy: the verify kernel reads the pinned host arena in place over PCIe
            t = _time_kernel(torch, lambda i: engine.verify_ptr(dptr, hview.size, descs, max_length_hint=w.max_length,
                                                                 counters=ctr), 5)
            out["host_zero_copy_verify_GiBps"] = round(nbytes / t / GIB, 2)
            ok = engine.read_counters(ctr)["buffers_failed"] == (5 + 1) * len(np.unique(w.corrupt_buf))  # + warm launch
            out["host_zero_copy_parity"] = bool(ok)
            # (b) pinned hipMemcpyAsync H2D then device verify
            host_t = torch.from_numpy(hview)
            dst = torch.empty_like(arenas[0])

            def h2d(i):
                dst.copy_(host_t, non_blocking=True)
                engine.verify(dst, descs, max_length_hint=w.max_length, counters=ctr)

            t = _time_kernel(torch, h2d, 5)
            out["host_h2d_then_verify_GiBps"] = round(nbytes / t / GIB, 2)
            del dst, host_t
            torch.cuda.synchronize()
            engine.host_free(hptr)
        except Exception as e:  # pragma: no cover
            out["host_error"] = repr(e)
    return out


def cpu_baseline(arena, w, seconds):
    """The oracle (g++/gcc restatement of VerifyBuffer, RtlCompareMemory semantics) on this host's
    cores over a host copy of the same batch. Bounded: ~`seconds` per leg."""
    import oracle

    host = arena.cpu().numpy()
    nthreads = max(1, min(16, os.cpu_count() or 1))
    legs = {}
    for nt in (1, nthreads):
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.verify_batch(host, w.descs, nthreads=nt, want_results=False)
            reps += 1
            if time.perf_counter() - t0 >= seconds:
                break
        el = time.perf_counter() - t0
        legs[nt] = w.verified_bytes() * reps / el / GIB
    loop = None
    try:
        # the same config-1 loopback run with the oracle answering VerifyBuffer on the CPU (one
        # verifying thread per connection), i.e. the reference's own arrangement
        from ctstraffic_amd import _pattern_abi as PA
        from ctstraffic_amd import loopback as LB
        from ctstraffic_amd.pattern import shared_buffer_attach

        S = oracle.sender_buffer(65536)
        shared_buffer_attach(S)
        hook = PA.BATCH_VERIFIER(oracle.batch_verifier_address())
        r = LB.run(connections=8, buffer_size=65536, transfer_size=1 << 30, verifier=hook,
                   verify_mode=PA.VERIFY_SYNC)
        loop = {"GBps_recv": round(r["GBps_recv"], 3), "connections_ok": r["connections_ok"],
                "seconds": round(r["seconds"], 3),
                "sample": "config 1: 8 conns x 1 GiB loopback push, 64 KiB, oracle VerifyBuffer (C) per completion "
                          "on each connection's receive thread"}
    except Exception as e:  # pragma: no cover
        loop = {"error": repr(e)}
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {
        "value": round(legs[nthreads], 2),
        "unit": "GiB/s",
        "cores": nthreads,
        "kind": "port",
        "sample": "config2 batch (%d x 64 KiB, 256 MiB host copy of the same arena), repeated for ~%.0f s per leg"
                  % (w.n, seconds),
        "single_thread_value": round(legs[1], 2),
        "cpu_model": model,
        "loopback_config1": loop,
    }


if __name__ == "__main__":
    main()
