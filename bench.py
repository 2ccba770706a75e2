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
i mod S (S = 2): one launch's tail overlaps the next one's ramp-up, as a receiver
verifying a stream of batches would run. roofline.achieved comes from a separate
serialized leg (one stream, HIP events), the per-kernel time rocprof reports.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        N>1: either form works; with no WORLD_SIZE in the environment, `bench.py --gpus N` starts the N ranks
        itself as a child `torch.distributed.run` (before anything touches the GPU) and exits with its code:
          python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
          python bench.py --gpus N
        A WORLD_SIZE that differs from --gpus is an error (exit 2): the line's n_gpus is what ran.
Each rank verifies its own shard (no data-path collective: "scaling": "weak");
one RCCL all-reduce of the 5 ctsStatistics-style counters closes the timed region.
After it, at every N, rank 0 times the CPU oracle over its own batch (cpu_baseline; the other ranks wait on a
gloo barrier) and the single-process leg (`--engines N`, one process driving all N GPUs, run as a child
process) and puts both into the same line. Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ENGINES_LEG_CAP_S = 300  # the single-process leg (a child process) normally takes ~20 s
ALLREDUCE_CAP_S = 120    # cts_counters_allreduce timing in that leg: a first 8-GPU communicator set-up takes seconds
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)
METRIC = "GiB/s verified, 64 KiB buffers device-resident; % MI355X HBM roofline"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20,
                   help="timed steps; a step = one rotation over the R arenas = R config-2 batches (R launches)")
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--arenas", type=int, default=8, help="rotated copies of the batch (defeat the 256 MiB MALL)")
    p.add_argument("--buffers", type=int, default=4096)
    p.add_argument("--cpu-seconds", type=float, default=6.0, help="budget per CPU-baseline leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip fill / datagram / host-path extras")
    p.add_argument("--extras-only", default="", help="comma list: fill,datagram,host,loopback")
    p.add_argument("--stream", choices=["new", "default"], default="default",
                   help="launch stream: a new HIP stream or the device's default stream")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    p.add_argument("--engines", type=int, default=0,
                   help="single-process multi-GPU leg (the ctsTraffic process model): N engines on GPUs 0..N-1 in "
                        "this one process, one host thread and stream set per GPU, connections by cts_shard_of, "
                        "counters folded on the host by cts_counters_read_multi (0 = off)")
    p.add_argument("--launcher", choices=["native", "python"], default="python",
                   help="who issues the headline's launches: python = one ctypes cts_verify call per launch; native = "
                        "cts_verify called from C++ (tools/bench_multi.cpp). Measured the same (the host runs ahead "
                        "either way: profiles/r03/launcher_ab/); the single-process leg always launches natively")
    p.add_argument("--no-serial-graph", action="store_true",
                   help="roofline leg from K*R host launches instead of replays of a HIP graph")
    p.add_argument("--serial-graph-rotations", type=int, default=0,
                   help="roofline leg: rotations (R launches each) per captured graph; 0 = all K in one graph, replayed "
                        "once after an untimed upload replay; 1 = round 3's K replays of one rotation")
    p.add_argument("--engines-same-gpu", action="store_true",
                   help="--engines N with every engine on GPU 0: a rehearsal of the single-process code path on a "
                        "one-GPU box (the line then says n_gpus 1)")
    p.add_argument("--graph", action="store_true", help="replay the timed steps from a HIP graph (measured: no gain; "
                   "implies --pipeline-streams 1)")
    p.add_argument("--pipeline-streams", type=int, default=2,
                   help="headline leg: launches round-robin over S engine streams, so one batch's tail overlaps the "
                        "next batch's ramp-up (1 = serialized launches; 2 measured best at the driver's 20 steps: "
                        "profiles/r02/pipeline_streams/)")
    p.add_argument("--pin-numa", action="store_true",
                   help="pin the process to the GPU's NUMA node (cts_engine_numa_node): tools/sync_probe's SYNC "
                        "verifies answer faster there, but whole loopback runs were not faster "
                        "(profiles/r02/numa/); the device-resident legs do not care")
    p.add_argument("--no-engines-leg", action="store_true",
                   help="skip the single-process leg (--engines N as a child process) in the line's extras")
    p.add_argument("--stub-gpu", action="store_true",
                   help="launcher test: every rank reports its RANK/WORLD_SIZE over gloo and rank 0 prints one line; "
                        "nothing touches a GPU (tests/test_bench_launcher.py)")
    p.add_argument("--dist-timeout", type=float, default=600.0,
                   help="seconds any collective or barrier may wait at N > 1 (process-group timeout). Above rank 0's "
                        "work after the timed region, which the other ranks wait out at a barrier: the CPU baseline "
                        "(~1 min) and the single-process leg (capped at %d s). A rank that stalls longer or dies makes "
                        "the others raise; a rank that raises exits non-zero, and the launcher with it" % ENGINES_LEG_CAP_S)
    p.add_argument("--stub-fail-rank", type=int, default=-1,
                   help="with --stub-gpu: this rank fails (tests/test_bench_launcher.py)")
    p.add_argument("--stub-fail-mode", choices=["raise", "stall"], default="raise",
                   help="with --stub-fail-rank: raise before the all-gather, or sleep past --dist-timeout")
    return p.parse_args()


# environment keys of a torch.distributed.run rank; a child started from a rank (the single-process leg) drops
# them so it runs as a 1-process job of its own
_DIST_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
             "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
             "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE",
             "TORCHELASTIC_ERROR_FILE", "TORCH_NCCL_ASYNC_ERROR_HANDLING")


_LINE_OUT = None  # this process's real stdout, kept for the one JSON line once fd 1 points at stderr


def _claim_stdout():
    """From here on fd 1 is stderr: whatever a library prints (RCCL's version banner when it creates a communicator,
    gloo's rendezvous) stays off stdout, where the driver reads exactly one JSON line (written by emit())."""
    global _LINE_OUT
    sys.stdout.flush()
    _LINE_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)


def emit(line: dict) -> None:
    out = _LINE_OUT if _LINE_OUT is not None else sys.stdout
    out.write(json.dumps(line) + "\n")
    out.flush()


class _StdoutToStderr:
    """Point fd 1 at fd 2 for a block: gloo's C++ rendezvous prints "[Gloo] Rank r is connected to ..." on stdout,
    and the driver reads exactly one JSON line from it."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`bench.py --gpus N` without WORLD_SIZE: start the N ranks as ONE child process tree
    (torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1) and return its exit code. This process
    never touches the GPU and never execs; rank 0's JSON line reaches our stdout unchanged."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.stdout.flush()
    return subprocess.call(cmd, env=env)


def rank_diagnostics(rows) -> dict:
    """The per-rank rows of gather_rank_rows([avg_kernel_us, engine device, torch device, placement ok, local rank])
    as the line's keys: one slow GPU or one misplaced rank in the driver's N-GPU run then shows by name."""
    return {"per_rank_avg_kernel_us": [round(r[0], 2) for r in rows],
            "per_rank_device": [int(r[1]) for r in rows],
            "per_rank_torch_device": [int(r[2]) for r in rows],
            "per_rank_local_rank": [int(r[4]) for r in rows],
            "placement_ok": all(r[3] == 1.0 for r in rows)}


def check_placement(torch, engine, B, gpu, local):
    """Before the timed region: this rank's engine, its current torch device and every buffer it launches over (arenas,
    descriptors, records, first-failure slots, counter block) sit on GPU `gpu` = LOCAL_RANK mod the visible GPUs.
    Raises otherwise (torch.distributed.run then stops the other ranks)."""
    where = {("arena", t.device.index) for t in B.arenas} | {("results", t.device.index) for t in B.results} | \
            {("first_fail", t.device.index) for t in B.cff} | {("descs", B.descs.device.index),
                                                              ("counters", B.counters.device.index)}
    bad = sorted(x for x in where if x[1] != gpu)
    eng_dev, cur = engine.device_ordinal(), torch.cuda.current_device()
    if bad or eng_dev != gpu or cur != gpu or gpu != local % torch.cuda.device_count():
        raise RuntimeError("bench.py: rank placement (LOCAL_RANK %d, GPU %d): engine on %d, torch current device %d, "
                           "buffers off the GPU: %s" % (local, gpu, eng_dev, cur, bad))
    return eng_dev, cur


def stub_main(args):
    """--stub-gpu: the launcher's CPU test. Each rank joins a gloo group from the torch.distributed.run
    environment and reports (RANK, WORLD_SIZE, LOCAL_RANK); rank 0 prints one line shaped like the real one."""
    import torch
    import torch.distributed as dist

    from ctstraffic_amd import distributed as D

    world, rank, local = D.dist_env()
    if world > 1:
        with _StdoutToStderr():
            D.init("gloo", timeout_s=args.dist_timeout)
    if rank == args.stub_fail_rank:
        if args.stub_fail_mode == "raise":
            raise RuntimeError("bench.py --stub-fail-rank %d: this rank fails" % rank)
        time.sleep(args.dist_timeout * 20)  # stall: the others time out at the all-gather
    me = torch.tensor([rank, world, local], dtype=torch.int64)
    seen = [torch.zeros_like(me) for _ in range(world)]
    if world > 1:
        dist.all_gather(seen, me)
    else:
        seen = [me]
    # a library printing on fd 1 (as RCCL prints its version banner when it creates a communicator) must not reach
    # the driver's stdout
    os.write(1, b"RCCL version : stand-in banner of bench.py --stub-gpu\n")
    # the per-rank diagnostics of the real line, with stand-in values (kernel time 40 + rank, device = LOCAL_RANK)
    diag = rank_diagnostics(D.gather_rank_rows([40.0 + rank, local, local, 1, local]))
    if rank == 0:
        emit({"metric": METRIC, "value": 0.0, "unit": "GiB/s", "n_gpus": world, "stub": True,
              "ranks": [[int(x) for x in t.tolist()] for t in seen],
              "roofline": {k: v for k, v in diag.items() if k == "per_rank_avg_kernel_us"},
              **{k: v for k, v in diag.items() if k != "per_rank_avg_kernel_us"}})
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def engines_leg(args, world):
    """The single-process leg at this N (`bench.py --engines N`: one process, one engine per GPU, counters folded
    on the host), run as a child process with the rank environment removed. Returns a dict for the line's extras."""
    env = {k: v for k, v in os.environ.items() if k not in _DIST_ENV}
    cmd = [sys.executable, os.path.abspath(__file__), "--engines", str(world), "--no-cpu-baseline", "--no-extras",
           "--steps", str(args.steps), "--warmup", str(args.warmup), "--arenas", str(args.arenas),
           "--buffers", str(args.buffers), "--pipeline-streams", str(args.pipeline_streams)]
    try:
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           timeout=ENGINES_LEG_CAP_S)
    except subprocess.TimeoutExpired:
        return {"error": "timed out after %d s" % ENGINES_LEG_CAP_S}
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    err = "exit %d: %s" % (r.returncode, r.stderr.strip().splitlines()[-1:] or "")
    if not lines:
        return {"error": err}
    j = json.loads(lines[-1])
    out = {"value": j["value"], "unit": j["unit"], "n_gpus": j["n_gpus"], "ms_per_step": j["ms_per_step"],
           "per_gpu_GiBps": j.get("per_gpu_GiBps"), "parity": j.get("parity"), "node_counters": j.get("node_counters"),
           "process_model": "one process, one engine per GPU (cts_engine_create(g)), one host thread + %d streams "
                            "each, connections by cts_shard_of, counters folded by cts_counters_read_multi_ex and "
                            "all-reduced over RCCL by cts_counters_allreduce_ex after cts_counters_allreduce_prepare "
                            "at start-up" % args.pipeline_streams}
    if r.returncode != 0:  # e.g. an RCCL call that never returned: the line was emitted, the leg still failed
        out["error"] = err
    return out


class Batch:
    """One GPU's config-2 work: R rotated arenas of one batch (4096 x 64 KiB received buffers), their descriptors,
    and the product's outputs per arena: the per-buffer records (cts_verify_result, what CompleteIo reads for the
    pass bit and the first-mismatch report) and the per-connection first-failure slots (the DataError decision,
    ctsSocketState.cpp:221-232). Every timed launch writes all three outputs plus the counter block."""

    def __init__(self, torch, engine, W, dev, n_buffers, R, conn_ids):
        self.engine, self.dev, self.R = engine, dev, R
        self.w = W.tcp_resident(n_buffers=n_buffers)
        self.conn_ids = np.asarray(conn_ids)  # the node-wide connection of each buffer (one buffer per connection)
        assert len(self.conn_ids) == n_buffers
        self.arenas = []
        for _ in range(R):
            a, _d = W.materialize(engine, self.w, device=dev)
            self.arenas.append(a)
        # descriptors carry the GPU-local connection slot i (conn_ids[i] on the host), so the first-failure
        # slots of this GPU's connections are one dense array
        d = self.w.descs.copy()
        d["conn_index"] = np.arange(n_buffers, dtype=np.uint32)
        self.descs = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
        self.first, self.count, self.exp_ctr, self.exp_cff = W.expected_results(self.w)
        self.results = [engine.new_results(self.w.n) for _ in range(R)]
        self.cff = [torch.full((self.w.n,), -1, dtype=torch.int32, device=dev) for _ in range(R)]
        self.counters = engine.new_counters()
        self.bytes_per_launch = self.w.verified_bytes()

    def launch(self, i, stream):
        r = i % self.R
        self.engine.verify(self.arenas[r], self.descs, max_length_hint=self.w.max_length, results=self.results[r],
                           counters=self.counters, conn_first_fail=self.cff[r], stream=stream)

    def outputs_ok(self):
        """Every arena's records and first-failure slots equal the analytic outcome of the corruption plan."""
        from ctstraffic_amd.engine import results_from_device

        ok = True
        for r in range(self.R):
            res = results_from_device(self.results[r])
            exp_pass = self.first < 0
            ok &= bool(np.array_equal(res["pass"].astype(bool), exp_pass))
            fail = ~exp_pass
            ok &= bool(np.array_equal(res["first_mismatch"][fail].astype(np.int64), self.first[fail]))
            ok &= bool(np.array_equal(res["mismatch_bytes"][fail].astype(np.int64), self.count[fail]))
            ok &= bool(np.all(res["first_mismatch"][exp_pass] == 65536))
            ok &= bool(np.array_equal(self.cff[r].cpu().numpy().view(np.uint32), self.exp_cff))
        return ok


def main():
    args = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and args.engines == 0:
        sys.exit(launch_ranks(args))  # before anything touches the GPU
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus and args.engines == 0:
        print("bench.py: WORLD_SIZE=%s but --gpus %d: the line's n_gpus must be what ran"
              % (os.environ.get("WORLD_SIZE", "1"), args.gpus), file=sys.stderr)
        sys.exit(2)
    _claim_stdout()
    if args.stub_gpu:
        sys.exit(stub_main(args))
    import torch

    from ctstraffic_amd.distributed import dist_env

    world, rank, local = dist_env()
    import torch.distributed as dist

    if not torch.cuda.is_available():
        print("bench.py: no HIP device visible", file=sys.stderr)
        sys.exit(2)
    if args.engines > 0:
        if world > 1:
            print("bench.py: --engines is the single-process leg; do not launch it under torch.distributed.run",
                  file=sys.stderr)
            sys.exit(2)
        return main_engines(args, torch)
    gpu = local % torch.cuda.device_count()  # one rank per GPU; ranks share a GPU only in rehearsals
    torch.cuda.set_device(gpu)
    dev = "cuda:%d" % gpu
    from ctstraffic_amd import Engine, _lib, workload as W
    from ctstraffic_amd import distributed as D
    from ctstraffic_amd.types import COUNTER_FIELDS_EX

    cpu_group = None
    if world > 1:
        with _StdoutToStderr():
            D.init(args.dist_backend, device=torch.device(dev) if args.dist_backend == "nccl" else None,
                   timeout_s=args.dist_timeout)
            # host-side waits (while rank 0 runs the CPU baseline and the single-process leg) go over gloo, so
            # the waiting ranks hold no spinning collective kernel on their GPUs
            cpu_group = D.new_cpu_group(timeout_s=args.dist_timeout)

    engine = Engine(gpu)
    near = engine.cpus_near() if args.pin_numa else []
    if near:  # threads started from here on (loopback sides, the mailbox watchdog) inherit it
        os.sched_setaffinity(0, near)
    stream = torch.cuda.Stream() if args.stream == "new" else torch.cuda.current_stream()

    # ---- workload (per rank: weak scaling) --------------------------------------------------
    # every rank verifies a config-2 batch of its own connections (rank-disjoint connection ids, so the
    # per-connection DataError decisions never span GPUs)
    R = max(1, args.arenas)
    B = Batch(torch, engine, W, dev, args.buffers, R, conn_ids=np.arange(args.buffers) + rank * args.buffers)
    w, counters = B.w, B.counters
    exp_ctr = B.exp_ctr
    bytes_per_launch = B.bytes_per_launch
    bytes_per_step = bytes_per_launch * R
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    # ---- HIP graph of one rotation (R launches), replayed in the timed region ----------------
    graph = None
    if args.graph:
        for i in range(R):  # first launches outside capture (module load, allocator)
            B.launch(i, stream)
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for i in range(R):
                B.launch(i, stream)
        torch.cuda.synchronize()

    # pipelined steps: launch i on engine stream i mod S (independent arenas; the counter block takes
    # device atomics from every stream), then `stream` waits for all S before anything reads it
    S = 1 if graph is not None else max(1, args.pipeline_streams)
    pipe = [torch.cuda.ExternalStream(engine.stream_create(), device=dev) for _ in range(S)] if S > 1 else []

    # --launcher native: the launches go through cts_verify from native code (tools/bench_multi.cpp, in
    # this thread), as ctsTraffic's completion threads call VerifyBuffer; python: one ctypes call per launch
    native = args.launcher == "native" and graph is None
    if native:
        NL = _bench_multi_lib()
        w_ser, keep_ser = _bench_work(B, engine, gpu, [stream.cuda_stream])
        w_pipe, keep_pipe = _bench_work(B, engine, gpu, [ps.cuda_stream for ps in pipe] or [stream.cuda_stream])
        nt0, nt1, nts = (ctypes.c_double * 1)(), (ctypes.c_double * 1)(), ctypes.c_double()

        def native_launches(w, k):
            rc = NL.cts_bench_run_multi(ctypes.byref(w), 1, k * R, nt0, nt1, ctypes.byref(nts), 0)
            if rc != 0:
                raise RuntimeError("cts_bench_run_multi failed: %d" % rc)

    def run_steps(k):
        """k steps (k rotations = k*R launches) on `stream` (graph: one replay per step)."""
        if native:
            native_launches(w_ser, k)
            return
        with torch.cuda.stream(stream):
            if graph is not None:
                for _ in range(k):
                    graph.replay()
                return
            for i in range(k * R):
                B.launch(i, stream)

    def run_pipelined(k):
        if not pipe:
            run_steps(k)
            return
        start = torch.cuda.Event()
        start.record(stream)
        for ps in pipe:
            ps.wait_event(start)
        if native:
            native_launches(w_pipe, k)
        else:
            for i in range(k * R):
                B.launch(i, pipe[i % S].cuda_stream)
        for ps in pipe:
            ev = torch.cuda.Event()
            ev.record(ps)
            stream.wait_event(ev)

    # ---- warmup -------------------------------------------------------------------------------
    run_steps(max(args.warmup, 1))
    run_pipelined(max(args.warmup, 1))
    torch.cuda.synchronize()
    K = args.steps
    launches = K * R

    # ---- roofline leg: serialized launches on one stream, HIP events around exactly the K*R launches.
    # This is the per-kernel duration rocprof reports (run with --pipeline-streams 1 for the trace).
    avg_kernel_s = None
    ser_ok = True
    serial_graph = False
    if pipe:
        engine.reset_counters(counters, stream=stream)
        ev_a = torch.cuda.Event(enable_timing=True)
        ev_b = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        sg = None
        # rotations per captured graph: all K by default (one replay of K*R launches), so no replay boundary and no
        # first-replay upload sits inside the timed interval
        G = K if args.serial_graph_rotations <= 0 else max(1, min(K, args.serial_graph_rotations))
        while K % G:
            G -= 1
        if not args.no_serial_graph:
            # launches captured on their own stream and replayed: the host's dispatch gaps between back-to-back
            # kernels leave the measured interval, so it is the kernels' own time, as rocprof reports it (host
            # launches: 41.74-42.41 us, graph of one rotation: 41.56-41.79 us, alternating on one box,
            # profiles/r03/serial_graph/)
            gs = torch.cuda.Stream()
            try:
                sg = torch.cuda.CUDAGraph()
                # thread_local: other threads' HIP calls (RCCL's watchdog at N > 1) stay legal during the capture
                with torch.cuda.graph(sg, stream=gs, capture_error_mode="thread_local"):
                    for i in range(G * R):
                        B.launch(i, gs)
                with torch.cuda.stream(gs):
                    sg.replay()  # untimed: the graph's first replay uploads it
            except Exception as e:  # pragma: no cover - keep the host-launch leg
                print("bench.py: graph capture failed (%r); roofline leg from host launches" % e, file=sys.stderr)
                sg = None
            torch.cuda.synchronize()
            engine.reset_counters(counters, stream=stream)
            torch.cuda.synchronize()
        if sg is not None:
            with torch.cuda.stream(gs):  # replay() launches on the current stream
                ev_a.record(gs)
                for _ in range(K // G):
                    sg.replay()
                ev_b.record(gs)
        else:
            ev_a.record(stream)
            run_steps(K)
            ev_b.record(stream)
        torch.cuda.synchronize()
        avg_kernel_s = ev_a.elapsed_time(ev_b) / 1e3 / launches
        ser_ok = engine.read_counters(counters) == {k: v * launches for k, v in exp_ctr.items()}
        serial_graph = sg is not None

    eng_dev, torch_dev = check_placement(torch, engine, B, gpu, local)
    engine.reset_counters(counters, stream=stream)
    for c in B.cff:
        c.fill_(-1)
    for r in B.results:
        r.zero_()
    if world > 1:
        # the counter all-reduce once before the clock starts (communicator and kernel set-up)
        with torch.cuda.stream(stream):
            D.allreduce_counters(D.fold_counters(counters, COUNTER_FIELDS_EX))
    torch.cuda.synchronize()

    # ---- timed region (headline) --------------------------------------------------------------
    ev_a = torch.cuda.Event(enable_timing=True)
    ev_b = torch.cuda.Event(enable_timing=True)
    ctr_reduced = None
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_a.record(stream)
    run_pipelined(K)
    t_enq = time.perf_counter()  # the host has issued every launch (how far ahead of the GPU it ran: below)
    ev_b.record(stream)
    if world > 1:
        # fold the shards on-device and all-reduce the 6 counters (bytes, buffers, DataError connections) over
        # RCCL/xGMI
        with torch.cuda.stream(stream):
            ctr_reduced = D.allreduce_counters(D.fold_counters(counters, COUNTER_FIELDS_EX))
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = D.max_over_ranks(t1 - t0, device=dev)
    # each rank's own rate over its own bytes and its own clock (the max-over-ranks clock sets `value`)
    per_rank = [bytes_per_step * K / (t1 - t0) / GIB]
    if world > 1:
        mine = torch.tensor([per_rank[0]], dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine, group=cpu_group)
        per_rank = [float(x.item()) for x in allr]
    pipe_launch_s = ev_a.elapsed_time(ev_b) / 1e3 / launches

    # S = 1: the events on the launch stream bracket exactly the K*R launches of the headline leg, and the
    # average launch duration includes the dispatch gaps, so it is an upper bound of the kernel time rocprof
    # reports
    if avg_kernel_s is None:
        avg_kernel_s = pipe_launch_s
    local_ctr = engine.read_counters(counters)
    # the DataError count: every arena's slots were emptied before the timed region, so its first launch claims
    # the batch's failed connections and the later rotations find them claimed (one per connection,
    # ctsSocketState.cpp:221-228)
    conns_failed = engine.read_counters_ex(counters)["connections_failed"]
    exp_conns = int((B.exp_cff != 0xFFFFFFFF).sum()) * R
    outputs_ok = B.outputs_ok()
    parity_ok = (ser_ok and outputs_ok and local_ctr == {k: v * launches for k, v in exp_ctr.items()} and
                 conns_failed == exp_conns)
    if world > 1:
        glob = D.counters_dict(ctr_reduced)
        exp_glob = {f: exp_ctr[f] * launches * world for f in exp_ctr}
        exp_glob["connections_failed"] = exp_conns * world
        parity_ok = parity_ok and glob == exp_glob
        ok_t = torch.tensor([1 if parity_ok else 0], device=dev)
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        parity_ok = bool(ok_t.item())

    total_bytes = bytes_per_step * K * world
    value = total_bytes / elapsed / GIB
    achieved_gbps = bytes_per_launch / avg_kernel_s / 1e9

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
    if rank == 0:
        want = set(x for x in args.extras_only.split(",") if x) or {"fill", "datagram", "host", "loopback", "shards"}
        if not args.no_extras and world == 1:
            extras = run_extras(engine, torch, W, w, B.arenas, B.descs, dev, want)
        if not args.no_cpu_baseline:
            # at every N: the reference's CPU verify beside the GPU number (rank 0's host, rank 0's batch)
            cpu = cpu_baseline(B.arenas[0], w, args.cpu_seconds)
            # config 3 and the MediaStream receive on the CPU, beside the datagram extras' GPU numbers
            cpu["config3"] = cpu_baseline_config3(W, max(1.0, args.cpu_seconds / 2))
            cpu["loopback_media_stream_oracle"] = loopback_media_stream_oracle()
        if not (args.no_engines_leg or args.no_extras or args.extras_only):
            if world <= torch.cuda.device_count():
                extras["engines_single_process"] = engines_leg(args, world)
            else:
                extras["engines_single_process"] = {"skipped": "%d ranks share %d visible GPU(s)"
                                                    % (world, torch.cuda.device_count())}
    if world > 1:
        dist.barrier(group=cpu_group)

    traffic, traffic_src = pmc_traffic(w.name, args.buffers)
    kernel = verify_kernel_name(engine)
    # every rank's serialized-leg kernel time and placement, beside per_rank_GiBps
    diag = rank_diagnostics(D.gather_rank_rows([avg_kernel_s * 1e6, eng_dev, torch_dev, 1, local], group=cpu_group))

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
                            "(RtlCompareMemory semantics) writing per-buffer records, per-connection first-failure "
                            "slots and the counter block; a step = one rotation over %d arenas of that batch "
                            "(%d launches, %d bytes verified per GPU)" % (args.buffers, R, R, bytes_per_step),
                "buffers_per_gpu": args.buffers,
                "buffer_bytes": 65536,
                "verified_bytes_per_launch_per_gpu": bytes_per_launch,
                "launches_per_step": R,
                "verified_bytes_per_step_per_gpu": bytes_per_step,
                "arenas_rotated": R,
                "pipeline_streams": S,
                "launcher": ("native (cts_verify called from C++, tools/bench_multi.cpp)" if native else
                             "python (one ctypes cts_verify call per launch)"),
                "host_numa_node": engine.numa_node() if near else None,
                "host_cpus_pinned": len(near),
                "parallelism": "%d rank(s), one config-2 batch of its own connections each, no data-path "
                               "collective; %s" % (world, "one rank: no collective" if world == 1 else
                                                   "%s all-reduce of the 6 counters (bytes, buffers, DataError connections) closes the timed "
                                                   "region"
                                                   % ("RCCL" if args.dist_backend == "nccl" else args.dist_backend)),
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
                "per_rank_avg_kernel_us": diag["per_rank_avg_kernel_us"],
                "timing": ("HIP events on the launch stream around the K*R timed launches (%s), / (K*R)"
                           % ("HIP-graph replays" if graph is not None else "host launches")) if not pipe else
                          ("separate serialized leg of K*R launches on one stream (%s), HIP events around them, "
                           "/ (K*R) (the per-kernel duration rocprof reports); the headline value is the pipelined leg"
                           % (("%d replay(s) of a HIP graph of %d rotation(s), after an untimed upload replay"
                               % (K // G, G)) if serial_graph else "host launches")),
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "pipelined": {
                    "streams": S,
                    "us_per_launch": round(pipe_launch_s * 1e6, 2),
                    "effective_GBps": round(bytes_per_launch / pipe_launch_s / 1e9, 1),
                    "frac": round(bytes_per_launch / pipe_launch_s / 1e9 / HBM_PEAK_GBPS, 4),
                    "timing": "HIP events around the headline leg's K*R launches, / (K*R): launch i on engine "
                              "stream i mod S, so one launch's tail overlaps the next launch's ramp-up",
                    # where the wall clock of the headline leg goes beyond the GPU's own span of it
                    "host_enqueue_us": round((t_enq - t0) * 1e6, 1),
                    "wall_minus_events_us": round((elapsed - pipe_launch_s * launches) * 1e6, 1),
                },
            },
            "cpu_baseline": cpu,
            "parity": {"counters_match_expected": bool(parity_ok), "records_and_first_fail_match": bool(outputs_ok),
                       "counters": {**local_ctr, "connections_failed": conns_failed},
                       "connections_failed_expected": exp_conns},
        }
        line["per_rank_GiBps"] = [round(x, 1) for x in per_rank]
        line.update({k: v for k, v in diag.items() if k != "per_rank_avg_kernel_us"})
        if allreduce_us is not None:
            line["allreduce_counters_us"] = round(allreduce_us, 1)
        if extras:
            line["extras"] = extras
        emit(line)
    torch.cuda.synchronize()
    for ps in pipe:
        engine.stream_destroy(ps.cuda_stream)
    engine.close()
    if world > 1:
        dist.destroy_process_group()


class _BenchGpu(ctypes.Structure):
    """tools/bench_multi.cpp's cts_bench_gpu: one GPU's batch, outputs and streams."""
    _fields_ = [("engine", ctypes.c_void_p), ("device", ctypes.c_int), ("arenas", ctypes.c_uint32),
                ("arena", ctypes.POINTER(ctypes.c_void_p)), ("arena_bytes", ctypes.c_uint64),
                ("descs", ctypes.c_void_p), ("n", ctypes.c_uint32), ("max_length_hint", ctypes.c_uint32),
                ("results", ctypes.POINTER(ctypes.c_void_p)), ("counters", ctypes.c_void_p),
                ("conn_first_fail", ctypes.POINTER(ctypes.c_void_p)), ("n_conns", ctypes.c_uint32),
                ("streams", ctypes.POINTER(ctypes.c_void_p)), ("nstreams", ctypes.c_uint32)]


def _bench_multi_lib():
    """tools/libcts_bench_multi.so (make): loaded after libcts_engine.so, so its cts_verify is the engine's."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "libcts_bench_multi.so")
    if not os.path.exists(path):
        raise RuntimeError("%s is missing: run make" % path)
    L = ctypes.CDLL(path)
    L.cts_bench_run_multi.restype = ctypes.c_int
    L.cts_bench_run_multi.argtypes = [ctypes.POINTER(_BenchGpu), ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    return L


def _bench_work(B, engine, device, streams):
    """One cts_bench_gpu for Batch B on `streams` (raw HIP stream handles), and the ctypes arrays it points into."""
    R, S = len(B.arenas), len(streams)
    arena = (ctypes.c_void_p * R)(*[a.data_ptr() for a in B.arenas])
    res = (ctypes.c_void_p * R)(*[r.data_ptr() for r in B.results])
    cff = (ctypes.c_void_p * R)(*[c.data_ptr() for c in B.cff])
    st = (ctypes.c_void_p * S)(*streams)
    w = _BenchGpu(engine._h.value, device, R, arena, B.arenas[0].numel(), B.descs.data_ptr(), B.w.n, B.w.max_length,
                  res, B.counters.data_ptr(), cff, B.w.n, st, S)
    return w, (arena, res, cff, st)


def _median_us(fn, reps: int) -> float:
    """Median wall time of fn() in microseconds over reps calls (host-synchronous calls)."""
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t) * 1e6)
    return float(np.median(ts))


def main_engines(args, torch):
    """The ctsTraffic process model on a node: ONE process, one engine per GPU (cts_engine_create(g)), one native
    host thread and stream set per GPU (tools/bench_multi.cpp: the launches go through the C ABI from std::threads,
    as ctsTraffic's completion threads call VerifyBuffer; Python threads would serialise every launch on the GIL),
    connections assigned to GPUs by cts_shard_of, counters folded on the host with cts_counters_read_multi. Each GPU
    verifies a config-2 batch of its own connections (weak scaling, like the torch.distributed leg);
    value = all bytes / (wall from the common start to the last GPU's end).
    --engines-same-gpu puts every engine on GPU 0 (a rehearsal of the code path on a one-GPU box)."""
    import threading

    from ctstraffic_amd import Engine, workload as W
    from ctstraffic_amd.engine import (_multi_args, counters_allreduce_ex, counters_allreduce_prepare,
                                       counters_allreduce_release, counters_allreduce_setup_times, counters_read_multi,
                                       counters_read_multi_ex)

    G = args.engines
    same = args.engines_same_gpu
    if G > torch.cuda.device_count() and not same:
        print("bench.py: --engines %d but %d GPUs are visible" % (G, torch.cuda.device_count()), file=sys.stderr)
        sys.exit(2)
    L = _bench_multi_lib()
    R, S, K = max(1, args.arenas), max(1, args.pipeline_streams), args.steps
    # the node's connections (G batches' worth), each on GPU cts_shard_of(conn, G)
    n_conns = args.buffers * G
    conns = np.arange(n_conns, dtype=np.uint32)
    owner = W.shard_of(conns, G)
    ctx = []
    keep = []  # ctypes arrays the descriptors point into
    work = (_BenchGpu * G)()
    for g in range(G):
        dev = 0 if same else g
        torch.cuda.set_device(dev)
        e = Engine(dev)
        mine = conns[owner == g]
        B = Batch(torch, e, W, "cuda:%d" % dev, len(mine), R, conn_ids=mine)
        check_placement(torch, e, B, dev, dev)  # engine g, its buffers and outputs on GPU g (0 in the rehearsal)
        streams = [e.stream_create() for _ in range(S)]
        ctx.append((e, B, streams, len(mine)))
        work[g], k = _bench_work(B, e, dev, streams)
        keep.append(k)
    for g in range(G):
        torch.cuda.synchronize(0 if same else g)
    engs, blocks = [c[0] for c in ctx], [c[1].counters for c in ctx]
    red = {}

    # the status thread: it builds the node's RCCL clique at start-up (cts_counters_allreduce_prepare, next to
    # cts_engine_create, before the status timer's first tick at t = 0, ctsTraffic.cpp:107-113), waits for the
    # timed region to end, then makes its counter reads (the first one timed apart); a collective that never returns
    # costs the leg only its own numbers (the waits on this thread are bounded)
    prepared, go = threading.Event(), threading.Event()

    def status_thread():
        try:
            t = time.perf_counter()
            counters_allreduce_prepare(engs)
            red["prepare_ms"] = round((time.perf_counter() - t) * 1e3, 2)
            red["allreduce_setup_breakdown_ms"] = {k: (round(v, 3) if isinstance(v, float) else v)
                                                   for k, v in counters_allreduce_setup_times().items()
                                                   if not k.startswith("last_")}
        except Exception as ex:  # reported, not fatal: the verify leg is the measurement
            red["allreduce_error"] = repr(ex)
        prepared.set()
        if "allreduce_error" in red or not go.wait(ALLREDUCE_CAP_S * 4):
            return
        try:
            _multi_args(engs, blocks, None)  # the ctypes array types of the binding, made once (not the C ABI's time)
            t = time.perf_counter()
            red["reduced"] = counters_allreduce_ex(engs, blocks)  # the first read: the prepared clique's
            red["allreduce_first_call_us"] = round((time.perf_counter() - t) * 1e6, 1)
            ph = counters_allreduce_setup_times()
            red["allreduce_first_call_phases_us"] = {k[5:]: round(ph[k], 1) for k in ph if k.startswith("last_")}
            # the same call from entry to return inside the C ABI (what a C++ host's status timer pays); the rest of
            # allreduce_first_call_us is this ctypes binding's first call
            red["allreduce_first_call_c_abi_us"] = round(ph["last_total_us"], 1)
            red["allreduce_counters_us"] = round(_median_us(lambda: counters_allreduce_ex(engs, blocks), 20), 1)
            ph = counters_allreduce_setup_times()
            red["allreduce_last_call_phases_us"] = {k[5:]: round(ph[k], 1) for k in ph if k.startswith("last_")}
            # a thread that never called HIP before (a timer callback landing on a new pool thread): its first HIP
            # call, a host fold (device-to-host copies and synchronizes only), then the all-reduce, then again
            first = {}

            def other_thread():
                for k, fn in (("hip", torch.cuda.synchronize),
                              ("host_fold", lambda: counters_read_multi_ex(engs, blocks)),
                              ("allreduce", lambda: counters_allreduce_ex(engs, blocks)),
                              ("allreduce_again", lambda: counters_allreduce_ex(engs, blocks))):
                    t = time.perf_counter()
                    fn()
                    first[k] = round((time.perf_counter() - t) * 1e6, 1)

            th2 = threading.Thread(target=other_thread)
            th2.start()
            th2.join()
            red["new_thread_first_calls_us"] = first
            counters_allreduce_release()
        except Exception as ex:  # reported, not fatal: the verify leg above is the measurement
            red["allreduce_error"] = repr(ex)

    st = threading.Thread(target=status_thread, daemon=True)
    st.start()
    hung = not prepared.wait(ALLREDUCE_CAP_S)
    if hung:
        red["allreduce_error"] = "cts_counters_allreduce_prepare did not return within %d s" % ALLREDUCE_CAP_S
    t0, t1, ts = (ctypes.c_double * G)(), (ctypes.c_double * G)(), ctypes.c_double()

    def run(k):
        rc = L.cts_bench_run_multi(work, G, k * R, t0, t1, ctypes.byref(ts), 1)
        if rc != 0:
            raise RuntimeError("cts_bench_run_multi failed: %d" % rc)

    run(max(args.warmup, 1))
    for e, B, _, _ in ctx:
        e.reset_counters(B.counters)
        for c in B.cff:  # empty slots: the timed launches claim every failed connection again
            c.fill_(-1)
    for g in range(G):
        torch.cuda.synchronize(0 if same else g)
    run(K)
    elapsed = max(t1) - min(min(t0), ts.value)
    per_gpu = [ctx[g][1].bytes_per_launch * R * K / (t1[g] - t0[g]) / GIB for g in range(G)]
    folded = counters_read_multi_ex(engs, blocks)
    per = [c[0].read_counters_ex(c[1].counters) for c in ctx]
    # after the timed region: the node-wide counters both ways, the host fold and the RCCL all-reduce issued from
    # the C ABI (cts_counters_allreduce_ex: per-device fold + ncclAllReduce sum u64 x 6 per device), each timed
    fold_us = _median_us(lambda: counters_read_multi(engs, blocks), 20)

    if not hung:
        go.set()
        st.join(ALLREDUCE_CAP_S)
        hung = st.is_alive()
        if hung:
            red["allreduce_error"] = "cts_counters_allreduce_ex did not return within %d s" % ALLREDUCE_CAP_S
    reduced = red.pop("reduced", None)
    total = sum(c[1].bytes_per_launch for c in ctx) * R * K
    exp = {k: sum(c[1].exp_ctr[k] for c in ctx) * K * R for k in ctx[0][1].exp_ctr}
    # each arena's slots were emptied before the timed region: its first launch claims the batch's failed
    # connections, the later rotations find them claimed (ctsSocketState.cpp:221-228 counts a connection once)
    exp["connections_failed"] = sum(int((c[1].exp_cff != 0xFFFFFFFF).sum()) for c in ctx) * R
    line = {
        "metric": METRIC, "value": round(total / elapsed / GIB, 2), "unit": "GiB/s", "n_gpus": 1 if same else G,
        "steps": K, "warmup": args.warmup, "ms_per_step": round(elapsed / K * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (as the default leg)",
        "config": {"workload": "config2 per engine, single process: %d engines%s, one native host thread + %d "
                               "streams each, a step = %d launches per engine"
                               % (G, " all on GPU 0 (rehearsal)" if same else "", S, R),
                   "process_model": "one process, one engine per GPU (the ctsTraffic host model); launches from "
                                    "std::threads through cts_verify (tools/bench_multi.cpp)",
                   "engines": G, "connections_per_gpu": [c[3] for c in ctx]},
        "per_gpu_GiBps": [round(x, 1) for x in per_gpu],
        "parity": {"folded_counters_match_expected": folded == exp,
                   "fold_equals_sum_of_reads": folded == {k: sum(p[k] for p in per) for k in exp},
                   "records_and_first_fail_match": all(c[1].outputs_ok() for c in ctx), "counters": folded,
                   "allreduce_equals_fold": reduced == folded},
        "node_counters": {"fold_counters_us": round(fold_us, 1), **red,
                          "devices": [c[0].device_ordinal() for c in ctx]},
    }
    emit(line)
    if hung:  # the RCCL call still holds the devices: leave without tearing down under it, and say it failed
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(3)
    for e, B, streams, _ in ctx:
        for s in streams:
            e.stream_destroy(s)
        e.close()


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


def verify_kernel_name(engine):
    """The large-buffer verify kernel the engine launches, demangled as rocprofv3 reports it."""
    from ctstraffic_amd import _lib

    return _lib.verify_kernel_name(bool(engine.get_attr(_lib.ATTR_NT_LOADS)))


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
        # config 2's "fill+verify" as HBM traffic: fill arena i, then verify arena i + R/2, which was filled R/2
        # launch pairs earlier (R/2 x 256 MiB written and as much read since: its lines have left the 256 MB
        # Infinity Cache). Beside it the series bound of the two kernels' own rotated rates, and the same-arena
        # pair, whose verify reads what the fill just left in the Infinity Cache (labelled _mall).
        ctr = engine.new_counters()
        t_ver = _time_kernel(torch, lambda i: engine.verify(arenas[i % R], descs, max_length_hint=w.max_length,
                                                           counters=ctr), 100)

        def fv(i):
            engine.fill(arenas[i % R], descs, max_length_hint=w.max_length)
            engine.verify(arenas[(i + R // 2) % R], descs, max_length_hint=w.max_length, counters=ctr)

        def fv_same(i):
            engine.fill(arenas[i % R], descs, max_length_hint=w.max_length)
            engine.verify(arenas[i % R], descs, max_length_hint=w.max_length, counters=ctr)

        t_fv = _time_kernel(torch, fv, 50)
        t_same = _time_kernel(torch, fv_same, 50)
        out["verify_GBps_rotated"] = round(nbytes / t_ver / 1e9, 1)
        out["fill_then_verify_GiBps_verified"] = round(nbytes / t_fv / GIB, 1)
        out["fill_then_verify_series_bound_GiBps"] = round(nbytes / (t + t_ver) / GIB, 1)
        out["fill_then_verify_pair"] = ("fill arena i, verify arena i+%d of %d (filled %d pairs earlier: HBM); "
                                        "series bound = verified bytes / (fill time + verify time), each rotated"
                                        % (R // 2, R, R // 2))
        out["fill_then_verify_mall_GiBps_verified"] = round(nbytes / t_same / GIB, 1)
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
            # the same verify over the ring's descriptor-free form (datagram i at i * 1472, lengths only:
            # 4 bytes of metadata per datagram instead of a 24-byte descriptor)
            lens = torch.from_numpy(wd.descs["length"].astype(np.uint32)).to(dev)
            ctr_s = engine.new_counters()
            t = _time_kernel(torch, lambda i: engine.verify_strided(ad, wd.max_length, lens, skip_head=26,
                                                                    expected_offset=0, counters=ctr_s), 10)
            out["datagram_1472_verify_strided_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            out["datagram_strided_parity"] = bool(
                engine.read_counters(ctr_s)["buffers_failed"] == 11 * len(np.unique(wd.corrupt_buf)))
            # the MediaStream client path: header parse + validate + payload verify + 32-byte record
            recs = torch.empty(wd.n * 32, dtype=torch.uint8, device=dev)
            res = engine.new_results(wd.n)
            t = _time_kernel(torch, lambda i: MS.verify(engine, ad, dd, records=recs, results=res), 10)
            out["media_stream_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            out["media_stream_verify_Mdgram_per_s"] = round(wd.n / t / 1e6, 1)
            # the same receive pass over the ring's descriptor-free form (datagram i at i * 1472, lengths only)
            t = _time_kernel(torch, lambda i: MS.verify_strided(engine, ad, wd.max_length, lens, records=recs,
                                                                results=res), 10)
            out["media_stream_strided_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            # the compact receive pass: one 16-byte cts_datagram_status per datagram instead of record + result
            st = torch.empty(wd.n * 16, dtype=torch.uint8, device=dev)
            ctr_c = engine.new_counters()
            t = _time_kernel(torch, lambda i: MS.verify_status(engine, ad, dd, status=st, counters=ctr_c), 10)
            out["media_stream_status_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            t = _time_kernel(torch, lambda i: MS.verify_strided_status(engine, ad, wd.max_length, lens, status=st), 10)
            out["media_stream_strided_status_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            out["media_stream_status_parity"] = bool(
                engine.read_counters(ctr_c)["buffers_failed"] == 11 * len(np.unique(wd.corrupt_buf)))
            # the receive pass with the client's frame accounting summed on the GPU (no per-datagram output;
            # a jitter window of 10 frames from sequence number 1: the config-3 datagrams carry seq = i + 1)
            win = MS.FrameWindow(1, wd.n, 10, 0)
            sums = MS.FrameSums(win.frames, device=dev)
            t = _time_kernel(torch, lambda i: MS.verify_frames(engine, ad, dd, win, sums), 10)
            out["media_stream_frames_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            t = _time_kernel(torch, lambda i: MS.verify_strided_frames(engine, ad, wd.max_length, lens, win, sums), 10)
            out["media_stream_strided_frames_verify_GiBps"] = round(wd.verified_bytes() / t / GIB, 1)
            ft, fb = sums.read()
            bad = np.unique(wd.corrupt_buf)
            in_win = 10 - int(np.sum(bad < 10))  # clean datagrams of sequence numbers 1..10
            out["media_stream_frames_parity"] = bool(
                ft.exceptions == len(bad) and ft.datagrams == wd.n - len(bad) and int(fb.sum()) == 1472 * in_win and
                ft.error_frames == wd.n - len(bad) - in_win and ft.first_exception == int(bad[0]))
            # the sender side: whole datagrams (header + payload, as the MediaStream server sends them) written into
            # the same ring by cts_media_stream_fill (descriptors) and cts_media_stream_fill_strided (the ring);
            # the corruption plan is overwritten, so the strided receive then finds every datagram clean
            from ctstraffic_amd.types import DGRAM_HEADER_DTYPE, DGRAM_STATUS_DTYPE

            hdr = np.zeros(wd.n, dtype=DGRAM_HEADER_DTYPE)
            hdr["sequence_number"] = np.arange(1, wd.n + 1)
            hd = torch.from_numpy(hdr.view(np.uint8)).to(dev)
            t = _time_kernel(torch, lambda i: MS.fill(engine, ad, dd, hd), 5)
            out["media_stream_fill_GBps_written"] = round(wd.arena_bytes / t / 1e9, 1)
            t = _time_kernel(torch, lambda i: MS.fill_strided(engine, ad, wd.max_length, lens, hd), 5)
            out["media_stream_fill_strided_GBps_written"] = round(wd.arena_bytes / t / 1e9, 1)
            ctr_f = engine.new_counters()
            MS.verify_strided_status(engine, ad, wd.max_length, lens, status=st, counters=ctr_f)
            cf = engine.read_counters(ctr_f)
            seq = st.cpu().numpy().view(DGRAM_STATUS_DTYPE)["sequence_number"]
            out["media_stream_fill_parity"] = bool(cf["buffers_failed"] == 0 and cf["buffers_checked"] == wd.n and
                                                   np.array_equal(seq, hdr["sequence_number"]))
            del hd
            del st
            del lens
            del recs, res
            del ad, dd
        except Exception as e:  # pragma: no cover
            out["datagram_error"] = repr(e)
    if "shards" in want:
        try:
            # configs 4 and 5 at full size: rank 0's connection-hash shard of 1 M x 64 KiB over 2 and 4 GPUs
            # (32 / 16 GiB) and of 8 M x 64 KiB over 8 GPUs (64 GiB), resident at once, verified in one launch each
            # (per-buffer records, per-connection first-failure slots, counters); per-GPU work of the N-GPU runs
            for name, kw in (("config4_shard_of_2", dict(world=2, rank=0)), ("config4_shard_of_4", dict(world=4, rank=0)),
                             ("config5_shard_of_8", dict(n_conns=8192, buffers_per_conn=1024, world=8, rank=0,
                                                         name="config5"))):
                ws = W.connection_streams(**kw)
                a_s, d_s = W.materialize(engine, ws, device=dev)
                res_s = engine.new_results(ws.n)
                cff_s = torch.full((ws.n_conns,), -1, dtype=torch.int32, device=dev)
                ctr_s = engine.new_counters()
                launches = 5
                t = _time_kernel(torch, lambda i: engine.verify(a_s, d_s, max_length_hint=ws.max_length, results=res_s,
                                                                counters=ctr_s, conn_first_fail=cff_s), launches)
                _, _, exp_c, exp_cff = W.expected_results(ws)
                ok = engine.read_counters(ctr_s) == {k: v * (launches + 1) for k, v in exp_c.items()}
                ok = ok and bool(np.array_equal(cff_s.cpu().numpy().view(np.uint32), exp_cff))
                out[name] = {"GiBps": round(ws.verified_bytes() / t / GIB, 1),
                             "GBps": round(ws.verified_bytes() / t / 1e9, 1), "ms_per_launch": round(t * 1e3, 3),
                             "buffers": ws.n, "verified_bytes": ws.verified_bytes(), "parity": ok}
                del a_s, d_s, res_s, cff_s
                torch.cuda.empty_cache()
        except Exception as e:  # pragma: no cover
            out["shards_error"] = repr(e)
    if "loopback" in want:
        try:
            # config 1 end to end: loopback TCP push, 8 conns, 64 KiB IO, 1 GiB/conn, -verify:data; the
            # sender buffer comes from the fill kernel, every received buffer is verified on the GPU
            from ctstraffic_amd import _lib, _pattern_abi as PA
            from ctstraffic_amd import loopback as LB

            for name, mode, pat, mailbox in (("deferred", PA.VERIFY_DEFERRED, PA.PATTERN_PUSH, 1),
                                             ("sync", PA.VERIFY_SYNC, PA.PATTERN_PUSH, 1),
                                             ("sync_launch", PA.VERIFY_SYNC, PA.PATTERN_PUSH, 0),
                                             ("duplex_deferred", PA.VERIFY_DEFERRED, PA.PATTERN_DUPLEX, 1)):
                # (duplex: each side sends and receives half of the 1 GiB at once, both directions verified;
                # sync: every completion's VerifyBuffer posted to the resident mailbox grid, the default;
                # sync_launch: one sliced launch + synchronize per completion instead)
                engine.set_attr(_lib.ATTR_SYNC_MAILBOX, mailbox)
                try:
                    r = LB.run(connections=8, buffer_size=65536, transfer_size=1 << 30, engine=engine,
                               verify_mode=mode, io_pattern=pat, sides=True)
                finally:
                    engine.set_attr(_lib.ATTR_SYNC_MAILBOX, 1)
                # the patterns' waits for DEFERRED batch verdicts (cts_pattern_stats.verify_wait_ns), as a share of
                # the 2 x 8 sides' wall time (every side of a Duplex run receives)
                wait_s = sum(sd["verify_wait_ns"] for sd in r["sides"]) * 1e-9
                out["loopback_config1_%s" % name] = {
                    "GBps_recv": round(r["GBps_recv"], 3), "seconds": round(r["seconds"], 3),
                    "connections_ok": r["connections_ok"], "data_errors": r["data_errors"],
                    "buffers_verified": r["buffers_verified"],
                    "recv_cpu_s_per_GiB": round(r["recv_cpu_s_per_GiB"], 4),
                    "recv_pattern_cpu_s_per_GiB": round(r["recv_pattern_cpu_s_per_GiB"], 4),
                    "verdict_wait_s_per_GiB": round(wait_s / max(r["bytes_recv"] / GIB, 1e-9), 4)}
                if mode == PA.VERIFY_DEFERRED:
                    # launches in flight per connection, as the patterns ran them (cts_pattern_stats.deferred_depth)
                    out["loopback_config1_%s" % name]["launches_in_flight"] = max(sd["deferred_depth"]
                                                                                  for sd in r["sides"])
            # the socket path alone (-verify:connection): what the receive threads spend without any VerifyBuffer
            r = LB.run(connections=8, buffer_size=65536, transfer_size=1 << 30, verify=False)
            out["loopback_config1_verify_off"] = {
                "GBps_recv": round(r["GBps_recv"], 3), "seconds": round(r["seconds"], 3),
                "connections_ok": r["connections_ok"], "recv_cpu_s_per_GiB": round(r["recv_cpu_s_per_GiB"], 4),
                "recv_pattern_cpu_s_per_GiB": round(r["recv_pattern_cpu_s_per_GiB"], 4)}
            # MediaStream over loopback UDP (README sizing, 52083-byte frames at 240 frames/s, 16 connections, ~1.3 s):
            # the client patterns verify every datagram per completion (SYNC) or in batches through the frame-sum
            # receive pass (DEFERRED); the stream is rate-paced, so the number is the receive threads' CPU per datagram
            for name, mode in (("sync", PA.VERIFY_SYNC), ("deferred", PA.VERIFY_DEFERRED)):
                r = LB.media_stream_run(connections=16, frame_size=52083, frames_per_second=240,
                                        stream_length_frames=240, buffered_frames=60, engine=engine, verify_mode=mode)
                c = r["clients"]
                out["loopback_media_stream_%s" % name] = {
                    "connections_ok": r["connections_ok"], "data_errors": r["data_errors"],
                    "datagrams_received": r["datagrams_received"], "successful_frames": c["successful_frames"],
                    "dropped_frames": c["dropped_frames"], "payload_MBps": round(r["payload_MBps"], 1),
                    "recv_cpu_us_per_datagram": round(1e6 * r["recv_cpu_seconds"] / max(1, r["datagrams_received"]),
                                                      3)}
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


def _cpu_threads():
    try:
        avail = len(os.sched_getaffinity(0))
    except Exception:  # pragma: no cover
        avail = os.cpu_count() or 1
    return avail, sorted({1, min(16, avail)})


def cpu_baseline_config3(W, seconds, n_datagrams=1 << 20, ring=16 * 1024 * 1024):
    """Config 3 on the CPU: the oracle's VerifyBuffer with the MediaStream client's arguments (skip the 26-byte
    header, expected pattern offset 0: ctsIOPatternMediaStream.cpp:185-192) over the first `n_datagrams` of the
    16 M x 1472 B ring in host memory (the datagram extras' ring: same layout, headers and corruption plan, restricted
    to the slice), on 1 and 16 threads, ~`seconds` per leg. GiB/s of payload, as the GPU's datagram numbers."""
    import oracle

    full = W.udp_datagrams(n_datagrams=ring)  # the ring's descriptors and corruption plan (host arrays only)
    keep = full.corrupt_buf < n_datagrams
    ws = W.Workload("config3_slice", full.descs[:n_datagrams].copy(), n_datagrams * int(full.max_length),
                    full.max_length, full.corrupt_buf[keep], full.corrupt_pos[keep], full.corrupt_xor[keep],
                    n_conns=1, datagram_headers=True)
    del full
    # the bytes as received: payloads from the sender's pattern, {flag 0, seq i + 1, 0, 0} headers, the corruptions
    host = np.zeros(ws.arena_bytes, dtype=np.uint8)
    oracle.fill(host, ws.descs)
    host.reshape(n_datagrams, -1)[:, :W.UDP_DATA_HEADER_LENGTH] = W.header_bytes(np.arange(1, n_datagrams + 1))
    host[ws.corrupt_abs_offsets()] ^= ws.corrupt_xor
    _, _, exp_ctr, _ = W.expected_results(ws)
    avail, counts = _cpu_threads()
    legs, parity = {}, True
    for nt in counts:
        reps, t0 = 0, time.perf_counter()
        while True:
            _, c, _ = oracle.verify_batch(host, ws.descs, nthreads=nt, want_results=False)
            parity &= c == exp_ctr
            reps += 1
            if time.perf_counter() - t0 >= seconds:
                break
        legs[nt] = ws.verified_bytes() * reps / (time.perf_counter() - t0) / GIB
    best = max(legs, key=lambda k: legs[k])
    return {"value": round(legs[best], 2), "unit": "GiB/s of payload", "cores": best, "kind": "port",
            "sample": "config3 slice: the first %d of the 16 M x 1472 B datagrams (%d MiB host copy), oracle "
                      "VerifyBuffer skip 26 / expected 0 per datagram, ~%.1f s per leg" %
                      (n_datagrams, ws.arena_bytes >> 20, seconds),
            "threads_GiBps": {str(k): round(v, 2) for k, v in legs.items()},
            "single_thread_value": round(legs[1], 2), "counters_match_expected": bool(parity)}


def loopback_media_stream_oracle():
    """The MediaStream loopback run of the extras (16 UDP connections, README frame size 52083 B at 240 frames/s)
    with the oracle as every client pattern's VerifyBuffer, per datagram on the receive thread: the reference's own
    arrangement (ctsIOPatternMediaStream.cpp:185-192 on the IOCP thread). Receive-thread CPU per datagram beside the
    GPU SYNC / DEFERRED legs (extras.loopback_media_stream_*)."""
    import oracle
    from ctstraffic_amd import _pattern_abi as PA
    from ctstraffic_amd import loopback as LB
    from ctstraffic_amd.pattern import shared_buffer_attach

    try:
        S = oracle.sender_buffer(65536)  # attached by pointer: kept alive for the run
        shared_buffer_attach(S)
        hook = PA.BATCH_VERIFIER(oracle.batch_verifier_address())
        r = LB.media_stream_run(connections=16, frame_size=52083, frames_per_second=240, stream_length_frames=240,
                                buffered_frames=60, verifier=hook, verify_mode=PA.VERIFY_SYNC)
        c = r["clients"]
        return {"connections_ok": r["connections_ok"], "data_errors": r["data_errors"],
                "datagrams_received": r["datagrams_received"], "successful_frames": c["successful_frames"],
                "dropped_frames": c["dropped_frames"], "payload_MBps": round(r["payload_MBps"], 1),
                "recv_cpu_us_per_datagram": round(1e6 * r["recv_cpu_seconds"] / max(1, r["datagrams_received"]), 3),
                "sample": "16 conns x 240 frames of 52083 B at 240 frames/s over loopback UDP, oracle VerifyBuffer "
                          "(C) per datagram on each client's receive thread", "sender_buffer_bytes": int(S.size)}
    except Exception as e:  # pragma: no cover
        return {"error": repr(e)}


# the BASELINE configs the CPU baseline times (BASELINE.md promises the full set or a labelled subset)
CPU_CONFIGS_TIMED = ["config1-loopback", "config2", "config3-slice(1/16)"]
CPU_CONFIGS_NOTE = ("configs 4 and 5 are not timed on the CPU: their buffers are 64 KiB completions of per-connection "
                    "streams, the per-byte work of config 2 (the same VerifyBuffer over 64 KiB at a prefix-sum offset), "
                    "so config 2's GiB/s per core stands for them; config 3 is timed on its first 1 M of 16 M datagrams")


def cpu_baseline(arena, w, seconds, loopback=True):
    """The oracle (g++/gcc restatement of VerifyBuffer, RtlCompareMemory semantics) on this host's
    cores over a host copy of the same batch. Bounded: ~`seconds` per leg. loopback=False skips the config-1
    loopback leg (the CPU tests)."""
    import oracle

    host = arena.cpu().numpy()
    # 1 thread, 16 threads (this pool's CPU share per GPU) and every CPU this process may run on
    avail, counts = _cpu_threads()
    counts = sorted(set(counts) | {avail})
    legs = {}
    for nt in counts:
        reps, t0 = 0, time.perf_counter()
        while True:
            oracle.verify_batch(host, w.descs, nthreads=nt, want_results=False)
            reps += 1
            if time.perf_counter() - t0 >= seconds:
                break
        el = time.perf_counter() - t0
        legs[nt] = w.verified_bytes() * reps / el / GIB
    best = max(legs, key=lambda k: legs[k])
    loop = None
    try:
        if not loopback:
            raise RuntimeError("skipped (loopback=False)")
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
                "seconds": round(r["seconds"], 3), "recv_cpu_s_per_GiB": round(r["recv_cpu_s_per_GiB"], 4),
                "recv_pattern_cpu_s_per_GiB": round(r["recv_pattern_cpu_s_per_GiB"], 4),
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
    quota = None
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q[0] != "max":
            quota = round(int(q[0]) / int(q[1]), 2)
    except Exception:
        pass
    return {
        "value": round(legs[best], 2),
        "unit": "GiB/s",
        "cores": best,
        "kind": "port",
        "sample": "config2 batch (%d x 64 KiB, 256 MiB host copy of the same arena), repeated for ~%.0f s per leg; "
                  "the best of %s threads" % (w.n, seconds, "/".join(str(c) for c in counts)),
        "threads_GiBps": {str(k): round(v, 2) for k, v in legs.items()},
        "single_thread_value": round(legs[1], 2),
        "cpus_available": avail,
        "cgroup_cpu_quota": quota,
        "cpu_model": model,
        "loopback_config1": loop,
        "configs_timed": list(CPU_CONFIGS_TIMED),
        "configs_note": CPU_CONFIGS_NOTE,
    }


if __name__ == "__main__":
    main()
