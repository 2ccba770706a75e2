"""GPU, one rank over RCCL ("nccl"): the collectives bench.py issues at N > 1, rehearsed at world size 1 on the one
GPU this box has (RCCL refuses two ranks on one device, and the 8-GPU run is the driver's).

The rank inits the group as bench.py does (``distributed.init`` with ``device_id`` and the bounded timeout, plus the
gloo group for host-side waits), verifies a config-4-shaped shard on the GPU, folds the device counter block and
all-reduces the five int64 counters (SUM), the parity flag (MIN) and the wall time (float64 MAX) over RCCL, and
all-gathers the per-rank rate over gloo: every dtype and op of the N > 1 path goes through RCCL on gfx950 once.
(``allreduce_counters`` skips the call at world size 1, so the rank issues the same all_reduce directly.)
"""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    try:
        import torch
        import torch.distributed as dist

        import oracle
        from ctstraffic_amd import Engine
        from ctstraffic_amd import distributed as D
        from ctstraffic_amd import workload as W

        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        D.init("nccl", device=dev, timeout_s=120)
        cpu_group = D.new_cpu_group(timeout_s=120)
        with Engine(0) as eng:
            w = W.connection_streams(world=4, rank=1, n_conns=64, buffers_per_conn=8, length=65536, corrupt_rate=9)
            arena, descs = W.materialize(eng, w, device="cuda:0")
            ctr = eng.new_counters()
            eng.verify(arena, descs, max_length_hint=65536, counters=ctr)
            torch.cuda.synchronize()
            local = eng.read_counters(ctr)
            _, exp, _ = oracle.verify_batch(arena.cpu().numpy(), w.descs)
            c5 = D.fold_counters(ctr)
            dist.all_reduce(c5, op=dist.ReduceOp.SUM)  # what allreduce_counters issues at N > 1
            ok = torch.tensor([1 if local == exp else 0], device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            t = torch.tensor([1.25], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            mine = torch.tensor([2.5], dtype=torch.float64)
            allr = [torch.zeros_like(mine)]
            dist.all_gather(allr, mine, group=cpu_group)
            dist.barrier(group=cpu_group)
            q.put((D.counters_dict(c5), local, exp, int(ok.item()), float(t.item()), float(allr[0].item()),
                   dist.get_backend()))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put(("error", repr(e)))


def test_rccl_world1_collectives_of_the_multi_gpu_path():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_main, args=(_free_port(), q), daemon=True)
    p.start()
    try:
        r = q.get(timeout=100)
        p.join(15)
    finally:
        if p.is_alive():  # a hung rank must not outlive the test
            p.kill()
            p.join(5)
    assert r[0] != "error", r[1]
    glob, local, exp, ok, t, gathered, backend = r
    assert backend == "nccl"
    assert glob == local == exp and exp["buffers_failed"] > 0
    assert ok == 1 and t == 1.25 and gathered == 2.5
    assert p.exitcode == 0


def _allreduce_main(q):
    """cts_counters_allreduce through the C ABI: one engine (a one-rank RCCL clique), then two engines on this GPU
    (folded into one device slot; each on its own stream), against cts_counters_read_multi and the oracle."""
    try:
        import torch

        import oracle
        from ctstraffic_amd import Engine
        from ctstraffic_amd import workload as W
        from ctstraffic_amd.engine import counters_allreduce, counters_allreduce_release, counters_read_multi

        torch.cuda.set_device(0)
        out = {}
        with Engine(0) as e0, Engine(0) as e1:
            blocks, exps = [], []
            for k, eng in enumerate((e0, e1)):
                w = W.connection_streams(world=2, rank=k, n_conns=64, buffers_per_conn=8, length=65536,
                                         corrupt_rate=7 + k)
                arena, descs = W.materialize(eng, w, device="cuda:0")
                ctr = eng.new_counters()
                eng.verify(arena, descs, max_length_hint=65536, counters=ctr)
                torch.cuda.synchronize()
                blocks.append(ctr)
                exps.append(oracle.verify_batch(arena.cpu().numpy(), w.descs)[1])
            out["one"] = (counters_allreduce([e0], blocks[:1]), counters_read_multi([e0], blocks[:1]), exps[0])
            s0, s1 = e0.stream_create(), e1.stream_create()
            out["two"] = (counters_allreduce([e0, e1], blocks, [s0, s1]), counters_read_multi([e0, e1], blocks),
                          {k: exps[0][k] + exps[1][k] for k in exps[0]})
            counters_allreduce_release()
            out["again"] = counters_allreduce([e0, e1], blocks)
            counters_allreduce_release()
            e0.stream_destroy(s0)
            e1.stream_destroy(s1)
        q.put(out)
    except Exception as e:  # pragma: no cover
        q.put(("error", repr(e)))


def test_counters_allreduce_c_abi_over_rccl():
    """north_star / config 5: the RCCL all-reduce of the ctsStatistics counters, issued from the C ABI (ctsTraffic's
    one-process C++ host cannot call torch.distributed). Run in a child so RCCL's threads end with it."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_allreduce_main, args=(q,), daemon=True)
    p.start()
    try:
        r = q.get(timeout=100)
        p.join(15)
    finally:
        if p.is_alive():
            p.kill()
            p.join(5)
    assert not (isinstance(r, tuple) and r[0] == "error"), r[1]
    red, fold, exp = r["one"]
    assert red == fold == exp and exp["buffers_failed"] > 0
    red, fold, exp = r["two"]
    assert red == fold == exp
    assert r["again"] == exp
    assert p.exitcode == 0


def _allreduce_ex_main(q):
    """cts_counters_allreduce_prepare, then cts_counters_allreduce_ex with the DataError count: one engine, then two
    engines on this GPU, each block carrying the connections_failed its verify counted on its slot array."""
    try:
        import time

        import numpy as np
        import torch

        import oracle
        from ctstraffic_amd import Engine
        from ctstraffic_amd import workload as W
        from ctstraffic_amd.engine import (counters_allreduce_ex, counters_allreduce_prepare,
                                           counters_allreduce_release, counters_allreduce_setup_times,
                                           counters_read_multi_ex)

        torch.cuda.set_device(0)
        out = {}
        with Engine(0) as e0, Engine(0) as e1:
            t = time.perf_counter()
            counters_allreduce_prepare([e0, e1])  # before any verify: the status timer's t = 0
            out["prepare_ms"] = (time.perf_counter() - t) * 1e3
            out["setup"] = counters_allreduce_setup_times()
            blocks, exps = [], []
            for k, eng in enumerate((e0, e1)):
                w = W.connection_streams(world=2, rank=k, n_conns=64, buffers_per_conn=8, length=65536,
                                         corrupt_rate=5 + k)
                arena, descs = W.materialize(eng, w, device="cuda:0")
                ctr = eng.new_counters()
                cff = torch.full((w.n_conns,), -1, dtype=torch.int32, device="cuda:0")
                eng.verify(arena, descs, max_length_hint=65536, counters=ctr, conn_first_fail=cff)
                torch.cuda.synchronize()
                blocks.append(ctr)
                _, c, ocff = oracle.verify_batch(arena.cpu().numpy(), w.descs, n_conns=w.n_conns)
                c["connections_failed"] = int((ocff != 0xFFFFFFFF).sum())
                exps.append(c)
            t = time.perf_counter()
            red2 = counters_allreduce_ex([e0, e1], blocks)  # the prepared clique: no set-up inside
            out["first_ex_us"] = (time.perf_counter() - t) * 1e6
            out["two"] = (red2, counters_read_multi_ex([e0, e1], blocks),
                          {k: exps[0][k] + exps[1][k] for k in exps[0]})
            out["setup_after"] = counters_allreduce_setup_times()
            out["one"] = (counters_allreduce_ex([e0], blocks[:1]), counters_read_multi_ex([e0], blocks[:1]), exps[0])
            counters_allreduce_release()
        q.put(out)
    except Exception as e:  # pragma: no cover
        q.put(("error", repr(e)))


def test_counters_allreduce_ex_prepared_carries_data_errors():
    """The node's DataError count through RCCL from the C ABI, after cts_counters_allreduce_prepare built the
    clique at start-up: the first all-reduce then pays no communicator set-up (< 100 ms here; the bench reports
    its microseconds), and the set-up breakdown names the prepared clique."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_allreduce_ex_main, args=(q,), daemon=True)
    p.start()
    try:
        r = q.get(timeout=100)
        p.join(15)
    finally:
        if p.is_alive():
            p.kill()
            p.join(5)
    assert not (isinstance(r, tuple) and r[0] == "error"), r[1]
    st = r["setup"]
    assert st["devices"] == 1 and st["prepared"] == 1  # two engines on one GPU: one rank
    assert st["comm_init_ms"] > 0 and st["first_allreduce_ms"] > 0
    after = r["setup_after"]  # the all-reduce reused the prepared clique
    assert {k: v for k, v in after.items() if not k.startswith("last_")} == \
        {k: v for k, v in st.items() if not k.startswith("last_")}
    assert after["last_fold_us"] > 0 and after["last_readback_us"] > 0
    assert after["last_total_us"] >= after["last_fold_us"] + after["last_allreduce_us"] + after["last_readback_us"]
    assert r["first_ex_us"] < 100e3, r["first_ex_us"]
    red, fold, exp = r["two"]
    assert red == fold == exp and exp["connections_failed"] > 0
    red, fold, exp = r["one"]
    assert red == fold == exp and exp["connections_failed"] > 0
    assert p.exitcode == 0
