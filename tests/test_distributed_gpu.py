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
