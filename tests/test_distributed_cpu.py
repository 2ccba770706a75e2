"""CPU, world_size 2 over gloo: the multi-GPU path's host logic.

Checks that the connection-hash sharding is disjoint and complete, that each
rank's expected offsets are the per-connection prefix sums of the unsharded
stream, and that folding a per-rank counter block and all-reducing it gives the
totals of the whole job (configs 4/5). The per-rank counter
blocks are produced by the oracle standing in for the device (no GPU here);
the GPU kernel's counters are checked against the same oracle in
tests/test_verify_gpu.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from ctstraffic_amd import distributed as D
from ctstraffic_amd import workload as W
from ctstraffic_amd.types import COUNTER_FIELDS, COUNTER_FIELDS_EX

KW = dict(n_conns=48, buffers_per_conn=6, length=4096, ragged=True, corrupt_rate=7, align=1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    try:
        D.init("gloo")
        w = W.connection_streams(world=world, rank=rank, **KW)
        arena = np.zeros(max(w.arena_bytes, 16), dtype=np.uint8)
        oracle.fill(arena, w.descs)
        if len(w.corrupt_buf):
            pos = w.corrupt_abs_offsets()
            arena[pos] ^= w.corrupt_xor
        _, ctr, cff = oracle.verify_batch(arena, w.descs, n_conns=w.n_conns)
        # a device-shaped counter block: 64 shards x 8 u64, this rank's totals spread over two shards
        block = torch.zeros(64 * 8, dtype=torch.int64)
        for k, f in enumerate(COUNTER_FIELDS):
            block[k] = ctr[f] // 2
            block[8 * 5 + k] = ctr[f] - ctr[f] // 2
        c5 = D.fold_counters(block)
        assert D.counters_dict(c5) == ctr
        D.allreduce_counters(c5)
        derr = D.data_error_count(torch.from_numpy(cff.view(np.int32).copy()))
        # the same block with its DataError slot (what the kernels count): six counters in one all-reduce
        block[5] = int((cff != 0xFFFFFFFF).sum())
        c6 = D.fold_counters(block, COUNTER_FIELDS_EX)
        assert D.counters_dict(c6) == {**ctr, "connections_failed": int(block[5])}
        D.allreduce_counters(c6)
        assert D.counters_dict(c6)["connections_failed"] == derr
        assert {f: v for f, v in D.counters_dict(c6).items() if f in COUNTER_FIELDS} == D.counters_dict(c5)
        wall = D.max_over_ranks(float(rank + 1))
        q.put((rank, sorted(set(w.descs["conn_index"].tolist())), D.counters_dict(c5), derr, wall, ctr))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e), 0, 0, None))


def test_world2_sharding_and_counter_allreduce():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r = q.get(timeout=240)
        out[r[0]] = r
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        assert out[r][1] != "error", out[r][2]
    conns = [set(out[r][1]) for r in range(world)]
    assert not (conns[0] & conns[1])                                # disjoint
    assert conns[0] | conns[1] == set(range(KW["n_conns"]))          # complete
    # all-reduced counters == sum of the per-rank truths == the analytic job totals
    total = {f: sum(out[r][5][f] for r in range(world)) for f in COUNTER_FIELDS}
    assert out[0][2] == out[1][2] == total
    exp = {f: 0 for f in COUNTER_FIELDS}
    derr = 0
    for r in range(world):
        w = W.connection_streams(world=world, rank=r, **KW)
        _, _, c, cff = W.expected_results(w)
        for f in COUNTER_FIELDS:
            exp[f] += c[f]
        derr += int((cff != 0xFFFFFFFF).sum())
    assert total == exp and total["buffers_failed"] > 0
    assert out[0][3] == out[1][3] == derr                           # DataError connections
    assert out[0][4] == out[1][4] == 2.0                             # max over ranks


def test_shard_offsets_match_unsharded_stream():
    """A connection's descriptors on its rank carry the same expected offsets as in the 1-rank job."""
    full = W.connection_streams(world=1, rank=0, **KW)
    per_conn = {}
    for d in full.descs:
        per_conn.setdefault(int(d["conn_index"]), []).append((int(d["length"]), int(d["expected_pattern_offset"])))
    for r in range(3):
        w = W.connection_streams(world=3, rank=r, **KW)
        got = {}
        for d in w.descs:
            got.setdefault(int(d["conn_index"]), []).append((int(d["length"]), int(d["expected_pattern_offset"])))
        for c, v in got.items():
            assert v == per_conn[c]
            # exclusive prefix sum of lengths mod 65536 (ctsIOPattern.cpp:491-492)
            acc = 0
            for ln, off in v:
                assert off == acc % 65536
                acc += ln
    shards = W.shard_of(np.arange(1 << 16, dtype=np.uint32), 8)
    counts = np.bincount(shards, minlength=8)
    assert counts.min() > 0.9 * counts.mean()  # the hash balances connections across 8 GPUs
