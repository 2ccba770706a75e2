"""Multi-GPU plumbing for the verify path.

The path shards embarrassingly: each buffer carries its own expected pattern
offset, and connections are assigned to ranks by ``fmix32(conn_index) mod G``
(:func:`ctstraffic_amd.workload.shard_of`), so a connection's first failing
buffer and its DataError decision (ctsSocketState.cpp:221-232) stay on one
rank. The only collective is an optional all-reduce (sum) of the five
ctsStatistics-style counters (ctsStatistics.hpp:87-198) and the DataError
count (ctsSocketState.cpp:221-228) — 48 bytes over RCCL/xGMI (backend
"nccl") or gloo on CPU.
"""
from __future__ import annotations

import os
from typing import Optional

from .types import COUNTER_FIELDS, COUNTER_FIELDS_EX

COUNTER_SLOTS = 8  # u64 per 64-byte counter shard (cts_internal.hpp kCounterSlots)


def dist_env():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


DEFAULT_TIMEOUT_S = 600.0


def init(backend: str, device=None, timeout_s: Optional[float] = DEFAULT_TIMEOUT_S):
    """init_process_group from the env; MASTER_ADDR defaults to 127.0.0.1.

    ``timeout_s`` bounds every collective and barrier of the group (the library default is 10 to 30 min): a rank
    that dies or stalls makes the others raise after that long instead of holding the whole job, and a rank that
    raises exits non-zero, so torch.distributed.run stops the group and returns non-zero."""
    import datetime

    import torch.distributed as dist

    world, rank, _ = dist_env()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {}
    if device is not None:
        kw["device_id"] = device
    if timeout_s is not None:
        kw["timeout"] = datetime.timedelta(seconds=float(timeout_s))
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return world, rank


def new_cpu_group(timeout_s: Optional[float] = DEFAULT_TIMEOUT_S):
    """A gloo group over all ranks for host-side waits, with the same bound."""
    import datetime

    import torch.distributed as dist

    kw = {} if timeout_s is None else {"timeout": datetime.timedelta(seconds=float(timeout_s))}
    return dist.new_group(backend="gloo", **kw)


def fold_counters(counter_block, fields=COUNTER_FIELDS):
    """Device counter block (CTS_COUNTER_SHARDS x 8 int64, cts_counters_device_bytes) -> int64[len(fields)], on the
    block's own device (no host round trip). fields=COUNTER_FIELDS_EX adds the DataError count (connections_failed,
    counted by the verifies given a conn_first_fail array)."""
    assert tuple(fields) == COUNTER_FIELDS_EX[: len(fields)], fields
    return counter_block.view(-1, COUNTER_SLOTS)[:, : len(fields)].sum(0)


def allreduce_counters(counters, group=None):
    """In-place sum of the folded counters over all ranks (ctsStatsTracking::Add across GPUs)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters


def counters_dict(counters) -> dict:
    """Folded counters (5, or 6 with connections_failed) -> {field: value}."""
    vals = [int(x) for x in counters.tolist()]
    return dict(zip(COUNTER_FIELDS_EX, vals))


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a float over ranks (the timed region's wall time)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def data_error_count(conn_first_fail, group=None) -> int:
    """DataError count: connections whose first failing buffer exists (slot != 0xFFFFFFFF),
    summed over ranks (connections are rank-local, so the sum is exact)."""
    import torch
    import torch.distributed as dist

    n = (conn_first_fail.view(torch.int32) != -1).sum().to(torch.int64).reshape(1)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(n, op=dist.ReduceOp.SUM, group=group)
    return int(n.item())


def gather_rank_rows(row, group=None) -> list:
    """Every rank's row of floats, in rank order (an all-gather over `group`, the gloo group in bench.py); at world
    size 1, [row]. bench.py's per-rank diagnostics: kernel time, engine device, torch device, placement check."""
    import torch
    import torch.distributed as dist

    mine = torch.tensor([float(x) for x in row], dtype=torch.float64)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return [mine.tolist()]
    rows = [torch.zeros_like(mine) for _ in range(dist.get_world_size(group))]
    dist.all_gather(rows, mine, group=group)
    return [r.tolist() for r in rows]


__all__ = ["dist_env", "init", "new_cpu_group", "DEFAULT_TIMEOUT_S", "fold_counters", "allreduce_counters", "counters_dict", "max_over_ranks",
           "data_error_count", "gather_rank_rows"]
