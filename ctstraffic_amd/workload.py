"""Synthetic workloads for the BASELINE.json configs (host-side descriptor/corruption plans).

Everything here is deterministic from the seeds SURVEY.md §8(d) fixes:

* config 2 — 4096 x 64 KiB resident buffers; expected offsets 75 % phase 0,
  25 % uniform in [0, 65535] (seed 0xC75); 1 in 1024 buffers corrupted by XOR of
  one random byte with a nonzero random value (seed 0xBAD).
* config 3 — 16 M x 1472-byte MediaStream datagrams: 26-byte data header
  (u16 flag 0, i64 seq = i+1, i64 qpc 0, i64 qpf 0 — ctsMediaStreamProtocol.hpp:43-52)
  + P[0..1445]; the payload is verified at expected offset 0
  (ctsIOPatternMediaStream.cpp:185-192). Same corruption rate/seed.
* config 4/5 — 1024 connections x 1024 buffers per 1 M, sharded by
  hash(conn_index) mod G; expected offsets = per-connection exclusive prefix
  sum of lengths mod 65536 (ctsIOPattern.cpp:491-492).

A corruption plan is (buffer index, byte position inside the verified region,
xor value). Because every injected position is distinct per buffer and the xor
is nonzero, the exact reference outcome follows analytically:
first_mismatch = min position, mismatch_bytes = # positions, and the counters
(see :func:`expected_results`) — this is what the full-size GPU tests check.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from .types import DESC_DTYPE

PATTERN_PERIOD = 65536
UDP_DATA_HEADER_LENGTH = 26
SEED_OFFSETS = 0xC75
SEED_CORRUPT = 0xBAD


@dataclass
class Workload:
    name: str
    descs: np.ndarray                    # DESC_DTYPE
    arena_bytes: int
    max_length: int
    corrupt_buf: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    corrupt_pos: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))  # within verified region
    corrupt_xor: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint8))
    n_conns: int = 0
    datagram_headers: bool = False       # write the 26-byte MediaStream data header per buffer

    @property
    def n(self) -> int:
        return len(self.descs)

    def verified_bytes(self) -> int:
        d = self.descs
        return int((d["length"].astype(np.int64) - d["skip_head"].astype(np.int64)).sum())

    def corrupt_abs_offsets(self) -> np.ndarray:
        """Arena byte offsets of the injected corruptions."""
        d = self.descs[self.corrupt_buf]
        return (d["byte_offset"].astype(np.int64) + d["skip_head"].astype(np.int64) + self.corrupt_pos)


def fmix32(x: np.ndarray) -> np.ndarray:
    """murmur3 finaliser: the connection hash used for sharding (hash(conn_index) mod G)."""
    x = np.asarray(x, dtype=np.uint32).astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(13)
    x = (x * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x.astype(np.uint32)


def shard_of(conn_index: np.ndarray, world: int) -> np.ndarray:
    return (fmix32(conn_index) % np.uint32(world)).astype(np.int64)


def _corruption_plan(lengths: np.ndarray, rate: int, seed: int, rng_count: Optional[int] = None):
    """Choose n // rate distinct buffers (none when rate <= 0), one corrupted byte each."""
    n = len(lengths)
    rng = np.random.default_rng(seed)
    if rate <= 0 or n == 0:
        k = 0
    else:
        k = (n // rate) if rng_count is None else rng_count
    eligible = np.nonzero(lengths > 0)[0]
    k = min(k, len(eligible))
    bufs = np.sort(rng.choice(eligible, size=k, replace=False)) if k else np.zeros(0, np.int64)
    pos = (rng.random(k) * lengths[bufs]).astype(np.int64) if k else np.zeros(0, np.int64)
    xor = rng.integers(1, 256, size=k, dtype=np.uint8) if k else np.zeros(0, np.uint8)
    return bufs.astype(np.int64), pos, xor


def tcp_resident(n_buffers: int = 4096, length: int = 65536, corrupt_rate: int = 1024,
                 random_phase_frac: float = 0.25, seed_offsets: int = SEED_OFFSETS,
                 seed_corrupt: int = SEED_CORRUPT, name: str = "config2", conn_base: int = 0) -> Workload:
    """Config 2: n x 64 KiB device-resident buffers, mixed phases, sparse corruption."""
    rng = np.random.default_rng(seed_offsets)
    d = np.zeros(n_buffers, dtype=DESC_DTYPE)
    d["byte_offset"] = np.arange(n_buffers, dtype=np.uint64) * np.uint64(length)
    d["length"] = length
    rand = rng.random(n_buffers) < random_phase_frac
    offs = rng.integers(0, PATTERN_PERIOD, size=n_buffers)
    d["expected_pattern_offset"] = np.where(rand, offs, 0).astype(np.uint32)
    d["conn_index"] = np.arange(n_buffers, dtype=np.uint32) + np.uint32(conn_base)  # rank-disjoint connections
    d["skip_head"] = 0
    lens = d["length"].astype(np.int64)
    cb, cp, cx = _corruption_plan(lens, corrupt_rate, seed_corrupt)
    return Workload(name, d, n_buffers * length, length, cb, cp, cx, n_conns=n_buffers)


def udp_datagrams(n_datagrams: int = 16 * 1024 * 1024, datagram: int = 1472, corrupt_rate: int = 1024,
                  seed_corrupt: int = SEED_CORRUPT, name: str = "config3") -> Workload:
    """Config 3: n x 1472-byte MediaStream datagrams (26-byte header + P[0..1445])."""
    d = np.zeros(n_datagrams, dtype=DESC_DTYPE)
    d["byte_offset"] = np.arange(n_datagrams, dtype=np.uint64) * np.uint64(datagram)
    d["length"] = datagram
    d["expected_pattern_offset"] = 0
    d["conn_index"] = 0
    d["skip_head"] = UDP_DATA_HEADER_LENGTH
    payload = np.full(n_datagrams, datagram - UDP_DATA_HEADER_LENGTH, dtype=np.int64)
    cb, cp, cx = _corruption_plan(payload, corrupt_rate, seed_corrupt)
    return Workload(name, d, n_datagrams * datagram, datagram, cb, cp, cx, n_conns=1, datagram_headers=True)


def connection_streams(n_conns: int = 1024, buffers_per_conn: int = 1024, length: int = 65536,
                       ragged: bool = False, corrupt_rate: int = 1024, seed: int = SEED_OFFSETS,
                       seed_corrupt: int = SEED_CORRUPT, world: int = 1, rank: int = 0,
                       align: int = 16, name: str = "config4") -> Workload:
    """Configs 4/5: per-connection streams, offsets = exclusive prefix sums mod 65536.

    ``ragged`` draws each completion length uniformly in [1, length] (the
    ``-buffer:[lo,hi]`` / partial-completion case); otherwise every completion
    is a full ``length``. Only the connections with hash(conn) mod world == rank
    are materialised; their buffers are packed contiguously in the rank's arena
    (``align``-byte aligned; align=1 packs them tightly so buffer starts take
    every alignment), connection-major in stream order, so
    ``conn_first_fail`` (min failing buffer index per connection) gives the
    first failing buffer in stream order.
    """
    rng = np.random.default_rng(seed)
    conns = np.arange(n_conns, dtype=np.uint32)
    mine = conns[shard_of(conns, world) == rank] if world > 1 else conns
    if ragged:
        all_lens = rng.integers(1, length + 1, size=(n_conns, buffers_per_conn)).astype(np.int64)
    else:
        all_lens = np.full((n_conns, buffers_per_conn), length, dtype=np.int64)
    lens = all_lens[mine]                              # [mine, bpc]
    excl = np.cumsum(lens, axis=1) - lens              # exclusive prefix sum per connection
    offs = (excl % PATTERN_PERIOD).astype(np.uint32)
    n = lens.size
    d = np.zeros(n, dtype=DESC_DTYPE)
    flat_lens = lens.reshape(-1)
    slot = (flat_lens + align - 1) // align * align
    starts = np.cumsum(slot) - slot
    d["byte_offset"] = starts.astype(np.uint64)
    d["length"] = flat_lens.astype(np.uint32)
    d["expected_pattern_offset"] = offs.reshape(-1)
    d["conn_index"] = np.repeat(mine, buffers_per_conn)
    d["skip_head"] = 0
    arena = int(slot.sum()) if n else 16
    cb, cp, cx = _corruption_plan(flat_lens, corrupt_rate, seed_corrupt + rank)
    return Workload(name, d, arena, int(flat_lens.max()) if n else 0, cb, cp, cx, n_conns=n_conns)


def expected_results(w: Workload):
    """Analytic reference outcome of a workload whose only defects are its corruption plan.

    Returns (fail_first[n] int64 (-1 = pass), fail_count[n] int64, counters dict,
    conn_first_fail uint32[n_conns]).
    """
    n = w.n
    first = np.full(n, -1, dtype=np.int64)
    count = np.zeros(n, dtype=np.int64)
    if len(w.corrupt_buf):
        order = np.lexsort((w.corrupt_pos, w.corrupt_buf))
        b, p = w.corrupt_buf[order], w.corrupt_pos[order]
        uniq, idx, cnt = np.unique(b, return_index=True, return_counts=True)
        first[uniq] = p[idx]
        # distinct positions per buffer
        pairs = np.unique(np.stack([b, p], axis=1), axis=0)
        ub, ucnt = np.unique(pairs[:, 0], return_counts=True)
        count[ub] = ucnt
    vlen = w.descs["length"].astype(np.int64) - w.descs["skip_head"].astype(np.int64)
    failed = first >= 0
    counters = {
        "bytes_checked": int(vlen.sum()),
        "bytes_ok": int(vlen[~failed].sum()),
        "buffers_checked": int(n),
        "buffers_failed": int(failed.sum()),
        "mismatched_bytes": int(count.sum()),
    }
    cff = np.full(w.n_conns, 0xFFFFFFFF, dtype=np.uint32)
    if failed.any() and w.n_conns:
        fi = np.nonzero(failed)[0]
        conns = w.descs["conn_index"][fi].astype(np.int64)
        keep = conns < w.n_conns
        np.minimum.at(cff, conns[keep], fi[keep].astype(np.uint32))
    return first, count, counters, cff


def header_bytes(seq: np.ndarray) -> np.ndarray:
    """26-byte MediaStream data headers: u16 flag 0, i64 seq, i64 qpc 0, i64 qpf 0."""
    seq = np.asarray(seq, dtype="<i8")
    h = np.zeros((len(seq), UDP_DATA_HEADER_LENGTH), dtype=np.uint8)
    h[:, 2:10] = seq.view(np.uint8).reshape(-1, 8)
    return h


def materialize(engine, w: Workload, device: str = "cuda", fill_stream=None):
    """Build a workload on the device: arena (the sender's bytes as received,
    produced by the product fill kernel), MediaStream headers, injected
    corruptions. Returns (arena uint8 tensor, descs uint8 tensor)."""
    import torch

    from .engine import descs_to_device

    arena = torch.zeros(((w.arena_bytes + 15) // 16) * 16 + 16, dtype=torch.uint8, device=device)
    arena = arena[: w.arena_bytes] if w.arena_bytes else arena[:16]
    descs = descs_to_device(w.descs, device)
    engine.fill(arena, descs, max_length_hint=w.max_length, stream=fill_stream)
    if w.datagram_headers and w.n:
        dg = int(w.descs["length"][0])
        assert np.all(w.descs["byte_offset"] == np.arange(w.n, dtype=np.uint64) * np.uint64(dg))
        a2 = arena[: w.n * dg].view(w.n, dg)
        seq = torch.arange(1, w.n + 1, dtype=torch.int64, device=device)
        a2[:, 0:2] = 0
        a2[:, 2:10] = seq.view(torch.uint8).view(w.n, 8)
        a2[:, 10:UDP_DATA_HEADER_LENGTH] = 0
    if len(w.corrupt_buf):
        pos = torch.from_numpy(w.corrupt_abs_offsets()).to(device)
        xor = torch.from_numpy(w.corrupt_xor).to(device)
        arena[pos] = arena[pos] ^ xor
    return arena, descs
