"""GPU: seeded fill -> corrupt -> verify round trips over every kernel path, against the oracle (integer work:
bit-exact).

Each case draws a descriptor set (lengths up to the case's maximum, byte offsets at any alignment, skips, phases
near the period's ends, some descriptors the reference would FAIL_FAST on, ctsIOPattern.cpp:723-725) and a
`max_length_hint` that selects the path: 0 (a workgroup per buffer), 64 / 1472 (the datagram kernels), 8192 / 65536
and hints below the true maximum (the fill's piece order, whose last piece of a buffer takes the rest). The GPU fills
a garbage arena and must leave exactly the bytes `oracle.fill` leaves; bytes are then flipped on the host (single,
bursts, first and last span bytes) and the GPU verify's per-buffer results, counters (DataError count included) and
per-connection first failures must equal `oracle.verify_batch` on the same bytes.
"""
import numpy as np
import pytest

import oracle
from ctstraffic_amd.types import DESC_DTYPE, RESULT_DTYPE

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda"
N_CONNS = 11


def _to_dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(DEV)


def _case(seed):
    rng = np.random.default_rng(0xF0220 + seed)
    max_len = int(rng.choice([40, 1472, 5000, 70000, 140000]))
    n = int(rng.integers(1, 400 if max_len <= 5000 else 80))
    hints = [0, 8192, 65536, max_len, max(1, max_len // 3)] + ([64, 1472] if max_len <= 1472 else [])
    hint = int(rng.choice(hints))
    descs = np.zeros(n, dtype=DESC_DTYPE)
    off = 0
    for i in range(n):
        off += int(rng.integers(0, 17)) if rng.random() < 0.5 else (-off) % 16
        ln = int(rng.integers(0, max_len + 1)) if rng.random() < 0.8 else max_len
        skip = min(ln, int(rng.integers(0, 40))) if rng.random() < 0.3 else 0
        exp = int(rng.integers(0, 65536)) if rng.random() < 0.7 else int(rng.choice([0, 1, 65535, 65534, 32767]))
        descs[i] = (off, ln, exp, int(rng.integers(0, N_CONNS)), skip)
        off += ln
    for i in rng.choice(n, size=n // 25, replace=False):  # FAIL_FAST shapes: nothing filled, flagged by the verify
        if rng.random() < 0.5:
            descs[i]["expected_pattern_offset"] = 65536
        else:
            descs[i]["skip_head"] = int(descs[i]["length"]) + 1
    garbage = rng.integers(0, 256, size=off + 64, dtype=np.uint8)
    return rng, descs, garbage, hint


def _corrupt(rng, arena, descs):
    for i in range(len(descs)):
        d = descs[i]
        v = int(d["length"]) - int(d["skip_head"])
        if v <= 0 or d["expected_pattern_offset"] >= 65536 or rng.random() > 0.3:
            continue
        base = int(d["byte_offset"]) + int(d["skip_head"])
        kind = int(rng.integers(0, 4))
        if kind == 0:
            ps = [int(rng.integers(0, v))]
        elif kind == 1:
            s = int(rng.integers(0, v))
            ps = list(range(s, min(v, s + int(rng.integers(1, 40)))))
        else:
            ps = [0 if kind == 2 else v - 1]
        for p in ps:
            arena[base + p] ^= int(rng.integers(1, 256))


@pytest.mark.parametrize("seed", range(64))
def test_fill_corrupt_verify_round_trip(engine, seed):
    rng, descs, garbage, hint = _case(seed)
    d = _to_dev(descs)
    # fill: the GPU's bytes are the oracle's, untouched bytes included
    exp = garbage.copy()
    oracle.fill(exp, descs)
    arena = _to_dev(garbage)
    engine.fill(arena, d, max_length_hint=hint)
    torch.cuda.synchronize()
    got = arena.cpu().numpy()
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, ("fill", seed, hint, bad[:8])
    # corrupt on the host, verify on the GPU, compare with the oracle on the same bytes
    _corrupt(rng, got, descs)
    arena = _to_dev(got)
    res = engine.new_results(len(descs))
    ctr = engine.new_counters()
    cff = torch.full((N_CONNS,), -1, dtype=torch.int32, device=DEV)
    engine.verify(arena, d, max_length_hint=hint, results=res, counters=ctr, conn_first_fail=cff)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(RESULT_DTYPE)
    er, ectr, ecff = oracle.verify_batch(got, descs, n_conns=N_CONNS)
    for f in ("first_mismatch", "mismatch_bytes", "expected", "actual", "pass", "flags"):
        diff = np.nonzero(r[f] != er[f])[0]
        assert diff.size == 0, ("verify", seed, hint, f, diff[:8])
    c = engine.read_counters_ex(ctr)
    assert {k: c[k] for k in ectr} == ectr, (seed, hint)
    f = cff.cpu().numpy().view(np.uint32)
    assert np.array_equal(f, ecff), (seed, hint)
    assert c["connections_failed"] == int((ecff != 0xFFFFFFFF).sum())
