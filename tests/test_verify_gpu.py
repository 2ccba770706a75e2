"""GPU parity: the gfx950 fill/verify kernels through the C ABI vs the oracle.

Every test compares the HIP path with the CPU oracle (oracle/cts_oracle.c) on
the same seeded bytes at sizes the oracle finishes in seconds, or with the
committed golden vectors; full BASELINE sizes are checked through the analytic
outcome of the injected corruption plan (ctstraffic_amd.workload.expected_results),
which test_workload.py pins against the oracle on CPU. Integer/byte work: the
bar is bit-exact.
"""
import json
import os

import numpy as np
import pytest

import oracle
from ctstraffic_amd import workload as W
from ctstraffic_amd.types import DESC_DTYPE, RESULT_DTYPE

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"


def to_dev(a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(DEV)


def run_verify(engine, arena_np, descs, hint, n_conns=0):
    arena = to_dev(arena_np) if arena_np.size else torch.zeros(16, dtype=torch.uint8, device=DEV)
    d = to_dev(descs)
    res = engine.new_results(len(descs))
    ctr = engine.new_counters()
    cff = torch.full((n_conns,), -1, dtype=torch.int32, device=DEV) if n_conns else None
    engine.verify(arena[: arena_np.size] if arena_np.size else arena[:0], d, max_length_hint=hint, results=res,
                  counters=ctr, conn_first_fail=cff)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(RESULT_DTYPE)
    c = engine.read_counters(ctr)
    f = cff.cpu().numpy().view(np.uint32) if n_conns else np.zeros(0, np.uint32)
    return r, c, f


def assert_results_equal(got, exp, ctx=""):
    for f in ("first_mismatch", "mismatch_bytes", "expected", "actual", "pass", "flags"):
        bad = np.nonzero(got[f] != exp[f])[0]
        assert bad.size == 0, "%s field %s differs at %s: got %s exp %s" % (
            ctx, f, bad[:8], got[f][bad[:8]], exp[f][bad[:8]])


# ---------------------------------------------------------------------------------------------
def test_golden_vectors(engine):
    vec = json.load(open(os.path.join(GOLDEN, "verify_vectors.json")))
    cases = vec["cases"]
    arena = bytearray()
    descs = np.zeros(len(cases), dtype=DESC_DTYPE)
    for i, c in enumerate(cases):
        arena += bytes(i % 13)
        b = bytes.fromhex(c["buffer_hex"])
        descs[i] = (len(arena), c["buffer_offset"] + c["transferred"], c["expected_offset"], i, c["buffer_offset"])
        arena += b
    a = np.frombuffer(bytes(arena), dtype=np.uint8).copy()
    for hint in (0, 1472):  # workgroup-per-buffer and wave-per-buffer kernels
        r, ctr, _ = run_verify(engine, a, descs, hint)
        for i, c in enumerate(cases):
            e = c["result"]
            assert r[i]["first_mismatch"] == e["first_mismatch"], c["name"]
            assert bool(r[i]["pass"]) == e["pass"], c["name"]
            assert r[i]["mismatch_bytes"] == e["mismatch_bytes"], c["name"]
            assert (r[i]["expected"], r[i]["actual"]) == (e["expected"], e["actual"]), c["name"]
        assert ctr["buffers_failed"] == sum(1 for c in cases if not c["result"]["pass"])


@pytest.mark.parametrize("max_buf", [0, 1, 15, 1446, 4096, 65536, 65537, 262144 + 3])
def test_sender_buffer_fill(engine, max_buf):
    S = engine.sender_buffer(max_buf)
    torch.cuda.synchronize()
    assert np.array_equal(S.cpu().numpy(), oracle.sender_buffer(max_buf))


def _random_case(rng, n, max_len, align_mix=True, corrupt_frac=0.3, skip=False, whole=False):
    """whole: every span starts on a 128-byte line and is a multiple of 16 bytes
    (the streamed-without-edges path of verify variants 9/10; a third are 64 KiB)."""
    lens = rng.integers(0, max_len + 1, size=n)
    if whole:
        lens = np.where(rng.random(n) < 0.33, 65536, lens // 16 * 16)
        skip = False
    descs = np.zeros(n, dtype=DESC_DTYPE)
    off = 0
    for i in range(n):
        if whole:
            off += (-off) % 128
        else:
            off += int(rng.integers(0, 17)) if align_mix else (-off) % 16
        descs[i]["byte_offset"] = off
        descs[i]["length"] = lens[i]
        descs[i]["skip_head"] = min(int(lens[i]), int(rng.integers(0, 40))) if skip else 0
        descs[i]["expected_pattern_offset"] = int(rng.integers(0, 65536)) if rng.random() < 0.7 else int(
            rng.choice([0, 1, 65535, 65534, 65520, 65521, 32767, 32768]))
        descs[i]["conn_index"] = int(rng.integers(0, 7))
        off += int(lens[i])
    arena = rng.integers(0, 256, size=off + 64, dtype=np.uint8)
    oracle.fill(arena, descs)
    # corrupt: single bytes, bursts, and edge bytes (first / last of the verified span)
    for i in range(n):
        v = int(descs[i]["length"]) - int(descs[i]["skip_head"])
        if v <= 0 or rng.random() > corrupt_frac:
            continue
        base = int(descs[i]["byte_offset"]) + int(descs[i]["skip_head"])
        kind = rng.integers(0, 5)
        if kind == 4:  # scattered bytes: several waves / lanes of one team see mismatches
            ps = sorted(set(int(x) for x in rng.integers(0, v, size=int(rng.integers(2, 9)))))
        elif kind == 0:
            ps = [int(rng.integers(0, v))]
        elif kind == 1:
            s = int(rng.integers(0, v))
            ps = list(range(s, min(v, s + int(rng.integers(1, 40)))))
        elif kind == 2:
            ps = [0]
        else:
            ps = [v - 1]
        for p in ps:
            arena[base + p] ^= int(rng.integers(1, 256))
    return arena, descs


@pytest.mark.parametrize("seed,n,max_len,hint,skip", [
    (1, 300, 200, 1472, False),
    (2, 300, 200, 0, False),
    (3, 200, 5000, 0, True),
    (4, 200, 5000, 8192, True),
    (5, 64, 70000, 0, False),
    (6, 64, 140000, 0, False),
    (7, 500, 40, 64, True),
])
def test_random_parity_vs_oracle(engine, seed, n, max_len, hint, skip):
    rng = np.random.default_rng(seed)
    arena, descs = _random_case(rng, n, max_len, skip=skip)
    r, ctr, cff = run_verify(engine, arena, descs, hint, n_conns=7)
    er, ectr, ecff = oracle.verify_batch(arena, descs, n_conns=7)
    assert_results_equal(r, er, "seed %d" % seed)
    assert ctr == ectr
    assert np.array_equal(cff, ecff)


def test_bad_descriptors(engine):
    arena = np.zeros(256, np.uint8)
    oracle.fill(arena, np.array([(0, 256, 0, 0, 0)], dtype=oracle.DESC_DTYPE))
    d = np.zeros(5, dtype=DESC_DTYPE)
    d[0] = (0, 10, 65536, 0, 0)   # expected offset out of period
    d[1] = (0, 10, 0, 0, 11)      # length < skip_head
    d[2] = (250, 10, 0, 0, 0)     # crosses the arena end
    d[3] = (2**40, 1, 0, 0, 0)    # far out of the arena
    d[4] = (16, 32, 16, 0, 0)     # valid
    r, ctr, _ = run_verify(engine, arena, d, 0)
    er, ectr, _ = oracle.verify_batch(arena, d)
    assert_results_equal(r, er)
    assert list(r["flags"]) == [1, 1, 1, 1, 0] and r[4]["pass"] == 1
    assert ctr == ectr and ctr["buffers_checked"] == 1


def test_bad_descriptors_interleaved(engine):
    """Bad descriptors interleaved with valid and corrupt buffers, one and many workgroups (each workgroup then walks
    bad, clean and corrupt buffers in turn), vs the oracle."""
    from ctstraffic_amd import _lib

    eng = engine
    dbpc = eng.get_attr(_lib.ATTR_BLOCKS_PER_CU)
    rng = np.random.default_rng(77)
    arena = np.zeros(1 << 20, np.uint8)
    oracle.fill(arena, np.array([(0, 1 << 20, 0, 0, 0)], dtype=oracle.DESC_DTYPE))
    d = np.zeros(203, dtype=DESC_DTYPE)
    for k in range(len(d)):
        if k % 5 == 3:
            d[k] = ((1 << 20) - 4, 64, 0, k % 7, 0)  # crosses the arena end
        else:
            ln = int(rng.integers(9000, 20000))
            off = int(rng.integers(0, (1 << 20) - ln))
            d[k] = (off, ln, off % 65536, k % 7, int(rng.integers(0, 30)))
    for k in rng.choice(len(d), 20, replace=False):  # corrupt some valid buffers
        if k % 5 != 3:
            arena[int(d[k]["byte_offset"]) + int(d[k]["length"]) - 1] ^= 0x11
    try:
        for bpc in (1, 16):
            eng.set_attr(_lib.ATTR_BLOCKS_PER_CU, bpc)
            r, ctr, cff = run_verify(eng, arena, d, 0, n_conns=7)
            er, ectr, ecff = oracle.verify_batch(arena, d, n_conns=7)
            assert_results_equal(r, er, "bpc %d" % bpc)
            assert ctr == ectr and np.array_equal(cff, ecff)
    finally:
        eng.set_attr(_lib.ATTR_BLOCKS_PER_CU, dbpc)


def test_misaligned_descriptor_array_is_rejected(engine):
    """The kernels read descriptors as u64 fields: a descriptor array that is not
    8-byte aligned is refused with CTS_E_INVALID, before any launch. So are outputs the kernels would write
    misaligned (dword records and DataError slots, 64-bit counter atomics)."""
    from ctstraffic_amd._lib import CtsError

    arena = torch.zeros(256, dtype=torch.uint8, device=DEV)
    raw = torch.zeros(DESC_DTYPE.itemsize * 2 + 8, dtype=torch.uint8, device=DEV)
    with pytest.raises(CtsError):
        engine.verify(arena, raw[4:4 + DESC_DTYPE.itemsize], max_length_hint=0)
    with pytest.raises(CtsError):
        engine.fill(arena, raw[4:4 + DESC_DTYPE.itemsize], max_length_hint=0)
    d = raw[:DESC_DTYPE.itemsize]
    res = engine.new_results(2)
    ctr = engine.new_counters()
    nb = ctr.numel() * ctr.element_size()
    ctr_raw = torch.zeros(nb + 16, dtype=torch.uint8, device=DEV)
    cff = torch.full((4,), -1, dtype=torch.int32, device=DEV).view(torch.uint8)
    with pytest.raises(CtsError):
        engine.verify(arena, d, max_length_hint=0, results=res.view(torch.uint8)[2:2 + 12])
    with pytest.raises(CtsError):
        engine.verify(arena, d, max_length_hint=0, counters=ctr_raw[4:4 + nb])
    with pytest.raises(CtsError):
        engine.verify(arena, d, max_length_hint=0, conn_first_fail=cff[2:10])
    engine.verify(arena, d, max_length_hint=0, results=res, counters=ctr_raw[8:8 + nb], conn_first_fail=cff[4:12])
    torch.cuda.synchronize()


@pytest.mark.parametrize("fill_nt", [0, 1, 2])
def test_fill_matches_oracle_and_leaves_neighbours(engine, fill_nt):
    from ctstraffic_amd import _lib

    default_nt = engine.get_attr(_lib.ATTR_FILL_NT)
    engine.set_attr(_lib.ATTR_FILL_NT, fill_nt)
    try:
        _fill_vs_oracle(engine)
    finally:
        engine.set_attr(_lib.ATTR_FILL_NT, default_nt)


def _fill_vs_oracle(engine):
    rng = np.random.default_rng(11)
    # aligned: 16-byte-aligned spans of whole chunks (the fill's straight-line store rounds;
    # a third are 64 KiB, phases odd and even), with 16-byte gaps that must stay untouched
    # hints: 0 (unknown: one workgroup per buffer), 1472 (the datagram path), 65536 and 70000 (the piece order,
    # fill_pieces_kernel: 8 and 9 pieces per buffer) and 9000 (under the true maximum: the last piece of a buffer
    # takes the rest)
    for hint, aligned in ((0, False), (1472, False), (0, True), (1472, True), (65536, False), (65536, True),
                          (70000, False), (9000, False), (9000, True)):
        n = 400
        descs = np.zeros(n, dtype=DESC_DTYPE)
        off = 0
        for i in range(n):
            if aligned:
                off += 16 * int(rng.integers(0, 3))
                ln = 65536 if rng.random() < 0.33 else 16 * int(rng.integers(0, (3000 if hint == 1472 else 70000) // 16))
                descs[i] = (off, ln, int(rng.integers(0, 65536)), 0, 0)
            else:
                off += int(rng.integers(0, 9))
                ln = int(rng.integers(0, 3000 if hint == 1472 else 70000))
                descs[i] = (off, ln, int(rng.integers(0, 65536)), 0, int(rng.integers(0, min(ln, 30) + 1)))
            off += ln
        init = rng.integers(0, 256, size=off + 32, dtype=np.uint8)
        exp = init.copy()
        oracle.fill(exp, descs)
        arena = to_dev(init)
        engine.fill(arena, to_dev(descs), max_length_hint=hint)
        torch.cuda.synchronize()
        got = arena.cpu().numpy()
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, bad[:10]


@pytest.mark.parametrize("hint", [0, 1472, 65536, 9000])
def test_fill_skips_bad_descriptors(engine, hint):
    """Descriptors the reference would FAIL_FAST on or that leave the arena (expected offset >= 65536,
    ctsIOPattern.cpp:723-725; a skip longer than the buffer; a span past the arena's end, straddling it or wholly
    beyond) write nothing on every fill path (hint 0: workgroup per buffer, 1472: the datagram path, 65536 / 9000: the
    piece order), the bytes past the arena inside the same allocation included; the valid ones around them are filled
    as the oracle fills them (it skips the same descriptors)."""
    rng = np.random.default_rng(0xBAD)
    n, N = 300, 0
    descs = np.zeros(n, dtype=DESC_DTYPE)
    big = hint in (65536, 9000)
    for i in range(n):
        ln = 65536 if big and rng.random() < 0.5 else int(rng.integers(1, 1473 if hint == 1472 else 70000))
        descs[i] = (N, ln, int(rng.integers(0, 65536)), i, int(rng.integers(0, min(ln, 30) + 1)))
        N += ln + int(rng.integers(0, 9))
    arena_bytes = N - 5000  # the last buffers straddle or lie past the end
    bad = rng.choice(n - 10, size=30, replace=False)
    for k, i in enumerate(bad):
        if k % 3 == 0:
            descs[i]["expected_pattern_offset"] = 65536 + k
        elif k % 3 == 1:
            descs[i]["skip_head"] = int(descs[i]["length"]) + 1
        else:
            descs[i]["byte_offset"] = arena_bytes + 64 * k  # past the end
    past = descs["byte_offset"].astype(np.int64) + descs["length"] > arena_bytes
    assert past.sum() > 10 and (descs["byte_offset"][past] < arena_bytes).any()  # straddling ones too
    init = rng.integers(0, 256, size=N + 4096, dtype=np.uint8)
    exp = init.copy()
    oracle.fill(exp[:arena_bytes], descs)
    base = to_dev(init)
    engine.fill(base[:arena_bytes], to_dev(descs), max_length_hint=hint)
    torch.cuda.synchronize()
    diff = np.nonzero(base.cpu().numpy() != exp)[0]
    assert diff.size == 0, diff[:10]
    assert not np.array_equal(exp, init)  # the valid buffers were written


def test_counters_accumulate_and_reset(engine):
    w = W.tcp_resident(n_buffers=256, corrupt_rate=64)
    arena, descs = W.materialize(engine, w)
    ctr = engine.new_counters()
    for _ in range(3):
        engine.verify(arena, descs, max_length_hint=w.max_length, counters=ctr)
    c = engine.read_counters(ctr)
    _, _, ec, _ = W.expected_results(w)
    assert c == {k: 3 * v for k, v in ec.items()}
    engine.reset_counters(ctr)
    assert all(v == 0 for v in engine.read_counters(ctr).values())


# ---- BASELINE configs ---------------------------------------------------------------------------
def _check_workload(engine, w, with_oracle: bool):
    arena, descs = W.materialize(engine, w)
    res = engine.new_results(w.n)
    ctr = engine.new_counters()
    cff = torch.full((w.n_conns,), -1, dtype=torch.int32, device=DEV) if w.n_conns else None
    engine.verify(arena, descs, max_length_hint=w.max_length, results=res, counters=ctr, conn_first_fail=cff)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(RESULT_DTYPE)
    c = engine.read_counters(ctr)
    first, count, ec, ecff = W.expected_results(w)
    assert c == ec
    failed = first >= 0
    assert np.array_equal(r["pass"] == 0, failed)
    vlen = w.descs["length"].astype(np.int64) - w.descs["skip_head"].astype(np.int64)
    assert np.array_equal(r["first_mismatch"].astype(np.int64), np.where(failed, first, vlen))
    assert np.array_equal(r["mismatch_bytes"].astype(np.int64), count)
    if w.n_conns:
        assert np.array_equal(cff.cpu().numpy().view(np.uint32), ecff)
    if with_oracle:
        host = arena.cpu().numpy()
        er, ectr, _ = oracle.verify_batch(host, w.descs, nthreads=8)
        assert_results_equal(r, er, w.name)
        assert c == ectr
    else:
        _sampled_oracle_check(arena, w, r)
    del arena, descs, res


def _sample_indices(w):
    """The buffers a full-size test re-checks with the oracle: every 4096th, every corrupted one, and the first
    and last buffer starting in each 4 GiB window of the arena (offsets past 4 GiB and 16 GiB included)."""
    off = w.descs["byte_offset"].astype(np.int64)
    win = off >> 32
    firsts = np.unique(win, return_index=True)[1]
    lasts = len(win) - 1 - np.unique(win[::-1], return_index=True)[1]
    step = max(1, min(4096, w.n // 4096))  # at least ~4 k buffers
    idx = np.unique(np.concatenate([np.arange(0, w.n, step), w.corrupt_buf, firsts, lasts]))
    return idx.astype(np.int64)


def _gather_spans(arena, offs, lens, chunk=512):
    """Copy buffers [offs[i], offs[i] + lens[i]) of a device arena into a compact host arena with a fixed
    16-byte-aligned stride (chunked gather on the device)."""
    stride = int(((int(lens.max()) + 15) // 16) * 16)
    out = np.zeros(len(offs) * stride, dtype=np.uint8)
    col = torch.arange(stride, device=arena.device, dtype=torch.int64)
    last = arena.numel() - 1
    for s in range(0, len(offs), chunk):
        o = torch.from_numpy(offs[s:s + chunk]).to(arena.device)
        idx = (o[:, None] + col[None, :]).clamp_(max=last)
        out[s * stride:(s + len(o)) * stride] = arena[idx.reshape(-1)].cpu().numpy()
    return out, stride


def _sampled_oracle_check(arena, w, r):
    """Breaks the common mode of a full-size test: the arena was written by the product fill kernel and is
    verified by the product verify kernel, which share one pattern generator. Here the sampled buffers' bytes
    are copied back and (1) compared with the oracle's own fill of the same spans plus the corruption plan, and
    (2) verified by the oracle, every result field compared with the GPU's."""
    idx = _sample_indices(w)
    assert len(idx) >= 4000 or len(idx) == w.n
    d = w.descs[idx]
    host, stride = _gather_spans(arena, d["byte_offset"].astype(np.int64), d["length"].astype(np.int64))
    cd = d.copy()
    cd["byte_offset"] = np.arange(len(idx), dtype=np.uint64) * np.uint64(stride)
    # (1) the fill's bytes vs the oracle's fill (payload only: MediaStream headers are not the fill's)
    exp = host.copy()
    oracle.fill(exp, cd)
    pos_in = np.searchsorted(idx, w.corrupt_buf)
    assert np.array_equal(idx[pos_in], w.corrupt_buf)
    at = cd["byte_offset"][pos_in].astype(np.int64) + cd["skip_head"][pos_in].astype(np.int64) + w.corrupt_pos
    exp[at] ^= w.corrupt_xor
    bad = np.nonzero(exp != host)[0]
    assert bad.size == 0, ("fill differs from the oracle's", bad[:8] // stride, bad[:8] % stride)
    # (2) the oracle's verify of the same bytes vs the GPU's records
    er, _, _ = oracle.verify_batch(host, cd, nthreads=8)
    assert_results_equal(r[idx], er, w.name + " (sampled)")
    far = d["byte_offset"].astype(np.int64)
    for gib in (4, 16):
        if w.arena_bytes > (gib + 1) << 30:
            assert (far >= gib << 30).sum() >= 2, gib


def test_config2_full_vs_oracle(engine):
    """4096 x 64 KiB resident, 25 % random phases, 1/1024 corrupted — exact vs the oracle."""
    _check_workload(engine, W.tcp_resident(), with_oracle=True)


def test_config2_dense_corruption_vs_oracle(engine):
    _check_workload(engine, W.tcp_resident(n_buffers=2048, corrupt_rate=3, random_phase_frac=0.9), with_oracle=True)


def test_config3_scaled_vs_oracle(engine):
    """MediaStream datagrams (26-byte header + P[0..1445]) at 1/64 of the config size, vs the oracle."""
    _check_workload(engine, W.udp_datagrams(n_datagrams=256 * 1024, corrupt_rate=97), with_oracle=True)


def test_config3_full_size(engine):
    """16 M x 1472 B (23 GiB) — checked against the analytic outcome of the corruption plan."""
    _check_workload(engine, W.udp_datagrams(), with_oracle=False)


def test_config4_ragged_unaligned_vs_oracle(engine):
    """Per-connection prefix-sum offsets with ragged completions and unaligned buffer starts."""
    w = W.connection_streams(n_conns=64, buffers_per_conn=64, ragged=True, align=1, corrupt_rate=50, world=2, rank=1)
    _check_workload(engine, w, with_oracle=True)


def test_config4_full_shard(engine):
    """1 M x 64 KiB hash-sharded over 4 GPUs: this GPU verifies rank 0's shard (~16 GiB)."""
    _check_workload(engine, W.connection_streams(world=4, rank=0), with_oracle=False)
    torch.cuda.empty_cache()


def test_config4_full_shard_two_gpus(engine):
    """Config 4's first step, 1 M x 64 KiB hash-sharded over 2 GPUs: this GPU verifies rank 0's shard (~32 GiB
    resident at once), checked against the analytic outcome and, for >= 4 k sampled buffers, the oracle."""
    w = W.connection_streams(world=2, rank=0)
    assert w.verified_bytes() > 30 * 2**30
    _check_workload(engine, w, with_oracle=False)
    torch.cuda.empty_cache()


def test_config5_full_shard(engine):
    """8 M x 64 KiB over 8 GPUs (512 GiB): this GPU verifies rank 0's hash shard, ~1 M buffers = ~64 GiB
    resident at once, checked against the analytic outcome (per-buffer records, counters, DataError slots)."""
    w = W.connection_streams(n_conns=8192, buffers_per_conn=1024, world=8, rank=0, name="config5")
    assert w.verified_bytes() > 60 * 2**30
    _check_workload(engine, w, with_oracle=False)
    torch.cuda.empty_cache()


# ---- host-buffer paths ------------------------------------------------------------------------------
@pytest.fixture(params=[1, 0], ids=["mailbox", "launch"])
def host_path(engine, request):
    """cts_verify_host through the mailbox grid (CTS_ATTR_SYNC_MAILBOX = 1, the default) or one sliced launch +
    synchronize per call (0)."""
    from ctstraffic_amd import _lib

    engine.set_attr(_lib.ATTR_SYNC_MAILBOX, request.param)
    yield engine
    engine.set_attr(_lib.ATTR_SYNC_MAILBOX, 1)


def test_verify_host_single(host_path):
    engine = host_path
    S = oracle.sender_buffer(70000)
    for e, n in [(0, 10), (0, 0), (4, 6), (65535, 100), (123, 65536), (1, 70000 - 1)]:
        buf = S[e:e + n].copy()
        assert engine.verify_host(buf, e)["pass"]
        if n:
            k = n // 2
            buf[k] ^= 0x80
            r = engine.verify_host(buf, e)
            o = oracle.verify_buffer(buf, 0, e, n)
            assert (r["pass"], r["first_mismatch"], r["expected"], r["actual"], r["mismatch_bytes"]) == (
                o["pass"], o["first_mismatch"], o["expected"], o["actual"], o["mismatch_bytes"])
    # MSTest TestBaseClass_InvalidBytesOnRecv: 10 zero bytes at offset 0 fail at byte 2
    r = engine.verify_host(np.zeros(10, np.uint8), 0)
    assert not r["pass"] and r["first_mismatch"] == 2


def test_verify_host_single_slice_edges(host_path):
    """cts_verify_host reads one buffer as up to 64 slices (csrc/cts_slices.hpp) or as the mailbox's 4 KiB
    pieces; corruptions on slice edges, in two slices at once, and ragged last slices fold back to the oracle's
    whole-buffer result."""
    engine = host_path
    S = oracle.sender_buffer(140000)
    rng = np.random.default_rng(0x51CE)
    for n in (1023, 1024, 1025, 4097, 65536, 65537, 100000, 131072):
        sl = max(1024, ((n + 63) // 64 + 15) // 16 * 16)
        for trial in range(6):
            e = int(rng.integers(0, 65536))
            buf = S[e:e + n].copy()
            picks = {0: [0], 1: [n - 1], 2: [min(sl, n - 1)], 3: [min(sl - 1, n - 1)],
                     4: [n - 1, int(rng.integers(0, n))], 5: sorted({int(x) for x in rng.integers(0, n, 3)})}[trial]
            for k in picks:
                buf[k] ^= int(rng.integers(1, 256))
            r = engine.verify_host(buf, e)
            o = oracle.verify_buffer(buf, 0, e, n)
            assert (r["pass"], r["first_mismatch"], r["expected"], r["actual"], r["mismatch_bytes"]) == (
                o["pass"], o["first_mismatch"], o["expected"], o["actual"], o["mismatch_bytes"]), (n, trial)


def test_verify_host_threads(engine):
    """cts_verify_host from 8 threads at once (a Level-1 VerifyBuffer drop-in called by concurrent IOCP threads):
    each call stages into a pinned buffer of its own and posts to the mailbox; every answer is the oracle's."""
    import threading

    S = oracle.sender_buffer(140000)
    errors = []

    def worker(t):
        rng = np.random.default_rng(0x4057 + t)
        try:
            for it in range(40):
                n = int(rng.choice([0, 1, 17, 4096, 65536, 70001]))
                e = int(rng.integers(0, 65536))
                buf = S[e:e + n].copy()
                if n and rng.random() < 0.5:
                    buf[int(rng.integers(0, n))] ^= int(rng.integers(1, 256))
                r = engine.verify_host(buf, e)
                o = oracle.verify_buffer(buf, 0, e, n)
                got = (r["pass"], r["first_mismatch"], r["expected"], r["actual"], r["mismatch_bytes"])
                want = (o["pass"], o["first_mismatch"], o["expected"], o["actual"], o["mismatch_bytes"])
                if got != want:
                    errors.append((t, it, n, e, got, want))
        except Exception as ex:  # surfaced below
            errors.append((t, repr(ex)))

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]


def test_verify_mapped_mailbox_threads(engine):
    """cts_verify_mapped from 16 threads at once (SYNC verifies of concurrent connections) through the
    resident mailbox grid, over buffers in separate pinned arenas that every thread rewrites between calls
    (a reused recv slot: nothing may be answered from a cache); every caller must get exactly the oracle's
    record for its own buffer (ctsIOPattern.cpp:745-775)."""
    import threading
    S = oracle.sender_buffer(140000)
    T, ITERS, CAP = 16, 40, 70000
    arenas = [engine.host_alloc(CAP) for _ in range(T)]
    errors = []

    def worker(t):
        arr, _, dev = arenas[t]
        rng = np.random.default_rng(0xC0A1 + t)
        try:
            for it in range(ITERS):
                n = int(rng.choice([0, 1, 1023, 1024, 1025, 4097, 65536, 65537, CAP - 16]))
                e = int(rng.integers(0, 65536))
                at = int(rng.integers(0, 16)) if n <= CAP - 16 else 0
                arr[at:at + n] = S[e:e + n]
                if n and rng.random() < 0.5:
                    for k in sorted({int(x) for x in rng.integers(0, n, int(rng.integers(1, 4)))}):
                        arr[at + k] ^= int(rng.integers(1, 256))
                r = engine.verify_mapped(dev + at, n, e)
                o = oracle.verify_buffer(arr[at:at + n].copy(), 0, e, n)
                got = (r["pass"], r["first_mismatch"], r["expected"], r["actual"], r["mismatch_bytes"])
                want = (o["pass"], o["first_mismatch"], o["expected"], o["actual"], o["mismatch_bytes"])
                if got != want:
                    errors.append((t, it, n, e, got, want))
        except Exception as ex:  # surfaced below
            errors.append((t, repr(ex)))

    try:
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    finally:
        for _, h, _ in arenas:
            engine.host_free(h)
    assert not errors, errors[:5]


def test_verify_mapped_mailbox_small_rings(monkeypatch):
    """A fresh engine whose mailbox has 2 groups of 8 job slots (CTS_MAILBOX_GROUPS / CTS_MAILBOX_SLOTS, read when
    the grid is first set up): 12 threads post at once, so each group's ring wraps many times, posters wait for
    slots whose previous job is still being answered, and the least-busy assignment keeps both groups busy.
    Every answer must still be the oracle's record for the caller's own buffer."""
    import threading

    from ctstraffic_amd import Engine

    monkeypatch.setenv("CTS_MAILBOX_GROUPS", "2")
    monkeypatch.setenv("CTS_MAILBOX_SLOTS", "16")
    eng = Engine(0)
    S = oracle.sender_buffer(70000)
    T, ITERS, CAP = 12, 60, 4096 + 32
    arenas = [eng.host_alloc(CAP) for _ in range(T)]
    errors = []

    def worker(t):
        arr, _, dev = arenas[t]
        rng = np.random.default_rng(0x5106 + t)
        try:
            for it in range(ITERS):
                n = int(rng.integers(0, 4097))
                e = int(rng.integers(0, 65536))
                at = int(rng.integers(0, 32))
                arr[at:at + n] = S[e:e + n]
                if n and rng.random() < 0.3:
                    arr[at + int(rng.integers(0, n))] ^= int(rng.integers(1, 256))
                r = eng.verify_mapped(dev + at, n, e)
                o = oracle.verify_buffer(arr[at:at + n].copy(), 0, e, n)
                got = (r["pass"], r["first_mismatch"], r["expected"], r["actual"], r["mismatch_bytes"])
                want = (o["pass"], o["first_mismatch"], o["expected"], o["actual"], o["mismatch_bytes"])
                if got != want:
                    errors.append((t, it, n, e, at, got, want))
        except Exception as ex:  # surfaced below
            errors.append((t, repr(ex)))

    try:
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    finally:
        for _, h, _ in arenas:
            eng.host_free(h)
        eng.close()
    assert not errors, errors[:5]


def test_verify_mapped_mailbox_stop_start_races(monkeypatch):
    """A fresh engine whose watchdog stops the grid after 5 ms without posts (CTS_MAILBOX_IDLE_MS): 6 threads post
    with random pauses of 0-20 ms, so stops race new posts and relaunches all through the run. Every answer must be
    the oracle's, the grid must have been relaunched many times, and the engine must close cleanly."""
    import random
    import threading
    import time

    from ctstraffic_amd import Engine

    monkeypatch.setenv("CTS_MAILBOX_IDLE_MS", "5")
    eng = Engine(0)
    S = oracle.sender_buffer(70000)
    arenas = [eng.host_alloc(65536 + 32) for _ in range(6)]
    errors = []

    def worker(t):
        arr, _, dev = arenas[t]
        rng = np.random.default_rng(0x5A0 + t)
        pause = random.Random(t)
        try:
            for it in range(40):
                n = int(rng.choice([1, 1500, 4096, 65536]))
                e = int(rng.integers(0, 65536))
                arr[:n] = S[e:e + n]
                if rng.random() < 0.3:
                    arr[int(rng.integers(0, n))] ^= 0x11
                r = eng.verify_mapped(dev, n, e)
                o = oracle.verify_buffer(arr[:n].copy(), 0, e, n)
                if (r["pass"], r["first_mismatch"], r["actual"], r["mismatch_bytes"]) != (
                        o["pass"], o["first_mismatch"], o["actual"], o["mismatch_bytes"]):
                    errors.append((t, it, n, e))
                time.sleep(pause.choice([0, 0, 0.002, 0.006, 0.012, 0.02]))
        except Exception as ex:  # surfaced below
            errors.append((t, repr(ex)))

    try:
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        launches = eng.mailbox_launches()
    finally:
        for _, h, _ in arenas:
            eng.host_free(h)
        eng.close()
    assert not errors, errors[:5]
    assert launches >= 3, launches


def test_verify_mapped_mailbox_group_keepalive(monkeypatch):
    """A fresh engine whose grid groups leave after 400 ms without a job (CTS_MAILBOX_EXIT_MS) and whose watchdog
    would wait 5 s (CTS_MAILBOX_IDLE_MS), i.e. a watchdog too slow to stop the grid first. One thread posts for
    1.2 s (least-busy assignment alone would use one group and let the others leave), then 8 threads post at once
    (jobs land on every group), then the process is silent for 0.8 s (the whole grid leaves on its own) and posts
    again (the engine must see the finished grid and relaunch it). Every answer must be the oracle's."""
    import threading
    import time

    from ctstraffic_amd import Engine

    monkeypatch.setenv("CTS_MAILBOX_EXIT_MS", "400")
    monkeypatch.setenv("CTS_MAILBOX_IDLE_MS", "5000")
    eng = Engine(0)
    S = oracle.sender_buffer(70000)
    arenas = [eng.host_alloc(65536 + 32) for _ in range(8)]
    errors = []

    def one(t, rng):
        arr, _, dev = arenas[t]
        n = int(rng.choice([1, 1500, 4096, 65536]))
        e = int(rng.integers(0, 65536))
        arr[:n] = S[e:e + n]
        if rng.random() < 0.3:
            arr[int(rng.integers(0, n))] ^= 0x24
        r = eng.verify_mapped(dev, n, e)
        o = oracle.verify_buffer(arr[:n].copy(), 0, e, n)
        if (r["pass"], r["first_mismatch"], r["actual"], r["mismatch_bytes"]) != (
                o["pass"], o["first_mismatch"], o["actual"], o["mismatch_bytes"]):
            errors.append((t, n, e))

    def burst(t):
        rng = np.random.default_rng(0x4EE + t)
        try:
            for _ in range(200):
                one(t, rng)
        except Exception as ex:  # surfaced below
            errors.append((t, repr(ex)))

    try:
        rng = np.random.default_rng(0x4EE)
        t_end = time.monotonic() + 1.2
        while time.monotonic() < t_end:
            one(0, rng)
        ths = [threading.Thread(target=burst, args=(t,)) for t in range(8)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        first = eng.mailbox_launches()
        time.sleep(0.8)
        for _ in range(50):
            one(0, rng)
        launches = eng.mailbox_launches()
    finally:
        for _, h, _ in arenas:
            eng.host_free(h)
        eng.close()
    assert not errors, errors[:5]
    assert first == 1, first
    assert launches == 2, launches


def test_host_free_after_the_grid_left_on_its_own(monkeypatch):
    """The grid leaves on its own (CTS_MAILBOX_EXIT_MS 40) long before the watchdog would stop it (10 s): a free then
    stops nothing and must not wait CTS_MAILBOX_TIMEOUT_MS for stop jobs no workgroup will answer (round 4 did), and
    the next post relaunches the grid with exact answers."""
    import time

    from ctstraffic_amd import Engine

    monkeypatch.setenv("CTS_MAILBOX_EXIT_MS", "40")
    monkeypatch.setenv("CTS_MAILBOX_IDLE_MS", "10000")
    eng = Engine(0)
    S = oracle.sender_buffer(70000)
    arr, h, dev = eng.host_alloc(65536 + 32)
    try:
        arr[:65536] = S[9:9 + 65536]
        assert eng.verify_mapped(dev, 65536, 9)["pass"]
        time.sleep(0.3)  # every group's idle exit has passed
        _, hh, _ = eng.host_alloc(1 << 20)
        t0 = time.monotonic()
        eng.host_free(hh)
        took = time.monotonic() - t0
        arr[777] ^= 0x08
        r = eng.verify_mapped(dev, 65536, 9)
        assert (r["pass"], r["first_mismatch"], r["mismatch_bytes"]) == (False, 777, 1)
        launches = eng.mailbox_launches()
    finally:
        eng.host_free(h)
        eng.close()
    assert took < 0.5, took
    assert launches == 2, launches


def _mapped_check(eng, arr, dev, S, n, e, flip=None):
    """verify_mapped of arr[:n] (= S[e:e + n], one byte flipped at `flip`) against the oracle's record."""
    arr[:n] = S[e:e + n]
    if flip is not None:
        arr[flip] ^= 0x3C
    r = eng.verify_mapped(dev, n, e)
    o = oracle.verify_buffer(arr[:n].copy(), 0, e, n)
    return (r["pass"], r["first_mismatch"], r["expected"], r["actual"], r["mismatch_bytes"]) == (
        o["pass"], o["first_mismatch"], o["expected"], o["actual"], o["mismatch_bytes"])


def test_verify_mapped_mailbox_late_poller(monkeypatch):
    """a job slot is reused once the workgroups that answer a job have answered, but every workgroup of
    the group reads every job. One group of 16 slots whose last workgroup starts polling 300 ms late
    (CTS_MAILBOX_DELAY_MS): 40 jobs of 1 KiB (one piece: answered by the group's first workgroup alone) wrap the
    ring twice before it polls, then 64 KiB jobs need all four workgroups. The late poller must take the jobs
    whose slots hold later jobs as no-ops and catch up, so the big jobs are answered by the grid (one launch, no
    2 s timeout), exactly."""
    import time

    from ctstraffic_amd import Engine

    monkeypatch.setenv("CTS_MAILBOX_GROUPS", "1")
    monkeypatch.setenv("CTS_MAILBOX_SLOTS", "16")
    monkeypatch.setenv("CTS_MAILBOX_DELAY_MS", "300")
    eng = Engine(0)
    S = oracle.sender_buffer(140000)
    arr, h, dev = eng.host_alloc(65536 + 64)
    try:
        t0 = time.monotonic()
        ok = [_mapped_check(eng, arr, dev, S, 1024, (7 * k) % 65536, flip=(k if k % 5 == 0 else None))
              for k in range(40)]
        ok += [_mapped_check(eng, arr, dev, S, 65536, 999 + k, flip=(4096 * k + 3 if k % 2 else None))
               for k in range(8)]
        took = time.monotonic() - t0
        launches = eng.mailbox_launches()
    finally:
        eng.host_free(h)
        eng.close()
    assert all(ok), ok
    assert launches == 1 and took < 1.5, (launches, took)


def test_verify_mapped_mailbox_timeout_recovers(monkeypatch):
    """one unanswered job used to break the mailbox for the engine's life. Here the first job times out
    (group 0's last workgroup starts 1.5 s late, CTS_MAILBOX_TIMEOUT_MS 200): that verify and the ones after it
    take the launch path and stay exact; once the grid has drained (its groups leave after 300 ms without a job)
    the next post resets the rings and relaunches, and the mailbox answers again."""
    import time

    from ctstraffic_amd import Engine

    monkeypatch.setenv("CTS_MAILBOX_GROUPS", "1")
    monkeypatch.setenv("CTS_MAILBOX_DELAY_MS", "1500")
    monkeypatch.setenv("CTS_MAILBOX_TIMEOUT_MS", "200")
    monkeypatch.setenv("CTS_MAILBOX_EXIT_MS", "300")
    eng = Engine(0)
    S = oracle.sender_buffer(140000)
    arr, h, dev = eng.host_alloc(65536 + 64)
    rng = np.random.default_rng(0x7E0)
    try:
        ok, slow = [], 0
        t_end = time.monotonic() + 2.6
        while time.monotonic() < t_end:
            n = int(rng.choice([100, 5000, 65536]))
            ok.append(_mapped_check(eng, arr, dev, S, n, int(rng.integers(0, 65536)),
                                    flip=int(rng.integers(0, n)) if rng.random() < 0.3 else None))
            time.sleep(0.005)
        launches_before = eng.mailbox_launches()
        for k in range(20):  # through the relaunched grid
            t0 = time.monotonic()
            ok.append(_mapped_check(eng, arr, dev, S, 65536, 17 * k, flip=(k * 1000 if k % 3 == 0 else None)))
            slow += time.monotonic() - t0 > 0.1
        launches = eng.mailbox_launches()
    finally:
        eng.host_free(h)
        eng.close()
    assert all(ok) and len(ok) > 100
    assert launches_before == 2 and launches == 2 and slow == 0, (launches_before, launches, slow)


def test_verify_mapped_mailbox_keepalive_many_groups(monkeypatch):
    """the keepalive refreshed at most one idle group per post. 32 groups whose workgroups leave after
    400 ms without a job, a watchdog that never stops the grid (CTS_MAILBOX_IDLE_MS 5 s) and one caller posting
    every 40 ms for 1.5 s (each post lands on one group): the watchdog's no-op jobs must keep all 32 groups
    resident, so a burst of 32 threads afterwards (jobs on every group) is answered by the same grid."""
    import threading
    import time

    from ctstraffic_amd import Engine

    monkeypatch.setenv("CTS_MAILBOX_GROUPS", "32")
    monkeypatch.setenv("CTS_MAILBOX_EXIT_MS", "400")
    monkeypatch.setenv("CTS_MAILBOX_IDLE_MS", "5000")
    eng = Engine(0)
    S = oracle.sender_buffer(140000)
    arenas = [eng.host_alloc(65536 + 64) for _ in range(32)]
    errors = []
    try:
        arr, _, dev = arenas[0]
        t_end = time.monotonic() + 1.5
        k = 0
        while time.monotonic() < t_end:
            if not _mapped_check(eng, arr, dev, S, 65536, k % 65536, flip=(k if k % 4 == 0 else None)):
                errors.append(("paced", k))
            k += 1
            time.sleep(0.04)

        def burst(t):
            a, _, d = arenas[t]
            for j in range(20):
                t0 = time.monotonic()
                if not _mapped_check(eng, a, d, S, 65536, (t * 977 + j) % 65536, flip=(j if j % 3 == 0 else None)):
                    errors.append((t, j))
                if time.monotonic() - t0 > 0.5:
                    errors.append((t, j, "slow"))

        ths = [threading.Thread(target=burst, args=(t,)) for t in range(32)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        launches = eng.mailbox_launches()
    finally:
        for _, h, _ in arenas:
            eng.host_free(h)
        eng.close()
    assert not errors, errors[:5]
    assert launches == 1, launches


def test_host_free_while_posting(engine):
    """hipHostFree waits for the device's kernels, and the resident mailbox grid never ends while
    other threads post. cts_host_free stops the grid first: frees return quickly while a thread posts 64 KiB
    verifies back to back, and every verify stays exact (those posted during a free take the launch path)."""
    import threading
    import time

    S = oracle.sender_buffer(140000)
    arr, h, dev = engine.host_alloc(65536 + 64)
    stop = threading.Event()
    errors = []

    def poster():
        k = 0
        while not stop.is_set():
            if not _mapped_check(engine, arr, dev, S, 65536, (31 * k) % 65536, flip=(k if k % 4 == 0 else None)):
                errors.append(k)
            k += 1

    th = threading.Thread(target=poster)
    th.start()
    frees = []
    try:
        time.sleep(0.1)
        for _ in range(6):
            _, hh, _ = engine.host_alloc(1 << 20)
            t0 = time.monotonic()
            engine.host_free(hh)
            frees.append(time.monotonic() - t0)
            time.sleep(0.05)
    finally:
        stop.set()
        th.join()
        engine.host_free(h)
    assert not errors, errors[:5]
    assert max(frees) < 0.5, frees


def test_host_free_while_another_engine_posts(engine):
    """hipHostFree is an implicit hipDeviceSynchronize: a second engine's resident grid on the same GPU, kept alive by
    a thread posting to it back to back, would hold a free on the first engine up for as long as the posts go on
    (round 4 paused only the freeing engine's own grid). A free now stops every engine's grid on the device, so each
    returns quickly, and both engines' verifies (the posting one's and a growing staging buffer's) stay exact."""
    import threading
    import time

    from ctstraffic_amd import Engine

    S = oracle.sender_buffer(300000)
    other = Engine(0)
    arr, h, dev = other.host_alloc(65536 + 64)
    stop = threading.Event()
    errors = []

    def poster():
        k = 0
        while not stop.is_set():
            if not _mapped_check(other, arr, dev, S, 65536, (17 * k) % 65536, flip=(k if k % 5 == 0 else None)):
                errors.append(k)
            k += 1

    th = threading.Thread(target=poster)
    th.start()
    frees = []
    try:
        time.sleep(0.1)
        for i in range(6):
            _, hh, _ = engine.host_alloc(1 << 20)
            t0 = time.monotonic()
            engine.host_free(hh)
            frees.append(time.monotonic() - t0)
            # the first engine's own staging buffer grows (its old one is freed the same way)
            n = 70000 + 40000 * i
            buf = S[3:3 + n].copy()
            buf[n // 2] ^= 0x11
            r = engine.verify_host(buf, 3)
            assert (r["pass"], r["first_mismatch"], r["mismatch_bytes"]) == (False, n // 2, 1)
            time.sleep(0.05)
    finally:
        stop.set()
        th.join()
        other.host_free(h)
        other.close()
    assert not errors, errors[:5]
    assert max(frees) < 0.5, frees


def test_verify_mapped_mailbox_restarts_after_idle(engine):
    """The mailbox grid stops after CTS_MAILBOX_IDLE_MS (50 ms) without posts and the next post starts it again;
    answers stay exact across the restart, including an HBM buffer and a buffer larger than the grid's
    64 x 4 KiB of pieces per round (several rounds per workgroup)."""
    import time

    import torch

    S = oracle.sender_buffer(3 << 20)
    arr, h, dev = engine.host_alloc(1 << 20)
    try:
        before = engine.mailbox_launches()
        for rnd in range(3):
            n = [65536, 1 << 20, 12345][rnd]
            e = [7, 65535, 0][rnd]
            arr[:n] = S[e:e + n]
            arr[n // 3] ^= 0x5A
            r = engine.verify_mapped(dev, n, e)
            o = oracle.verify_buffer(arr[:n].copy(), 0, e, n)
            assert (r["pass"], r["first_mismatch"], r["expected"], r["actual"], r["mismatch_bytes"]) == (
                o["pass"], o["first_mismatch"], o["expected"], o["actual"], o["mismatch_bytes"])
            time.sleep(0.3)
        assert engine.mailbox_launches() - before == 3
        # an HBM buffer (the ABI takes any GPU-addressable pointer)
        d = torch.from_numpy(S[100:100 + 300001].copy()).cuda()
        r = engine.verify_mapped(d.data_ptr(), 300001, 100)
        assert r["pass"] and r["first_mismatch"] == 300001 and r["mismatch_bytes"] == 0
        d[299999] ^= 1
        torch.cuda.synchronize()
        r = engine.verify_mapped(d.data_ptr(), 300001, 100)
        assert (r["pass"], r["first_mismatch"], r["mismatch_bytes"]) == (False, 299999, 1)
    finally:
        engine.host_free(h)


def test_verify_host_batch(engine):
    """Repeated calls reuse (and grow) the engine's pinned staging: small, larger, small again."""
    for seed, n, max_len in ((5, 100, 3000), (6, 3000, 70000), (7, 17, 200)):
        rng = np.random.default_rng(seed)
        arena, descs = _random_case(rng, n, max_len, skip=True)
        bufs = [arena[int(d["byte_offset"]): int(d["byte_offset"]) + int(d["length"])] for d in descs]
        r, c = engine.verify_host_batch(bufs, descs["expected_pattern_offset"], descs["skip_head"])
        er, ec, _ = oracle.verify_batch(arena, descs)
        assert_results_equal(r, er, "seed %d" % seed)
        assert c == ec


# ---- every launch geometry and load policy is bit-identical ----------------------------------------
@pytest.mark.parametrize("nt", [1, 0])
def test_launch_geometry_parity(engine, nt):
    """The workgroup-per-buffer kernel and the small-buffer kernel under nontemporal and plain loads, 1 and 16
    workgroups per CU: random lengths, alignments, phases and skips, spans longer than the small-path hint, whole-line
    arenas, fewer buffers than workgroups, more than 1024 buffers per workgroup, vs the oracle."""
    from ctstraffic_amd import _lib

    default_bpc = engine.get_attr(_lib.ATTR_BLOCKS_PER_CU)
    default_small_bpc = engine.get_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU)
    try:
        engine.set_attr(_lib.ATTR_NT_LOADS, nt)
        for seed, n, max_len, hint, skip, whole in [
                (21, 200, 3000, 1472, True, False), (22, 64, 140000, 0, False, False),
                (23, 300, 1472, 1472, True, False), (24, 100, 70000, 0, True, False),
                (25, 6000, 9000, 0, False, False),
                (26, 400, 140000, 0, False, True), (27, 300, 2000, 1472, False, True),
                (28, 3, 70000, 0, False, False)]:
            for bpc in (1, 16):
                engine.set_attr(_lib.ATTR_BLOCKS_PER_CU, bpc)
                engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, bpc)
                rng = np.random.default_rng(seed)
                arena, descs = _random_case(rng, n, max_len, skip=skip, whole=whole)
                r, ctr, cff = run_verify(engine, arena, descs, hint, n_conns=7)
                er, ectr, ecff = oracle.verify_batch(arena, descs, n_conns=7)
                assert_results_equal(r, er, "nt %d seed %d bpc %d" % (nt, seed, bpc))
                assert ctr == ectr
                assert np.array_equal(cff, ecff)
        w = W.udp_datagrams(n_datagrams=4099, corrupt_rate=7)
        _check_workload(engine, w, with_oracle=True)
        w = W.tcp_resident(n_buffers=300, corrupt_rate=5)
        _check_workload(engine, w, with_oracle=True)
    finally:
        engine.set_attr(_lib.ATTR_NT_LOADS, 1)
        engine.set_attr(_lib.ATTR_BLOCKS_PER_CU, default_bpc)
        engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, default_small_bpc)


# ---- the small-buffer (datagram) kernel under every walk ------------------------------------------------
def test_small_path_parity(engine):
    """Small-buffer path (max_length_hint <= 8192, four buffers per wave in 16-lane teams) under block-contiguous and
    chunked walks and 1 / 2 / 64 workgroups per CU, vs the oracle. Includes spans longer than the hint (multi-round
    teams), empty spans, all start alignments, bad descriptors, a batch whose size is not a multiple of the team count,
    and config-3 datagrams."""
    from ctstraffic_amd import _lib

    default_sbpc = engine.get_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU)
    default_chunk = engine.get_attr(_lib.ATTR_SMALL_CHUNK)
    try:
        for seed, n, max_len, hint, skip in [(31, 301, 1500, 1472, True), (32, 257, 200, 64, False),
                                             (33, 120, 20000, 1472, True), (34, 1000, 3000, 8192, False),
                                             (35, 7, 40, 40, True)]:
            for sbpc, chunk in ((1, 0), (64, 0), (1, 16), (2, 48)):
                engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, sbpc)
                engine.set_attr(_lib.ATTR_SMALL_CHUNK, chunk)
                rng = np.random.default_rng(seed)
                arena, descs = _random_case(rng, n, max_len, skip=skip)
                r, ctr, cff = run_verify(engine, arena, descs, hint, n_conns=7)
                er, ectr, ecff = oracle.verify_batch(arena, descs, n_conns=7)
                assert_results_equal(r, er, "seed %d sbpc %d chunk %d" % (seed, sbpc, chunk))
                assert ctr == ectr
                assert np.array_equal(cff, ecff)
        arena = np.zeros(256, np.uint8)
        oracle.fill(arena, np.array([(0, 256, 0, 0, 0)], dtype=oracle.DESC_DTYPE))
        d = np.zeros(5, dtype=DESC_DTYPE)
        d[0] = (0, 10, 65536, 0, 0)
        d[1] = (0, 10, 0, 0, 11)
        d[2] = (250, 10, 0, 0, 0)
        d[3] = (2**40, 1, 0, 0, 0)
        d[4] = (16, 32, 16, 0, 0)
        r, ctr, _ = run_verify(engine, arena, d, 1472)
        er, ectr, _ = oracle.verify_batch(arena, d)
        assert_results_equal(r, er)
        assert ctr == ectr and ctr["buffers_checked"] == 1
        w = W.udp_datagrams(n_datagrams=4099, corrupt_rate=7)
        _check_workload(engine, w, with_oracle=True)
    finally:
        engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, default_sbpc)
        engine.set_attr(_lib.ATTR_SMALL_CHUNK, default_chunk)


def test_kernel_ids_are_fixed(engine):
    """One kernel per path: the variant attributes report its id (verify 25, small 15, MediaStream 3) and refuse any
    other value."""
    from ctstraffic_amd import _lib
    from ctstraffic_amd._lib import CtsError

    for attr, dflt, others in ((_lib.ATTR_VERIFY_VARIANT, 25, (0, 4, 12, 13, 17)), (_lib.ATTR_SMALL_VARIANT, 15, (0, 5, 9)),
                               (_lib.ATTR_MS_VARIANT, 3, (0, 2))):
        assert engine.get_attr(attr) == dflt
        engine.set_attr(attr, dflt)
        for v in others:
            with pytest.raises(CtsError):
                engine.set_attr(attr, v)
        assert engine.get_attr(attr) == dflt


# ---- maximum sizes: one buffer of 2^32 - 1 bytes, buffers past the 4 GiB arena offset -----------------------
def test_max_length_buffers(engine):
    """ctsTask::m_bufferLength is a u32: a single 2^32 - 1-byte buffer (last byte corrupted) and a 2^31 + 77-byte
    buffer starting past 2^32 in the arena at an odd address with the MediaStream skip. Both kernel paths (workgroup
    per buffer, four buffers per wave); the fill writes them first (its 64-bit offsets are checked at sampled positions
    against the oracle's pattern)."""
    L0, L1 = 2**32 - 1, 2**31 + 77
    off1 = 2**32 + 3
    total = off1 + L1 + 64
    try:
        arena = torch.zeros(total, dtype=torch.uint8, device=DEV)
    except RuntimeError:  # pragma: no cover
        pytest.skip("not enough device memory")
    descs = np.zeros(2, dtype=DESC_DTYPE)
    descs[0] = (0, L0, 12345, 0, 0)
    descs[1] = (off1, L1, 65535, 1, 26)
    d = to_dev(descs)
    engine.fill(arena, d, max_length_hint=0)
    torch.cuda.synchronize()
    pat = oracle.sender_buffer(65536)  # P(j) for j < 65536 + 65536
    for b, (off, ln, exp, skip) in enumerate([(0, L0, 12345, 0), (off1, L1, 65535, 26)]):
        for rel in (0, 1, 2**31 - 5, 2**32 - 2 - 2 * skip if b == 0 else ln - skip - 1, ln - skip - 1):
            got = int(arena[off + skip + rel].item())
            assert got == int(pat[(exp + rel) % 65536]), (b, rel)
        assert int(arena[off + ln].item()) == 0 if b == 1 else True  # the byte after the buffer is untouched
    # the piece-order fill (a length hint above the datagram threshold) writes the same bytes: with a hint far
    # below the lengths (the last piece of each buffer takes the rest) and with the exact one
    ref = arena.clone()
    for hint in (65536, L0):
        arena.fill_(0x33)
        engine.fill(arena, d, max_length_hint=hint)
        torch.cuda.synchronize()
        for off, ln, skip in ((0, L0, 0), (off1, L1, 26)):
            assert torch.equal(arena[off + skip:off + ln], ref[off + skip:off + ln]), hint
        assert int(arena[off1 + L1].item()) == 0x33 and int(arena[off1 + 25].item()) == 0x33  # neighbours, header
    del ref
    # corrupt: buffer 0 at its last byte, buffer 1 at span byte 2^31 + 9 (past 2^31)
    c0, c1 = L0 - 1, 2**31 + 9
    arena[c0] ^= 0x5A
    arena[off1 + 26 + c1] ^= 0xFF
    exp_first = [c0, c1]
    exp_bytes = [int(pat[(12345 + c0) % 65536]), int(pat[(65535 + c1) % 65536])]
    act_bytes = [exp_bytes[0] ^ 0x5A, exp_bytes[1] ^ 0xFF]
    for hint in (0, 1472):  # workgroup per buffer, four buffers per wave
        res = engine.new_results(2)
        ctr = engine.new_counters()
        engine.verify(arena, d, max_length_hint=hint, results=res, counters=ctr)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(RESULT_DTYPE)
        for b in range(2):
            assert (int(r[b]["first_mismatch"]), int(r[b]["mismatch_bytes"]), int(r[b]["expected"]),
                    int(r[b]["actual"]), int(r[b]["pass"])) == (exp_first[b], 1, exp_bytes[b], act_bytes[b], 0), (
                        hint, b)
        c = engine.read_counters(ctr)
        assert c == {"bytes_checked": L0 + L1 - 26, "bytes_ok": 0, "buffers_checked": 2, "buffers_failed": 2,
                     "mismatched_bytes": 2}
    del arena
    torch.cuda.empty_cache()


def test_engine_stream(engine):
    """cts_engine_stream_create: a stream on the engine's device that cts_verify runs on."""
    import ctypes

    from ctstraffic_amd import _lib

    s = ctypes.c_void_p()
    assert _lib.lib().cts_engine_stream_create(engine._h, ctypes.byref(s)) == 0 and s.value
    w = W.tcp_resident(n_buffers=32, corrupt_rate=8)
    arena, descs = W.materialize(engine, w, device=DEV)
    ctr = engine.new_counters()
    torch.cuda.synchronize()
    engine.verify(arena, descs, max_length_hint=w.max_length, counters=ctr, stream=s.value)
    exp = W.expected_results(w)[2]
    assert engine.read_counters(ctr, stream=s.value) == exp
    assert _lib.lib().cts_engine_stream_destroy(engine._h, s) == 0


# ---- strided receive rings (cts_verify_strided) -----------------------------------------------------------------
@pytest.mark.parametrize("stride,skip,expected", [(1472, 26, 0), (1536, 26, 0), (9017, 0, 777), (64, 3, 65535)])
def test_verify_strided_matches_oracle(engine, stride, skip, expected):
    """cts_verify_strided: buffer i of a ring at i * stride (16-byte-aligned slots and odd strides) with only its
    completed length, one skip / expected offset / connection for the ring (MediaStream payloads: skip 26,
    expected 0). Results, counters and the connection's first failure equal the oracle's over the same buffers
    described by descriptors; a length above the stride is BAD_DESC and counts nowhere."""
    rng = np.random.default_rng(stride)
    n = 6000
    S = oracle.sender_buffer(stride + 65536)
    ring = np.full(n * stride + 64, 0xEE, dtype=np.uint8)
    lens = rng.integers(0, stride + 1, size=n).astype(np.uint32)
    lens[:6] = [0, max(0, skip - 1), skip, min(stride, skip + 1), stride, stride]
    for i in range(n):
        ln = int(lens[i])
        if ln > skip:
            body = S[expected:expected + ln - skip].copy()
            if rng.random() < 0.05:
                body[int(rng.integers(0, ln - skip))] ^= int(rng.integers(1, 256))
            ring[i * stride + skip:i * stride + ln] = body
    descs = np.zeros(n, dtype=DESC_DTYPE)
    descs["byte_offset"] = np.arange(n, dtype=np.uint64) * stride
    descs["length"] = lens
    descs["expected_pattern_offset"] = expected
    descs["conn_index"] = 3
    descs["skip_head"] = skip
    er, ectr, ecff = oracle.verify_batch(ring, descs, n_conns=5)
    a = to_dev(ring)
    res = engine.new_results(n)
    ctr = engine.new_counters()
    cff = torch.full((5,), -1, dtype=torch.int32, device=DEV)
    engine.verify_strided(a, stride, to_dev(lens), skip_head=skip, expected_offset=expected, conn_index=3, results=res,
                          counters=ctr, conn_first_fail=cff)
    torch.cuda.synchronize()
    assert_results_equal(res.cpu().numpy().view(RESULT_DTYPE), er, "stride %d" % stride)
    assert engine.read_counters(ctr) == ectr
    assert np.array_equal(cff.cpu().numpy().view(np.uint32), ecff)
    # a completion longer than its slot is flagged, not read
    lens2 = lens.copy()
    lens2[7] = stride + 1
    res2 = engine.new_results(n)
    ctr2 = engine.new_counters()
    engine.verify_strided(a, stride, to_dev(lens2), skip_head=skip, expected_offset=expected, results=res2, counters=ctr2)
    torch.cuda.synchronize()
    r2 = res2.cpu().numpy().view(RESULT_DTYPE)
    assert r2["flags"][7] == 1 and r2["pass"][7] == 0
    keep = np.arange(n) != 7
    assert_results_equal(r2[keep], er[keep], "stride %d, one long" % stride)
    c2 = engine.read_counters(ctr2)
    assert c2["buffers_checked"] == ectr["buffers_checked"] - 1


def test_verify_strided_rejects_bad_arguments(engine):
    from ctstraffic_amd import CtsError

    a = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    lens = torch.zeros(4, dtype=torch.int32, device=DEV)
    for kw in [dict(stride=0), dict(expected_offset=65536)]:
        args = dict(stride=1024, expected_offset=0)
        args.update(kw)
        with pytest.raises(CtsError):
            engine.verify_strided(a, args["stride"], lens, expected_offset=args["expected_offset"])
    with pytest.raises(CtsError):
        engine.verify_strided(a[1:], 1024, lens)  # arena not 16-byte aligned
