"""CPU: the oracle (oracle/cts_oracle.c) against the committed golden fixtures.

The fixtures are produced by tests/golden/make_golden.py, an independent
pure-Python transcription of ctsTraffic/ctsIOPattern.cpp:52-90 and :745-775
(the reference itself is Windows-only and cannot be built here).
"""
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def closed_form(j):
    j = np.asarray(j, dtype=np.int64) % 65536
    return np.where(j & 1, j >> 9, (j >> 1) & 0xFF).astype(np.uint8)


def test_pattern_table_is_u16_le_ramp():
    t = oracle.pattern_table()
    assert t.size == 131072
    assert np.array_equal(t.view("<u2"), np.arange(65536, dtype=np.uint16))


def test_sender_buffer_kat():
    kat = _load("pattern_kat.json")
    S = oracle.sender_buffer(4096)
    assert S.size == kat["sender_size_for_max_4096"] == 65536 + 4096
    assert S[:16].tobytes().hex() == kat["first_16"]
    assert S[65530:65542].tobytes().hex() == kat["bytes_65530_65541"]
    assert "%016x" % oracle.fnv1a64(S[:65536]) == kat["fnv1a64_one_period"]
    assert "%016x" % oracle.fnv1a64(oracle.pattern_table()) == kat["fnv1a64_table_131072"]
    assert "%016x" % oracle.fnv1a64(S) == kat["sender_fnv1a64_max_4096"]
    for p, v in kat["probe_bytes"].items():
        assert S[int(p)] == v


@pytest.mark.parametrize("max_buf", [0, 1, 1446, 1472, 65535, 65536, 65537, 200000])
def test_sender_buffer_periodic_and_closed_form(max_buf):
    S = oracle.sender_buffer(max_buf)
    assert S.size == 65536 + max_buf
    assert np.array_equal(S, closed_form(np.arange(S.size)))


def test_pattern_byte_closed_form_all_positions():
    pos = np.arange(0, 65536 * 2 + 7, 1)
    got = np.array([oracle.pattern_byte(int(p)) for p in pos[::97]], dtype=np.uint8)
    assert np.array_equal(got, closed_form(pos[::97]))
    assert oracle.pattern_byte(2**40 + 3) == closed_form(3)


def test_compare_memory_semantics():
    a = np.arange(10000, dtype=np.uint8)
    b = a.copy()
    assert oracle.compare_memory(a, b, 10000) == 10000
    assert oracle.compare_memory(a, b, 0) == 0
    for k in (0, 1, 4095, 4096, 4097, 9999):
        c = b.copy()
        c[k] ^= 1
        assert oracle.compare_memory(a, c, 10000) == k
        assert oracle.compare_memory(a, c, k) == k


VEC = _load("verify_vectors.json")


@pytest.mark.parametrize("case", VEC["cases"], ids=[c["name"] for c in VEC["cases"]])
def test_verify_buffer_vectors(case):
    buf = np.frombuffer(bytes.fromhex(case["buffer_hex"]), dtype=np.uint8)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    r = oracle.verify_buffer(buf, case["buffer_offset"], case["expected_offset"], case["transferred"])
    exp = case["result"]
    assert r["pass"] == exp["pass"]
    assert r["first_mismatch"] == exp["first_mismatch"]
    assert r["mismatch_bytes"] == exp["mismatch_bytes"]
    if not exp["pass"]:
        assert (r["expected"], r["actual"]) == (exp["expected"], exp["actual"])


def test_verify_batch_matches_vectors():
    """All vectors packed into one arena at ragged offsets, verified in one batch (1 and 4 threads)."""
    cases = VEC["cases"]
    arena = bytearray()
    descs = np.zeros(len(cases), dtype=oracle.DESC_DTYPE)
    for i, c in enumerate(cases):
        arena += bytes(i % 7)  # ragged alignment
        b = bytes.fromhex(c["buffer_hex"])
        descs[i] = (len(arena), c["buffer_offset"] + c["transferred"], c["expected_offset"], i % 5, c["buffer_offset"])
        arena += b
    a = np.frombuffer(bytes(arena), dtype=np.uint8).copy()
    for nt in (1, 4):
        res, ctr, cff = oracle.verify_batch(a, descs, n_conns=5, nthreads=nt)
        for i, c in enumerate(cases):
            e = c["result"]
            assert res[i]["first_mismatch"] == e["first_mismatch"], c["name"]
            assert bool(res[i]["pass"]) == e["pass"], c["name"]
            assert res[i]["mismatch_bytes"] == e["mismatch_bytes"], c["name"]
        fails = [i for i, c in enumerate(cases) if not c["result"]["pass"]]
        assert ctr["buffers_checked"] == len(cases)
        assert ctr["buffers_failed"] == len(fails)
        assert ctr["bytes_checked"] == sum(c["transferred"] for c in cases)
        assert ctr["bytes_ok"] == sum(c["transferred"] for c in cases if c["result"]["pass"])
        assert ctr["mismatched_bytes"] == sum(c["result"]["mismatch_bytes"] for c in cases)
        for conn in range(5):
            fc = [i for i in fails if i % 5 == conn]
            assert cff[conn] == (min(fc) if fc else 0xFFFFFFFF)


@pytest.mark.parametrize("name", sorted(VEC["streams"]))
def test_offset_advance_streams(name):
    s = VEC["streams"][name]
    o = 0
    for c, e in zip(s["completions"], s["expected_offsets"]):
        assert o == e
        o = oracle.advance_offset(o, c)
    assert o == s["final_offset"]


def test_bad_descriptors_flagged_not_counted():
    a = np.zeros(64, np.uint8)
    d = np.zeros(3, dtype=oracle.DESC_DTYPE)
    d[0] = (0, 10, 65536, 0, 0)   # offset out of period
    d[1] = (0, 10, 0, 0, 11)      # length < skip_head
    d[2] = (60, 10, 0, 0, 0)      # beyond the arena
    res, ctr, _ = oracle.verify_batch(a, d)
    assert list(res["flags"]) == [1, 1, 1]
    assert ctr["buffers_checked"] == 0 and ctr["bytes_checked"] == 0
