"""GPU: the node's DataError count on the device (cts_counters_ex.connections_failed) vs the oracle.

The reference counts a DataError once per connection whose verify failed, at the connection's close
(ctsSocketState.cpp:221-228: ConnectionStatusDetails.m_protocolErrorCount), however many of its buffers failed. The
kernels count it where the per-connection first-failure slot is claimed: the atomicMin on dev_conn_first_fail[c]
that finds the slot still 0xFFFFFFFF. The oracle's count is the number of slots its own verify left set
(oracle.verify_batch's conn_first_fail), and the analytic one the same from the corruption plan. Integer work:
bit-exact.
"""
import numpy as np
import pytest

import oracle
from ctstraffic_amd import workload as W

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda"
EMPTY = 0xFFFFFFFF


def _slots(n):
    return torch.full((n,), -1, dtype=torch.int32, device=DEV)


def _failed_conns(cff_u32) -> int:
    return int((np.asarray(cff_u32, dtype=np.uint32) != EMPTY).sum())


def _verify_ex(engine, w, arena, descs, cff, ctr, stream=None):
    engine.verify(arena, descs, max_length_hint=w.max_length, counters=ctr, conn_first_fail=cff, stream=stream)


def _check(engine, w, oracle_bytes=True):
    arena, descs = W.materialize(engine, w)
    ctr, cff = engine.new_counters(), _slots(w.n_conns)
    _verify_ex(engine, w, arena, descs, cff, ctr)
    torch.cuda.synchronize()
    got = engine.read_counters_ex(ctr)
    _, _, ec, ecff = W.expected_results(w)
    want = _failed_conns(ecff)
    assert got["connections_failed"] == want > 0, (got, want)
    assert {k: got[k] for k in ec} == ec  # the five counters read alongside are unchanged
    assert engine.read_counters(ctr) == ec
    assert np.array_equal(cff.cpu().numpy().view(np.uint32), ecff)
    if oracle_bytes:
        _, octr, ocff = oracle.verify_batch(arena.cpu().numpy(), w.descs, n_conns=w.n_conns, nthreads=8)
        assert got["connections_failed"] == _failed_conns(ocff)
        assert {k: got[k] for k in octr} == octr
    return arena, descs, got


def test_config2_connections_failed_vs_oracle(engine):
    """Config 2 (4096 x 64 KiB, one buffer per connection, 1/1024 corrupted): the workgroup-per-buffer kernel."""
    _check(engine, W.tcp_resident())


def test_dense_corruption_many_failures_per_connection(engine):
    """Configs 4/5 shaped streams with a third of the buffers corrupt: most connections fail many times and must
    count once each (64 KiB buffers: the workgroup kernel)."""
    w = W.connection_streams(n_conns=96, buffers_per_conn=48, length=65536, corrupt_rate=3)
    _, _, got = _check(engine, w)
    per_conn = np.bincount(w.descs["conn_index"][np.unique(w.corrupt_buf)].astype(np.int64), minlength=w.n_conns)
    assert per_conn.max() >= 8 and got["buffers_failed"] > 4 * got["connections_failed"]


def test_dense_corruption_datagram_sized_buffers(engine):
    """The same on ragged completions of at most 1472 bytes, so the four-buffers-per-wave kernel counts."""
    w = W.connection_streams(n_conns=200, buffers_per_conn=64, length=1472, ragged=True, corrupt_rate=5, align=1)
    assert w.max_length <= engine.get_attr(3)  # CTS_ATTR_SMALL_THRESHOLD: the quad path
    _check(engine, w)


def test_strided_ring_counts_its_one_connection_once(engine):
    """cts_verify_strided (one connection for the whole ring, MediaStream payloads): one DataError however many
    datagrams fail, and none when every datagram is clean."""
    n, stride, skip = 4096, 1536, 26
    rng = np.random.default_rng(0x5EED)
    lens = rng.integers(skip + 1, stride + 1, size=n).astype(np.uint32)
    ring = np.zeros(n * stride, dtype=np.uint8)
    pat = oracle.sender_buffer(stride)
    for i in range(n):
        ring[i * stride + skip:i * stride + lens[i]] = pat[:lens[i] - skip]
    bad = rng.choice(n, size=40, replace=False)
    for i in bad:
        ring[i * stride + skip + rng.integers(0, lens[i] - skip)] ^= 0x5A
    lens_d = torch.from_numpy(lens.copy()).to(DEV)
    for arena_np, want in ((ring, 1), (np.zeros_like(ring), 1)):
        ctr, cff = engine.new_counters(), _slots(3)
        engine.verify_strided(torch.from_numpy(arena_np).to(DEV), stride, lens_d, skip_head=skip, conn_index=2,
                              counters=ctr, conn_first_fail=cff)
        torch.cuda.synchronize()
        assert engine.read_counters_ex(ctr)["connections_failed"] == want
    clean = ring.copy()
    for i in bad:
        clean[i * stride + skip:i * stride + lens[i]] = pat[:lens[i] - skip]
    ctr, cff = engine.new_counters(), _slots(3)
    engine.verify_strided(torch.from_numpy(clean).to(DEV), stride, lens_d, skip_head=skip, conn_index=2,
                          counters=ctr, conn_first_fail=cff)
    torch.cuda.synchronize()
    c = engine.read_counters_ex(ctr)
    assert c["connections_failed"] == 0 and c["buffers_failed"] == 0


def test_two_launches_share_one_slot_array(engine):
    """A connection's buffers verified by two launches (interleaved halves of its stream) that share the slot
    array and the counter block, in series and at once on two streams: each failed connection counts once, and
    a connection that fails in both launches is claimed by exactly one of them."""
    w = W.connection_streams(n_conns=128, buffers_per_conn=32, length=65536, corrupt_rate=6)
    arena, _ = W.materialize(engine, w)
    _, _, ocff = oracle.verify_batch(arena.cpu().numpy(), w.descs, n_conns=w.n_conns, nthreads=8)
    want = _failed_conns(ocff)
    halves = [w.descs[0::2], w.descs[1::2]]
    host = arena.cpu().numpy()
    claimed = [oracle.verify_batch(host, h, n_conns=w.n_conns, nthreads=8)[2] != EMPTY for h in halves]
    assert (claimed[0] & claimed[1]).sum() > 8  # connections failing in both halves: the race this test is about
    assert (claimed[0] | claimed[1]).sum() == want
    dd = [torch.from_numpy(np.ascontiguousarray(h).view(np.uint8).copy()).to(DEV) for h in halves]
    s1, s2 = engine.stream_create(), engine.stream_create()
    try:
        for mode in ("series", "concurrent", "concurrent"):
            ctr, cff = engine.new_counters(), _slots(w.n_conns)
            torch.cuda.synchronize()
            if mode == "series":
                for d in dd:
                    engine.verify(arena, d, max_length_hint=65536, counters=ctr, conn_first_fail=cff)
            else:
                engine.verify(arena, dd[0], max_length_hint=65536, counters=ctr, conn_first_fail=cff, stream=s1)
                engine.verify(arena, dd[1], max_length_hint=65536, counters=ctr, conn_first_fail=cff, stream=s2)
            torch.cuda.synchronize()
            got = engine.read_counters_ex(ctr)
            assert got["connections_failed"] == want, (mode, got, want)
            assert _failed_conns(cff.cpu().numpy().view(np.uint32)) == want
            # the same slots again, not re-initialised: every connection was already claimed
            engine.reset_counters(ctr)
            for d in dd:
                engine.verify(arena, d, max_length_hint=65536, counters=ctr, conn_first_fail=cff)
            torch.cuda.synchronize()
            again = engine.read_counters_ex(ctr)
            assert again["connections_failed"] == 0 and again["buffers_failed"] == got["buffers_failed"]
    finally:
        engine.stream_destroy(s1)
        engine.stream_destroy(s2)


def test_no_slot_array_no_count(engine):
    """Without dev_conn_first_fail there is no per-connection claim, so the count stays 0 (documented in
    include/cts_engine.h); slots past n_conns are not claimed either."""
    w = W.tcp_resident(n_buffers=512, corrupt_rate=16)
    arena, descs = W.materialize(engine, w)
    ctr = engine.new_counters()
    engine.verify(arena, descs, max_length_hint=65536, counters=ctr)
    torch.cuda.synchronize()
    c = engine.read_counters_ex(ctr)
    assert c["buffers_failed"] > 0 and c["connections_failed"] == 0
    engine.reset_counters(ctr)
    cff = _slots(100)  # connections 100.. of the batch have no slot
    engine.verify(arena, descs, max_length_hint=65536, counters=ctr, conn_first_fail=cff)
    torch.cuda.synchronize()
    _, _, _, ecff = W.expected_results(w)
    assert engine.read_counters_ex(ctr)["connections_failed"] == _failed_conns(ecff[:100])


def test_status_line_from_the_device_counters(engine):
    """§8f-4 on the device-resident path ("device-resident receive"): two status ticks, each adding
    what the GPU verified since the previous tick into the status counters (never SetValue), give the TCP status
    line's RecvBps and DataError columns and the exit summary the oracle's totals: DataError = the failed connections
    (ctsSocketState.cpp:221-228), counted once each although both ticks' batches carry failing buffers of the same
    connections."""
    from ctstraffic_amd import status as S

    w = W.connection_streams(n_conns=64, buffers_per_conn=16, length=65536, corrupt_rate=5)
    arena, _ = W.materialize(engine, w)
    host = arena.cpu().numpy()
    halves = [w.descs[0::2], w.descs[1::2]]  # every connection's stream, split over two batches
    ctr, cff = engine.new_counters(), _slots(w.n_conns)
    last = dict.fromkeys(("bytes_checked", "connections_failed"), 0)
    recv, data_errors, lines = 0, 0, []
    for tick, h in enumerate(halves):
        engine.verify(arena, torch.from_numpy(np.ascontiguousarray(h).view(np.uint8).copy()).to(DEV),
                      max_length_hint=65536, counters=ctr, conn_first_fail=cff)
        torch.cuda.synchronize()
        node = engine.read_counters_ex(ctr)
        d_bytes = node["bytes_checked"] - last["bytes_checked"]
        d_conns = node["connections_failed"] - last["connections_failed"]
        last = node
        recv += d_bytes
        data_errors += d_conns
        lines.append(S.line(S.CSV, current_time_ms=1000 * (tick + 1), start_time_ms=1000 * tick,
                            end_time_ms=1000 * (tick + 1), bytes_sent=0, bytes_recv=d_bytes, active_connections=64,
                            successful=0, connection_errors=0, protocol_errors=data_errors))
    _, octr, ocff = oracle.verify_batch(host, w.descs, n_conns=w.n_conns, nthreads=8)
    assert recv == octr["bytes_checked"]
    assert data_errors == _failed_conns(ocff) > 0
    for tick, (ln, h) in enumerate(zip(lines, halves)):
        fields = ln.strip().split(",")
        assert int(fields[2]) == int(h["length"].astype(np.int64).sum())  # RecvBps over a 1 s slice
        assert int(fields[6]) <= data_errors
    assert int(lines[-1].strip().split(",")[6]) == data_errors  # DataError is cumulative
    s = S.summary(64 - data_errors, 0, data_errors, recv, 0)
    assert "ProtocolErrors [%d]" % data_errors in s and "Total Bytes Recv : %d" % recv in s
