"""Loopback-TCP feeder: whole connections over 127.0.0.1
through the ctsIoPattern mirror, the reference's config 1 in miniature.

CPU: the oracle answers VerifyBuffer through the pattern's batch-verifier hook
(the reference's tests replace ctsConfig with fakes the same way); GPU: the
fill kernel writes the sender buffer and the verify kernel checks every
received buffer. A fault-injection knob flips one byte on the wire.
"""
import pytest

import oracle
from ctstraffic_amd import _pattern_abi as A
from ctstraffic_amd import loopback
from ctstraffic_amd.pattern import shared_buffer_attach

_SENDER = oracle.sender_buffer(2 * 65536)
_SENDER_WIDE = oracle.sender_buffer(98304)  # g_senderSharedBuffer for -Buffer:[32768,98304] (the pattern keeps a pointer)


def _oracle_verifier(arena, descs):
    return oracle.verify_batch(arena, descs)[0]


@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
@pytest.mark.parametrize("pattern", [A.PATTERN_PUSH, A.PATTERN_PULL], ids=["push", "pull"])
def test_loopback_clean_cpu(mode, pattern):
    shared_buffer_attach(_SENDER)
    r = loopback.run(connections=4, buffer_size=65536, transfer_size=3 * 1024 * 1024 + 12345, verifier=_oracle_verifier,
                     io_pattern=pattern, verify_mode=mode, batch_buffers=16, sides=True)
    assert r["connections_ok"] == 4 and r["connections_failed"] == 0 and r["data_errors"] == 0
    # a CPU hook answers synchronously: no device verdict is ever waited for, nothing stays held after the run
    assert all(sd["verify_wait_ns"] == 0 and sd["bytes_recv_held"] == 0 for sd in r["sides"])
    # every data byte crosses once; connection ids (37 B) and DONE (4 B) are counted too (ctsIOPattern.cpp:505-516)
    data = 4 * (3 * 1024 * 1024 + 12345)
    assert r["bytes_recv"] == data + 4 * (37 + 4)
    assert r["buffers_verified"] >= data // 65536


@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
def test_loopback_detects_wire_corruption_cpu(mode):
    shared_buffer_attach(_SENDER)
    r = loopback.run(connections=3, buffer_size=16384, transfer_size=2 * 1024 * 1024, verifier=_oracle_verifier,
                     verify_mode=mode, batch_buffers=8, corrupt_connection=1, corrupt_send_index=17)
    assert r["data_errors"] == 1 and r["connections_failed"] == 1 and r["connections_ok"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
def test_loopback_gpu(engine, mode):
    r = loopback.run(connections=4, buffer_size=65536, transfer_size=16 * 1024 * 1024 + 7, engine=engine,
                     verify_mode=mode, sides=True)
    assert r["connections_ok"] == 4 and r["data_errors"] == 0
    # cts_pattern_stats.verify_wait_ns: the receiving sides of a DEFERRED run waited for device verdicts (at least the
    # final flush's synchronize); SYNC has no batch to wait for
    waits = [sd["verify_wait_ns"] for sd in r["sides"][4:]]
    assert all(w > 0 for w in waits) if mode == A.VERIFY_DEFERRED else all(w == 0 for w in waits), waits
    assert all(sd["bytes_recv_held"] == 0 and sd["bytes_sent_held"] == 0 for sd in r["sides"])
    r = loopback.run(connections=4, buffer_size=65536, transfer_size=8 * 1024 * 1024, engine=engine, verify_mode=mode,
                     corrupt_connection=2, corrupt_send_index=40)
    assert r["data_errors"] == 1 and r["connections_ok"] == 3
    # small batches: DEFERRED's zero-copy recv ring (2 x 8 + 2 slots) has wrapped several times before send 100, so
    # the kernel must see the slot's new bytes, not a line cached from an earlier batch
    r = loopback.run(connections=4, buffer_size=65536, transfer_size=8 * 1024 * 1024, engine=engine, verify_mode=mode,
                     batch_buffers=8, corrupt_connection=1, corrupt_send_index=100)
    assert r["data_errors"] == 1 and r["connections_ok"] == 3


@pytest.mark.gpu
@pytest.mark.parametrize("wait", ["0", "1", "2"], ids=["spin", "event", "sleep_poll"])
def test_loopback_deferred_retire_waits_gpu(engine, wait, monkeypatch):
    """Every way DEFERRED's Retire can wait for the in-flight batch (CTS_DEFERRED_BLOCKING_SYNC, read when a pattern is
    created; 2 = sleep between event queries, the default) gives the same outcome: clean connections complete, the
    corrupt one fails with exactly one DataError, and every buffer of the clean ones was verified."""
    monkeypatch.setenv("CTS_DEFERRED_BLOCKING_SYNC", wait)
    n, total = 4, 8 * 1024 * 1024
    r = loopback.run(connections=n, buffer_size=65536, transfer_size=total, engine=engine,
                     verify_mode=A.VERIFY_DEFERRED, batch_buffers=16, recv_whole=True,
                     corrupt_connection=3, corrupt_send_index=50)
    assert (r["connections_ok"], r["connections_failed"], r["data_errors"]) == (n - 1, 1, 1)
    assert r["buffers_verified"] >= (n - 1) * total // 65536


def test_loopback_with_c_oracle_hook():
    """The CPU baseline's arrangement: the oracle's C entry point as the pattern's verifier."""
    shared_buffer_attach(_SENDER)
    hook = A.BATCH_VERIFIER(oracle.batch_verifier_address())
    r = loopback.run(connections=8, buffer_size=65536, transfer_size=8 * 1024 * 1024, verifier=hook,
                     verify_mode=A.VERIFY_SYNC)
    assert r["connections_ok"] == 8 and r["data_errors"] == 0
    r = loopback.run(connections=2, buffer_size=65536, transfer_size=8 * 1024 * 1024, verifier=hook,
                     verify_mode=A.VERIFY_SYNC, corrupt_connection=0, corrupt_send_index=3)
    assert r["data_errors"] == 1


def test_loopback_thread_cpu_accounting():
    """recv_cpu_seconds / send_cpu_seconds: RUSAGE_THREAD of the threads that ran the data recvs / sends. Verifying
    on the receive thread (the reference's arrangement) costs that thread CPU that verification off does not;
    a verifier that burns 2 ms per batch shows up in the receive side only."""
    import time

    shared_buffer_attach(_SENDER)
    cfg = dict(connections=2, buffer_size=65536, transfer_size=4 * 1024 * 1024)
    off = loopback.run(verify=False, **cfg)
    assert off["connections_ok"] == 2
    assert 0 < off["recv_cpu_seconds"] and 0 < off["send_cpu_seconds"]

    def slow(arena, descs):  # the oracle after 2 ms of spinning on the calling (receive) thread
        t_end = time.thread_time() + 0.002
        while time.thread_time() < t_end:
            pass
        return _oracle_verifier(arena, descs)

    r = loopback.run(verifier=slow, verify_mode=A.VERIFY_SYNC, **cfg)
    assert r["connections_ok"] == 2 and r["data_errors"] == 0
    calls = r["buffers_verified"]
    # every VerifyBuffer ran on a receive thread: at least 2 ms of its CPU each
    assert r["recv_cpu_seconds"] >= 0.002 * calls * 0.9, (r["recv_cpu_seconds"], calls)
    assert r["send_cpu_seconds"] < 0.002 * calls / 2
    assert r["recv_cpu_s_per_GiB"] == pytest.approx(r["recv_cpu_seconds"] / (r["bytes_recv"] / (1 << 30)))
    # the split: the socket calls' share, and the rest (here the spinning verifier) in the pattern's share
    for x in (off, r):
        assert 0 < x["recv_io_cpu_seconds"] <= x["recv_cpu_seconds"] * 1.01
    assert r["recv_pattern_cpu_s_per_GiB"] * r["bytes_recv"] / (1 << 30) >= 0.002 * calls * 0.9
    assert r["recv_io_cpu_seconds"] < r["recv_cpu_seconds"] - 0.002 * calls * 0.9


# ---- PushPull (sync functor) and Duplex (async functor: a send and a recv in flight per side) -----------------
@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
def test_loopback_pushpull_cpu(mode):
    """-Pattern:pushpull: the client pushes PushBytes, then pulls PullBytes, alternating (ctsIOPattern.cpp:888-966);
    both directions are verified, and segment ends shift the receive phase (odd sizes)."""
    shared_buffer_attach(_SENDER)
    total = 5 * 1024 * 1024 + 333
    r = loopback.run(connections=3, buffer_size=65536, transfer_size=total, verifier=_oracle_verifier,
                     io_pattern=A.PATTERN_PUSHPULL, verify_mode=mode, batch_buffers=8, push_bytes=100003,
                     pull_bytes=65537)
    assert r["connections_ok"] == 3 and r["data_errors"] == 0
    assert r["bytes_recv"] == 3 * (total + 37 + 4)
    r = loopback.run(connections=2, buffer_size=65536, transfer_size=total, verifier=_oracle_verifier,
                     io_pattern=A.PATTERN_PUSHPULL, verify_mode=mode, batch_buffers=8, push_bytes=100003,
                     pull_bytes=65537, corrupt_connection=1, corrupt_send_index=9)
    assert r["data_errors"] == 1 and r["connections_ok"] == 1


@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
def test_loopback_duplex_cpu(mode):
    """-Pattern:duplex: each side sends and receives half the transfer at once (ctsIOPattern.cpp:968-1031), which
    only the async functor can run; both receive directions are verified."""
    shared_buffer_attach(_SENDER)
    total = 6 * 1024 * 1024 + 10
    r = loopback.run(connections=4, buffer_size=65536, transfer_size=total, verifier=_oracle_verifier,
                     io_pattern=A.PATTERN_DUPLEX, verify_mode=mode, batch_buffers=8)
    assert r["connections_ok"] == 4 and r["connections_failed"] == 0 and r["data_errors"] == 0
    assert r["bytes_recv"] == 4 * (total + 37 + 4)
    assert r["bytes_sent"] == r["bytes_recv"]
    # a flipped byte in either direction fails that connection only
    r = loopback.run(connections=3, buffer_size=65536, transfer_size=total, verifier=_oracle_verifier,
                     io_pattern=A.PATTERN_DUPLEX, verify_mode=mode, batch_buffers=8, corrupt_connection=1,
                     corrupt_send_index=21)
    assert r["data_errors"] == 1 and r["connections_failed"] == 1 and r["connections_ok"] == 2


# ---- the reference's acceptance scenario "verify:data with randomized buffers" ---------------------------------
# (TestScripts/ctsTraffic_acceptance_test.cmd:124-140: -Buffer:[32768,98304] -verify:data for each pattern)
@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
@pytest.mark.parametrize("pattern", [A.PATTERN_PUSH, A.PATTERN_PULL, A.PATTERN_PUSHPULL, A.PATTERN_DUPLEX],
                         ids=["push", "pull", "pushpull", "duplex"])
def test_loopback_randomized_buffers_cpu(mode, pattern):
    """Every send and recv draws its size in [32768, 98304] (GetBufferSize, ctsConfig.cpp:4679-4684); the sender
    buffer and the recv slots are sized for the maximum; every connection completes clean, and a byte flipped on
    the wire fails exactly its connection."""
    shared_buffer_attach(_SENDER_WIDE)
    total = 7 * 1024 * 1024 + 4321
    kw = dict(buffer_size=32768, buffer_size_high=98304, transfer_size=total, verifier=_oracle_verifier,
              io_pattern=pattern, verify_mode=mode, batch_buffers=8, random_seed=7)
    r = loopback.run(connections=3, **kw)
    assert r["connections_ok"] == 3 and r["data_errors"] == 0
    # (Duplex makes an odd transfer even, ctsIOPattern.cpp:1004-1009)
    assert r["bytes_recv"] == 3 * (total + (total % 2 if pattern == A.PATTERN_DUPLEX else 0) + 37 + 4)
    r = loopback.run(connections=3, corrupt_connection=2, corrupt_send_index=11, **kw)
    assert r["data_errors"] == 1 and r["connections_ok"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
@pytest.mark.parametrize("pattern", [A.PATTERN_PUSH, A.PATTERN_DUPLEX], ids=["push", "duplex"])
def test_loopback_randomized_buffers_gpu(engine, mode, pattern):
    """The same acceptance scenario with every VerifyBuffer on the GPU."""
    total = 16 * 1024 * 1024 + 99
    kw = dict(buffer_size=32768, buffer_size_high=98304, transfer_size=total, engine=engine, io_pattern=pattern,
              verify_mode=mode, random_seed=3)
    r = loopback.run(connections=4, **kw)
    even = total % 2 if pattern == A.PATTERN_DUPLEX else 0  # (Duplex makes an odd transfer even)
    assert r["connections_ok"] == 4 and r["data_errors"] == 0 and r["bytes_recv"] == 4 * (total + even + 37 + 4)
    r = loopback.run(connections=4, corrupt_connection=1, corrupt_send_index=30, **kw)
    assert r["data_errors"] == 1 and r["connections_ok"] == 3


def test_loopback_functor_choice():
    """The async functor runs the one-IO-at-a-time patterns too; Duplex refuses the sync functor."""
    from ctstraffic_amd._lib import CtsError

    shared_buffer_attach(_SENDER)
    r = loopback.run(connections=2, buffer_size=32768, transfer_size=3 * 1024 * 1024, verifier=_oracle_verifier,
                     io_pattern=A.PATTERN_PULL, verify_mode=A.VERIFY_SYNC, functor=loopback.FUNCTOR_ASYNC)
    assert r["connections_ok"] == 2 and r["data_errors"] == 0
    with pytest.raises(CtsError):
        loopback.run(connections=1, buffer_size=65536, transfer_size=1 << 20, verifier=_oracle_verifier,
                     io_pattern=A.PATTERN_DUPLEX, functor=loopback.FUNCTOR_SYNC)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
def test_loopback_duplex_gpu(engine, mode):
    r = loopback.run(connections=4, buffer_size=65536, transfer_size=16 * 1024 * 1024 + 6, engine=engine,
                     io_pattern=A.PATTERN_DUPLEX, verify_mode=mode)
    assert r["connections_ok"] == 4 and r["data_errors"] == 0
    r = loopback.run(connections=4, buffer_size=65536, transfer_size=8 * 1024 * 1024, engine=engine,
                     io_pattern=A.PATTERN_DUPLEX, verify_mode=mode, corrupt_connection=3, corrupt_send_index=30)
    assert r["data_errors"] == 1 and r["connections_ok"] == 3


def test_loopback_multi_engine_validation():
    from ctstraffic_amd._lib import CtsError

    shared_buffer_attach(_SENDER)
    # no engines + a hook: the hook verifies (n_engines == 0)
    r = loopback.run(connections=2, buffer_size=65536, transfer_size=1 << 20, verifier=_oracle_verifier, engine=[])
    assert r["connections_ok"] == 2
    with pytest.raises(CtsError):  # nothing to verify with
        loopback.run(connections=1, buffer_size=65536, transfer_size=1 << 20, engine=[])


@pytest.mark.gpu
@pytest.mark.parametrize("pattern", [A.PATTERN_PUSH, A.PATTERN_DUPLEX], ids=["push", "duplex"])
def test_loopback_two_engines_gpu(engine, pattern):
    """Connections spread over two engines by cts_shard_of (two engines on one GPU here; one per GPU on a node)."""
    from ctstraffic_amd import Engine

    with Engine(0) as e2:
        r = loopback.run(connections=8, buffer_size=65536, transfer_size=8 * 1024 * 1024 + 2, engine=[engine, e2],
                         io_pattern=pattern, verify_mode=A.VERIFY_DEFERRED)
        assert r["connections_ok"] == 8 and r["data_errors"] == 0
        for bad in (0, 5):  # connections on either engine (cts_shard_of(0, 2) != cts_shard_of(5, 2))
            r = loopback.run(connections=8, buffer_size=65536, transfer_size=4 * 1024 * 1024, engine=[engine, e2],
                             io_pattern=pattern, verify_mode=A.VERIFY_DEFERRED, corrupt_connection=bad,
                             corrupt_send_index=11)
            assert r["data_errors"] == 1 and r["connections_ok"] == 7


# ---- counter parity across verify arrangements (SYNC = the reference's timing; DEFERRED must report the same) -------
def _side_view(r, connections, corrupt):
    """Everything a run reports that the reference's own run would report identically. With recv_whole every data
    completion is a whole buffer, so completion sizes do not depend on the socket's timing. The one quantity the
    reference itself leaves to timing is left out: how many bytes the corrupted connection's *sender* got out (and
    the error its send saw) before the receiver's reset reached it."""
    sides = [dict(s) for s in r["sides"]]
    for s in sides:  # wall time spent waiting for device verdicts: a timing, not a count (0 without a device)
        s.pop("verify_wait_ns", None)
        s.pop("deferred_depth", None)  # how the arrangement verifies, not what it reports
    if corrupt is not None:
        for k in ("bytes_sent", "final_error", "last_error"):
            sides[corrupt].pop(k)
    totals = {k: r[k] for k in ("bytes_recv", "connections_ok", "connections_failed", "data_errors",
                                "buffers_verified")}
    if corrupt is None:
        totals["bytes_sent"] = r["bytes_sent"]
    return totals, sides


def _three_way(run, connections, transfer, corrupt, send_index, arrangements, depths=None):
    """Runs every arrangement and checks that each reports what the first does; `depths` (a dict), when given, gets
    each arrangement's DEFERRED launches in flight per connection (cts_pattern_stats.deferred_depth, max over sides)."""
    views = {}
    for name, kw in arrangements.items():
        r = run(connections=connections, buffer_size=65536, transfer_size=transfer, recv_whole=True, sides=True,
                corrupt_connection=corrupt, corrupt_send_index=send_index, **kw)
        if depths is not None:
            depths[name] = max(s["deferred_depth"] for s in r["sides"])
        views[name] = _side_view(r, connections, corrupt)
    names = list(views)
    for n in names[1:]:
        assert views[n][0] == views[names[0]][0], (n, views[n][0], views[names[0]][0])
        for i, (a, b) in enumerate(zip(views[n][1], views[names[0]][1])):
            assert a == b, (n, i, a, b)
    return views[names[0]]


@pytest.mark.parametrize("corrupt", [None, 3], ids=["clean", "corrupt"])
def test_deferred_counters_equal_sync_cpu(corrupt):
    """A data error in DEFERRED mode is found up to a batch later; the flush takes back every completion after the
    failing buffer, so TcpStatusDetails, every connection's statistics, its failure record, final status and last
    error equal SYNC's (the reference's timing: ctsIOPattern.cpp:486-489 fails the connection on that completion)."""
    shared_buffer_attach(_SENDER)
    hook = A.BATCH_VERIFIER(oracle.batch_verifier_address())
    arr = {"sync": dict(verifier=hook, verify_mode=A.VERIFY_SYNC),
           "deferred": dict(verifier=hook, verify_mode=A.VERIFY_DEFERRED, batch_buffers=64),
           "deferred_py": dict(verifier=_oracle_verifier, verify_mode=A.VERIFY_DEFERRED, batch_buffers=7)}
    totals, sides = _three_way(loopback.run, 6, 24 * 1024 * 1024 + 4321, corrupt, 150, arr)
    if corrupt is None:
        assert totals["data_errors"] == 0 and totals["connections_ok"] == 6
    else:
        assert totals["data_errors"] == 1 and totals["connections_ok"] == 5
        srv = sides[6 + corrupt]
        # the 151st data buffer carries the flipped byte at len/2: the server stops right there
        assert srv["has_failure"] == 1 and srv["fail_completion"] == 150 and srv["fail_offset"] == 32768
        assert srv["buffers_verified"] == 151 and srv["buffers_failed"] == 1
        assert srv["bytes_recv"] == 151 * 65536 and srv["bytes_recv_at_failure"] == srv["bytes_recv"]
        assert srv["final_error"] == 2147483644 and srv["queued"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("corrupt", [None, 5], ids=["clean", "corrupt"])
def test_config1_three_arrangements_gpu(engine, corrupt):
    """BASELINE configs[0] at full size: loopback TCP push, 8 connections x 1 GiB, 64 KiB IO, -verify:data. The CPU
    oracle answering VerifyBuffer in each receive thread (the reference's arrangement), the GPU per completion
    (SYNC) and the GPU in batches (DEFERRED) report identical status details, per-connection statistics, failure
    records, statuses and last errors, clean and with one corrupted connection."""
    hook = A.BATCH_VERIFIER(oracle.batch_verifier_address())

    def run(**kw):
        if "verifier" in kw:
            shared_buffer_attach(_SENDER)
        return loopback.run(**kw)

    arr = {"cpu_oracle": dict(verifier=hook, verify_mode=A.VERIFY_SYNC),
           "gpu_sync": dict(engine=engine, verify_mode=A.VERIFY_SYNC),
           "gpu_deferred": dict(engine=engine, verify_mode=A.VERIFY_DEFERRED)}
    totals, sides = _three_way(run, 8, 1 << 30, corrupt, 9000, arr)
    if corrupt is None:
        assert totals["connections_ok"] == 8 and totals["data_errors"] == 0
        assert totals["bytes_recv"] == 8 * ((1 << 30) + 37 + 4)
        assert all(s["buffers_verified"] == 16384 for s in sides[8:])
    else:
        assert totals["connections_ok"] == 7 and totals["data_errors"] == 1
        srv = sides[8 + corrupt]
        assert srv["fail_completion"] == 9000 and srv["buffers_verified"] == 9001
        assert srv["bytes_recv"] == 9001 * 65536 and srv["queued"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [0, 16])
@pytest.mark.parametrize("depth", [1, 3])
@pytest.mark.parametrize("corrupt", [None, 5], ids=["clean", "corrupt"])
def test_config1_deferred_depths_gpu(engine, monkeypatch, depth, corrupt, batch):
    """Config 1 at full size with 1 and 3 DEFERRED batches in flight per connection (CTS_DEFERRED_DEPTH; the default,
    2, runs in test_config1_three_arrangements_gpu): the same
    status details, per-connection statistics, failure records and statuses as the CPU oracle in each receive
    thread, clean and with one corrupted connection (a failing batch drops the ones launched after it); at the
    feeder's batch and at 16 buffers (launches of 8 or 4 buffers, thousands per connection)."""
    hook = A.BATCH_VERIFIER(oracle.batch_verifier_address())

    def run(**kw):
        if "verifier" in kw:
            shared_buffer_attach(_SENDER)
            monkeypatch.delenv("CTS_DEFERRED_DEPTH", raising=False)
        else:
            monkeypatch.setenv("CTS_DEFERRED_DEPTH", str(depth))
        try:
            return loopback.run(**kw)
        finally:
            monkeypatch.delenv("CTS_DEFERRED_DEPTH", raising=False)

    arr = {"cpu_oracle": dict(verifier=hook, verify_mode=A.VERIFY_SYNC),
           "gpu_deferred": dict(engine=engine, verify_mode=A.VERIFY_DEFERRED, batch_buffers=batch)}
    depths = {}
    totals, sides = _three_way(run, 8, 1 << 30, corrupt, 9000, arr, depths)
    # the patterns ran the depth asked for (clamped to batch - 1: 3 at batch 16 and at the feeder's batch)
    assert depths == {"cpu_oracle": 0, "gpu_deferred": depth}
    if corrupt is None:
        assert totals["connections_ok"] == 8 and totals["data_errors"] == 0
        assert all(s["buffers_verified"] == 16384 for s in sides[8:])
    else:
        assert totals["connections_ok"] == 7 and totals["data_errors"] == 1
        srv = sides[8 + corrupt]
        assert srv["fail_completion"] == 9000 and srv["buffers_verified"] == 9001
        assert srv["bytes_recv"] == 9001 * 65536 and srv["queued"] == 0


def test_loopback_diagnostic_recv_ring_cpu():
    """The feeder's diagnostic recv ring (verify off, sync functor): data recvs land round robin in a ring of
    buffers, as a DEFERRED pattern's do; counters and statuses are the plain verify-off run's. It refuses to run
    with verification on, with the async functor, or pinned without an engine."""
    shared_buffer_attach(_SENDER)
    base = loopback.run(connections=3, buffer_size=65536, transfer_size=40 * 65536 + 123, verify=False,
                        recv_whole=True, sides=True)
    ring = loopback.run(connections=3, buffer_size=65536, transfer_size=40 * 65536 + 123, verify=False,
                        recv_whole=True, sides=True, recv_ring_buffers=7)
    for r in (base, ring):
        assert r["connections_ok"] == 3 and r["data_errors"] == 0
        assert r["bytes_recv"] == 3 * (40 * 65536 + 123 + 37 + 4)
    assert [s["bytes_recv"] for s in ring["sides"]] == [s["bytes_recv"] for s in base["sides"]]
    with pytest.raises(Exception):
        loopback.run(connections=1, buffer_size=4096, transfer_size=8192, verifier=_oracle_verifier,
                     verify_mode=A.VERIFY_SYNC, recv_ring_buffers=4)
    with pytest.raises(Exception):
        loopback.run(connections=1, buffer_size=4096, transfer_size=8192, verify=False, recv_ring_buffers=4,
                     io_pattern=A.PATTERN_DUPLEX)
    with pytest.raises(Exception):
        loopback.run(connections=1, buffer_size=4096, transfer_size=8192, verify=False, recv_ring_buffers=4,
                     recv_ring_pinned=True)


@pytest.mark.gpu
def test_loopback_diagnostic_recv_ring_pinned_gpu(engine):
    """The diagnostic recv ring in pinned host memory (cts_host_alloc on the engine, as a DEFERRED pattern's ring):
    a verify-off run's counters and statuses are the plain run's."""
    base = loopback.run(connections=4, buffer_size=65536, transfer_size=300 * 65536 + 77, verify=False,
                        recv_whole=True, sides=True, engine=engine)
    ring = loopback.run(connections=4, buffer_size=65536, transfer_size=300 * 65536 + 77, verify=False,
                        recv_whole=True, sides=True, engine=engine, recv_ring_buffers=2 * 512 + 2,
                        recv_ring_pinned=True)
    for r in (base, ring):
        assert r["connections_ok"] == 4 and r["data_errors"] == 0
        assert r["bytes_recv"] == 4 * (300 * 65536 + 77 + 37 + 4)
    assert [s["bytes_recv"] for s in ring["sides"]] == [s["bytes_recv"] for s in base["sides"]]


def test_loopback_send_pacing_cpu():
    """Send pacing end to end: the feeder's senders wait each task's time offset (ctsSendRecvIocp.cpp:378-383).
    4 Push connections x 40 x 8 KiB at 1 MiB/s each (100 ms quanta of 104 857 B, 13 buffers) are deferred into
    their third quantum, so the run takes at least 200 ms; -burstcount:4 -burstdelay:30 with 16 sends per
    connection waits 4 x 30 ms. Data and counters stay exact."""
    shared_buffer_attach(_SENDER)
    hook = A.BATCH_VERIFIER(oracle.batch_verifier_address())
    for kw, n_bufs, floor in [(dict(tcp_bytes_per_second=1 << 20), 40, 0.2),
                              (dict(burst_count=4, burst_delay=30), 16, 0.12)]:
        r = loopback.run(connections=4, buffer_size=8192, transfer_size=n_bufs * 8192, verifier=hook,
                         verify_mode=A.VERIFY_SYNC, functor=loopback.FUNCTOR_SYNC, recv_whole=True, **kw)
        assert r["connections_ok"] == 4 and r["data_errors"] == 0
        assert r["bytes_recv"] == 4 * (n_bufs * 8192 + 37 + 4)
        assert r["seconds"] >= floor, (kw, r["seconds"])
