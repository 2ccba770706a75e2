"""MediaStream (UDP) framing around the verify path.

CPU: the frame -> datagram split against the reference's MSTest known answers
(MSTest/ctsMediaStreamSendBuffer/ctsMediaStreamProtocolUnitTest.cpp:74-160) and a
pure-Python transcription; the client's frame accounting against the Python
restatement (oracle/media_stream.py) on random datagram streams; the oracle's
header parsing on crafted datagrams.
GPU: cts_media_stream_fill / cts_media_stream_verify through the C ABI vs the
oracle, bit-exact, and an end-to-end stream (fill -> verify -> client -> render).
"""
import numpy as np
import pytest

import oracle
from oracle import media_stream as OM
from ctstraffic_amd import media_stream as M
from ctstraffic_amd.types import DESC_DTYPE, DGRAM_HEADER_DTYPE, DGRAM_RECORD_DTYPE, DGRAM_STATUS_DTYPE, RESULT_DTYPE

MAX = 1400  # c_udpDatagramMaximumSizeBytes in the MSTest (ctsMediaStreamProtocolUnitTest.cpp:22)


# ---- split: MSTest KATs -------------------------------------------------------------------------
@pytest.mark.parametrize("frame,count", [
    (26 + 1, 1),          # TinySendRequest :74-83
    (MAX, 1),             # OneDatagramSendRequest :85-94
    (MAX - 1, 1),         # OneDatagramMinusOneSendRequest :96-105
    (MAX + 1, 2),         # OneDatagramPlusOneSendRequest :107-116
    (2 * MAX, 2),         # ExactlyTwoDatagramSendRequest :118-127
    (123456789, 88184),   # LargeSendRequest :129-138
])
def test_split_mstest_kats(frame, count):
    lens = M.split(frame, MAX)
    assert len(lens) == count
    assert int(lens.sum()) == frame  # verify_byte_count: every byte of the frame is sent once
    assert lens.min() >= 27 and lens.max() <= MAX  # header + at least one data byte, never above the max


def test_split_matches_transcription_and_rejects_tiny():
    rng = np.random.default_rng(7)
    for _ in range(400):
        mx = int(rng.integers(27, 9000))
        fr = int(rng.integers(27, 200000))
        assert M.split(fr, mx).tolist() == OM.split(fr, mx)
    assert len(M.split(26, MAX)) == 0 and len(M.split(0, MAX)) == 0  # the ctor FAIL_FASTs on <= 26


# ---- client frame accounting vs the Python restatement -----------------------------------------------
def _random_stream(rng, frame_size, n_frames, max_dgram, p_drop, p_dup, p_bad, p_corrupt, shuffle):
    recs = []
    for f in range(1, n_frames + 1):
        for ln in OM.split(frame_size, max_dgram):
            if rng.random() < p_drop:
                continue
            copies = 2 if rng.random() < p_dup else 1
            for _ in range(copies):
                recs.append((0, f, ln, True))
    extra = []
    for _ in range(int(len(recs) * p_bad)):
        kind = int(rng.choice([0, 0, 2, 3, 4]))
        seq = int(rng.integers(-5, n_frames + 20))
        extra.append((kind, seq, int(rng.integers(27, max_dgram)), True))
    recs += extra
    if shuffle:
        # local reordering only (datagrams overtake each other within a small window)
        idx = np.arange(len(recs)) + rng.random(len(recs)) * shuffle
        recs = [recs[i] for i in np.argsort(idx, kind="stable")]
    out = []
    for k, s, ln, ok in recs:
        if k == 0 and rng.random() < p_corrupt:
            ok = False
        out.append((k, s, ln, ok))
    return out


def _status_of(recs, res):
    """The compact statuses (cts_datagram_status) of records + results."""
    st = np.zeros(len(recs), dtype=DGRAM_STATUS_DTYPE)
    for f in ("sequence_number", "completed_bytes", "flag", "kind"):
        st[f] = recs[f]
    st["pass"] = (recs["kind"] == 0) & (res["pass"] == 1)
    return st


def _sums_of(st, w):
    """What cts_media_stream_verify_frames writes for statuses st under window w (media_stream_verify_quad_kernel,
    FRAMES): FrameTotals and the bytes per window slot."""
    t = M.FrameTotals()
    t.first_exception = M.NO_EXCEPTION
    fb = np.zeros(w.frames, dtype=np.uint64)
    for i, d in enumerate(st):
        if d["kind"] == M.DGRAM_DATA and d["pass"]:
            seq = int(d["sequence_number"])
            t.bits_received += 8 * int(d["completed_bytes"])
            t.datagrams += 1
            k = seq - w.head_sequence_number
            if seq > w.final_frame or k < 0 or k >= w.frames:
                t.error_frames += 1
            else:
                fb[k] += int(d["completed_bytes"])
        elif not (d["kind"] == M.DGRAM_ZERO and w.finished):
            t.exceptions += 1
            t.first_exception = min(t.first_exception, i)
    return t, fb


def _complete_by_sums(cf, st):
    """A batch through the sums path; a batch holding an exception is replayed from its statuses."""
    w = cf.window()
    t, fb = _sums_of(st, w)
    rc = cf.complete_frames(w, t, fb, len(st))
    return cf.complete_status(st)[0] if rc == M.FRAMES_REPLAY else rc


def _run_both(frame_size, buffered, n_frames, stream, renders_between):
    """The client over records + results, the client over compact statuses, the client over per-batch sums (the GPU
    frame accounting, replaying batches with an exception) and the Python restatement, in lockstep: every render
    code and the final statistics agree."""
    cm = M.MediaStreamClient(frame_size, buffered, n_frames)
    cs = M.MediaStreamClient(frame_size, buffered, n_frames)
    cf = M.MediaStreamClient(frame_size, buffered, n_frames)
    om = OM.ClientModel(frame_size, buffered, n_frames)
    recs = np.zeros(len(stream), dtype=DGRAM_RECORD_DTYPE)
    res = np.zeros(len(stream), dtype=RESULT_DTYPE)
    for i, (k, s, ln, ok) in enumerate(stream):
        recs[i] = (s, 0, 0, 0, k, 0, ln if k != 2 else 0)
        res[i]["pass"] = 1 if ok else 0
    st = _status_of(recs, res)
    i = 0
    status = 0
    while i < len(stream) and status == 0:
        j = min(len(stream), i + renders_between)
        status, consumed = cm.complete(recs[i:j], res[i:j])
        assert cs.complete_status(st[i:j]) == (status, consumed)
        assert _complete_by_sums(cf, st[i:j]) == status
        for q in range(i, i + consumed):
            k, s, ln, ok = stream[q]
            om.complete(k, s, ln if k != 2 else 0, ok)
        assert consumed == j - i or status != 0
        i += consumed
        if status == 0:
            code = cm.render()
            assert code == om.render() == cs.render() == cf.render()
            if code != 0:
                break  # the stream finished (Abort) or aborted: the functor stops receiving
    while cm.stats()["finished"] == 0 and cm.stats()["last_error"] == OM.RUNNING:
        assert cm.render() == om.render() == cs.render() == cf.render()
    got = cm.stats()
    exp = om.stats()
    for k in exp:
        assert got[k] == exp[k], (k, got, exp)
    assert cs.stats() == got
    assert cf.stats() == got
    cm.close()
    cs.close()
    cf.close()
    return got


def test_complete_frames_refuses_a_moved_window():
    """A batch summed for one window cannot be applied after a render tick moved it."""
    from ctstraffic_amd._lib import CtsError

    c = M.MediaStreamClient(3000, 2, 6)
    w = c.window()
    assert (w.head_sequence_number, w.final_frame, w.frames, w.finished) == (1, 6, 4, 0)
    st = np.zeros(3, dtype=DGRAM_STATUS_DTYPE)  # frame 1 in three clean datagrams
    st["kind"], st["pass"], st["completed_bytes"], st["sequence_number"] = M.DGRAM_DATA, 1, 1000, 1
    t, fb = _sums_of(st, w)
    assert fb.tolist() == [3000, 0, 0, 0] and t.bits_received == 24000
    assert c.complete_frames(w, t, fb, 3) == 0
    assert c.render() == 0 and c.stats()["successful_frames"] == 1
    with pytest.raises(CtsError):
        c.complete_frames(w, t, fb, 0)
    t.exceptions, t.first_exception = 1, 0
    assert c.complete_frames(c.window(), t, fb, 4) == M.FRAMES_REPLAY
    with pytest.raises(CtsError):  # sums of 3 clean datagrams cannot be a batch of 1
        c.complete_frames(c.window(), t, fb, 1)


@pytest.mark.parametrize("seed", range(6))
def test_client_accounting_matches_model(seed):
    rng = np.random.default_rng(seed)
    frame = int(rng.choice([1400, 4096, 52083]))
    n_frames = int(rng.integers(10, 60))
    buffered = int(rng.integers(1, 10))
    stream = _random_stream(rng, frame, n_frames, MAX, p_drop=0.05, p_dup=0.05, p_bad=0.02 if seed % 2 else 0,
                            p_corrupt=0.002 if seed >= 4 else 0, shuffle=8)
    per_tick = max(1, len(stream) // n_frames)
    _run_both(frame, buffered, n_frames, stream, per_tick)


def test_client_clean_stream_renders_every_frame():
    frame, n_frames = 52083, 30  # README MediaStream sizing (FrameSize 52083 B)
    stream = [(0, f, ln, True) for f in range(1, n_frames + 1) for ln in OM.split(frame, MAX)]
    s = _run_both(frame, 5, n_frames, stream, len(OM.split(frame, MAX)))
    assert s["successful_frames"] == n_frames and s["dropped_frames"] == 0 and s["error_frames"] == 0
    assert s["bits_received"] == 8 * frame * n_frames and s["finished"] == 1 and s["last_error"] == 0


def test_client_nothing_received_is_fatal_abort():
    cm = M.MediaStreamClient(1000, 3, 10)
    codes = [cm.render() for _ in range(3)]
    assert codes[-1] == 2 and cm.stats()["dropped_frames"] == 10 and cm.stats()["last_error"] == OM.NOT_ALL_DATA


def test_client_connection_id():
    cm = M.MediaStreamClient(1000, 3, 10)
    cid = b"0123456789abcdef0123456789abcdef0123"
    cm.set_connection_id(b"\x00\x10" + cid + b"\x00")
    assert cm.connection_id() == cid.decode()


# ---- oracle header parsing on crafted datagrams ---------------------------------------------------
def _crafted():
    S = oracle.sender_buffer(4096)
    dgs = []
    hdr = lambda seq, qpc, qpf: (np.array([0], "<u2").tobytes() + np.array([seq, qpc, qpf], "<i8").tobytes())
    dgs.append(hdr(7, 111, 222) + S[:100].tobytes())                      # data, clean
    bad = bytearray(hdr(8, 1, 2) + S[:300].tobytes())
    bad[26 + 57] ^= 0x40
    dgs.append(bytes(bad))                                                 # data, corrupt at payload byte 57
    dgs.append(b"\x00\x10" + b"x" * 37)                                    # id datagram (39 B)
    dgs.append(b"\x00\x10" + b"x" * 10)                                    # id too short
    dgs.append(b"\x00\x00" + b"\x01" * 10)                                 # data too short (< 26)
    dgs.append(b"\x34\x12" + b"\x00" * 40)                                 # unknown flag 0x1234
    dgs.append(b"")                                                        # zero bytes
    dgs.append(b"\x00")                                                    # 1 byte
    dgs.append(hdr(9, 5, 6))                                               # data with an empty payload
    return dgs


def _pack(dgs, align=1):
    descs = np.zeros(len(dgs), dtype=DESC_DTYPE)
    off = 3  # unaligned on purpose
    blob = bytearray(b"\xee" * off)
    for i, d in enumerate(dgs):
        descs[i]["byte_offset"] = off
        descs[i]["length"] = len(d)
        blob += d
        pad = (-len(blob)) % align
        blob += b"\xee" * pad
        off = len(blob)
    blob += b"\xee" * 64
    return np.frombuffer(bytes(blob), dtype=np.uint8).copy(), descs


def test_oracle_parses_crafted_datagrams():
    arena, descs = _pack(_crafted())
    recs, res, ctr = oracle.media_stream_verify(arena, descs)
    assert recs["kind"].tolist() == [0, 0, 1, 3, 3, 4, 2, 3, 0]
    assert recs["sequence_number"][:2].tolist() == [7, 8]
    # the reference reads "qpc" at +8 and "qpf" at +16 (ctsIOPatternMediaStream.cpp:218-219):
    # bytes 8..15 = seq's top 2 bytes + qpc's low 6 bytes
    assert recs["sender_qpc"][0] == int.from_bytes(arena[descs[0]["byte_offset"] + 8:][:8].tobytes(), "little",
                                                   signed=True)
    assert res["pass"].tolist() == [1, 0, 0, 0, 0, 0, 0, 0, 1]
    assert res["first_mismatch"][1] == 57 and res["flags"][2] == 2
    assert ctr["buffers_checked"] == 3 and ctr["buffers_failed"] == 1 and ctr["bytes_checked"] == 100 + 300


# ---- GPU: fill + verify through the C ABI vs the oracle ---------------------------------------------
def _to_dev(a, torch):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to("cuda")


@pytest.mark.gpu
def test_gpu_media_stream_verify_matches_oracle(engine):
    """The MediaStream receive (four datagrams per wave, header by 16-byte chunk loads gathered with DPP row shifts,
    block-contiguous datagram ranges, outputs written every 64 rounds from a per-wave LDS ring) vs the oracle under
    several walks: several rounds per workgroup, chunked walks (partial last rings, chunk ends and the launch end
    inside a ring), and outputs at 4-byte-aligned (not 16) addresses."""
    from ctstraffic_amd import _lib

    default_sbpc = engine.get_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU)
    default_chunk = engine.get_attr(_lib.ATTR_SMALL_CHUNK)
    try:
        # sbpc 1: several rounds per workgroup (5 000+ datagrams over 256 workgroups); chunked walks
        for sbpc, chunk in ((1, 0), (64, 0), (1, 16), (2, 48), (1, 200)):
            engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, sbpc)
            engine.set_attr(_lib.ATTR_SMALL_CHUNK, chunk)
            _media_stream_verify_vs_oracle(engine)
        _media_stream_verify_vs_oracle(engine, out_shift=4)
    finally:
        engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, default_sbpc)
        engine.set_attr(_lib.ATTR_SMALL_CHUNK, default_chunk)


def _media_stream_verify_vs_oracle(engine, out_shift=0):
    import torch

    rng = np.random.default_rng(11)
    dgs = _crafted()
    S = oracle.sender_buffer(9000)
    for _ in range(5000):  # random valid/corrupt data datagrams of random sizes
        ln = int(rng.integers(26, 9000))
        d = bytearray(np.array([0], "<u2").tobytes() + np.array([rng.integers(-9, 1 << 40), rng.integers(0, 1 << 62),
                                                                 rng.integers(0, 1 << 62)], "<i8").tobytes())
        d += S[:ln - 26].tobytes()
        if ln > 26 and rng.random() < 0.1:
            for p in rng.integers(26, ln, size=int(rng.integers(1, 5))):
                d[int(p)] ^= int(rng.integers(1, 256))
        dgs.append(bytes(d))
    order = rng.permutation(len(dgs))
    dgs = [dgs[i] for i in order]
    arena, descs = _pack(dgs)
    er, eres, ectr = oracle.media_stream_verify(arena, descs)
    a = _to_dev(arena, torch)
    d = _to_dev(descs, torch)
    recs = torch.zeros(len(dgs) * 32 + out_shift, dtype=torch.uint8, device="cuda")[out_shift:]
    res = torch.zeros(len(dgs) * 12 + out_shift, dtype=torch.uint8, device="cuda")[out_shift:]
    ctr = engine.new_counters()
    M.verify(engine, a, d, records=recs, results=res, counters=ctr)
    torch.cuda.synchronize()
    gr = recs.cpu().numpy().view(DGRAM_RECORD_DTYPE)
    gres = res.cpu().numpy().view(RESULT_DTYPE)
    for f in DGRAM_RECORD_DTYPE.names:
        assert np.array_equal(gr[f], er[f]), f
    for f in RESULT_DTYPE.names:
        bad = np.nonzero(gres[f] != eres[f])[0]
        assert bad.size == 0, (f, [(int(i), int(descs[i]["byte_offset"]), int(descs[i]["length"]), gres[i].tolist(),
                                    eres[i].tolist()) for i in bad[:6]])
    assert engine.read_counters(ctr) == ectr
    # the compact form: 16-byte statuses, same counters
    st = torch.zeros(len(dgs) * 16 + out_shift, dtype=torch.uint8, device="cuda")[out_shift:]
    ctr2 = engine.new_counters()
    M.verify_status(engine, a, d, status=st, counters=ctr2)
    torch.cuda.synchronize()
    gs = st.cpu().numpy().view(DGRAM_STATUS_DTYPE)
    es = _status_of(er, eres)
    for f in DGRAM_STATUS_DTYPE.names:
        assert np.array_equal(gs[f], es[f]), f
    assert engine.read_counters(ctr2) == ectr


def _media_stream_fill_expected(arena, descs, hdrs):
    """What cts_media_stream_fill writes (ctsMediaStreamProtocol.hpp:230-243): per datagram the header {u16 0, i64 seq,
    i64 qpc, i64 qpf} then P[0 .. length - 26) -- the oracle's payload fill (skip 26, pattern offset 0) plus the
    header bytes; every other byte of the arena untouched."""
    d = descs.copy()
    d["skip_head"] = 26
    d["expected_pattern_offset"] = 0
    oracle.fill(arena, d)
    for i in range(len(descs)):
        o = int(descs["byte_offset"][i])
        arena[o:o + 26] = np.frombuffer(b"\0\0" + hdrs[i].tobytes(), dtype=np.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("fill_nt", [0, 1])
def test_gpu_media_stream_fill_matches_oracle(engine, fill_nt):
    """cts_media_stream_fill byte for byte: datagrams on 16-byte boundaries (the whole-chunk path, header assembled in
    registers) and off them (the per-byte-edge path), lengths 26 (header only) to 26 + 1446 and past, partial last
    chunks, sentinel gaps between datagrams that must stay untouched, random 64-bit header values; plain and
    nontemporal stores."""
    import torch

    from ctstraffic_amd import _lib

    rng = np.random.default_rng(0x5E4D + fill_nt)
    lens = [26, 27, 31, 32, 33, 42, 47, 48, 1471, 1472, 1473, 1488, 2048 + 26, 9000, 26 + 65536 - 7]
    lens += rng.integers(26, 1600, size=300).tolist()
    n = len(lens)
    descs = np.zeros(n, dtype=DESC_DTYPE)
    off = 0
    for i, ln in enumerate(lens):
        mis = 0 if i % 3 else int(rng.integers(1, 16))  # two in three on a 16-byte boundary
        off = ((off + 15) // 16) * 16 + mis + int(rng.integers(0, 3)) * 16
        descs[i]["byte_offset"] = off
        descs[i]["length"] = ln
        off += ln + int(rng.integers(0, 5))
    hdrs = np.zeros(n, dtype=DGRAM_HEADER_DTYPE)
    for f in ("sequence_number", "qpc", "qpf"):
        hdrs[f] = rng.integers(-(1 << 62), 1 << 62, size=n)
    arena_bytes = off + 64
    base = rng.integers(0, 256, size=arena_bytes, dtype=np.uint8)
    expect = base.copy()
    _media_stream_fill_expected(expect, descs, hdrs)
    default = engine.get_attr(_lib.ATTR_FILL_NT)
    engine.set_attr(_lib.ATTR_FILL_NT, fill_nt)
    try:
        a = torch.from_numpy(base.copy()).to("cuda")
        M.fill(engine, a, _to_dev(descs, torch), _to_dev(hdrs, torch))
        torch.cuda.synchronize()
    finally:
        engine.set_attr(_lib.ATTR_FILL_NT, default)
    got = a.cpu().numpy()
    bad = np.nonzero(got != expect)[0]
    assert bad.size == 0, (bad[:8].tolist(), got[bad[:8]].tolist(), expect[bad[:8]].tolist())


@pytest.mark.gpu
@pytest.mark.parametrize("fill_nt", [0, 1])
@pytest.mark.parametrize("stride", [32, 48, 1024, 1472, 1536, 4096])
def test_gpu_media_stream_fill_strided_matches_oracle(engine, fill_nt, stride):
    """cts_media_stream_fill_strided byte for byte against the same datagrams through descriptors: full slots, short
    datagrams (26 bytes, partial last chunks), lengths that must leave their slot unwritten (below 26, above the
    stride, past the arena's end), the gap after each datagram untouched; strides below 1024 (per-lane loads) and
    from 1024 (two headers per round as scalar loads); several waves' runs, so run ends fall inside datagrams."""
    import torch

    from ctstraffic_amd import _lib

    rng = np.random.default_rng(stride * 3 + fill_nt)
    n = 3000 if stride < 1024 else 700
    lens = np.full(n, stride, dtype=np.uint32)
    pick = rng.random(n)
    lens[pick < 0.3] = rng.integers(26, stride + 1, size=int(np.sum(pick < 0.3)))
    lens[(pick >= 0.3) & (pick < 0.35)] = 26
    lens[(pick >= 0.35) & (pick < 0.38)] = rng.integers(0, 26, size=int(np.sum((pick >= 0.35) & (pick < 0.38))))
    lens[(pick >= 0.38) & (pick < 0.40)] = stride + 1 + rng.integers(0, 64, size=int(np.sum((pick >= 0.38) & (pick < 0.40))))
    arena_bytes = n * stride - 5  # the last slot ends past the arena: written only if its length still fits
    lens[-1] = stride
    hdrs = np.zeros(n, dtype=DGRAM_HEADER_DTYPE)
    for f in ("sequence_number", "qpc", "qpf"):
        hdrs[f] = rng.integers(-(1 << 62), 1 << 62, size=n)
    base = rng.integers(0, 256, size=arena_bytes, dtype=np.uint8)
    expect = base.copy()
    ok = (lens >= 26) & (lens <= stride) & (np.arange(n, dtype=np.uint64) * stride + lens <= arena_bytes)
    descs = np.zeros(int(ok.sum()), dtype=DESC_DTYPE)
    descs["byte_offset"] = np.nonzero(ok)[0].astype(np.uint64) * stride
    descs["length"] = lens[ok]
    _media_stream_fill_expected(expect, descs, hdrs[ok])
    default = engine.get_attr(_lib.ATTR_FILL_NT)
    engine.set_attr(_lib.ATTR_FILL_NT, fill_nt)
    try:
        a = torch.from_numpy(base.copy()).to("cuda")
        M.fill_strided(engine, a, stride, torch.from_numpy(lens).to("cuda"), _to_dev(hdrs, torch))
        torch.cuda.synchronize()
    finally:
        engine.set_attr(_lib.ATTR_FILL_NT, default)
    got = a.cpu().numpy()
    bad = np.nonzero(got != expect)[0]
    assert bad.size == 0, (bad[:8].tolist(), got[bad[:8]].tolist(), expect[bad[:8]].tolist())


@pytest.mark.gpu
def test_gpu_media_stream_fill_strided_refuses_bad_shapes(engine):
    import torch

    a = torch.zeros(4096 + 16, dtype=torch.uint8, device="cuda")
    lens = torch.full((2,), 64, dtype=torch.int32, device="cuda")
    hd = torch.zeros(2 * 24 + 8, dtype=torch.uint8, device="cuda")
    for stride, arena, ln, h in ((40, a[:4096], lens, hd), (16, a[:4096], lens, hd), (64, a[1:4097], lens, hd),
                                 ((1 << 20) + 16, a[:4096], lens, hd),  # above 1 MiB
                                 (64, a[:4096], lens.view(torch.uint8)[1:5], hd),  # lengths not 4-byte aligned
                                 (64, a[:4096], lens, hd[4:4 + 48])):  # headers not 8-byte aligned
        with pytest.raises(Exception):
            M.fill_strided(engine, arena, stride, ln, h)


@pytest.mark.gpu
def test_gpu_media_stream_end_to_end(engine):
    """Server frames -> datagrams (split) -> GPU fill -> GPU verify -> client accounting -> render."""
    import torch

    frame, n_frames, buffered = 52083, 40, 5
    lens = M.split(frame, 1472)
    per = len(lens)
    n = per * n_frames
    descs = np.zeros(n, dtype=DESC_DTYPE)
    descs["length"] = np.tile(lens, n_frames)
    descs["byte_offset"] = np.concatenate([[0], np.cumsum(descs["length"][:-1].astype(np.uint64))])
    hdrs = np.zeros(n, dtype=DGRAM_HEADER_DTYPE)
    hdrs["sequence_number"] = np.repeat(np.arange(1, n_frames + 1), per)
    hdrs["qpc"] = np.arange(n) * 1000
    hdrs["qpf"] = 10_000_000
    arena_bytes = int(descs["length"].sum())
    a = torch.zeros(arena_bytes + 64, dtype=torch.uint8, device="cuda")[:arena_bytes]
    dd, hd = _to_dev(descs, torch), _to_dev(hdrs, torch)
    M.fill(engine, a, dd, hd)
    # corrupt one datagram of frame 30
    bad = 29 * per + 3
    pos = int(descs["byte_offset"][bad]) + 26 + 100
    a[pos] ^= 0x5A
    recs = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    res = engine.new_results(n)
    M.verify(engine, a, dd, records=recs, results=res)
    torch.cuda.synchronize()
    host = a.cpu().numpy()
    er, eres, _ = oracle.media_stream_verify(host, descs)
    gr = recs.cpu().numpy().view(DGRAM_RECORD_DTYPE)
    gres = res.cpu().numpy().view(RESULT_DTYPE)
    assert np.array_equal(gr, er) and np.array_equal(gres, eres)
    assert gr["sequence_number"].tolist() == hdrs["sequence_number"].tolist()
    # header bytes on the wire: flag 0, seq, qpc, qpf (ctsMediaStreamProtocol.hpp:230-243)
    d0 = host[int(descs["byte_offset"][5]):][:26]
    assert d0[:2].tolist() == [0, 0] and int.from_bytes(d0[2:10].tobytes(), "little") == 1
    assert int.from_bytes(d0[10:18].tobytes(), "little") == 5000
    cm = M.MediaStreamClient(frame, buffered, n_frames)
    status, consumed = cm.complete(gr, gres)
    assert status == 2 and consumed == bad + 1  # the corrupt datagram fails the stream (CorruptedBytes)
    s = cm.stats()
    assert s["last_error"] == OM.DATA_MISMATCH and s["fail_datagram"] == bad
    # the compact receive pass drives the client to the same failure
    st = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    M.verify_status(engine, a, dd, status=st)
    torch.cuda.synchronize()
    gs = st.cpu().numpy().view(DGRAM_STATUS_DTYPE)
    assert np.array_equal(gs, _status_of(gr, gres))
    cs = M.MediaStreamClient(frame, buffered, n_frames)
    assert cs.complete_status(gs) == (2, bad + 1) and cs.stats() == s
    # without the corruption every frame renders successfully
    fixed = gres.copy()
    fixed["pass"][bad] = 1
    cm2 = M.MediaStreamClient(frame, buffered, n_frames)
    for f in range(n_frames):  # one frame arrives per renderer tick
        assert cm2.complete(gr[f * per:(f + 1) * per], fixed[f * per:(f + 1) * per]) == (0, per)
        code = cm2.render()
    assert code == 1
    s2 = cm2.stats()
    assert s2["successful_frames"] == n_frames and s2["dropped_frames"] == 0 and s2["last_error"] == 0


def _frames_case(rng, n, head, frames, final, with_exceptions, finished=False):
    """Random datagrams around a window: clean DATA of random sizes with sequence numbers before, in, after the window
    and past the final frame; optionally corrupt payloads, zero-byte, short, ID and unknown-flag datagrams."""
    S = oracle.sender_buffer(4000)
    dgs = []
    for _ in range(n):
        ln = int(rng.integers(26, 3000))
        seq = int(rng.choice([rng.integers(head - 30, head), rng.integers(head, head + frames),
                              rng.integers(head, head + frames), rng.integers(head + frames, head + frames + 40),
                              rng.integers(final + 1, final + 50), -int(rng.integers(1, 1 << 40))]))
        d = bytearray(np.array([0], "<u2").tobytes() + np.array([seq, 0, 0], "<i8").tobytes()) + S[:ln - 26].tobytes()
        if with_exceptions and ln > 26 and rng.random() < 0.01:
            d[int(rng.integers(26, ln))] ^= 0x20
        dgs.append(bytes(d))
    if with_exceptions:
        for c in _crafted()[2:]:
            dgs.insert(int(rng.integers(0, len(dgs))), c)
    elif finished:
        for _ in range(5):
            dgs.insert(int(rng.integers(0, len(dgs))), b"")  # zero-byte datagrams after the stream finished
    return dgs


@pytest.mark.gpu
def test_gpu_media_stream_frames_match_statuses(engine):
    """cts_media_stream_verify_frames / _strided_frames: the GPU sums of the batch's frame accounting equal the sums
    of the oracle's per-datagram statuses (bits, error frames, clean DATA datagrams, the bytes of every window slot,
    the first exception and their count), for windows summed in LDS (<= 512 slots) and with global atomics, several
    walks, both forms; the counter block is the oracle's."""
    import torch

    from ctstraffic_amd import _lib

    rng = np.random.default_rng(0xF4A)
    sbpc0, chunk0 = engine.get_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU), engine.get_attr(_lib.ATTR_SMALL_CHUNK)
    try:
        for head, frames, final, exc, fin in ((100, 10, 10**6, False, False), (100, 10, 10**6, True, False),
                                              (5, 2000, 1500, True, False), (40, 512, 45, False, True),
                                              (7, 513, 10**9, False, False)):
            dgs = _frames_case(rng, 6000, head, frames, final, exc, fin)
            arena, descs = _pack(dgs)
            er, eres, ectr = oracle.media_stream_verify(arena, descs)
            w = M.FrameWindow(head, final, frames, 1 if fin else 0)
            et, efb = _sums_of(_status_of(er, eres), w)
            assert (et.exceptions > 0) == exc and et.error_frames > 0
            a, d = _to_dev(arena, torch), _to_dev(descs, torch)
            # the strided form: the same datagrams in a ring of 3072-byte slots (16-byte aligned)
            ring = np.zeros(len(dgs) * 3072 + 16, dtype=np.uint8)
            lens = np.array([len(x) for x in dgs], dtype=np.uint32)
            for i, x in enumerate(dgs):
                ring[i * 3072:i * 3072 + len(x)] = np.frombuffer(x, dtype=np.uint8)
            ra, rl = _to_dev(ring, torch), _to_dev(lens, torch)
            for sbpc, chunk in ((64, 0), (1, 0), (1, 48)):
                engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, sbpc)
                engine.set_attr(_lib.ATTR_SMALL_CHUNK, chunk)
                for strided in (False, True):
                    sums = M.FrameSums(frames)
                    ctr = engine.new_counters()
                    if strided:
                        M.verify_strided_frames(engine, ra, 3072, rl, w, sums, counters=ctr)
                    else:
                        M.verify_frames(engine, a, d, w, sums, counters=ctr)
                    torch.cuda.synchronize()
                    t, fb = sums.read()
                    case = (head, frames, final, exc, fin, sbpc, chunk, strided)
                    assert t.as_dict() == et.as_dict(), (case, t.as_dict(), et.as_dict())
                    assert np.array_equal(fb[:frames], efb), case
                    assert engine.read_counters(ctr) == ectr, case
    finally:
        engine.set_attr(_lib.ATTR_SMALL_BLOCKS_PER_CU, sbpc0)
        engine.set_attr(_lib.ATTR_SMALL_CHUNK, chunk0)


@pytest.mark.gpu
def test_gpu_media_stream_frames_edges(engine):
    """cts_media_stream_verify_frames at its edges: an empty batch zeroes the sums, a zero-slot window counts every
    clean datagram as an error frame without touching frame_bytes, misaligned or missing outputs are refused."""
    import torch

    rng = np.random.default_rng(0xED6)
    dgs = _frames_case(rng, 300, 10, 5, 10**6, False)
    arena, descs = _pack(dgs)
    a, d = _to_dev(arena, torch), _to_dev(descs, torch)
    sums = M.FrameSums(5)
    sums.totals.fill_(0x5A)
    sums.frame_bytes.fill_(77)
    M.verify_frames(engine, a, d[:0], M.FrameWindow(10, 10**6, 5, 0), sums)  # n = 0
    torch.cuda.synchronize()
    t, fb = sums.read()
    assert t.as_dict() == {"bits_received": 0, "error_frames": 0, "datagrams": 0,
                           "first_exception": M.NO_EXCEPTION, "exceptions": 0} and not fb.any()
    w0 = M.FrameWindow(10, 10**6, 0, 0)  # no window slot: every clean datagram is an error frame
    M.verify_frames(engine, a, d, w0, sums)
    torch.cuda.synchronize()
    t, _ = sums.read()
    er, eres, _ = oracle.media_stream_verify(arena, descs)
    et, _ = _sums_of(_status_of(er, eres), w0)
    assert t.as_dict() == et.as_dict() and t.error_frames == t.datagrams == len(dgs)
    import ctypes

    def raw(totals_ptr, frame_bytes_ptr, w):
        return engine._L.cts_media_stream_verify_frames(engine._h, a.data_ptr(), a.numel(), d.data_ptr(), len(dgs),
                                                        ctypes.byref(w), totals_ptr, frame_bytes_ptr, None, None)

    w5 = M.FrameWindow(10, 10**6, 5, 0)
    assert raw(sums.totals.data_ptr(), sums.frame_bytes.data_ptr(), w5) == 0
    assert raw(sums.totals.data_ptr() + 4, sums.frame_bytes.data_ptr(), w5) < 0  # totals not 8-byte aligned
    assert raw(None, sums.frame_bytes.data_ptr(), w5) < 0                      # no totals
    assert raw(sums.totals.data_ptr(), None, w5) < 0                           # a window with slots needs frame_bytes
    assert raw(sums.totals.data_ptr(), None, w0) == 0                          # ... a zero-slot one does not
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_gpu_media_stream_client_by_frames(engine, seed):
    """A whole MediaStream stream (split frames, drops, duplicates, local reordering, stray sequence numbers, a
    corrupt payload for seed 2) received in batches between render ticks: the client fed by the GPU sums (replaying
    batches with an exception from compact statuses) ends with the same statistics as the client fed every
    datagram's status (ctsIOPatternMediaStream.cpp:150-530)."""
    import torch

    rng = np.random.default_rng(0xC11 + seed)
    frame, n_frames, buffered = 52083, 40, 4
    stream = _random_stream(rng, frame, n_frames, 1472, p_drop=0.01, p_dup=0.01, p_bad=0.0, p_corrupt=0, shuffle=6)
    stream += [(0, int(s), 700, True) for s in rng.integers(-3, n_frames + 30, size=20)]  # strays
    if seed == 2:
        stream.insert(len(stream) // 2, (0, n_frames // 2, 1000, False))
    S = oracle.sender_buffer(2000)
    dgs = []
    for k, sq, ln, ok in stream:
        d = bytearray(np.array([0], "<u2").tobytes() + np.array([sq, 0, 0], "<i8").tobytes()) + S[:ln - 26].tobytes()
        if not ok:
            d[26 + 5] ^= 1
        dgs.append(bytes(d))
    arena, descs = _pack(dgs)
    a = _to_dev(arena, torch)
    per = max(1, len(dgs) // n_frames)
    cg = M.MediaStreamClient(frame, buffered, n_frames)
    cs = M.MediaStreamClient(frame, buffered, n_frames)
    replays = 0
    for b, i in enumerate(range(0, len(dgs), per)):
        d = _to_dev(descs[i:i + per], torch)
        rc, replayed = cg.complete_batch_on_gpu(engine, a, d)
        replays += replayed
        st = torch.zeros(len(descs[i:i + per]) * 16, dtype=torch.uint8, device="cuda")
        M.verify_status(engine, a, d, status=st)
        torch.cuda.synchronize()
        rs, _ = cs.complete_status(st.cpu().numpy().view(DGRAM_STATUS_DTYPE))
        assert rc == rs
        if rc != 0:
            break
        if b >= buffered - 1:  # rendering starts once the first frames are buffered
            assert cg.render() == cs.render()
    while cs.stats()["finished"] == 0 and cs.stats()["last_error"] == OM.RUNNING:
        assert cg.render() == cs.render()
    assert cg.stats() == cs.stats()
    assert (replays > 0) == (seed == 2)
    assert cs.stats()["successful_frames"] > 0


@pytest.mark.gpu
def test_gpu_media_stream_udp_status_line(engine):
    """The UDP status output (ctsPrintStatus.hpp:314-446, ctsTraffic.cpp:173-200) over a GPU-verified stream:
    fill -> one extra datagram with an unknown sequence number -> a corrupt payload in frame 7 -> the compact
    receive pass -> the client, one frame per render tick. The process-wide counters equal the client's, and
    the Errors column shows its error frames; the corruption itself fails the stream (CorruptedBytes) and is
    the connection's ProtocolError, not an error frame (:185-190)."""
    import torch

    from ctstraffic_amd import status as S

    frame, n_frames, buffered = 52083, 10, 3
    lens = M.split(frame, 1472)
    per = len(lens)
    seqs = np.repeat(np.arange(1, n_frames + 1), per)
    extra = 2 * per  # after frame 2: a datagram of frame 999 (> the final frame: an error frame, :198-208)
    seqs = np.insert(seqs, extra, 999)
    lengths = np.insert(np.tile(lens, n_frames), extra, 1472)
    n = len(seqs)
    descs = np.zeros(n, dtype=DESC_DTYPE)
    descs["length"] = lengths
    descs["byte_offset"] = np.concatenate([[0], np.cumsum(lengths[:-1].astype(np.uint64))])
    hdrs = np.zeros(n, dtype=DGRAM_HEADER_DTYPE)
    hdrs["sequence_number"], hdrs["qpf"] = seqs, 10_000_000
    arena_bytes = int(lengths.sum())
    a = torch.zeros(arena_bytes + 64, dtype=torch.uint8, device="cuda")[:arena_bytes]
    dd = _to_dev(descs, torch)
    M.fill(engine, a, dd, _to_dev(hdrs, torch))
    bad = 6 * per + 1 + 2  # the third datagram of frame 7
    a[int(descs["byte_offset"][bad]) + 26 + 500] ^= 0x81
    st = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    M.verify_status(engine, a, dd, status=st)
    torch.cuda.synchronize()
    gs = st.cpu().numpy().view(DGRAM_STATUS_DTYPE)
    er, eres, _ = oracle.media_stream_verify(a.cpu().numpy(), descs)
    assert np.array_equal(gs, _status_of(er, eres))
    M.udp_status_details_reset()
    c = M.MediaStreamClient(frame, buffered, n_frames)
    # the datagrams of frame f + 1, the extra one arriving with frame 2
    starts = [0] + [f * per + (1 if f >= 2 else 0) for f in range(1, n_frames)] + [n]
    status = 0
    for f in range(n_frames):
        status, consumed = c.complete_status(gs[starts[f]:starts[f + 1]])
        if status != 0:
            break
        c.render()
    s = c.stats()
    assert status == 2 and s["last_error"] == OM.DATA_MISMATCH and s["fail_datagram"] == bad
    assert s["error_frames"] == 1 and s["successful_frames"] == 6
    udp = M.udp_status_details()
    assert udp == {f: s[f] for f in udp}
    line = S.udp_line(S.CONSOLE, current_time_ms=1000, start_time_ms=0, end_time_ms=1000, active_streams=1,
                      **udp)
    assert line[79 - 7:79].strip() == str(s["error_frames"]) == "1"
    assert line[48 - 9:48].strip() == str(s["successful_frames"])
    summ = S.udp_summary(0, 0, 1, **udp)
    assert "ProtocolErrors [1]" in summ and "  Total Error Frames : 1 (" in summ
    assert "  Total Bytes Recv : %d\n" % (udp["bits_received"] // 8) in summ
    M.udp_status_details_reset()


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1536, 1500, 9017])
def test_gpu_media_stream_verify_strided_matches_oracle(engine, stride):
    """cts_media_stream_verify_strided: a receive ring of datagrams at i * stride (16-byte-aligned slots and
    odd strides) with their completed lengths only; records, results and counters equal the oracle's over the
    same datagrams described by descriptors. Lengths above the stride are BAD_DESC."""
    import torch

    rng = np.random.default_rng(stride)
    S = oracle.sender_buffer(stride + 64)
    n = 7000
    ring = np.full(n * stride + 64, 0xEE, dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint32)
    crafted = _crafted()
    for i in range(n):
        if i < len(crafted) * 3 and i % 3 == 0:
            d = crafted[i // 3]
        else:
            ln = int(rng.integers(26, stride + 1))
            d = bytearray(np.array([0], "<u2").tobytes() + np.array([i, rng.integers(0, 1 << 62),
                                                                     rng.integers(0, 1 << 62)], "<i8").tobytes())
            d += S[:ln - 26].tobytes()
            if rng.random() < 0.05:
                d[int(rng.integers(26, ln))] ^= int(rng.integers(1, 256)) if ln > 26 else 0
            d = bytes(d)
        ring[i * stride:i * stride + len(d)] = np.frombuffer(d, dtype=np.uint8)
        lens[i] = len(d)
    descs = np.zeros(n, dtype=DESC_DTYPE)
    descs["byte_offset"] = np.arange(n, dtype=np.uint64) * stride
    descs["length"] = lens
    er, eres, ectr = oracle.media_stream_verify(ring, descs)
    a = _to_dev(ring, torch)
    ld = _to_dev(lens, torch)
    recs = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
    res = engine.new_results(n)
    ctr = engine.new_counters()
    M.verify_strided(engine, a, stride, ld, records=recs, results=res, counters=ctr)
    torch.cuda.synchronize()
    gr = recs.cpu().numpy().view(DGRAM_RECORD_DTYPE)
    gres = res.cpu().numpy().view(RESULT_DTYPE)
    for f in DGRAM_RECORD_DTYPE.names:
        assert np.array_equal(gr[f], er[f]), f
    for f in RESULT_DTYPE.names:
        assert np.array_equal(gres[f], eres[f]), f
    assert engine.read_counters(ctr) == ectr
    # the compact form over the same ring
    st = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    ctr2 = engine.new_counters()
    M.verify_strided_status(engine, a, stride, ld, status=st, counters=ctr2)
    torch.cuda.synchronize()
    gs = st.cpu().numpy().view(DGRAM_STATUS_DTYPE)
    es = _status_of(er, eres)
    for f in DGRAM_STATUS_DTYPE.names:
        assert np.array_equal(gs[f], es[f]), f
    assert engine.read_counters(ctr2) == ectr
    # a completion longer than its slot is a bad descriptor, not read
    lens2 = lens.copy()
    lens2[5] = stride + 1
    recs.zero_()
    M.verify_strided(engine, a, stride, _to_dev(lens2, torch), records=recs, results=res)
    M.verify_strided_status(engine, a, stride, _to_dev(lens2, torch), status=st)
    torch.cuda.synchronize()
    gr = recs.cpu().numpy().view(DGRAM_RECORD_DTYPE)
    gres = res.cpu().numpy().view(RESULT_DTYPE)
    assert gr["kind"][5] == 5 and gres["flags"][5] == 1 and gres["pass"][5] == 0
    gs = st.cpu().numpy().view(DGRAM_STATUS_DTYPE)
    assert gs["kind"][5] == 5 and gs["pass"][5] == 0 and gs["completed_bytes"][5] == stride + 1
