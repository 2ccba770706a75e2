"""MediaStream (UDP) patterns of the ctsIoPattern mirror: MakeIoPattern for -Pattern:MediaStream returns
ctsIoPatternMediaStreamServer when listening (ctsIOPattern.cpp:1100-1175) and ctsIoPatternMediaStreamClient
otherwise (ctsIOPatternMediaStream.cpp:46-530), both driven through InitiateIo / CompleteIo like every other
pattern (ctsMediaStreamClient.cpp:136-144,268,404; ctsMediaStreamServerConnectedSocket.cpp:111-133).

The reference holds no MSTest of these patterns; the checks below follow its source line by line:
- server: the connection-id datagram, one tracked send of one frame per frame timed to the frame rate, bits
  counted per completed send, completion after the last frame;
- client: untracked one-datagram recvs, header validation, payload verify (the oracle on CPU, the gfx950 kernel
  on the GPU), frame accounting in lockstep with the Python restatement (oracle/media_stream.py ClientModel),
  the START / renderer timers and the Abort / FatalAbort tasks they hand to the registered callback.
"""
import threading
import time

import numpy as np
import pytest

import oracle
from oracle import media_stream as OM
from ctstraffic_amd import _pattern_abi as A
from ctstraffic_amd import media_stream as M
from ctstraffic_amd.pattern import IoPattern, PatternConfig, clock_set, shared_buffer_attach

_SENDER = oracle.sender_buffer(4 * 65536)
Send, Recv = A.TASK_SEND, A.TASK_RECV


def _oracle_verifier(arena, descs):
    return oracle.verify_batch(arena, descs)[0]


class FakeClock:
    def __init__(self, t=100000):
        self.t = t

    def __call__(self):
        return self.t


@pytest.fixture
def clock():
    c = FakeClock()
    clock_set(c)
    yield c
    clock_set(None)


def _make(cfg, engine=None):
    if engine is None:
        shared_buffer_attach(_SENDER)
        return IoPattern.MakeIoPattern(cfg, None, verifier=_oracle_verifier)
    return IoPattern.MakeIoPattern(cfg, engine)


# ---- server ---------------------------------------------------------------------------------------------
def test_server_connection_id_then_timed_frames(clock):
    M.udp_status_details_reset()
    frame, fps, frames = 4000, 50, 6
    p = _make(PatternConfig.media_stream(listening=True, frame_size=frame, frames_per_second=fps,
                                         stream_length_frames=frames))
    cid = p.connection_id()
    assert len(cid) == 36
    t = p.InitiateIo()  # MakeConnectionIdTask over a recv buffer (ctsMediaStreamProtocol.hpp:389-405)
    assert (t.io_action, t.buffer_type, t.track_io, t.buffer_length) == (Send, A.BUFFER_UDP_CONNECTION_ID, 0, 39)
    assert IoPattern.read_task_buffer(t, 39) == b"\x00\x10" + cid.encode() + b"\x00"
    assert p.CompleteIo(t, 39) == A.IO_CONTINUE
    clock.t += 3
    base = clock.t  # the stream's base time: the first frame request after the connection id (:1131-1134)
    for f in range(1, frames + 1):
        clock.t = base + 7 * (f - 1)  # the sender gets ahead of the frame clock
        t = p.InitiateIo()
        assert (t.io_action, t.track_io, t.buffer_length) == (Send, 1, frame)
        assert t.buffer == IoPattern.AccessSharedBuffer()
        # base + frame * 1000 / fps - now (ctsIOPattern.cpp:1140-1146)
        assert t.time_offset_ms == base + f * 1000 // fps - clock.t
        assert p.InitiateIo().io_action == A.TASK_NONE  # one task per frame in flight
        st = p.CompleteIo(t, frame)
        assert st == (A.IO_COMPLETED if f == frames else A.IO_CONTINUE)
    assert p.GetLastPatternError() == 0
    s = p.media_stream_stats()
    assert s["bits_received"] == 8 * frame * frames
    assert M.udp_status_details()["bits_received"] == 8 * frame * frames
    assert p.InitiateIo().io_action == A.TASK_NONE
    p.close()


def test_server_failed_send_fails_the_stream(clock):
    p = _make(PatternConfig.media_stream(listening=True, frame_size=1000, frames_per_second=10,
                                         stream_length_frames=3))
    p.CompleteIo(p.InitiateIo(), 39)
    t = p.InitiateIo()
    assert p.CompleteIo(t, 0, 10054) == A.IO_FAILED  # WSAECONNRESET: UDP fails on any error (ctsIOPatternState.hpp:263-271)
    assert p.GetLastPatternError() == 10054
    p.close()


# ---- client -----------------------------------------------------------------------------------------------
def _datagram(seq, length, qpc=0, qpf=0, corrupt_at=None):
    b = bytearray(np.array([0], "<u2").tobytes() + np.array([seq, qpc, qpf], "<i8").tobytes())
    b += _SENDER[:length - 26].tobytes()
    if corrupt_at is not None:
        b[26 + corrupt_at] ^= 0x5A
    return bytes(b)


class ClientRun:
    """A MediaStream client pattern with manual timers on a fake clock, fed datagrams one recv at a time, beside
    the Python restatement of the client (oracle ClientModel) fed the same datagrams and render ticks."""

    def __init__(self, clock, frame, buffered, frames, fps=100, max_dgram=1400, recvs=3, engine=None,
                 complete_in_callback=False, mode=A.VERIFY_SYNC, batch=0):
        self.clock, self.frame, self.fps = clock, frame, fps
        cfg = PatternConfig.media_stream(listening=False, frame_size=frame, frames_per_second=fps,
                                         stream_length_frames=frames, buffered_frames=buffered,
                                         datagram_max_size=max_dgram, pre_post_recvs=recvs, ms_manual_timers=True,
                                         verify_mode=mode, batch_buffers=batch)
        self.p = _make(cfg, engine)
        self.model = OM.ClientModel(frame, buffered, frames)
        self.tasks = []  # tasks handed to the callback
        self.in_callback = []

        def cb(task):
            self.tasks.append(task)
            if complete_in_callback and task.io_action in (A.TASK_ABORT, A.TASK_FATAL_ABORT):
                self.in_callback.append(self.p.CompleteIo(task, 0, 0))  # re-entrant, as ctsMediaStreamClient.cpp:317-331

        self.p.RegisterCallback(cb)
        self.base = clock.t
        self.posted = [self.p.InitiateIo() for _ in range(recvs)]
        assert self.p.InitiateIo().io_action == A.TASK_NONE
        for t in self.posted:
            assert (t.io_action, t.track_io, t.buffer_type) == (Recv, 0, A.BUFFER_DYNAMIC)
            assert t.buffer_length == min(frame, max_dgram)
            assert IoPattern.read_task_buffer(t, 8) == b"\0" * 8  # the seq number zeroed (:130-132)

    def deliver(self, payload, model_kind=0, seq=0, ok=True):
        t = self.posted.pop(0)
        IoPattern.write_task_buffer(t, payload)
        st = self.p.CompleteIo(t, len(payload))
        self.model.complete(model_kind, seq, len(payload), ok)
        n = self.p.InitiateIo()
        if n.io_action == Recv:
            self.posted.append(n)
        return st

    def tick(self):
        """One renderer tick: the clock at the renderer's due time, so TimerCallback renders exactly one frame."""
        _, due = self.p.media_stream_timers()
        assert due >= 0
        self.clock.t = max(self.clock.t, due)
        before = len(self.tasks)
        self.p.media_stream_fire(A.MS_TIMER_RENDER)
        code = self.model.render()
        got = self.tasks[before:]
        if code == 0:
            assert not got
        else:
            assert [t.io_action for t in got] == [A.TASK_ABORT if code == 1 else A.TASK_FATAL_ABORT]
        return code

    def check_stats(self):
        got = self.p.media_stream_stats()
        exp = self.model.stats()
        for k in ("bits_received", "successful_frames", "dropped_frames", "duplicate_frames", "error_frames",
                  "datagrams", "finished", "head_sequence_number"):
            assert got[k] == exp[k], (k, got, exp)
        return got


def test_client_timers_armed_at_first_initiate(clock):
    r = ClientRun(clock, frame=3000, buffered=2, frames=8, fps=100)
    start, render = r.p.media_stream_timers()
    assert start == r.base + 10 + 500  # msPerFrame + 500 (:351-364)
    assert render == r.base + 2 * 10   # base + BufferedFrames * msPerFrame (:321-349, initial)
    # START is re-sent until a datagram arrives (:440-468)
    clock.t = start
    r.p.media_stream_fire(A.MS_TIMER_START)
    t = r.tasks[-1]
    assert (t.io_action, t.track_io, t.buffer_type, t.buffer_length) == (Send, 0, A.BUFFER_STATIC, 5)
    assert IoPattern.read_task_buffer(t, 5) == b"START"
    assert r.p.CompleteIo(t, 5) == A.IO_CONTINUE
    assert r.p.media_stream_timers()[0] == clock.t + 510
    r.p.close()


MODES = [pytest.param((A.VERIFY_SYNC, 0), id="sync"), pytest.param((A.VERIFY_DEFERRED, 0), id="deferred"),
         pytest.param((A.VERIFY_DEFERRED, 5), id="deferred-batch5")]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("complete_in_callback", [False, True])
def test_client_clean_stream_in_lockstep_with_model(clock, complete_in_callback, mode):
    M.udp_status_details_reset()
    frame, frames = 3000, 8
    r = ClientRun(clock, frame=frame, buffered=2, frames=frames, complete_in_callback=complete_in_callback,
                  mode=mode[0], batch=mode[1])
    cid = b"0123456789abcdef0123456789abcdef0123"
    assert r.deliver(b"\x00\x10" + cid + b"\x00", model_kind=1) == A.IO_CONTINUE
    assert r.p.connection_id() == cid.decode()
    # START is not re-sent once data arrived
    for f in range(1, frames + 1):
        for ln in OM.split(frame, 1400):
            assert r.deliver(_datagram(f, ln, qpc=f, qpf=1000), seq=f) == A.IO_CONTINUE
        if f >= 2:
            assert r.tick() == 0
    while (code := r.tick()) == 0:
        pass
    assert code == 1
    abort = r.tasks[-1]
    if complete_in_callback:
        assert r.in_callback == [A.IO_COMPLETED]
    else:
        assert r.p.CompleteIo(abort, 0, 0) == A.IO_COMPLETED
    s = r.check_stats()
    assert s["successful_frames"] == frames and s["dropped_frames"] == 0 and s["finished"] == 1
    assert s["bits_received"] == 8 * frame * frames and s["last_error"] == 0
    assert r.p.GetLastPatternError() == 0
    assert r.p.stats()["buffers_verified"] == frames * len(OM.split(frame, 1400))
    u = M.udp_status_details()
    assert u["successful_frames"] == frames and u["bits_received"] == 8 * frame * frames
    r.p.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", range(4))
def test_client_random_stream_matches_model(clock, seed, mode):
    rng = np.random.default_rng(seed)
    frame = int(rng.choice([1400, 3000, 5000]))
    frames = int(rng.integers(6, 20))
    buffered = int(rng.integers(1, 5))
    r = ClientRun(clock, frame=frame, buffered=buffered, frames=frames, recvs=int(rng.integers(1, 4)), mode=mode[0],
                  batch=mode[1])
    st = A.IO_CONTINUE
    for f in range(1, frames + 1):
        lens = OM.split(frame, 1400)
        for ln in lens:
            if rng.random() < 0.1:
                continue  # dropped
            seq = f if rng.random() > 0.05 else int(rng.integers(-3, frames + 8))  # stale / future / past-final
            st = r.deliver(_datagram(seq, ln), seq=seq)
            assert st == A.IO_CONTINUE
            if rng.random() < 0.05:
                st = r.deliver(_datagram(seq, ln), seq=seq)  # duplicate
        if r.tick() != 0:
            break
    while r.model.finished == 0:
        r.tick()
    assert r.p.CompleteIo(r.tasks[-1], 0, 0) == A.IO_COMPLETED
    r.check_stats()
    r.p.close()


def test_client_corrupt_payload_fails_the_stream(clock):
    r = ClientRun(clock, frame=3000, buffered=2, frames=5)
    assert r.deliver(_datagram(1, 1400), seq=1) == A.IO_CONTINUE
    assert r.deliver(_datagram(1, 1400, corrupt_at=700), seq=1, ok=False) == A.IO_FAILED
    _check_corrupt_failure(r)
    r.p.close()


def _check_corrupt_failure(r):
    assert r.p.GetLastPatternError() == A.STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN
    s = r.p.media_stream_stats()
    assert s["has_failure"] == 1 and s["fail_datagram"] == 1 and s["bits_received"] == 8 * 1400
    ps = r.p.stats()
    assert (ps["buffers_failed"], ps["fail_offset"], ps["fail_length"]) == (1, 700, 1374)


@pytest.mark.parametrize("batch", [0, 4])
def test_client_deferred_corrupt_payload(clock, batch):
    """DEFERRED: the corrupt datagram fails the stream when its batch is verified (a full batch, a render tick or
    any completion that is not a queued data datagram), with the same failure record and counters as SYNC; the
    datagrams queued after it are not applied."""
    r = ClientRun(clock, frame=3000, buffered=2, frames=5, mode=A.VERIFY_DEFERRED, batch=batch)
    assert r.deliver(_datagram(1, 1400), seq=1) == A.IO_CONTINUE
    assert r.deliver(_datagram(1, 1400, corrupt_at=700), seq=1, ok=False) == A.IO_CONTINUE  # queued
    st = r.deliver(_datagram(2, 1400), seq=2)  # the model stops at the corrupt one
    if batch == 4:
        assert st == A.IO_CONTINUE
        st = r.p.CompleteIo(r.posted.pop(0), 0)  # a zero-byte datagram: not queued, flushes first
    else:
        assert st == A.IO_CONTINUE
        assert r.p.Flush() == A.IO_FAILED
        st = A.IO_FAILED
    assert st == A.IO_FAILED
    _check_corrupt_failure(r)
    r.p.close()


def _failing_verifier(arena, descs):
    raise RuntimeError("the batched verify fails (a device error stand-in)")


@pytest.mark.parametrize("first_timer", ["start", "render"])
def test_client_deferred_device_failure_on_the_first_tick(clock, first_timer):
    """DEFERRED: the batched verify of the datagrams queued before the first timer fails (the hook returns an error,
    as a failed kernel launch would). Whichever timer flushes first, START (before the renderer ever ran) or the
    renderer, hands exactly one FatalAbort task to the callback (ctsIOPatternMediaStream.cpp:490-508), and the
    pattern reports the latched failure; the other timer sends nothing more."""
    cfg = PatternConfig.media_stream(listening=False, frame_size=3000, frames_per_second=100, stream_length_frames=5,
                                     buffered_frames=2, datagram_max_size=1400, pre_post_recvs=2,
                                     ms_manual_timers=True, verify_mode=A.VERIFY_DEFERRED, batch_buffers=4)
    shared_buffer_attach(_SENDER)
    p = IoPattern.MakeIoPattern(cfg, None, verifier=_failing_verifier)
    tasks = []
    p.RegisterCallback(tasks.append)
    posted = [p.InitiateIo() for _ in range(2)]
    t = posted.pop(0)
    IoPattern.write_task_buffer(t, _datagram(1, 1400))
    assert p.CompleteIo(t, 1400) == A.IO_CONTINUE  # queued for the batch
    start, render = p.media_stream_timers()
    first, second = (A.MS_TIMER_START, A.MS_TIMER_RENDER) if first_timer == "start" else (A.MS_TIMER_RENDER,
                                                                                          A.MS_TIMER_START)
    clock.t = max(start, render)
    p.media_stream_fire(first)
    assert [x.io_action for x in tasks] == [A.TASK_FATAL_ABORT]
    assert p.GetLastPatternError() != 0
    p.media_stream_fire(second)
    assert [x.io_action for x in tasks] == [A.TASK_FATAL_ABORT]
    p.close()


@pytest.mark.parametrize("payload,why", [
    (b"", "zero-byte datagram before the stream finished"),
    (b"\x00", "shorter than the flag"),
    (b"\x00\x00" + b"\x01" * 10, "data datagram shorter than its header"),
    (b"\x00\x10" + b"x" * 10, "id datagram shorter than its header"),
    (b"\x34\x12" + b"\x00" * 40, "unknown flag"),
])
def test_client_rejects_invalid_datagrams(clock, payload, why):
    r = ClientRun(clock, frame=3000, buffered=2, frames=5)
    assert r.deliver(payload) == A.IO_FAILED, why
    assert r.p.GetLastPatternError() == A.STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED  # TooFewBytes
    assert r.p.media_stream_stats()["fail_datagram"] == 0
    r.p.close()


def test_client_zero_byte_after_finish_is_fine(clock):
    r = ClientRun(clock, frame=1400, buffered=1, frames=2)
    for f in (1, 2):
        r.deliver(_datagram(f, 1400), seq=f)
    while r.tick() == 0:
        pass
    assert r.deliver(b"", model_kind=2) == A.IO_CONTINUE  # :158-167: finished, zero bytes are NoError
    assert r.p.CompleteIo(r.tasks[-1], 0, 0) == A.IO_COMPLETED
    r.p.close()


def test_client_nothing_received_is_fatal_abort(clock):
    r = ClientRun(clock, frame=1000, buffered=3, frames=10)
    # the first renderer tick (base + 3 frames) finds the buffer empty: FatalAbort (:486-500)
    assert r.tick() == 2
    assert r.tasks[-1].io_action == A.TASK_FATAL_ABORT
    assert r.p.media_stream_timers()[1] == -1  # no renderer tick after that
    assert r.p.CompleteIo(r.tasks[-1], 0, 0) == A.IO_FAILED
    assert r.p.GetLastPatternError() == A.STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED
    assert r.check_stats()["dropped_frames"] == 10
    r.p.close()


def test_client_abort_before_finish_is_a_fail_fast(clock):
    r = ClientRun(clock, frame=1000, buffered=3, frames=10)
    t = A.CtsTask()
    t.io_action = A.TASK_ABORT
    assert r.p.CompleteIo(t, 0, 0) == A.IO_FAILED
    assert "Abort before the stream was finished" in r.p.fail_fast_reason()
    r.p.close()


def test_client_renderer_catches_up_when_late(clock):
    """TimerCallback renders until its next tick lies more than 2 ms ahead (:470-530)."""
    r = ClientRun(clock, frame=1400, buffered=3, frames=6, fps=100)
    for f in range(1, 7):
        r.deliver(_datagram(f, 1400), seq=f)
    assert r.p.media_stream_timers()[1] == r.base + 30  # the first tick: 3 buffered frames of 10 ms
    clock.t = r.base + 45  # late: the ticks at +30 and +40 are both due, +50 is more than 2 ms ahead
    r.p.media_stream_fire(A.MS_TIMER_RENDER)
    assert r.model.render() == 0 and r.model.render() == 0
    assert r.check_stats()["successful_frames"] == 2
    assert r.p.media_stream_timers()[1] == r.base + 50
    r.p.close()


def test_client_auto_timers_real_clock():
    """Without manual timers a thread fires the START and renderer timers at the reference's times."""
    clock_set(None)
    shared_buffer_attach(_SENDER)
    frames = 5
    cfg = PatternConfig.media_stream(listening=False, frame_size=1400, frames_per_second=100,
                                     stream_length_frames=frames, buffered_frames=frames, pre_post_recvs=1)
    p = IoPattern.MakeIoPattern(cfg, None, verifier=_oracle_verifier)
    done = threading.Event()
    got = []

    def cb(task):
        if task.io_action in (A.TASK_ABORT, A.TASK_FATAL_ABORT):
            got.append(p.CompleteIo(task, 0, 0))
            done.set()

    p.RegisterCallback(cb)
    t = p.InitiateIo()
    for f in range(1, frames + 1):
        IoPattern.write_task_buffer(t, _datagram(f, 1400))
        assert p.CompleteIo(t, 1400) == A.IO_CONTINUE
        t = p.InitiateIo()
    assert done.wait(5.0), "the renderer never finished the stream"
    assert got == [A.IO_COMPLETED]
    assert p.media_stream_stats()["successful_frames"] == frames
    p.close()


def test_media_stream_config_is_checked(clock):
    from ctstraffic_amd._lib import CtsError

    ok = dict(listening=False, frame_size=3000, frames_per_second=100, stream_length_frames=5, buffered_frames=2)
    bad = [
        PatternConfig(**{**PatternConfig.media_stream(**ok).__dict__, "transfer_size": 3000 * 5 + 1}),
        PatternConfig(**{**PatternConfig.media_stream(**ok).__dict__, "verify_mode": 7}),
        PatternConfig(**{**PatternConfig.media_stream(**ok).__dict__, "ms_buffered_frames": 0}),
        PatternConfig.media_stream(**{**ok, "frame_size": 39, "stream_length_frames": 5}),
        PatternConfig(**{**PatternConfig.media_stream(**ok).__dict__, "registered_io": True}),
    ]
    for cfg in bad:
        with pytest.raises(CtsError):
            _make(cfg)
    p = _make(PatternConfig.media_stream(**ok))
    p.close()


def test_tcp_patterns_refuse_the_media_stream_calls():
    from ctstraffic_amd._lib import CtsError

    shared_buffer_attach(_SENDER)
    p = IoPattern.MakeIoPattern(PatternConfig(), None, verifier=_oracle_verifier)
    with pytest.raises(CtsError):
        p.media_stream_fire(A.MS_TIMER_RENDER)
    with pytest.raises(CtsError):
        p.media_stream_stats()
    p.close()


# ---- GPU: the payload verify on the gfx950 kernel ----------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_client_stream_with_corruption(engine, clock, mode):
    """The client pattern on a device engine: every data datagram's payload is verified on the GPU (the SYNC
    mailbox over the pattern's pinned recv buffers); a clean stream renders every frame, and a corrupted
    payload fails the stream at that datagram with the first mismatch the kernel found."""
    frame, frames = 5000, 6
    r = ClientRun(clock, frame=frame, buffered=2, frames=frames, engine=engine, mode=mode[0], batch=mode[1])
    for f in range(1, frames + 1):
        for ln in OM.split(frame, 1400):
            assert r.deliver(_datagram(f, ln), seq=f) == A.IO_CONTINUE
        if f >= 2:
            assert r.tick() == 0
    while r.tick() == 0:
        pass
    assert r.p.CompleteIo(r.tasks[-1], 0, 0) == A.IO_COMPLETED
    s = r.check_stats()
    assert s["successful_frames"] == frames
    assert r.p.stats()["buffers_verified"] == frames * len(OM.split(frame, 1400))
    r.p.close()

    r = ClientRun(clock, frame=frame, buffered=2, frames=frames, engine=engine, mode=mode[0], batch=mode[1])
    assert r.deliver(_datagram(1, 1400), seq=1) == A.IO_CONTINUE
    st = r.deliver(_datagram(1, 1400, corrupt_at=1001), seq=1, ok=False)
    if mode[0] == A.VERIFY_DEFERRED:
        assert st == A.IO_CONTINUE and r.p.Flush() == A.IO_FAILED  # the batch's verdict
    else:
        assert st == A.IO_FAILED
    ps = r.p.stats()
    assert (ps["buffers_failed"], ps["fail_offset"], ps["fail_length"]) == (1, 1001, 1374)
    assert ps["fail_expected"] == int(_SENDER[1001]) and ps["fail_actual"] == int(_SENDER[1001]) ^ 0x5A
    assert r.p.GetLastPatternError() == A.STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN
    r.p.close()


@pytest.mark.gpu
def test_gpu_server_sends_frames(engine, clock):
    p = _make(PatternConfig.media_stream(listening=True, frame_size=52083, frames_per_second=60,
                                         stream_length_frames=4), engine)
    p.CompleteIo(p.InitiateIo(), 39)
    S = IoPattern.AccessSharedBuffer()
    for f in range(4):
        t = p.InitiateIo()
        assert t.buffer == S and t.buffer_length == 52083
        # the sender buffer the fill kernel wrote holds the pattern the frame's datagrams carry
        assert IoPattern.read_task_buffer(t, 64, offset=-t.buffer_offset) == _SENDER[:64].tobytes()
        p.CompleteIo(t, 52083)
    assert p.GetLastPatternError() == 0
    p.close()


@pytest.mark.parametrize("backend", ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
@pytest.mark.parametrize("frame,max_dgram,slot", [(52083, 1400, 1408), (1000, 1400, 1008), (3000, 1472, 1472),
                                                  (64, 30, 32)])
def test_client_recv_slots_sized_to_one_datagram(request, clock, backend, mode, frame, max_dgram, slot):
    """A client recv is one datagram of min(frame, DatagramMaxSize) bytes (ctsIOPatternMediaStream.cpp:115-138), so
    its recv slots (and every slot of the DEFERRED recv ring) are that many bytes rounded up to 16, not a frame's:
    at the README frame size (52083 B) a frame-sized slot left 97 % of the pinned ring unused. The posted recvs sit
    `slot` bytes apart, the ring hands its slots out in order and wraps after 2 x batch + PrePostRecvs + 1 slots on a
    device (batch + PrePostRecvs + 1 with a CPU hook), and the stream still verifies."""
    engine = request.getfixturevalue("engine") if backend == "gpu" else None
    recvs, batch = 3, 4
    cfg = PatternConfig.media_stream(listening=False, frame_size=frame, frames_per_second=100, stream_length_frames=50,
                                     buffered_frames=50, datagram_max_size=max_dgram, pre_post_recvs=recvs,
                                     ms_manual_timers=True, verify_mode=mode, batch_buffers=batch)
    p = _make(cfg, engine)
    posted = [p.InitiateIo() for _ in range(recvs)]
    post_len = min(frame, max_dgram)
    assert all(t.buffer_length == post_len for t in posted)
    base = posted[0].buffer
    # the free list hands out its back first (ctsIOPattern.cpp:708-715)
    assert sorted(t.buffer - base for t in posted) == [-slot * k for k in range(recvs)][::-1]
    base = min(t.buffer for t in posted)
    ring = mode == A.VERIFY_DEFERRED
    slots = (batch * (2 if engine is not None else 1) + recvs + 1) if ring else recvs
    n = 3 * slots
    length = post_len
    seen = []
    for i in range(n):
        t = posted.pop(0)
        IoPattern.write_task_buffer(t, _datagram(1 + i // 40, length))
        assert p.CompleteIo(t, length) == A.IO_CONTINUE
        nxt = p.InitiateIo()
        assert nxt.io_action == Recv
        off = nxt.buffer - base
        assert off % slot == 0 and 0 <= off < slots * slot
        seen.append(off // slot)
        posted.append(nxt)
    if ring:  # recycled in ring order: slot recvs, recvs + 1, ... wrapping at `slots`
        assert seen == [(recvs + i) % slots for i in range(n)]
    assert p.Flush() == A.IO_CONTINUE
    s = p.media_stream_stats()
    assert s["datagrams"] == n and s["has_failure"] == 0
    p.close()


@pytest.mark.parametrize("mode", [A.VERIFY_SYNC, A.VERIFY_DEFERRED], ids=["sync", "deferred"])
def test_server_keeps_no_recv_ring(clock, mode):
    """The server receives nothing to verify: its one recv buffer only ever holds the 39-byte connection-id datagram
    (ctsIOPattern.cpp:1119-1128), whatever the frame size and verify mode, and it builds that datagram correctly."""
    p = _make(PatternConfig.media_stream(listening=True, frame_size=60000, frames_per_second=10,
                                         stream_length_frames=2, verify_mode=mode))
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_type, t.buffer_length) == (Send, A.BUFFER_UDP_CONNECTION_ID, 39)
    assert IoPattern.read_task_buffer(t, 39) == b"\x00\x10" + p.connection_id().encode() + b"\x00"
    assert p.CompleteIo(t, 39) == A.IO_CONTINUE
    p.close()
