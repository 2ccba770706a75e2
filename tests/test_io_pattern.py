"""The ctsIoPattern mirror (include/cts_pattern.h) replaying the reference's own
MSTest scenarios (MSTest/ctsIOPatternUnitTest_{Server,Client,Duplex}), plus
randomized long streams with injected corruption.

Each scenario runs against four backends:
  cpu-sync / cpu-deferred : VerifyBuffer answered by the CPU oracle through the
                            pattern's batch-verifier hook (the reference's tests
                            replace ctsConfig by link-time fakes the same way);
  gpu-sync / gpu-deferred : VerifyBuffer on the gfx950 verify kernel (zero-copy
                            over the pattern's pinned recv buffers), sender
                            buffer written by the gfx950 fill kernel.
Assertions follow the reference tests line by line (file:line cited per test); all 101 TEST_METHODs of
the three MSTest projects are replayed (identical flows folded into parametrized cases).
"""
import ctypes

import numpy as np
import pytest

import oracle
from ctstraffic_amd import _pattern_abi as A
from ctstraffic_amd._lib import ATTR_SYNC_MAILBOX
from ctstraffic_amd.pattern import IoPattern, PatternConfig, shared_buffer_attach

ContinueIo, CompletedIo, FailedIo = A.IO_CONTINUE, A.IO_COMPLETED, A.IO_FAILED
Send, Recv, NoneAction = A.TASK_SEND, A.TASK_RECV, A.TASK_NONE
ConnectionIdLength = A.CONNECTION_ID_LENGTH
g_TestBufferLength = 4  # completion message "DONE"
g_TestRecvBufferLength = 1024
WSAECONNRESET = 10054

BACKENDS = [
    pytest.param(("cpu", A.VERIFY_SYNC, False), id="cpu-sync"),
    pytest.param(("cpu", A.VERIFY_DEFERRED, False), id="cpu-deferred"),
    pytest.param(("gpu", A.VERIFY_SYNC, False), id="gpu-sync", marks=pytest.mark.gpu),  # the mailbox grid
    pytest.param(("gpu-launch", A.VERIFY_SYNC, False), id="gpu-sync-launch", marks=pytest.mark.gpu),
    pytest.param(("gpu", A.VERIFY_DEFERRED, False), id="gpu-deferred", marks=pytest.mark.gpu),
    # -io:rioiocp: buffers registered with the RIO fakes (tests/cpp/rio_fake.c), ids checked per task
    pytest.param(("cpu", A.VERIFY_SYNC, True), id="cpu-sync-rio"),
    pytest.param(("cpu", A.VERIFY_DEFERRED, True), id="cpu-deferred-rio"),
    pytest.param(("gpu", A.VERIFY_SYNC, True), id="gpu-sync-rio", marks=pytest.mark.gpu),
    pytest.param(("gpu", A.VERIFY_DEFERRED, True), id="gpu-deferred-rio", marks=pytest.mark.gpu),
]

_SENDER = oracle.sender_buffer(4 * 65536)  # g_senderSharedBuffer stand-in for device-less harnesses


def _oracle_verifier(arena, descs):
    return oracle.verify_batch(arena, descs)[0]


class RioCheckedPattern(IoPattern):
    """A pattern under -io:rioiocp, checked the way ctsRioIocp.cpp relies on it: every send/recv task carries a
    live RIO_BUFFERID whose registered memory holds the task's buffer (ctsRioIocp.cpp:446-448 FAIL_FASTs on
    RIO_INVALID_BUFFERID; :733-736 builds the RIO_BUF from id + m_bufferOffset + m_bufferLength), and an id is
    never in two tasks in flight at once (RIO cannot reuse one in concurrent sends, ctsIOPattern.cpp:683-692)."""

    rio = None  # the RioFake

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.in_flight = {}

    def InitiateIo(self):
        t = super().InitiateIo()
        if t.io_action in (Send, Recv):
            assert t.rio_buffer_id != A.RIO_INVALID_BUFFERID
            reg = self.rio.lookup(t.rio_buffer_id)
            assert reg is not None, "task carries an id that is not registered"
            base, n = reg
            lo = t.buffer + t.buffer_offset
            assert base == t.buffer and t.buffer_offset + t.buffer_length <= n, (hex(base), n, hex(lo))
            if t.buffer_type == A.BUFFER_DYNAMIC:
                assert t.rio_buffer_id not in self.in_flight, "one RIO_BUFFERID in two IOs at once"
                self.in_flight[t.rio_buffer_id] = lo
        else:
            assert t.rio_buffer_id == A.RIO_INVALID_BUFFERID
        return t

    def CompleteIo(self, task, current_transfer, status_code=0):
        if task.buffer_type == A.BUFFER_DYNAMIC and task.io_action in (Send, Recv):
            self.in_flight.pop(task.rio_buffer_id, None)
        return super().CompleteIo(task, current_transfer, status_code)


RIO_BACKENDS = [b for b in BACKENDS if b.values[0][2]]  # the registered-IO backends (tests of RIO ids only)


@pytest.fixture(params=BACKENDS)
def make(request):
    kind, mode, rio = request.param
    made = []
    fake = request.getfixturevalue("rio_fake") if rio else None
    if fake is not None:
        fake.reset()
    cls = IoPattern
    if rio:
        cls = type("RioChecked", (RioCheckedPattern,), {"rio": fake})

    def factory(**kw):
        kw.setdefault("verify_mode", mode)
        kw.setdefault("registered_io", rio)
        cfg = PatternConfig(**kw)
        if kind == "cpu":
            shared_buffer_attach(_SENDER)
            p = cls.MakeIoPattern(cfg, None, verifier=_oracle_verifier)
        else:
            eng = request.getfixturevalue("engine")
            # gpu-launch: SYNC verifies as one sliced launch + synchronize per completion instead of the mailbox
            eng.set_attr(ATTR_SYNC_MAILBOX, 0 if kind == "gpu-launch" else 1)
            p = cls.MakeIoPattern(cfg, eng)
        if rio:
            # ids on the free lists + connection id + completion message (ctsIOPattern.h:114-123)
            sends = (1 << 24) // cfg.buffer_size + 1  # g_maxNumberOfRioSendBuffers (ctsIOPattern.cpp:61)
            recvs = {A.PATTERN_PUSH: cfg.pre_post_recvs if cfg.listening else 0,
                     A.PATTERN_PULL: 0 if cfg.listening else cfg.pre_post_recvs,
                     A.PATTERN_PUSHPULL: 1, A.PATTERN_DUPLEX: cfg.pre_post_recvs}[cfg.io_pattern]
            assert p.GetRioBufferIdCount() == recvs + sends + 2
        made.append(p)
        return p

    factory.kind, factory.mode, factory.rio = kind, mode, rio
    yield factory
    for p in made:
        p.close()
    if kind == "gpu-launch":
        request.getfixturevalue("engine").set_attr(ATTR_SYNC_MAILBOX, 1)
    if fake is not None:
        assert fake.live() == 0, "ids left registered after the patterns were destroyed"
        assert fake.errors() == 0, "deregistration of an id that was not live"


def recv_correct(task, n=None):
    IoPattern.recv_from_wire(task, task.buffer_length if n is None else n)


def zero(task):
    ctypes.memset(task.buffer + task.buffer_offset, 0, task.buffer_length)


def server_defaults(**kw):  # ctsIOPatternUnitTest_Server.cpp:250-274 SetTestBaseClassDefaults(Server)
    d = dict(io_pattern=A.PATTERN_PUSH, listening=True, verify_buffers=True, pre_post_recvs=1, pre_post_sends=1,
             buffer_size=1024, transfer_size=10)
    d.update(kw)
    return d


def client_defaults(**kw):
    d = server_defaults(listening=False)
    d.update(kw)
    return d


# ---- ctsIOPatternUnitTest_Server.cpp ---------------------------------------------------------------
def test_TestBaseClass_SingleSuccessfulRecv_Server(make):  # :280-312
    p = make(**server_defaults())
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Send)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (10, Recv)
    recv_correct(t)
    assert p.CompleteIo(t, 10, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Send, g_TestBufferLength)
    assert IoPattern.read_task_buffer(t, 4) == b"DONE"
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, 0, 0) == CompletedIo
    assert p.GetLastPatternError() == 0
    s = p.stats()
    assert s["buffers_verified"] == 1 and s["buffers_failed"] == 0 and s["bytes_recv"] == 10


def test_TestBaseClass_FailSendingConnectionId(make):  # :314-324
    p = make(**server_defaults())
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Send)
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


def test_TestBaseClass_FailRecv(make):  # :326-342
    p = make(**server_defaults())
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (10, Recv)
    assert p.CompleteIo(t, 10, 1) == FailedIo
    assert p.GetLastPatternError() == 1


def _server_to_fin(p):
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    recv_correct(t)
    assert p.CompleteIo(t, 10, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Send and IoPattern.read_task_buffer(t, 4) == b"DONE"
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    return t


def test_TestServerBaseClass_FailFINAfterRecv(make):  # :344-377
    p = make(**server_defaults())
    t = _server_to_fin(p)
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


@pytest.mark.parametrize("case", ["AfterSend", "AfterRecv"])
def test_TestServerBaseClass_TooManyBytesOnFIN(make, case):  # :379-412 (AfterSend), :414-447 (AfterRecv)
    p = make(**server_defaults())
    t = _server_to_fin(p)
    assert p.CompleteIo(t, 1, 0) == FailedIo
    assert p.GetLastPatternError() == A.STATUS_ERROR_TOO_MUCH_DATA_TRANSFERRED


def test_TestBaseClass_InvalidBytesOnRecv(make):  # :449-467
    p = make(**server_defaults())
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (10, Recv)
    zero(t)  # ::ZeroMemory(test_task.m_buffer, test_task.m_bufferLength)
    assert p.CompleteIo(t, 10, 0) == FailedIo
    assert p.GetLastPatternError() == A.STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN
    s = p.stats()
    # P = 00 00 01 00 02 00 ...: the zeroed buffer first differs at byte 2 (expected 0x01, got 0x00)
    assert (s["has_failure"], s["fail_offset"], s["fail_expected"], s["fail_actual"]) == (1, 2, 1, 0)
    assert s["bytes_recv"] == 10  # a corrupt buffer is still counted (ctsIOPattern.cpp:505-521)
    assert "offset (2)" in p.failure_message() and "'0x1' didn't match '0x0'" in p.failure_message()


def _push_server_loop(p, n, post, complete):
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Send)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    offsets = []
    for _ in range(n):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action) == (post, Recv)
        assert p.InitiateIo().io_action == NoneAction
        offsets.append(t.expected_pattern_offset)
        recv_correct(t)
        assert p.CompleteIo(t, complete, 0) == ContinueIo
    return offsets


def _server_finish(p):
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Send, g_TestBufferLength)
    assert p.InitiateIo().io_action == NoneAction
    assert IoPattern.read_task_buffer(t, 4) == b"DONE"
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.InitiateIo().io_action == NoneAction
    assert p.CompleteIo(t, 0, 0) == CompletedIo


def test_PushServer_VerifyingBuffersNotUsingSharedBuffer(make):  # :609-667
    p = make(**server_defaults(buffer_size=1024, transfer_size=1024 * 10))
    offs = _push_server_loop(p, 10, 1024, 1024)
    assert offs == [1024 * i for i in range(10)]  # m_recvPatternOffset advances by completed bytes
    _server_finish(p)
    s = p.stats()
    assert s["buffers_verified"] == 10 and s["bytes_verified"] == 10240 and s["recv_pattern_offset"] == 10240


def test_PushServer_VerifyingBuffersNotUsingSharedBuffer_SmallRecvs(make):  # :669-740
    p = make(**server_defaults(buffer_size=2048, transfer_size=1024 * 10))
    offs = _push_server_loop(p, 9, 2048, 1024)
    assert offs == [1024 * i for i in range(9)]
    t = p.InitiateIo()  # the final recv is just 1024 bytes
    assert (t.buffer_length, t.io_action, t.expected_pattern_offset) == (1024, Recv, 9 * 1024)
    assert p.InitiateIo().io_action == NoneAction
    recv_correct(t)
    assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _server_finish(p)
    assert p.GetLastPatternError() == 0


def test_PushServer_NotVerifyingBuffersUsingSharedBuffer(make):  # :742-808
    p = make(**server_defaults(buffer_size=1024, transfer_size=1024 * 10, verify_buffers=False,
                               use_shared_buffer=True))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for _ in range(10):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action) == (1024, Recv)
        zero(t)  # not verifying: garbage is fine
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _server_finish(p)
    assert p.stats()["buffers_verified"] == 0


@pytest.mark.parametrize("post,complete", [(1024, 1024), (2048, 1024)], ids=["", "SmallRecvs"])
def test_PushServer_NotVerifyingBuffersNotUsingSharedBuffer(make, post, complete):  # :476-607
    p = make(**server_defaults(buffer_size=post, transfer_size=1024 * 10, verify_buffers=False))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for i in range(10):
        t = p.InitiateIo()
        # the last small recv is capped to the 1024 bytes left
        assert (t.buffer_length, t.io_action) == (post if (post == complete or i < 9) else 1024, Recv)
        zero(t)  # not verifying: any bytes are accepted
        assert p.CompleteIo(t, complete, 0) == ContinueIo
    _server_finish(p)
    assert p.stats()["buffers_verified"] == 0 and p.stats()["bytes_recv"] == 10240


@pytest.mark.parametrize("shared", [False, True], ids=["NotUsingSharedBuffer", "UsingSharedBuffer"])
def test_PullServer_NotVerifyingBuffers(make, shared):  # :810-866, :926-990
    p = make(**server_defaults(io_pattern=A.PATTERN_PULL, buffer_size=1024, transfer_size=1024 * 10,
                               verify_buffers=False, use_shared_buffer=shared))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for i in range(10):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action, t.buffer_offset) == (1024, Send, 1024 * i)
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _server_finish(p)
    assert p.stats()["bytes_sent"] == 10240


def test_PullServer_VerifyingBuffersNotUsingSharedBuffer(make):  # :868-924
    p = make(**server_defaults(io_pattern=A.PATTERN_PULL, buffer_size=1024, transfer_size=1024 * 10))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    base = IoPattern.AccessSharedBuffer()
    for i in range(10):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action) == (1024, Send)
        # Send tasks point into g_senderSharedBuffer at m_sendPatternOffset (ctsIOPattern.cpp:676-681)
        assert t.buffer == base and t.buffer_offset == 1024 * i
        assert p.InitiateIo().io_action == NoneAction
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _server_finish(p)
    assert p.stats()["send_pattern_offset"] == 10240 and p.stats()["bytes_sent"] == 10240


# ---- ctsIOPatternUnitTest_Client.cpp ------------------------------------------------------------
def test_TestBaseClass_SuccessfulSend(make):  # Client :280-313
    p = make(**client_defaults())
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (10, Send)
    assert p.CompleteIo(t, 10, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, g_TestBufferLength)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == A.TASK_GRACEFUL_SHUTDOWN
    assert p.CompleteIo(t, 0, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, 0, 0) == CompletedIo


@pytest.mark.parametrize("shutdown", [A.SHUTDOWN_GRACEFUL, A.SHUTDOWN_HARD], ids=["Graceful", "Rude"])
def test_PullClient_VerifyingBuffersNotUsingSharedBuffer_SmallRecvs(make, shutdown):  # Client :1662-1774
    p = make(**client_defaults(io_pattern=A.PATTERN_PULL, buffer_size=2048, transfer_size=10240,
                               tcp_shutdown=shutdown))
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for i in range(9):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action, t.expected_pattern_offset) == (2048, Recv, 1024 * i)
        recv_correct(t)
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (1024, Recv)
    recv_correct(t)
    assert p.CompleteIo(t, 1024, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, g_TestBufferLength)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    if shutdown == A.SHUTDOWN_GRACEFUL:
        assert t.io_action == A.TASK_GRACEFUL_SHUTDOWN
        assert p.CompleteIo(t, 0, 0) == ContinueIo
        t = p.InitiateIo()
        assert t.io_action == Recv
        assert p.CompleteIo(t, 0, 0) == CompletedIo
    else:
        assert t.io_action == A.TASK_HARD_SHUTDOWN
        assert p.CompleteIo(t, 0, 0) == CompletedIo
    assert p.stats()["buffers_verified"] == 10


def _client_to_status(p):
    """Connection id in, the 10-byte send out, then the server's 4-byte status recv (the common prefix of the
    client base-class tests, ctsIOPatternUnitTest_Client.cpp:360-760)."""
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (10, Send)
    assert p.CompleteIo(t, 10, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, g_TestBufferLength)
    return t


def test_TestBaseClass_SuccessfulMultipleSends(make):  # Client :315-358
    p = make(**client_defaults(pre_post_sends=2, buffer_size=10, transfer_size=20))
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t1 = p.InitiateIo()
    t2 = p.InitiateIo()  # two sends in flight (PrePostSends = 2)
    assert (t1.buffer_length, t1.io_action, t2.buffer_length, t2.io_action) == (10, Send, 10, Send)
    assert t2.buffer_offset == t1.buffer_offset + 10  # m_sendPatternOffset advances per created task (:695-697)
    assert p.CompleteIo(t1, 10, 0) == ContinueIo
    assert p.CompleteIo(t2, 10, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, g_TestBufferLength)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == A.TASK_GRACEFUL_SHUTDOWN
    assert p.CompleteIo(t, 0, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, 0, 0) == CompletedIo


def test_TestBaseClass_SuccessfulSend_HardShutdown(make):  # Client :360-387
    p = make(**client_defaults(tcp_shutdown=A.SHUTDOWN_HARD))
    t = _client_to_status(p)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == A.TASK_HARD_SHUTDOWN
    assert p.CompleteIo(t, 0, 0) == CompletedIo


@pytest.mark.parametrize("transferred,status", [(0, 0), (0, 1)], ids=["NoBytes", "Failed"])
def test_TestBaseClass_ServerStatusRecv(make, transferred, status):
    """ReceivedNoBytesWithServerStatus (Client :389-410) and FailedReceivingServerStatus (:412-433)."""
    p = make(**client_defaults())
    t = _client_to_status(p)
    assert p.CompleteIo(t, transferred, status) == FailedIo
    if status:
        assert p.GetLastPatternError() == status


def test_TestBaseClass_FailSend(make):  # Client :435-451
    p = make(**client_defaults())
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (10, Send)
    assert p.CompleteIo(t, 10, 1) == FailedIo
    assert p.GetLastPatternError() == 1


def test_TestBaseClass_FailMultipleSends(make):  # Client :453-480
    p = make(**client_defaults(pre_post_sends=2, buffer_size=10, transfer_size=20))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t1, t2 = p.InitiateIo(), p.InitiateIo()
    assert (t1.io_action, t2.io_action) == (Send, Send)
    assert p.CompleteIo(t1, 10, 1) == FailedIo
    assert p.GetLastPatternError() == 1
    assert p.CompleteIo(t2, 10, 1) == FailedIo
    assert p.GetLastPatternError() == 1


@pytest.mark.parametrize("shutdown", [A.SHUTDOWN_GRACEFUL, A.SHUTDOWN_HARD], ids=["Graceful", "Hard"])
def test_TestBaseClass_FailShutdown(make, shutdown):
    """FailGracefulShutdownAfterSend/-AFterRecv (Client :494-520, :554-580) and FailHardShutdownAfterSend/-AFterRecv
    (:524-550, :584-610): the shutdown task completes with an error."""
    p = make(**client_defaults(tcp_shutdown=shutdown))
    t = _client_to_status(p)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == (A.TASK_GRACEFUL_SHUTDOWN if shutdown == A.SHUTDOWN_GRACEFUL else A.TASK_HARD_SHUTDOWN)
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


@pytest.mark.parametrize("transferred,status,err", [(0, 1, 1), (1, 0, A.STATUS_ERROR_TOO_MUCH_DATA_TRANSFERRED)],
                         ids=["FailFIN", "TooManyBytesOnFIN"])
def test_TestClientBaseClass_FinalFin(make, transferred, status, err):
    """FailFINAfterSend / FailFINAfterRecv (Client :614-684) and TooManyBytesOnFINAfterSend / -AfterRecv (:686-760):
    the recv that waits for the server's FIN fails, or returns data."""
    p = make(**client_defaults())
    t = _client_to_status(p)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == A.TASK_GRACEFUL_SHUTDOWN
    assert p.CompleteIo(t, 0, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, transferred, status) == FailedIo
    assert p.GetLastPatternError() == err


def _client_finish(p, shutdown=A.SHUTDOWN_GRACEFUL):
    """Server status in, then the client's shutdown (graceful: FIN + wait for the server's FIN; rude: RST)."""
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, g_TestBufferLength)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    if shutdown == A.SHUTDOWN_GRACEFUL:
        assert t.io_action == A.TASK_GRACEFUL_SHUTDOWN
        assert p.CompleteIo(t, 0, 0) == ContinueIo
        t = p.InitiateIo()
        assert t.io_action == Recv
        assert p.CompleteIo(t, 0, 0) == CompletedIo
    else:
        assert t.io_action == A.TASK_HARD_SHUTDOWN
        assert p.CompleteIo(t, 0, 0) == CompletedIo


_CLIENT_VARIANTS = [pytest.param(False, False, id="NotVerifyingBuffersNotUsingSharedBuffer"),
                    pytest.param(True, False, id="VerifyingBuffersNotUsingSharedBuffer"),
                    pytest.param(False, True, id="NotVerifyingBuffersUsingSharedBuffer")]


@pytest.mark.parametrize("shutdown", [A.SHUTDOWN_GRACEFUL, A.SHUTDOWN_HARD], ids=["Graceful", "Rude"])
@pytest.mark.parametrize("verify,shared", _CLIENT_VARIANTS)
def test_PushClient(make, verify, shared, shutdown):
    """PushClient_{Not,}VerifyingBuffers{Not,}UsingSharedBuffer_{Graceful,Rude} (Client :765-1036): ten 1024-byte
    sends out of g_senderSharedBuffer at the advancing send offset, then status and shutdown."""
    p = make(**client_defaults(buffer_size=1024, transfer_size=10240, verify_buffers=verify, use_shared_buffer=shared,
                               tcp_shutdown=shutdown))
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    base = IoPattern.AccessSharedBuffer()
    for i in range(10):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action) == (1024, Send)
        assert t.buffer == base and t.buffer_offset == 1024 * i
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _client_finish(p, shutdown)
    assert p.stats()["bytes_sent"] == 10240


@pytest.mark.parametrize("shutdown", [A.SHUTDOWN_GRACEFUL, A.SHUTDOWN_HARD], ids=["Graceful", "Rude"])
@pytest.mark.parametrize("verify,shared", _CLIENT_VARIANTS)
def test_PullClient(make, verify, shared, shutdown):
    """PullClient_{Not,}VerifyingBuffers{Not,}UsingSharedBuffer_{Graceful,Rude} (Client :1359-1452, :1567-1660,
    :1775-1870): ten 1024-byte recvs; verified at expected offsets 0, 1024, ... when verifying, garbage accepted
    (and the offset left at 0) when not."""
    p = make(**client_defaults(io_pattern=A.PATTERN_PULL, buffer_size=1024, transfer_size=10240, verify_buffers=verify,
                               use_shared_buffer=shared, tcp_shutdown=shutdown))
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for i in range(10):
        t = p.InitiateIo()
        # m_recvPatternOffset advances only inside the verify gate (ctsIOPattern.cpp:475-493)
        assert (t.buffer_length, t.io_action, t.expected_pattern_offset) == (1024, Recv, 1024 * i if verify else 0)
        recv_correct(t) if verify else zero(t)
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _client_finish(p, shutdown)
    s = p.stats()
    # per-connection statistics count the pattern's own IO only; the status message goes to TcpStatusDetails
    # (ctsIOPattern.cpp:505-520)
    assert s["bytes_recv"] == 10240 and s["buffers_verified"] == (10 if verify else 0)


@pytest.mark.parametrize("shutdown", [A.SHUTDOWN_GRACEFUL, A.SHUTDOWN_HARD], ids=["Graceful", "Rude"])
def test_PullClient_NotVerifyingBuffersNotUsingSharedBuffer_SmallRecvs(make, shutdown):  # Client :1454-1565
    p = make(**client_defaults(io_pattern=A.PATTERN_PULL, buffer_size=2048, transfer_size=10240, verify_buffers=False,
                               tcp_shutdown=shutdown))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for _ in range(9):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action) == (2048, Recv)
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (1024, Recv)
    assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _client_finish(p, shutdown)


# ideal send backlog (SetIdealSendBacklog, PrePostSends = 0): Client :1038-1357
def _isb_client(make, isb):
    p = make(**client_defaults(buffer_size=1024, transfer_size=10240, verify_buffers=False, pre_post_sends=0))
    p.SetIdealSendBacklog(isb)
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    return p


@pytest.mark.parametrize("isb", [2048, 2047], ids=["MultipleSendsWithISBEnabled", "OffsetFromBufferSize"])
def test_PushClient_MultipleSendsWithISB(make, isb):  # Client :1038-1098, :1290-1357
    p = _isb_client(make, isb)
    for _ in range(5):  # two sends in flight, then nothing until one completes
        t1, t2 = p.InitiateIo(), p.InitiateIo()
        assert (t1.buffer_length, t1.io_action, t2.buffer_length, t2.io_action) == (1024, Send, 1024, Send)
        t3 = p.InitiateIo()
        assert (t3.buffer_length, t3.io_action) == (0, NoneAction)
        assert p.CompleteIo(t1, 1024, 0) == ContinueIo
        assert p.CompleteIo(t2, 1024, 0) == ContinueIo
    _client_finish(p)


def test_PushClient_MultipleSendsWithISBEnabledInterleaving(make):  # Client :1100-1161
    p = _isb_client(make, 2048)
    first = p.InitiateIo()
    assert (first.buffer_length, first.io_action) == (1024, Send)
    for _ in range(1, 10):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action) == (1024, Send)
        assert p.InitiateIo().io_action == NoneAction
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    assert p.CompleteIo(first, 1024, 0) == ContinueIo
    _client_finish(p)


def test_PushClient_LargeNumberOfSendsWithISBEnabled(make):  # Client :1163-1232
    p = _isb_client(make, 10240)
    pended = [p.InitiateIo() for _ in range(10)]
    assert all((t.buffer_length, t.io_action) == (1024, Send) for t in pended)
    assert p.InitiateIo().io_action == NoneAction
    for i, t in enumerate(pended):
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
        if i < 9:
            assert p.InitiateIo().io_action == NoneAction
    _client_finish(p)


def test_PushClient_OneSendInFlightWithISBEnabledWhenISBIsSmallerThanBufferSize(make):  # Client :1234-1288
    p = _isb_client(make, 512)
    for _ in range(10):
        t = p.InitiateIo()
        assert (t.buffer_length, t.io_action) == (1024, Send)
        t2 = p.InitiateIo()
        assert (t2.buffer_length, t2.io_action) == (0, NoneAction)
        assert p.CompleteIo(t, 1024, 0) == ContinueIo
    _client_finish(p)


def test_TestBaseClass_FailReceivingConnectionId(make):  # Client :482-492
    p = make(**client_defaults())
    t = p.InitiateIo()
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


# ---- ctsIOPatternUnitTest_Duplex.cpp --------------------------------------------------------------
def duplex_defaults(role_server=False, **kw):  # :208-229 SetTestDuplexDefaults
    d = dict(io_pattern=A.PATTERN_DUPLEX, listening=role_server, verify_buffers=True, pre_post_recvs=1,
             pre_post_sends=1, buffer_size=1024, transfer_size=20)
    d.update(kw)
    return d


def _complete_connection_id(p, server):
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Send if server else Recv)
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo


def _pended_data_tasks(p):
    r = p.InitiateIo()
    assert (r.io_action, r.buffer_length) == (Recv, 10)
    s = p.InitiateIo()
    assert (s.io_action, s.buffer_length) == (Send, 10)
    assert p.InitiateIo().io_action == NoneAction
    return r, s


def _complete_data_recv(p, t, n):
    IoPattern.recv_from_wire(t, n)
    return p.CompleteIo(t, n, 0)


def _successful_shutdown(p, server, hard=False):
    if server:
        t = p.InitiateIo()
        assert (t.io_action, t.buffer_length) == (Send, 4)
        assert p.CompleteIo(t, 4, 0) == ContinueIo
        t = p.InitiateIo()
        assert t.io_action == Recv
        assert p.CompleteIo(t, 0, 0) == CompletedIo
        return
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, 4)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    if hard:
        assert t.io_action == A.TASK_HARD_SHUTDOWN
        assert p.CompleteIo(t, 0, 0) == CompletedIo
        return
    assert t.io_action == A.TASK_GRACEFUL_SHUTDOWN
    assert p.CompleteIo(t, 0, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, 0, 0) == CompletedIo


@pytest.mark.parametrize("server,recv_first,hard", [(False, True, False), (False, False, False), (False, True, True),
                                                    (True, False, False), (True, True, False)],
                         ids=["Client_Graceful_RecvThenSend", "Client_Graceful_SendThenRecv", "Client_HardShutdown",
                              "Server_Graceful_SendThenRecv", "Server_Graceful_RecvThenSend"])
def test_Duplex_success_paths(make, server, recv_first, hard):  # :492-590
    p = make(**duplex_defaults(server, tcp_shutdown=A.SHUTDOWN_HARD if hard else A.SHUTDOWN_GRACEFUL))
    _complete_connection_id(p, server)
    r, s = _pended_data_tasks(p)
    if recv_first:
        assert _complete_data_recv(p, r, 10) == ContinueIo
        assert p.CompleteIo(s, 10, 0) == ContinueIo
    else:
        assert p.CompleteIo(s, 10, 0) == ContinueIo
        assert _complete_data_recv(p, r, 10) == ContinueIo
    _successful_shutdown(p, server, hard)
    assert p.GetLastPatternError() == 0


def test_Duplex_Client_PartialRecv_RepostsRemainder(make):  # :592-622
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r = p.InitiateIo()
    assert (r.io_action, r.buffer_length) == (Recv, 10)
    s = p.InitiateIo()
    assert (s.io_action, s.buffer_length) == (Send, 10)
    assert _complete_data_recv(p, r, 4) == ContinueIo
    rr = p.InitiateIo()
    assert (rr.io_action, rr.buffer_length) == (Recv, 6)
    assert rr.expected_pattern_offset == 4  # the unaligned phase the next buffer is verified at
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    assert _complete_data_recv(p, rr, 6) == ContinueIo
    _successful_shutdown(p, False)
    assert p.GetLastPatternError() == 0
    assert p.stats()["buffers_verified"] == 2


def test_Duplex_Server_TolerateRstWhileAwaitingFin(make):  # :626-655
    p = make(**duplex_defaults(True))
    _complete_connection_id(p, True)
    r, s = _pended_data_tasks(p)
    assert _complete_data_recv(p, r, 10) == ContinueIo
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Send
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, 0, WSAECONNRESET) == CompletedIo
    assert p.GetLastPatternError() == 0


def test_Duplex_Client_FailDataRecv(make):  # :700-715
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r, s = _pended_data_tasks(p)
    assert p.CompleteIo(r, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


def test_Duplex_Client_CorruptedRecv(make):
    """Not an MSTest case: a corrupted Duplex recv fails the connection with the bit-pattern error."""
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r, s = _pended_data_tasks(p)
    IoPattern.recv_from_wire(r, 10)
    IoPattern.write_task_buffer(r, b"\xff", 7)
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    assert p.CompleteIo(r, 10, 0) == FailedIo
    assert p.GetLastPatternError() == A.STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN
    s = p.stats()
    assert (s["fail_offset"], s["fail_expected"], s["fail_actual"]) == (7, 0, 0xFF)
    assert "'0x0' didn't match '0xffffffff'" in p.failure_message()  # char through %x sign-extends


WSAECONNABORTED, WSAETIMEDOUT = 10053, 10060


def _duplex_data_phase(p, server, send_last):  # :318-336 CompleteDataPhase
    _complete_connection_id(p, server)
    r, s = _pended_data_tasks(p)
    if send_last:
        assert _complete_data_recv(p, r, 10) == ContinueIo
        assert p.CompleteIo(s, 10, 0) == ContinueIo
    else:
        assert p.CompleteIo(s, 10, 0) == ContinueIo
        assert _complete_data_recv(p, r, 10) == ContinueIo


def _duplex_client_to_fin(p):  # :341-354 DriveClientToFinRecv
    t = p.InitiateIo()
    assert t.io_action == Recv
    IoPattern.write_task_buffer(t, b"DONE", 0)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == A.TASK_GRACEFUL_SHUTDOWN
    assert p.CompleteIo(t, 0, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    return t


def _duplex_server_to_fin(p):  # :358-367 DriveServerToFinRecv
    t = p.InitiateIo()
    assert t.io_action == Send
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    return t


@pytest.mark.parametrize("server", [False, True], ids=["Client", "Server"])
def test_Duplex_FailConnectionId(make, server):  # :657-681
    p = make(**duplex_defaults(server))
    t = p.InitiateIo()
    assert (t.buffer_length, t.io_action) == (ConnectionIdLength, Send if server else Recv)
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


def test_Duplex_Client_FailDataSend(make):  # :683-698 (the recv is still outstanding)
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r, s = _pended_data_tasks(p)
    assert p.CompleteIo(s, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


def test_Duplex_Client_PrematureFinDuringTransfer(make):  # :717-737
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r, s = _pended_data_tasks(p)
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    assert p.CompleteIo(r, 0, 0) == FailedIo  # a FIN before the expected data
    assert p.GetLastPatternError() == A.STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED


def test_Duplex_Client_ExtraBytesWhenExpectingFin(make):  # :739-769
    p = make(**duplex_defaults(False))
    _duplex_data_phase(p, False, send_last=True)
    t = _duplex_client_to_fin(p)
    assert p.CompleteIo(t, 1, 0) == FailedIo
    assert p.GetLastPatternError() == A.STATUS_ERROR_TOO_MUCH_DATA_TRANSFERRED


def test_Duplex_Client_FailReceivingServerCompletion(make):  # :771-790
    p = make(**duplex_defaults(False))
    _duplex_data_phase(p, False, send_last=True)
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


@pytest.mark.parametrize("hard", [False, True], ids=["FailGracefulShutdown", "HardShutdown_Fails"])
def test_Duplex_Client_ShutdownFails(make, hard):  # :792-816, :1000-1021
    p = make(**duplex_defaults(False, tcp_shutdown=A.SHUTDOWN_HARD if hard else A.SHUTDOWN_GRACEFUL))
    _duplex_data_phase(p, False, send_last=not hard)
    t = p.InitiateIo()
    assert t.io_action == Recv
    IoPattern.write_task_buffer(t, b"DONE", 0)
    assert p.CompleteIo(t, 4, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == (A.TASK_HARD_SHUTDOWN if hard else A.TASK_GRACEFUL_SHUTDOWN)
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


@pytest.mark.parametrize("status,completed,err", [(WSAECONNRESET, FailedIo, WSAECONNRESET),
                                                  (WSAECONNABORTED, FailedIo, WSAECONNABORTED),
                                                  (WSAETIMEDOUT, FailedIo, WSAETIMEDOUT), (0, CompletedIo, 0)],
                         ids=["FailFinWithRst", "FailFinWithConnAborted", "FailFinWithTimeout", "CleanFin_RecvLast"])
def test_Duplex_Client_FinStatus(make, status, completed, err):  # :818-850, :1060-1099: the client tolerates none
    p = make(**duplex_defaults(False))
    _duplex_data_phase(p, False, send_last=False)
    t = _duplex_client_to_fin(p)
    assert p.CompleteIo(t, 0, status) == completed
    assert p.GetLastPatternError() == err


@pytest.mark.parametrize("server,status", [(False, 1), (False, WSAECONNRESET), (True, 1)],
                         ids=["Client_SendLast_SendFails", "Client_SendLast_SendRst", "Server_SendLast_SendFails"])
def test_Duplex_SendLast_Fails(make, server, status):  # :852-906
    p = make(**duplex_defaults(server))
    _complete_connection_id(p, server)
    r, s = _pended_data_tasks(p)
    assert _complete_data_recv(p, r, 10) == ContinueIo
    assert p.CompleteIo(s, 0, status) == FailedIo
    assert p.GetLastPatternError() == status


@pytest.mark.parametrize("server,status", [(False, 1), (False, WSAECONNRESET), (True, 1)],
                         ids=["Client_RecvLast_RecvFails", "Client_RecvLast_RecvRst", "Server_RecvLast_RecvFails"])
def test_Duplex_RecvLast_Fails(make, server, status):  # :908-941, :968-987
    p = make(**duplex_defaults(server))
    _complete_connection_id(p, server)
    r, s = _pended_data_tasks(p)
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    assert p.CompleteIo(r, 0, status) == FailedIo
    assert p.GetLastPatternError() == status


def test_Duplex_Client_RecvLast_PartialThenComplete(make):  # :943-966
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r, s = _pended_data_tasks(p)
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    assert _complete_data_recv(p, r, 4) == ContinueIo
    rr = p.InitiateIo()
    assert (rr.io_action, rr.buffer_length, rr.expected_pattern_offset) == (Recv, 6, 4)
    assert _complete_data_recv(p, rr, 6) == ContinueIo
    _successful_shutdown(p, False)
    assert p.GetLastPatternError() == 0 and p.stats()["buffers_verified"] == 2


def test_Duplex_Client_HardShutdown_SendLast(make):  # :989-998
    p = make(**duplex_defaults(False, tcp_shutdown=A.SHUTDOWN_HARD))
    _duplex_data_phase(p, False, send_last=True)
    _successful_shutdown(p, False, hard=True)
    assert p.GetLastPatternError() == 0


@pytest.mark.parametrize("n,content", [(2, b"DONE"), (4, b"FAIL")], ids=["CompletionTooFewBytes",
                                                                          "CompletionWrongContent"])
def test_Duplex_Client_BadCompletion(make, n, content):  # :1023-1058
    p = make(**duplex_defaults(False))
    _duplex_data_phase(p, False, send_last=True)
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, 4)
    IoPattern.write_task_buffer(t, content, 0)
    assert p.CompleteIo(t, n, 0) == FailedIo
    assert p.GetLastPatternError() == A.STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED


@pytest.mark.parametrize("send_last,status,completed,err",
                         [(False, WSAETIMEDOUT, CompletedIo, 0), (True, WSAECONNABORTED, CompletedIo, 0),
                          (False, 1, FailedIo, 1)],
                         ids=["TolerateTimeoutAwaitingFin", "TolerateConnAbortedAwaitingFin", "FailFinWithError"])
def test_Duplex_Server_FinStatus(make, send_last, status, completed, err):  # :1101-1136
    p = make(**duplex_defaults(True))
    _duplex_data_phase(p, True, send_last)
    t = _duplex_server_to_fin(p)
    assert p.CompleteIo(t, 0, status) == completed
    assert p.GetLastPatternError() == err


def test_Duplex_Server_ExtraBytesWhenExpectingFin(make):  # :1138-1148
    p = make(**duplex_defaults(True))
    _duplex_data_phase(p, True, send_last=True)
    t = _duplex_server_to_fin(p)
    assert p.CompleteIo(t, 1, 0) == FailedIo
    assert p.GetLastPatternError() == A.STATUS_ERROR_TOO_MUCH_DATA_TRANSFERRED


def test_Duplex_Server_FailSendingCompletion(make):  # :1150-1162
    p = make(**duplex_defaults(True))
    _duplex_data_phase(p, True, send_last=False)
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Send, 4)
    assert p.CompleteIo(t, 0, 1) == FailedIo
    assert p.GetLastPatternError() == 1


@pytest.mark.parametrize("n", [1, 2, 3], ids=["OneByteFails", "ShortFirstPieceFailsWithoutReassembly",
                                             "ThreeBytesFails"])
def test_Duplex_Client_CompletionDoneSplitRecv(make, n):  # :1178-1228: a split 'DONE' is not reassembled
    p = make(**duplex_defaults(False))
    _duplex_data_phase(p, False, send_last=True)
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Recv, 4)
    assert p.CompleteIo(t, n, 0) == FailedIo
    assert p.GetLastPatternError() == A.STATUS_ERROR_NOT_ALL_DATA_TRANSFERRED
    assert p.InitiateIo().io_action == NoneAction


@pytest.mark.parametrize("n,send_last", [(2, False), (1, True)], ids=["ShortSendAdvancesWithoutResend",
                                                                      "OneByteAdvances"])
def test_Duplex_Server_CompletionDoneSplitSend(make, n, send_last):  # :1230-1265: a short 'DONE' send advances
    p = make(**duplex_defaults(True))
    _duplex_data_phase(p, True, send_last)
    t = p.InitiateIo()
    assert (t.io_action, t.buffer_length) == (Send, 4)
    assert p.CompleteIo(t, n, 0) == ContinueIo
    t = p.InitiateIo()
    assert t.io_action == Recv
    assert p.CompleteIo(t, 0, 0) == CompletedIo
    assert p.GetLastPatternError() == 0


def test_Duplex_Client_DataRecvCappedBelowSocketBuffer_DoneCannotCoalesce(make):  # :1284-1310
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r, s = _pended_data_tasks(p)
    assert r.buffer_length < 1024  # capped to the outstanding data, not the buffer size: 'DONE' cannot ride along
    assert _complete_data_recv(p, r, 10) == ContinueIo
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    _successful_shutdown(p, False)
    assert p.GetLastPatternError() == 0


def test_Duplex_Client_PartialFinalData_ThenDone_Deframed(make):  # :1312-1353
    p = make(**duplex_defaults(False))
    _complete_connection_id(p, False)
    r, s = _pended_data_tasks(p)
    assert _complete_data_recv(p, r, 6) == ContinueIo
    rr = p.InitiateIo()
    assert (rr.io_action, rr.buffer_length, rr.expected_pattern_offset) == (Recv, 4, 6)
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    assert _complete_data_recv(p, rr, 4) == ContinueIo
    _successful_shutdown(p, False)
    assert p.GetLastPatternError() == 0 and p.stats()["buffers_verified"] == 2


def test_Duplex_Server_DataRecvCapped_FinCannotCoalesce(make):  # :1355-1393
    p = make(**duplex_defaults(True))
    _complete_connection_id(p, True)
    r = p.InitiateIo()
    assert (r.io_action, r.buffer_length) == (Recv, 10) and r.buffer_length < 1024
    s = p.InitiateIo()
    assert s.io_action == Send
    assert _complete_data_recv(p, r, 10) == ContinueIo
    assert p.CompleteIo(s, 10, 0) == ContinueIo
    _successful_shutdown(p, True)
    assert p.GetLastPatternError() == 0


def _multi_send_defaults(server, pre_post_sends, chunks):  # :384-394 SetTestDuplexMultiSendDefaults
    return duplex_defaults(server, pre_post_sends=pre_post_sends, buffer_size=10, transfer_size=2 * chunks * 10)


def _recv_half(p, r, chunks):  # CompleteMultiSendRecvHalf: the recv half, one 10-byte chunk at a time
    for i in range(chunks):
        assert r.expected_pattern_offset == 10 * i
        assert _complete_data_recv(p, r, 10) == ContinueIo
        if i < chunks - 1:
            r = p.InitiateIo()
            assert (r.io_action, r.buffer_length) == (Recv, 10)


def test_Duplex_Client_MultipleConcurrentSends_ReDriveAfterCompletion(make):  # :1443-1475
    p = make(**_multi_send_defaults(False, 3, 4))
    _complete_connection_id(p, False)
    r = p.InitiateIo()
    assert (r.io_action, r.buffer_length) == (Recv, 10)
    sends = [p.InitiateIo() for _ in range(3)]  # only three fit the backlog though four chunks remain
    assert [t.io_action for t in sends] == [Send] * 3
    assert p.InitiateIo().io_action == NoneAction
    assert p.CompleteIo(sends[0], 10, 0) == ContinueIo
    again = p.InitiateIo()  # the freed backlog re-drives the fourth send
    assert (again.io_action, again.buffer_length, again.buffer_offset) == (Send, 10, 30)
    assert p.CompleteIo(again, 10, 0) == ContinueIo
    assert p.CompleteIo(sends[1], 10, 0) == ContinueIo
    assert p.CompleteIo(sends[2], 10, 0) == ContinueIo
    assert p.InitiateIo().io_action == NoneAction
    _recv_half(p, r, 4)
    _successful_shutdown(p, False)
    assert p.GetLastPatternError() == 0


def test_Duplex_Client_IsbMode_DynamicBacklogGatesSends(make):  # :1477-1513
    p = make(**_multi_send_defaults(False, 0, 3))
    _complete_connection_id(p, False)
    r = p.InitiateIo()
    assert (r.io_action, r.buffer_length) == (Recv, 10)
    s1 = p.InitiateIo()
    assert (s1.io_action, s1.buffer_length) == (Send, 10)
    assert p.InitiateIo().io_action == NoneAction  # the initial backlog is one chunk
    p.SetIdealSendBacklog(30)  # the stack raises the ideal send backlog
    s2, s3 = p.InitiateIo(), p.InitiateIo()
    assert (s2.io_action, s3.io_action) == (Send, Send)
    assert p.InitiateIo().io_action == NoneAction
    for t in (s1, s2, s3):
        assert p.CompleteIo(t, 10, 0) == ContinueIo
    _recv_half(p, r, 3)
    _successful_shutdown(p, False)
    assert p.GetLastPatternError() == 0


@pytest.mark.parametrize("reverse", [False, True], ids=["CompleteInOrder", "CompleteReverseOrder"])
def test_Duplex_Server_MultipleConcurrentSends(make, reverse):  # :1515-1553
    p = make(**_multi_send_defaults(True, 3, 3))
    _complete_connection_id(p, True)
    r = p.InitiateIo()
    assert (r.io_action, r.buffer_length) == (Recv, 10)
    sends = [p.InitiateIo() for _ in range(3)]
    assert [t.io_action for t in sends] == [Send] * 3
    assert p.InitiateIo().io_action == NoneAction
    for t in (sends[::-1] if reverse else sends):
        assert p.CompleteIo(t, 10, 0) == ContinueIo
    _recv_half(p, r, 3)
    _successful_shutdown(p, True)
    assert p.GetLastPatternError() == 0


@pytest.mark.parametrize("reverse", [False, True], ids=["InOrder", "ReverseOrder"])
def test_Duplex_MultipleConcurrentSends(make, reverse):  # :1401-1553 (send offsets advance per created task)
    p = make(**duplex_defaults(False, pre_post_sends=3, buffer_size=10, transfer_size=2 * 3 * 10))
    _complete_connection_id(p, False)
    r = p.InitiateIo()
    assert (r.io_action, r.buffer_length) == (Recv, 10)
    sends = [p.InitiateIo() for _ in range(3)]
    assert [t.io_action for t in sends] == [Send] * 3
    assert [t.buffer_offset for t in sends] == [0, 10, 20]
    assert p.InitiateIo().io_action == NoneAction
    for t in (sends[::-1] if reverse else sends):
        assert p.CompleteIo(t, 10, 0) == ContinueIo
    assert p.InitiateIo().io_action == NoneAction  # the send half is done; the recv is still pending
    for i in range(3):
        assert r.expected_pattern_offset == 10 * i
        assert _complete_data_recv(p, r, 10) == ContinueIo
        if i < 2:
            r = p.InitiateIo()
    _successful_shutdown(p, False)
    assert p.GetLastPatternError() == 0


# ---- configuration guards (ctsConfig.cpp:2169-2171, 3440-3446; ctsIOPattern.cpp:225-227) ----------
def test_config_guards():
    shared_buffer_attach(_SENDER)
    from ctstraffic_amd import CtsError

    with pytest.raises(CtsError):  # -PrePostRecvs > 1 requires -Verify:connection with TCP
        IoPattern(PatternConfig(pre_post_recvs=2, verify_buffers=True, buffer_size=1024), verifier=_oracle_verifier)
    with pytest.raises(CtsError):  # UseSharedBuffer && ShouldVerifyBuffers
        IoPattern(PatternConfig(use_shared_buffer=True, verify_buffers=True, buffer_size=1024),
                  verifier=_oracle_verifier)
    with pytest.raises(CtsError):  # PrePostRecvs == 0
        IoPattern(PatternConfig(pre_post_recvs=0, verify_buffers=False, buffer_size=1024))


def test_no_verifier_fails_loudly():
    """Without an engine or a hook a verifying pattern refuses to complete a data recv: the product
    has no CPU verify path."""
    shared_buffer_attach(_SENDER)
    from ctstraffic_amd import CtsError

    p = IoPattern(PatternConfig(**server_defaults()))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    t = p.InitiateIo()
    recv_correct(t)
    with pytest.raises(CtsError):
        p.CompleteIo(t, 10, 0)
    p.close()


# ---- randomized long streams: sync vs deferred vs the oracle ----------------------------------------
def _expected_stream(lens, corrupt):
    """Walk the completions with the oracle: (first failing completion, bytes_recv at it, result)."""
    S = oracle.sender_buffer(65536 * 2)
    off = 0
    recv = 0
    for i, n in enumerate(lens):
        buf = S[off:off + n].copy()
        if i in corrupt:
            buf[corrupt[i][0]] ^= corrupt[i][1]
        recv += n
        r = oracle.verify_buffer(buf, 0, off, n)
        if not r["pass"]:
            return i, recv, r
        off = (off + n) % 65536
    return None, recv, None


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_random_push_server_stream(make, seed):
    rng = np.random.default_rng(seed)
    bufsize = int(rng.choice([1000, 4096, 65536]))
    n = 300
    lens = [int(x) for x in rng.integers(1, bufsize + 1, size=n)]
    total = sum(lens)
    corrupt = {}
    if seed != 1:
        k = int(rng.integers(5, n - 5))
        corrupt[k] = (int(rng.integers(0, lens[k])), int(rng.integers(1, 256)))
    p = make(**server_defaults(buffer_size=bufsize, transfer_size=total, batch_buffers=16))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    statuses = []
    for i, ln in enumerate(lens):
        t = p.InitiateIo()
        assert t.io_action == Recv
        # the wire delivers fewer bytes than posted (partial completions shift the phase)
        take = min(ln, t.buffer_length)
        IoPattern.recv_from_wire(t, take)
        if i in corrupt:
            pos, x = corrupt[i]
            pos = min(pos, take - 1)
            corrupt[i] = (pos, x)
            b = IoPattern.read_task_buffer(t, 1, pos)[0] ^ x
            IoPattern.write_task_buffer(t, bytes([b]), pos)
        lens[i] = take
        st = p.CompleteIo(t, take, 0)
        statuses.append(st)
        if st == FailedIo:
            break
    flushed = p.Flush() if statuses[-1] != FailedIo else FailedIo  # drain a deferred queue
    fail_at, recv_at, r = _expected_stream(lens[:len(statuses)], corrupt)
    s = p.stats()
    if fail_at is None:
        assert all(x == ContinueIo for x in statuses[:-1])
        assert s["has_failure"] == 0 and p.GetLastPatternError() == 2147483647
        assert s["buffers_verified"] == len(statuses)
        return
    assert s["has_failure"] == 1 and s["fail_completion"] == fail_at
    assert (s["fail_offset"], s["fail_expected"], s["fail_actual"]) == (r["first_mismatch"], r["expected"], r["actual"])
    assert s["bytes_recv_at_failure"] == recv_at
    assert p.GetLastPatternError() == A.STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN
    if make.mode == A.VERIFY_SYNC:
        assert statuses[-1] == FailedIo and len(statuses) == fail_at + 1
    else:
        # deferred: the failure surfaces when its batch is retired -- on the device half batches of 8 are
        # launched and left in flight while the next half fills, and an in-flight half is retired as soon as
        # a completion sees its kernel done, or at the latest when the next half is full -- or at the final
        # flush: at most one batch (16) of completions after the corrupt one is told ContinueIo
        assert flushed == FailedIo and fail_at + 1 <= len(statuses)
        assert sum(1 for x in statuses[fail_at + 1:] if x == ContinueIo) < 16
    # either way every counter is the reference's, which stopped at the failing completion: the completions
    # a deferred pattern accepted after it are taken back at the flush
    assert s["bytes_recv"] == recv_at and s["buffers_verified"] == fail_at + 1 and s["buffers_failed"] == 1
    assert s["bytes_verified"] == recv_at and s["queued"] == 0
    assert s["recv_pattern_offset"] == (sum(lens[:fail_at + 1])) % 65536


GPU_DEFERRED_BACKENDS = [b for b in BACKENDS if b.values[0][0] == "gpu" and b.values[0][1] == A.VERIFY_DEFERRED]


@pytest.mark.parametrize("depth", [1, 3])
@pytest.mark.parametrize("seed,corrupt", [(21, False), (22, True), (23, True)])
@pytest.mark.parametrize("make", GPU_DEFERRED_BACKENDS, indirect=True)
def test_deferred_counters_never_decrease_pipelined(make, seed, corrupt, depth, monkeypatch):
    """The same with 1 and 3 DEFERRED batches in flight (CTS_DEFERRED_DEPTH, read when the pattern is made; the
    default, 2, runs in test_deferred_counters_never_decrease): a batch that fails drops the ones launched after it,
    and nothing published is taken back."""
    monkeypatch.setenv("CTS_DEFERRED_DEPTH", str(depth))
    _check_counters_never_decrease(make, seed, corrupt)


@pytest.mark.parametrize("seed,corrupt", [(11, False), (12, True), (13, True), (14, True)])
def test_deferred_counters_never_decrease(make, seed, corrupt):
    """TcpStatusDetails and the per-connection byte counters only ever grow. The reference only Adds to them
    (ctsIOPattern.cpp:505-516, ctsStatistics.hpp:153-186) and its status timer prints their SnapValueDifference
    (ctsStatistics.hpp:363), so a slice can never be negative. A DEFERRED pattern holds back the bytes of every
    completion behind a pending batch verdict and publishes them when the batch verifies. Here a paced Duplex client
    completes its sends and recvs in random order, with a corrupt recv in the middle of a batch. Both counters are
    read after every completion; the end totals must be the reference's: everything up to and including the failing
    recv, nothing after it, in every verify mode."""
    _check_counters_never_decrease(make, seed, corrupt)


def _check_counters_never_decrease(make, seed, corrupt):
    """The body of test_deferred_counters_never_decrease (and of its pipelined form)."""
    from ctstraffic_amd.pattern import status_details, status_details_reset

    rng = np.random.default_rng(seed)
    size, n_each = 1024, 200
    p = make(**duplex_defaults(False, buffer_size=size, transfer_size=2 * n_each * size, pre_post_sends=2,
                               batch_buffers=16, tcp_bytes_per_second=40 * size, tcp_bytes_per_second_period=100))
    status_details_reset()
    _complete_connection_id(p, False)
    bad_recv = int(rng.integers(20, n_each - 20)) if corrupt else None
    pending, log = [], []  # data completions in order: (action, bytes)
    recvs = 0
    prev = (status_details(), p.stats())
    st = ContinueIo
    while st == ContinueIo:
        while True:
            t = p.InitiateIo()
            if t.io_action == NoneAction:
                break
            pending.append(t)
        assert pending, "the pattern stalled"
        t = pending.pop(int(rng.integers(0, len(pending))))
        if t.io_action == Recv and t.buffer_type == A.BUFFER_DYNAMIC:
            n = int(t.buffer_length)
            IoPattern.recv_from_wire(t, n)
            if recvs == bad_recv:
                pos = int(rng.integers(0, n))
                IoPattern.write_task_buffer(t, bytes([IoPattern.read_task_buffer(t, 1, pos)[0] ^ 0x5A]), pos)
            recvs += 1
            log.append((Recv, n))
        elif t.io_action == Send and t.buffer_type != A.BUFFER_COMPLETION_MESSAGE:
            n = int(t.buffer_length)
            log.append((Send, n))
        elif t.buffer_type == A.BUFFER_COMPLETION_MESSAGE:
            n = 4  # "DONE": the client's completion buffer already holds it
        else:
            n = 0  # graceful shutdown, then the FIN
        st = p.CompleteIo(t, n, 0)
        cur = (status_details(), p.stats())
        for k in ("bytes_sent", "bytes_recv"):
            assert cur[0][k] >= prev[0][k], ("TcpStatusDetails", k, prev[0], cur[0])
            assert cur[1][k] >= prev[1][k], ("per-connection", k, prev[1], cur[1])
        if make.mode == A.VERIFY_SYNC:
            assert cur[1]["bytes_recv_held"] == 0 and cur[1]["bytes_sent_held"] == 0
        prev = cur
    p.Flush()
    s, g = p.stats(), status_details()
    # the reference's totals: it fails the connection at the corrupt recv's completion
    upto = log
    if corrupt:
        k = [i for i, (a, _) in enumerate(log) if a == Recv][bad_recv]
        upto = log[:k + 1]
    want_recv = sum(n for a, n in upto if a == Recv)
    want_sent = sum(n for a, n in upto if a == Send)
    assert (s["bytes_recv"], s["bytes_sent"]) == (want_recv, want_sent)
    assert s["bytes_recv_held"] == 0 and s["bytes_sent_held"] == 0 and s["queued"] == 0
    if corrupt:
        assert st == FailedIo and p.GetLastPatternError() == A.STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN
        assert s["fail_completion"] == bad_recv and s["bytes_recv_at_failure"] == want_recv
        assert (g["bytes_recv"], g["bytes_sent"]) == (ConnectionIdLength + want_recv, want_sent)
        assert g["data_errors"] == 1
    else:
        assert st == CompletedIo and p.GetLastPatternError() == 0
        assert (g["bytes_recv"], g["bytes_sent"]) == (ConnectionIdLength + want_recv + 4, want_sent)
        assert want_recv == want_sent == n_each * size


# ---- RIO buffer ids (ctsIOPattern.cpp:133-217, :369-386, :683-692, :716-725) ------------------------
@pytest.mark.parametrize("make", RIO_BACKENDS, indirect=True)
def test_rio_send_ids_unique_and_recycled(make):
    """A Push client under -io:rioiocp: concurrent sends carry distinct ids of the sender buffer's
    registrations; a completed send's id goes back on the list and is the next one handed out (the
    reference pops and pushes at the back)."""
    p = make(**client_defaults(pre_post_sends=3, transfer_size=100000))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    sends = [p.InitiateIo() for _ in range(3)]
    assert [t.io_action for t in sends] == [Send] * 3
    assert all(t.buffer_type == A.BUFFER_DYNAMIC for t in sends)  # Static without RIO
    assert len({t.rio_buffer_id for t in sends}) == 3
    base = p.GetRioBufferIdCount()
    assert p.CompleteIo(sends[1], 1024, 0) == ContinueIo
    assert p.GetRioBufferIdCount() == base + 1
    nxt = p.InitiateIo()
    assert nxt.rio_buffer_id == sends[1].rio_buffer_id


@pytest.mark.parametrize("make", RIO_BACKENDS, indirect=True)
def test_rio_send_ids_exhausted_returns_no_io(make):
    """-io:rioiocp registers the sender buffer 16 MiB / min buffer + 1 times (ctsIOPattern.cpp:61, 195-217). With
    every one of those ids in flight the next send request is an empty task, not a send (ctsIOPattern.cpp:580-587);
    a completed send's id makes the next request a send again, and the send offsets stay contiguous."""
    size = 65536
    p = make(**client_defaults(pre_post_sends=400, buffer_size=size, transfer_size=400 * size))
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    ids = (1 << 24) // size + 1
    sends = [p.InitiateIo() for _ in range(ids)]
    assert [t.io_action for t in sends] == [Send] * ids
    assert len({t.rio_buffer_id for t in sends}) == ids
    assert [t.buffer_offset for t in sends] == [(k * size) % 65536 for k in range(ids)]
    none = p.InitiateIo()
    assert none.io_action == A.TASK_NONE and none.rio_buffer_id == A.RIO_INVALID_BUFFERID
    assert p.CompleteIo(sends[0], size, 0) == ContinueIo
    nxt = p.InitiateIo()
    assert nxt.io_action == Send and nxt.rio_buffer_id == sends[0].rio_buffer_id
    assert nxt.buffer_offset == (ids * size) % 65536


def test_rio_without_functions_or_failing_register(rio_fake):
    """RIORegisterBuffer failing anywhere in the constructor (recv slots, connection id, completion message,
    the sender registrations) fails MakeIoPattern and leaves nothing registered."""
    from ctstraffic_amd import CtsError
    from ctstraffic_amd.pattern import rio_functions_set

    shared_buffer_attach(_SENDER)
    cfg = PatternConfig(**server_defaults(registered_io=True, buffer_size=65536))
    total = 1 + 2 + (1 << 24) // 65536 + 1  # recv slot, connection id, completion message, sends
    for k in [0, 1, 2, 3, total - 1]:
        rio_fake.reset(fail_after=k)
        with pytest.raises(CtsError):
            IoPattern(cfg, verifier=_oracle_verifier)
        assert rio_fake.live() == 0 and rio_fake.errors() == 0
    rio_fake.reset(fail_after=total)
    p = IoPattern(cfg, verifier=_oracle_verifier)
    assert rio_fake.live() == total and p.GetRioBufferIdCount() == total
    p.close()
    assert rio_fake.live() == 0
    rio_fake.reset()
    rio_functions_set(None, None)
    try:
        with pytest.raises(CtsError):
            IoPattern(cfg, verifier=_oracle_verifier)
    finally:
        rio_functions_set(rio_fake.register_ptr, rio_fake.deregister_ptr)
    p = IoPattern(PatternConfig(**server_defaults(buffer_size=65536)), verifier=_oracle_verifier)
    assert p.GetRioBufferIdCount() == 0  # ctsIOPattern.h:116-119
    t = p.InitiateIo()
    assert t.rio_buffer_id == A.RIO_INVALID_BUFFERID
    p.close()


# ---- send pacing: ctsTask::m_timeOffsetMilliseconds (ctsIOPattern.cpp:219-224, 593-674) ------------------------
# No MSTest drives the pattern's pacing (ctsIOPatternRateLimitPolicyUnitTest tests a policy class the product does
# not include), so these tests pin the C++ against a line-by-line Python restatement of CreateNewTask's branch and
# hand-worked cases: parity with the reference's source, not with a reference fixture.
class _Pacer:
    """CreateNewTask's send-time offset (ctsIOPattern.cpp:593-674), restated."""

    def __init__(self, bps, period, burst_count, burst_delay, start_ms):
        self.period = period
        self.per = bps * period // 1000
        self.this = 0
        self.start = start_ms
        self.burst_count, self.burst_delay, self.burst = burst_count, burst_delay, burst_count

    def offset(self, now, size):
        off = 0
        if self.per > 0:
            if self.this < self.per:
                self.this += size
                if now > self.start + self.period:
                    skipped = (now - self.start) // self.period
                    self.start += skipped * self.period
                    adjust = self.per * skipped
                    self.this = 0 if adjust > self.this else self.this - adjust
            else:
                ahead = self.this // self.per
                skip = (ahead - 1) * self.period
                self.this -= self.per * ahead
                self.this += size
                if now < self.start + self.period:
                    off = self.start + self.period - now
                off += skip
                self.start += skip + self.period
        elif self.burst_count:
            if self.burst == 0:
                self.burst = self.burst_count
            self.burst -= 1
            if self.burst == 0:
                off = self.burst_delay
        return off


class _FakeClock:
    def __init__(self, t):
        self.t = t

    def __call__(self):
        return self.t


def _paced_client(clock, **kw):
    from ctstraffic_amd.pattern import clock_set

    clock_set(clock)
    shared_buffer_attach(_SENDER)
    cfg = PatternConfig(**client_defaults(**kw))
    p = IoPattern.MakeIoPattern(cfg, None, verifier=_oracle_verifier)
    t = p.InitiateIo()  # the connection id
    assert t.io_action == Recv and t.time_offset_ms == 0
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    return p


def test_send_pacing_one_buffer_per_quantum():
    """10 x 64 KiB per second in 100 ms quanta is one buffer per quantum: with the clock standing still the
    sends are scheduled 0, 100, 200, ... ms ahead; once the clock reaches a send's slot it goes out at once."""
    from ctstraffic_amd.pattern import clock_set

    clock = _FakeClock(5000)
    try:
        p = _paced_client(clock, pre_post_sends=64, buffer_size=65536, transfer_size=1 << 30,
                          tcp_bytes_per_second=655360, tcp_bytes_per_second_period=100)
        offs = [p.InitiateIo().time_offset_ms for _ in range(5)]
        assert offs == [0, 100, 200, 300, 400]
        clock.t += 450  # the clock passes the five scheduled quanta
        assert p.InitiateIo().time_offset_ms == 50
        p.close()
    finally:
        clock_set(None)


def test_send_burst_delay():
    """-burstcount:3 -burstdelay:50 without a rate limit: every third send waits 50 ms (:657-674); recvs never."""
    from ctstraffic_amd.pattern import clock_set

    try:
        p = _paced_client(None, pre_post_sends=64, transfer_size=1 << 30, burst_count=3, burst_delay=50)
        ts = [p.InitiateIo() for _ in range(9)]
        assert [t.io_action for t in ts] == [Send] * 9
        assert [t.time_offset_ms for t in ts] == [0, 0, 50] * 3
        p.close()
        # a rate limit takes precedence over the burst settings
        p = _paced_client(_FakeClock(0), pre_post_sends=64, transfer_size=1 << 30, burst_count=1, burst_delay=7,
                          tcp_bytes_per_second=10 ** 9)
        assert [p.InitiateIo().time_offset_ms for _ in range(4)] == [0, 0, 0, 0]
        p.close()
    finally:
        clock_set(None)


@pytest.mark.parametrize("seed", range(6))
def test_send_pacing_matches_restatement(seed):
    """Random rates, quanta, buffer sizes ([lo, hi] draws) and clock steps (standing, within a quantum, skipping
    several): every send's time offset equals the restated CreateNewTask branch, including carried-over bytes
    and quantums skipped forward."""
    from ctstraffic_amd.pattern import clock_set

    rng = np.random.default_rng(seed)
    bps = int(rng.choice([1, 100_000, 655_360, 3_000_000, 50_000_000]))
    period = int(rng.choice([1, 10, 100, 250]))
    lo = int(rng.integers(1000, 30000))
    clock = _FakeClock(int(rng.integers(0, 10 ** 6)))
    try:
        p = _paced_client(clock, pre_post_sends=1 << 20, transfer_size=1 << 40, buffer_size=lo,
                          buffer_size_high=lo + int(rng.integers(0, 60000)), random_seed=seed,
                          tcp_bytes_per_second=bps, tcp_bytes_per_second_period=period)
        model = _Pacer(bps, period, 0, 0, clock.t)
        for _ in range(400):
            step = int(rng.choice([0, 0, 1, period // 2, period, 3 * period + 1, 17]))
            clock.t += step
            t = p.InitiateIo()
            assert t.io_action == Send
            assert t.time_offset_ms == model.offset(clock.t, t.buffer_length), (bps, period, clock.t)
        p.close()
    finally:
        clock_set(None)


def test_deferred_destroy_publishes_held_bytes(make):
    """A DEFERRED pattern destroyed while completions wait for their batch verdict verifies them first, so their bytes
    reach TcpStatusDetails: the reference verified and counted every completion inside its CompleteIo
    (ctsIOPattern.cpp:461-521) whenever the connection was torn down."""
    from ctstraffic_amd.pattern import status_details, status_details_reset

    p = make(**server_defaults(buffer_size=4096, transfer_size=100 * 4096, batch_buffers=64))
    status_details_reset()
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for _ in range(5):
        t = p.InitiateIo()
        assert _complete_data_recv(p, t, 4096) == ContinueIo
    s = p.stats()
    held = s["bytes_recv_held"]
    if make.mode == A.VERIFY_SYNC:
        assert held == 0 and s["bytes_recv"] == 5 * 4096
    else:
        assert held == 5 * 4096 and s["bytes_recv"] == 0 and s["queued"] == 5
    assert status_details()["bytes_recv"] == 5 * 4096 - held
    p.close()
    assert status_details()["bytes_recv"] == 5 * 4096


def test_deferred_destroy_reports_a_failed_final_verify():
    """cts_io_pattern_destroy returns the final flush's error (here the verifier hook failing on the batch destroy
    verifies) instead of CTS_OK, the pattern is freed all the same, and IoPattern.close() raises it once: a second
    close is a no-op (a CTS_E_TIMEOUT, by contrast, keeps the handle for another close: tests/cpp/engine_devices.cpp)."""
    from ctstraffic_amd._lib import CTS_E_INVALID, CtsError

    fail = [False]

    def verifier(arena, descs):
        if fail[0]:
            raise RuntimeError("the final verify fails")
        return _oracle_verifier(arena, descs)

    shared_buffer_attach(_SENDER)
    p = IoPattern(PatternConfig(**server_defaults(buffer_size=4096, transfer_size=100 * 4096, batch_buffers=64,
                                                  verify_mode=A.VERIFY_DEFERRED)), verifier=verifier)
    t = p.InitiateIo()
    assert p.CompleteIo(t, ConnectionIdLength, 0) == ContinueIo
    for _ in range(3):
        t = p.InitiateIo()
        assert _complete_data_recv(p, t, 4096) == ContinueIo
    assert p.stats()["queued"] == 3
    fail[0] = True
    with pytest.raises(CtsError) as e:
        p.close()
    assert e.value.status == CTS_E_INVALID
    assert p._h is None
    p.close()
