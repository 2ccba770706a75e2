"""ctsIoPatternState (include/cts_pattern.h: cts_io_pattern_state_*) replaying the reference's own
MSTest project MSTest/ctsIOPatternStateUnitTest/ctsIOPatternStateUnitTest.cpp, all 27 TEST_METHODs,
assertion for assertion (file:line per test). Pure host logic: CPU only.

The reference fakes ctsConfig (ctsIOPatternStateUnitTest.cpp:80-141): IsListening() = the role,
GetTransferSize() = GetMaxBufferSize() = the test's transfer size, Protocol TCP, TcpShutdown per test.
"""
import ctypes

import pytest

from ctstraffic_amd import _pattern_abi as A
from ctstraffic_amd._lib import lib

ConnectionIdLength = A.CONNECTION_ID_LENGTH
NO_ERROR = 0
WSAECONNRESET, WSAECONNABORTED = 10054, 10053
Client, Server = 0, 1

NoError, TooManyBytes, TooFewBytes, ErrorIoFailed, SuccessfullyCompleted = (
    A.PE_NO_ERROR, A.PE_TOO_MANY_BYTES, A.PE_TOO_FEW_BYTES, A.PE_ERROR_IO_FAILED, A.PE_SUCCESSFULLY_COMPLETED)


class PatternState:
    """ctsIoPatternState through the C ABI, with the test class's Request* helpers (:179-351)."""

    def __init__(self, transfer, role, shutdown, protocol=A.PROTOCOL_TCP):
        c = A.CtsPatternConfig()
        c.io_pattern = A.PATTERN_PUSH
        c.protocol = protocol
        c.listening = 1 if role == Server else 0
        c.tcp_shutdown = shutdown
        c.transfer_size = transfer
        c.buffer_size_low = max(1, min(transfer, 0xFFFFFFFF))  # GetMaxBufferSize() fake = transfer size
        h = ctypes.c_void_p()
        assert lib().cts_io_pattern_state_create(ctypes.byref(c), ctypes.byref(h)) == 0
        self.h = h
        self.listening = role == Server
        self._keep = []

    def __del__(self):
        if getattr(self, "h", None):
            lib().cts_io_pattern_state_destroy(self.h)

    # the reference's member functions
    def GetRemainingTransfer(self):
        return int(lib().cts_io_pattern_state_get_remaining_transfer(self.h))

    def GetMaxTransfer(self):
        return int(lib().cts_io_pattern_state_get_max_transfer(self.h))

    def SetMaxTransfer(self, v):
        assert lib().cts_io_pattern_state_set_max_transfer(self.h, v) == 0

    def IsCompleted(self):
        return lib().cts_io_pattern_state_is_completed(self.h) == 1

    def GetNextPatternType(self):
        return lib().cts_io_pattern_state_get_next_pattern_type(self.h)

    def NotifyNextTask(self, t):
        assert lib().cts_io_pattern_state_notify_next_task(self.h, ctypes.byref(t)) == 0

    def CompletedTask(self, t, n):
        return lib().cts_io_pattern_state_completed_task(self.h, ctypes.byref(t), n)

    def UpdateError(self, e):
        return lib().cts_io_pattern_state_update_error(self.h, e)

    # test helpers
    def _task(self, action, track, length, buf=None):
        t = A.CtsTask()
        t.io_action = action
        t.track_io = 1 if track else 0
        t.buffer_length = length
        if buf is not None:
            t.buffer = ctypes.cast(buf, ctypes.c_void_p).value
        return t

    def RequestConnectionId(self):  # :193-217
        pt = self.GetNextPatternType()
        assert pt == (A.PT_SEND_CONNECTION_ID if self.listening else A.PT_RECV_CONNECTION_ID)
        t = self._task(A.TASK_SEND if self.listening else A.TASK_RECV, False, ConnectionIdLength)
        self.NotifyNextTask(t)
        assert not self.IsCompleted()
        return t

    def RequestMoreIo(self, n):  # :219-232
        assert self.GetNextPatternType() == A.PT_MORE_IO
        t = self._task(A.TASK_RECV, True, n)
        self.NotifyNextTask(t)
        assert not self.IsCompleted()
        return t

    def _status(self, expect, action):
        assert self.GetNextPatternType() == expect
        buf = ctypes.create_string_buffer(4)  # uint32_t statusBuffer
        self._keep.append(buf)
        t = self._task(action, False, 4, buf)
        self.NotifyNextTask(t)
        assert not self.IsCompleted()
        self.VerifyNoMoreIo()
        return t, buf

    def RequestSendStatus(self):  # :234-254
        return self._status(A.PT_SEND_COMPLETION, A.TASK_SEND)[0]

    def RequestRecvStatus(self, write_done):  # :256-276 (+ the test's memcpy_s of "DONE")
        t, buf = self._status(A.PT_RECV_COMPLETION, A.TASK_RECV)
        if write_done:
            ctypes.memmove(buf, b"DONE", 4)
        return t

    def _plain(self, expect, action, length):
        assert self.GetNextPatternType() == expect
        t = self._task(action, False, length)
        self.NotifyNextTask(t)
        assert not self.IsCompleted()
        self.VerifyNoMoreIo()
        return t

    def RequestFin(self):  # :278-296
        return self._plain(A.PT_REQUEST_FIN, A.TASK_RECV, 16)

    def RequestGracefulShutdown(self):  # :298-316
        return self._plain(A.PT_GRACEFUL_SHUTDOWN, A.TASK_GRACEFUL_SHUTDOWN, 0)

    def RequestHardShutdown(self):  # :318-336
        return self._plain(A.PT_HARD_SHUTDOWN, A.TASK_HARD_SHUTDOWN, 0)

    def VerifyNoMoreIo(self):  # :338-342
        assert self.GetNextPatternType() == A.PT_NO_IO


def InitGracefulShutdownTest(transfer, role=Client):  # :161-170
    s = PatternState(transfer, role, A.SHUTDOWN_GRACEFUL)
    assert not s.IsCompleted() and s.GetRemainingTransfer() == transfer
    return s


def InitHardShutdownTest(transfer):  # :172-181 (client only)
    s = PatternState(transfer, Client, A.SHUTDOWN_HARD)
    assert not s.IsCompleted() and s.GetRemainingTransfer() == transfer
    return s


def test_TestGetMaxTransfer():  # :364-371
    for s in (InitGracefulShutdownTest(100), InitHardShutdownTest(100)):
        assert s.GetMaxTransfer() == 100


def test_TestGetRemainingTransfer():  # :373-380
    for s in (InitGracefulShutdownTest(100), InitHardShutdownTest(100)):
        assert s.GetRemainingTransfer() == 100


def test_TestSetMaxTransfer():  # :382-395
    for s in (InitGracefulShutdownTest(250), InitHardShutdownTest(250)):
        assert s.GetMaxTransfer() == 250
        s.SetMaxTransfer(100)
        assert s.GetMaxTransfer() == 100


def test_TestGetRemainingTransferAfterSetMaxTransfer():  # :397-416
    for s in (InitGracefulShutdownTest(250), InitHardShutdownTest(250)):
        assert s.GetMaxTransfer() == 250 and s.GetRemainingTransfer() == 250
        s.SetMaxTransfer(100)
        assert s.GetMaxTransfer() == 100 and s.GetRemainingTransfer() == 100


def test_TestClientIsCompletedNoIo():  # :418-425
    assert not InitGracefulShutdownTest(100, Client).IsCompleted()
    assert not InitHardShutdownTest(100).IsCompleted()


def test_TestServerIsCompletedNoIo():  # :427-431
    assert not InitGracefulShutdownTest(100, Server).IsCompleted()


def test_TestSuccessfullySendConnectionId():  # :433-440
    s = InitGracefulShutdownTest(100, Server)
    t = s.RequestConnectionId()
    assert t.buffer_length == ConnectionIdLength
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    assert not s.IsCompleted()


def test_TestFailedSendConnectionId():  # :442-450
    s = InitGracefulShutdownTest(100, Server)
    t = s.RequestConnectionId()
    assert t.buffer_length == ConnectionIdLength
    assert s.UpdateError(1) == ErrorIoFailed
    assert s.IsCompleted()


def test_TestSuccessfullyReceiveConnectionId():  # :452-465
    for s in (InitGracefulShutdownTest(100, Client), InitHardShutdownTest(100)):
        t = s.RequestConnectionId()
        assert t.buffer_length == ConnectionIdLength
        assert s.CompletedTask(t, ConnectionIdLength) == NoError
        assert not s.IsCompleted()


def test_TestFailedReceiveConnectionId():  # :467-484
    for s in (InitGracefulShutdownTest(100, Client), InitHardShutdownTest(100)):
        t = s.RequestConnectionId()
        assert t.buffer_length == ConnectionIdLength
        assert s.UpdateError(1) == ErrorIoFailed
        assert s.IsCompleted()
        s.VerifyNoMoreIo()


def test_TestReceivedTooFewBytesForConnectionId():  # :486-499
    for s in (InitGracefulShutdownTest(100, Client), InitHardShutdownTest(100)):
        t = s.RequestConnectionId()
        assert t.buffer_length == ConnectionIdLength
        assert s.CompletedTask(t, ConnectionIdLength - 1) == TooFewBytes
        assert s.IsCompleted()


@pytest.mark.parametrize("init", [lambda: InitGracefulShutdownTest(100, Client), lambda: InitHardShutdownTest(100),
                                  lambda: InitGracefulShutdownTest(100, Server)],
                         ids=["client-graceful", "client-hard", "server"])
def test_TestClientFailIo_TestServerFailIo(init):  # :501-528 (client), :530-545 (server)
    s = init()
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    t = s.RequestMoreIo(50)
    assert s.UpdateError(1) == ErrorIoFailed  # indicate an error
    assert s.IsCompleted()
    assert s.CompletedTask(t, 50) == ErrorIoFailed
    assert s.IsCompleted()
    assert s.UpdateError(1) == ErrorIoFailed
    assert s.IsCompleted()
    s.VerifyNoMoreIo()


@pytest.mark.parametrize("init", [lambda: InitGracefulShutdownTest(150, Client), lambda: InitHardShutdownTest(150),
                                  lambda: InitGracefulShutdownTest(150, Server)],
                         ids=["client-graceful", "client-hard", "server"])
def test_TestClientFailTooManyBytes_TestServerFailTooManyBytes(init):  # :547-574, :576-590
    s = init()
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    t = s.RequestMoreIo(100)
    assert s.CompletedTask(t, 100) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted()
    t = s.RequestMoreIo(100)
    assert s.CompletedTask(t, 100) == TooManyBytes
    assert s.UpdateError(0) == ErrorIoFailed
    assert s.IsCompleted()
    s.VerifyNoMoreIo()


@pytest.mark.parametrize("init", [lambda: InitGracefulShutdownTest(100, Client), lambda: InitHardShutdownTest(100),
                                  lambda: InitGracefulShutdownTest(100, Server)],
                         ids=["client-graceful", "client-hard", "server"])
def test_TestClientFailTooFewBytes_TestServerFailTooFewBytes(init):  # :592-621, :623-638
    s = init()
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    t = s.RequestMoreIo(100)  # 2 IO tasks - completing too few bytes
    assert s.CompletedTask(t, 50) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted()
    t = s.RequestMoreIo(100)
    assert s.CompletedTask(t, 0) == TooFewBytes
    assert s.UpdateError(0) == ErrorIoFailed
    assert s.IsCompleted()
    s.VerifyNoMoreIo()


def test_TestClient_GracefulShutdown_FINFailedTooManyBytes():  # :640-675
    s = InitGracefulShutdownTest(100, Client)
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    t = s.RequestMoreIo(100)
    assert s.CompletedTask(t, 100) == NoError
    assert s.GetRemainingTransfer() == 0 and not s.IsCompleted()
    assert s.UpdateError(0) == NoError
    t = s.RequestRecvStatus(write_done=True)
    assert s.CompletedTask(t, 4) == NoError
    assert s.GetRemainingTransfer() == 0 and not s.IsCompleted()
    assert s.UpdateError(0) == NoError
    t = s.RequestGracefulShutdown()
    assert s.CompletedTask(t, 0) == NoError
    assert s.GetRemainingTransfer() == 0 and not s.IsCompleted()
    assert s.UpdateError(0) == NoError
    t = s.RequestFin()
    assert s.CompletedTask(t, 1) == TooManyBytes
    assert s.GetRemainingTransfer() == 0 and s.IsCompleted()
    assert s.UpdateError(0) == ErrorIoFailed
    s.VerifyNoMoreIo()


def test_TestServerFINFailedTooManyBytes():  # :677-702
    s = InitGracefulShutdownTest(100, Server)
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    t = s.RequestMoreIo(100)
    assert s.CompletedTask(t, 100) == NoError
    assert s.GetRemainingTransfer() == 0 and not s.IsCompleted()
    assert s.UpdateError(0) == NoError
    t = s.RequestSendStatus()
    assert s.CompletedTask(t, 4) == NoError
    assert s.GetRemainingTransfer() == 0 and not s.IsCompleted()
    assert s.UpdateError(0) == NoError
    t = s.RequestFin()
    assert s.CompletedTask(t, 1) == TooManyBytes
    assert s.GetRemainingTransfer() == 0 and s.IsCompleted()
    assert s.UpdateError(0) == ErrorIoFailed
    s.VerifyNoMoreIo()


def _single_io_to_status(s):
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    t = s.RequestMoreIo(100)
    assert s.UpdateError(0) == NoError
    assert s.CompletedTask(t, 100) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0


def test_TestClientSingleIo():  # :704-770
    s = InitGracefulShutdownTest(100, Client)
    _single_io_to_status(s)
    t = s.RequestRecvStatus(write_done=False)
    assert s.UpdateError(0) == NoError
    ctypes.memmove(t.buffer, b"DONE", 4)  # write "DONE" in the message to complete it
    assert s.CompletedTask(t, 4) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestGracefulShutdown()
    assert s.UpdateError(0) == NoError
    assert s.CompletedTask(t, 0) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestFin()
    assert s.UpdateError(0) == NoError
    assert s.CompletedTask(t, 0) == SuccessfullyCompleted
    assert s.UpdateError(0) == NoError
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()

    s = InitHardShutdownTest(100)
    _single_io_to_status(s)
    t = s.RequestRecvStatus(write_done=True)
    assert s.UpdateError(0) == NoError
    assert s.CompletedTask(t, 4) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestHardShutdown()
    assert s.UpdateError(0) == NoError
    assert s.CompletedTask(t, 0) == SuccessfullyCompleted
    assert s.UpdateError(0) == NoError
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()


@pytest.mark.parametrize("fin_error", [NO_ERROR, WSAECONNRESET, WSAECONNABORTED],
                         ids=["TestServerSingleIo_FIN", "TestServerSingleIo_RST", "TestServerSingleIo_RST_with_other_error"])
def test_TestServerSingleIo(fin_error):  # :772-800 (FIN), :802-830 (RST), :832-860 (RST with WSAECONNABORTED)
    s = InitGracefulShutdownTest(100, Server)
    _single_io_to_status(s)
    t = s.RequestSendStatus()
    assert s.UpdateError(0) == NoError
    assert s.CompletedTask(t, 4) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    # the FIN recv may fail with a reset: fine while a server waits for the FIN (ctsIOPatternState.hpp:277-285)
    t = s.RequestFin()
    assert s.UpdateError(fin_error) == NoError
    assert s.CompletedTask(t, 0) == SuccessfullyCompleted
    assert s.UpdateError(0) == NoError
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()


def _three_ios(s):
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    for remaining in (200, 100, 0):
        t = s.RequestMoreIo(100)
        assert not s.IsCompleted() and s.GetRemainingTransfer() == remaining
        assert s.CompletedTask(t, 100) == NoError
        assert s.UpdateError(0) == NoError
        assert not s.IsCompleted() and s.GetRemainingTransfer() == remaining


def test_TestClientMultipleIo():  # :862-1005
    s = InitGracefulShutdownTest(300, Client)
    _three_ios(s)
    t = s.RequestRecvStatus(write_done=True)
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    assert s.CompletedTask(t, 4) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestGracefulShutdown()
    assert s.CompletedTask(t, 0) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestFin()
    assert s.CompletedTask(t, 0) == SuccessfullyCompleted
    assert s.UpdateError(0) == NoError
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()

    s = InitGracefulShutdownTest(300, Client)
    _three_ios(s)
    t = s.RequestRecvStatus(write_done=False)  # not writing "DONE" in the message - should fail the completion
    assert s.CompletedTask(t, 4) == TooFewBytes
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()

    s = InitHardShutdownTest(300)
    _three_ios(s)
    t = s.RequestRecvStatus(write_done=True)
    assert s.CompletedTask(t, 4) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestHardShutdown()
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    assert s.CompletedTask(t, 0) == SuccessfullyCompleted
    assert s.UpdateError(0) == NoError
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()


def test_TestServerMultipleIo():  # :1007-1055
    s = InitGracefulShutdownTest(300, Server)
    _three_ios(s)
    t = s.RequestSendStatus()
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    assert s.CompletedTask(t, 4) == NoError
    assert s.UpdateError(0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestFin()
    assert s.CompletedTask(t, 0) == SuccessfullyCompleted
    assert s.UpdateError(0) == NoError
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    assert s.UpdateError(0) == NoError
    s.VerifyNoMoreIo()


def _overlapping(s):
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    tasks = []
    for remaining in (200, 100, 0):
        tasks.append(s.RequestMoreIo(100))
        assert s.GetRemainingTransfer() == remaining
    s.VerifyNoMoreIo()  # all IO is now posted
    for k, t in enumerate(tasks):
        assert s.CompletedTask(t, 100) == NoError
        assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
        if k < 2:  # NoIo while IO is still pended
            assert s.GetNextPatternType() == A.PT_NO_IO
            s.VerifyNoMoreIo()


def test_TestClientOverlappingMultipleIo():  # :1057-1180
    s = InitGracefulShutdownTest(300, Client)
    _overlapping(s)
    t = s.RequestRecvStatus(write_done=True)
    assert s.CompletedTask(t, 4) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestGracefulShutdown()
    assert s.CompletedTask(t, 0) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    final_fin = s.RequestFin()
    assert s.CompletedTask(final_fin, 0) == SuccessfullyCompleted
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()

    s = InitHardShutdownTest(300)
    _overlapping(s)
    t = s.RequestRecvStatus(write_done=True)
    assert s.CompletedTask(t, 4) == NoError
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.RequestHardShutdown()
    # the reference completes the previous sub-test's FIN task here (:1175): any untracked completion ends a
    # hard shutdown
    assert s.CompletedTask(final_fin, 0) == SuccessfullyCompleted
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0
    s.VerifyNoMoreIo()


def test_TestServerOverlappingMultipleIo():  # :1182-1236
    s = InitGracefulShutdownTest(300, Server)
    _overlapping(s)
    t = s.RequestSendStatus()
    assert s.CompletedTask(t, 100) == NoError  # an untracked task: its byte count is not checked
    assert not s.IsCompleted() and s.GetRemainingTransfer() == 0
    t = s.RequestFin()
    assert s.CompletedTask(t, 0) == SuccessfullyCompleted
    assert s.IsCompleted() and s.GetRemainingTransfer() == 0


# ---- beyond the MSTest project: UDP byte tracking and the FAIL_FAST latch -------------------------------
def test_udp_state_only_tracks_bytes():
    """UDP starts in MoreIo and completes when the confirmed bytes reach the transfer (ctsIOPatternState.hpp:108-114,
    :263-272, :346-354); any IO error fails it."""
    s = PatternState(300, Client, A.SHUTDOWN_GRACEFUL, protocol=A.PROTOCOL_UDP)
    assert s.GetNextPatternType() == A.PT_MORE_IO
    t = s._task(A.TASK_RECV, True, 150)
    s.NotifyNextTask(t)
    assert s.CompletedTask(t, 150) == NoError
    t = s._task(A.TASK_RECV, True, 150)
    s.NotifyNextTask(t)
    assert s.CompletedTask(t, 150) == SuccessfullyCompleted
    u = PatternState(300, Client, A.SHUTDOWN_GRACEFUL, protocol=A.PROTOCOL_UDP)
    assert u.UpdateError(5) == ErrorIoFailed and u.IsCompleted()


def test_inconsistent_completion_latches_fail_fast():
    """A completion of more bytes than were in flight is a FAIL_FAST in the reference
    (ctsIOPatternState.hpp:317-330): latched, and every later call fails."""
    s = InitGracefulShutdownTest(100, Server)
    t = s.RequestConnectionId()
    assert s.CompletedTask(t, ConnectionIdLength) == NoError
    t = s.RequestMoreIo(50)
    assert s.CompletedTask(t, 60) < 0
    assert lib().cts_io_pattern_state_fail_fast_reason(s.h)
    assert s.GetNextPatternType() < 0
