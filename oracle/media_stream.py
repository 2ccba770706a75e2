"""Pure-Python restatement of the MediaStream host logic — TEST INFRASTRUCTURE ONLY.

Checker for the product's C++ (ctstraffic_amd/csrc/cts_media_stream.cpp):

* :func:`split` — ctsMediaStreamSendRequests::iterator (ctsTraffic/ctsMediaStreamProtocol.hpp:151-205)
* :class:`ClientModel` — ctsIoPatternMediaStreamClient: constructor (ctsIOPatternMediaStream.cpp:46-96),
  CompleteTaskBackToPattern (:140-272), FindSequenceNumber (:280-300), ReceivedBufferedFrames (:302-318),
  RenderFrame (:360-414), TimerCallback (:470-530) with one call per timer tick.
"""
from __future__ import annotations

HEADER = 26  # c_udpDatagramDataHeaderLength
NOT_ALL_DATA = 2147483646  # c_statusErrorNotAllDataTransferred
DATA_MISMATCH = 2147483644  # c_statusErrorDataDidNotMatchBitPattern
RUNNING = 2147483647


def split(frame_bytes: int, max_datagram: int) -> list:
    if frame_bytes <= HEADER:
        return []

    def update(bytes_to_send):  # UpdateBufferLength
        if bytes_to_send > max_datagram:
            payload = max_datagram - HEADER
        else:
            payload = bytes_to_send - HEADER
        total = HEADER + payload
        remaining = bytes_to_send - total
        if 0 < remaining <= HEADER:
            delta = HEADER + 1 - remaining
            total -= delta
        return total

    out = []
    b = frame_bytes
    b -= (first := update(b))  # iterator constructor
    out.append(first)
    while b != 0:  # operator++: end() once m_bytesToSend == 0
        n = update(b)
        out.append(n)
        b -= n
    return out


class ClientModel:
    def __init__(self, frame_size, buffered_frames, stream_length_frames):
        self.frame_size = frame_size
        self.final = stream_length_frames
        self.initial = min(stream_length_frames, buffered_frames)
        self.wheel = self.initial
        q = 2 * self.initial
        assert q >= 2
        self.seq = list(range(1, q + 1))
        self.bytes = [0] * q
        self.head = 0
        self.finished = 0
        self.last_error = RUNNING
        self.bits = self.ok = self.dropped = self.dup = self.err = 0
        self.datagrams = 0
        self.fail_datagram = None

    def _latch(self, e):
        if self.last_error == RUNNING:
            self.last_error = e

    def _find(self, s):
        hs = self.seq[self.head]
        tail = hs + len(self.seq) - 1
        vend = self.seq[-1]
        if s > tail or s < hs:
            return None
        if s <= vend:
            return self.head + (s - hs)
        return s - vend - 1

    def complete(self, kind, seq, completed, passed):
        """One datagram (kind 0 data, 1 id, 2 zero, 3 short, 4 unknown, 5 bad). Returns True while running."""
        if self.last_error != RUNNING:
            return False
        self.datagrams += 1
        err = 0
        if kind == 2:
            if not self.finished:
                err = NOT_ALL_DATA
        elif kind in (3, 4, 5):
            err = NOT_ALL_DATA
        elif kind == 0:
            if not passed:
                err = DATA_MISMATCH
            else:
                self.bits += completed * 8
                if seq > self.final:
                    self.err += 1
                else:
                    slot = self._find(seq)
                    if slot is None:
                        self.err += 1
                    else:
                        self.bytes[slot] += completed
        if err:
            self._latch(err)
            self.fail_datagram = self.datagrams - 1
        return self.last_error == RUNNING

    def _received_buffered(self):
        return self.seq[0] > 1 or self.head != 0 or any(b > 0 for b in self.bytes)

    def render(self):
        if self.finished:
            return self.finished
        self.wheel += 1
        if self.wheel >= self.initial and self.seq[self.head] <= self.final:
            if not self._received_buffered():
                self.dropped += self.final
                self.finished = 2
                self._latch(NOT_ALL_DATA)
                return 2
            b = self.bytes[self.head]
            if b == self.frame_size:
                self.ok += 1
            elif b < self.frame_size:
                self.dropped += 1
            else:
                self.dup += 1
            self.seq[self.head] += len(self.seq)
            self.bytes[self.head] = 0
            self.head = (self.head + 1) % len(self.seq)
        if self.seq[self.head] <= self.final:
            return 0
        self.finished = 1
        self._latch(0)
        return 1

    def stats(self):
        return {"bits_received": self.bits, "successful_frames": self.ok, "dropped_frames": self.dropped,
                "duplicate_frames": self.dup, "error_frames": self.err, "datagrams": self.datagrams,
                "last_error": self.last_error, "finished": self.finished,
                "head_sequence_number": self.seq[self.head]}
