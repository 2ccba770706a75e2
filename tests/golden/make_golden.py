#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ — committed, small, deterministic.

This script is an INDEPENDENT pure-Python transcription of the reference's
pattern construction and verify semantics (it does not use oracle/ or the
product), so the C oracle and the HIP engine are both checked against it:

* ``ctsTraffic/ctsIOPattern.cpp:35-36``  c_bufferPatternSize = 0x10000,
  g_bufferPattern[c_bufferPatternSize * 2]
* ``ctsTraffic/ctsIOPattern.cpp:55-58``  u16 little-endian ramp 0..0xffff
* ``ctsTraffic/ctsIOPattern.cpp:60,72-80`` sender buffer = repeated copies of
  at most c_bufferPatternSize bytes of the table
* ``ctsTraffic/ctsIOPattern.cpp:753-774`` RtlCompareMemory prefix length,
  pass iff == transferred, printed expected/actual bytes
* ``ctsTraffic/ctsIOPattern.cpp:491-492,695-697`` offsets advance mod 65536

The reference itself cannot be built or run here (Windows-only, SURVEY.md
§8c), so byte values are pinned by its source; SURVEY.md §0.1 recorded the
byte known answers independently (first 16 bytes, bytes 65530..65541), which
this script asserts (the survey's FNV value is not reproducible; see below).

Run:  python tests/golden/make_golden.py   (rewrites pattern_kat.json, verify_vectors.json)
"""
from __future__ import annotations

import json
import os
import random
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
C_BUFFER_PATTERN_SIZE = 0xFFFF + 0x1


def build_table() -> bytes:
    # for (fillSlot = 0; fillSlot < c_bufferPatternSize; ++fillSlot)
    #     *(unsigned short*)&g_bufferPattern[fillSlot * 2] = (unsigned short)fillSlot;
    return b"".join(struct.pack("<H", slot & 0xFFFF) for slot in range(C_BUFFER_PATTERN_SIZE))


def build_sender(table: bytes, max_buffer_size: int) -> bytes:
    total = C_BUFFER_PATTERN_SIZE + max_buffer_size
    out = bytearray()
    remaining = total
    while remaining > 0:
        n = C_BUFFER_PATTERN_SIZE if remaining > C_BUFFER_PATTERN_SIZE else remaining
        out += table[:n]
        remaining -= n
    return bytes(out)


def rtl_compare_memory(a: bytes, b: bytes, n: int) -> int:
    for i in range(n):
        if a[i] != b[i]:
            return i
    return n


def fnv1a64(data: bytes) -> int:
    h = 0xCBF29CE484222325
    for x in data:
        h ^= x
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def verify(sender: bytes, buf: bytes, buffer_offset: int, expected: int, transferred: int) -> dict:
    pattern = sender[expected: expected + transferred]
    received = buf[buffer_offset: buffer_offset + transferred]
    matched = rtl_compare_memory(pattern, received, transferred)
    ok = matched == transferred
    return {
        "first_mismatch": matched,
        "pass": ok,
        "expected": 0 if ok else pattern[matched],
        "actual": 0 if ok else received[matched],
        "mismatch_bytes": sum(1 for i in range(transferred) if pattern[i] != received[i]),
    }


def main() -> None:
    table = build_table()
    assert len(table) == 2 * C_BUFFER_PATTERN_SIZE
    max_buf = 4096
    S = build_sender(table, max_buf)
    period = S[:C_BUFFER_PATTERN_SIZE]

    kat = {
        "source": "ctsTraffic/ctsIOPattern.cpp:35-36,55-60,72-80 (pure-Python transcription)",
        "period": C_BUFFER_PATTERN_SIZE,
        "first_16": S[:16].hex(),
        "bytes_65530_65541": S[65530:65542].hex(),
        "fnv1a64_one_period": "%016x" % fnv1a64(period),
        "fnv1a64_table_131072": "%016x" % fnv1a64(table),
        "sender_size_for_max_4096": len(S),
        "sender_fnv1a64_max_4096": "%016x" % fnv1a64(S),
        "probe_bytes": {str(p): S[p] for p in (0, 1, 2, 3, 510, 511, 512, 513, 32767, 32768, 65533, 65534, 65535,
                                                65536, 65537, 65536 + 4095)},
    }
    # SURVEY.md §0.1 known answers (recorded independently during the survey)
    assert kat["first_16"] == "00000100020003000400050006000700"
    assert kat["bytes_65530_65541"] == "fd7ffe7fff7f000001000200"
    # SURVEY.md §0.1 also quotes "FNV-1a-64 of one period = e5e9f74086d8f183"; standard FNV-1a-64
    # (basis 0xcbf29ce484222325, prime 0x100000001b3) over these 65536 bytes gives
    # 7337f32238221f25 instead, and no FNV-1/1a variant over the period, the table or the
    # sender buffer reproduces the survey's value, so that number is not used as a pin
    # (DESIGN.md "Parity pinning"). The byte-level KATs above agree with the survey.
    assert kat["fnv1a64_one_period"] == "7337f32238221f25"
    # S is periodic with period 65536 over its whole length
    assert all(S[i] == S[i % C_BUFFER_PATTERN_SIZE] for i in range(0, len(S), 7))

    with open(os.path.join(HERE, "pattern_kat.json"), "w") as f:
        json.dump(kat, f, indent=1, sort_keys=True)

    # ---- verify vectors: small buffers, every phase class, wrap, corruption ----
    rng = random.Random(0xC75)
    cases = []

    def add(name, buf, buffer_offset, expected, transferred):
        r = verify(S, buf, buffer_offset, expected, transferred)
        cases.append({"name": name, "buffer_hex": bytes(buf).hex(), "buffer_offset": buffer_offset,
                      "expected_offset": expected, "transferred": transferred, "result": r})

    # MSTest TestBaseClass_InvalidBytesOnRecv (ctsIOPatternUnitTest_Server.cpp:449-467):
    # 10-byte all-zero recv at expected offset 0 -> fails (pattern starts 00 00 01 00 ...)
    add("mstest_invalid_bytes_on_recv_zero10", bytes(10), 0, 0, 10)
    # MSTest TestBaseClass_SingleSuccessfulRecv_Server (:280-312): correct 10 bytes
    add("mstest_single_successful_recv_10", S[0:10], 0, 0, 10)
    # MSTest Duplex_Client_PartialRecv_RepostsRemainder (ctsIOPatternUnitTest_Duplex.cpp:592-622)
    add("mstest_duplex_partial_first4", S[0:10], 0, 0, 4)
    add("mstest_duplex_partial_remainder6_at4", S[4:10], 0, 4, 6)
    # empty verify: RtlCompareMemory(.., 0) == 0 -> pass
    add("empty", b"", 0, 0, 0)
    add("empty_at_offset", b"\x00" * 4, 4, 12345, 0)
    # wrap-around of the 64 KiB period
    for e in (65530, 65535, 65534, 65520, 65521):
        add("wrap_e%d" % e, S[e:e + 40], 0, e, 40)
    # UDP MediaStream datagram: 26-byte header then P[0..]
    hdr = struct.pack("<HqqQ", 0, 7, 0, 0)
    assert len(hdr) == 26
    add("udp_datagram_1472", hdr + S[0:1446], 26, 0, 1446)
    bad = bytearray(hdr + S[0:1446])
    bad[26 + 1000] ^= 0x5A
    add("udp_datagram_1472_corrupt_1000", bytes(bad), 26, 0, 1446)
    # random phases / lengths / offsets, half corrupted
    for i in range(40):
        e = rng.randrange(C_BUFFER_PATTERN_SIZE)
        n = rng.choice([1, 2, 3, 15, 16, 17, 31, 33, 64, 100, 255, 256, 257, 1000])
        off = rng.randrange(0, 20)
        buf = bytearray(rng.randrange(256) for _ in range(off)) + bytearray(S[e:e + n]) + bytearray(
            rng.randrange(256) for _ in range(rng.randrange(0, 5)))
        if i % 2 == 1 and n > 0:
            k = rng.randrange(n)
            buf[off + k] ^= rng.randrange(1, 256)
            if i % 4 == 3 and n > 2:
                k2 = rng.randrange(n)
                buf[off + k2] ^= 0xFF
        add("random_%02d" % i, bytes(buf), off, e, n)
    # high-bit bytes (>= 0x80) in the received data: the reference prints chars through %x
    add("high_byte_actual", bytes([0x00, 0x00, 0x81]), 0, 0, 3)

    # offset-advance scenarios (pattern-offset bookkeeping; ctsIOPattern.cpp:491-492, :695-697)
    streams = {
        # PushServer_VerifyingBuffersNotUsingSharedBuffer (Server.cpp:609-667): 10 x 1024 full recvs
        "push_server_10x1024": {"completions": [1024] * 10},
        # PushServer_..._SmallRecvs (Server.cpp:669-740): 9 x (post 2048, complete 1024) then 1024
        "push_server_small_recvs": {"completions": [1024] * 10},
        # Duplex partial recv: 4 then 6
        "duplex_partial": {"completions": [4, 6]},
        # wraps the 64 KiB period
        "wrap_stream": {"completions": [65000, 1000, 70000, 3, 65536, 65535]},
    }
    for v in streams.values():
        offs, o = [], 0
        for c in v["completions"]:
            offs.append(o)
            o = (o + c) % C_BUFFER_PATTERN_SIZE
        v["expected_offsets"] = offs
        v["final_offset"] = o

    with open(os.path.join(HERE, "verify_vectors.json"), "w") as f:
        json.dump({"source": "pure-Python RtlCompareMemory over ctsIOPattern.cpp:52-90 sender buffer",
                   "cases": cases, "streams": streams}, f, indent=0, sort_keys=True)
    print("wrote %d verify cases, %d streams" % (len(cases), len(streams)))


if __name__ == "__main__":
    main()
