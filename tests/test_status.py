"""Status output: ctsTcpStatusInformation's header, legend and
status line (ctsTraffic/ctsPrintStatus.hpp:452-600) and the exit summary
(ctsTraffic.cpp:155-171). The header/legend strings are pinned by the reference
source; the README's sample run (README.md:119-141) supplies the values."""
from ctstraffic_amd import status as S

HEADER = " TimeSlice      SendBps      RecvBps  In-Flight  Completed  NetError  DataError \n"


def _expect(cols):
    """Independent layout: every value right-justified to end at its column offset (ctsPrintStatus.hpp:582-597)."""
    line = [" "] * 79
    for text, end in cols:
        for i, ch in enumerate(text):
            line[end - len(text) + i] = ch
    return "".join(line) + "\n"


def test_header_and_legend_are_the_reference_strings():
    assert S.header(S.CONSOLE) == HEADER
    assert S.header(S.CSV) == "TimeSlice,SendBps,RecvBps,In-Flight,Completed,NetError,DataError\r\n"
    assert S.header(S.CLEAR_TEXT) == HEADER[:-1] + "\r\n"
    leg = S.legend(S.CONSOLE)
    assert leg.startswith("Legend:\n* TimeSlice - (seconds) cumulative runtime\n")
    assert "* Data Errors - cumulative count of failed IO patterns due to data errors\n" in leg
    assert S.legend(S.CSV) == ""


def test_readme_sample_lines():
    # README.md:123-127: | 5.002 | 2635357062 | 124 | 8 | 8 | 0 | 0 | (5 s slices)
    got = S.line(S.CONSOLE, current_time_ms=5002, start_time_ms=0, end_time_ms=5000, bytes_sent=2635357062 * 5,
                 bytes_recv=124 * 5, active_connections=8, successful=8, connection_errors=0, protocol_errors=0)
    assert got == _expect([("5.002", 10), ("2635357062", 23), ("124", 36), ("8", 47), ("8", 58), ("0", 68), ("0", 79)])
    # the columns line up under the header's labels
    assert got.index("2635357062") + len("2635357062") == HEADER.index("SendBps") + len("SendBps")
    csv = S.line(S.CSV, current_time_ms=15001, start_time_ms=10000, end_time_ms=15000, bytes_sent=2437002784 * 5,
                 bytes_recv=202 * 5, active_connections=8, successful=32, connection_errors=0, protocol_errors=0)
    assert csv == "15.001,2437002784,202,8,32,0,0\r\n"


def test_wide_values_fall_back_to_exponent_notation():
    got = S.line(S.CONSOLE, current_time_ms=1000, start_time_ms=0, end_time_ms=1000, bytes_sent=123456789012,
                 bytes_recv=99999999999999, active_connections=1, successful=12345678, connection_errors=0,
                 protocol_errors=10 ** 13)
    assert got[23 - 11:23] == "123456.8x^6"  # 12 digits > 11 columns
    assert got[36 - 11:36] == "100000.0x^9"  # x^6 is still too wide
    assert got[58 - 7:58] == "12.3x^6"       # Completed column is 7 wide
    assert got[79 - 5:79] == "9+++T"         # does not fit even as x^12


def test_summary():
    s = S.summary(59, 0, 0, 5194, 67358818304)  # README.md:131-139
    assert "  SuccessfulConnections [59]   NetworkErrors [0]   ProtocolErrors [0]\n" in s
    assert "  Total Bytes Recv : 5194\n  Total Bytes Sent : 67358818304\n" in s


# ---- MSTest/ctsPrintStatusUnitTest/ctsPrintStatusUnitTest.cpp, replayed ----------------------------------
# ConnectionStatusDetails: In-Flight = active connections, Completed = successful, NetError = connection
# errors, DataError = protocol errors; TcpStatusDetails bytes and times are 0 (TestcaseInit, :24-37).
def _conn(v):
    return dict(active_connections=v, successful=v, connection_errors=v, protocol_errors=v)


def test_ctsTcpStatusInformationCsvAllZeroTest():  # :39-68
    assert S.header(S.CSV) == "TimeSlice,SendBps,RecvBps,In-Flight,Completed,NetError,DataError\r\n"
    assert S.legend(S.CSV) == ""  # nullptr
    assert S.line(S.CSV, current_time_ms=1000) == "1.000,0,0,0,0,0,0\r\n"
    assert S.line(S.CSV, current_time_ms=2000, **_conn(1)) == "2.000,0,0,1,1,1,1\r\n"


def test_ctsTcpStatusInformationConsoleOutputAllZeroTest():  # :70-96
    assert S.line(S.CONSOLE, current_time_ms=1000) == \
        "     1.000            0            0          0          0         0          0\n"
    assert S.line(S.CONSOLE, current_time_ms=2000, **_conn(1)) == \
        "     2.000            0            0          1          1         1          1\n"


def test_ctsTcpStatusInformationCsvMaxValueTest():  # :98-137
    assert S.line(S.CSV, current_time_ms=1000) == "1.000,0,0,0,0,0,0\r\n"
    assert S.line(S.CSV, current_time_ms=2000, **_conn(2**63 - 1)) == \
        "2.000,0,0,9223372036854775807,9223372036854775807,9223372036854775807,9223372036854775807\r\n"
    # UINT64_MAX: the CSV form prints the counters unsigned
    assert S.line(S.CSV, current_time_ms=3000, **_conn(-1)) == \
        "3.000,0,0,18446744073709551615,18446744073709551615,18446744073709551615,18446744073709551615\r\n"


def test_ctsTcpStatusInformationConsoleOutputMaxValueTest():  # :139-176
    assert S.line(S.CONSOLE, current_time_ms=2000, **_conn(2**63 - 1)) == \
        "     2.000            0            0      9+++T      9+++T     9+++T      9+++T\n"
    # "if we go greater than INT64_MAX, we will print -1 to the console. that's fine."
    assert S.line(S.CONSOLE, current_time_ms=3000, **_conn(-1)) == \
        "     3.000            0            0         -1         -1        -1         -1\n"


def test_ctsTcpStatusInformationConsoleOutputIterativeValuesTest():  # :178-392
    expect = {
        9: "          9          9         9          9",
        99: "         99         99        99         99",
        999: "        999        999       999        999",
        9999: "       9999       9999      9999       9999",
        99999: "      99999      99999     99999      99999",
        999999: "     999999     999999    999999     999999",
        9999999: "    9999999    9999999   9999999    9999999",
        99999999: "     0.1x^9     0.1x^9    0.1x^9     0.1x^9",
        999999999: "     1.0x^9     1.0x^9    1.0x^9     1.0x^9",
        9999999999: "    10.0x^9    10.0x^9   10.0x^9    10.0x^9",
        99999999999: "    0.1x^12    0.1x^12   0.1x^12    0.1x^12",
        999999999999: "    1.0x^12    1.0x^12   1.0x^12    1.0x^12",
    }
    for v in [9999999999999, 99999999999999, 999999999999999, 9999999999999999, 99999999999999999]:
        expect[v] = "      9+++T      9+++T     9+++T      9+++T"
    assert S.line(S.CONSOLE, current_time_ms=1000) == \
        "     1.000            0            0          0          0         0          0\n"
    t = 2000
    for v, cols in expect.items():
        got = S.line(S.CONSOLE, current_time_ms=t, **_conn(v))
        assert got == "%10.3f            0            0%s\n" % (t / 1000, cols), (v, got)
        t += 1000
