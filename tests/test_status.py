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
