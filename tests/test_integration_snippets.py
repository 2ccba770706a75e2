"""INTEGRATION.md's reference-side bindings and call sequences compile against the real headers.

The C++ blocks of INTEGRATION.md that a ctsTraffic maintainer would paste (Level 1's InitOnceIoPatternCallback and
VerifyBuffer, the zero-copy VerifyBuffer, Level 2's ctsIoPatternGpu adapter) are extracted from the document and
compiled with g++ -fsyntax-only against include/, each in its own translation unit. The reference's own types and
macros they use are declared by a small prelude written here from their documented shapes (ctsIOTask.hpp:37-60,
ctsIOPattern.h:38-43 and :329, the Windows typedefs): it declares names, it compiles nothing of the reference. The
statement fragments (the device-resident sequence, the node counters, the MediaStream receive forms) are compiled as
the body of a function whose parameters declare their free variables. A renamed entry point or a changed argument
list in the ABI fails this test before it strands the document.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRELUDE = r"""
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
typedef int BOOL;
typedef void* PVOID;
typedef void* PINIT_ONCE;
typedef uintptr_t ULONG_PTR;
typedef struct RIO_BUFFERID_t* RIO_BUFFERID;
#define CALLBACK
#define TRUE 1
#define FAIL_FAST_IF(c) do { if (c) std::abort(); } while (0)
enum class ctsTaskAction : uint8_t { None, Send, Recv, GracefulShutdown, HardShutdown, Abort, FatalAbort };
enum class ctsIoStatus : uint32_t { ContinueIo, CompletedIo, FailedIo };
struct ctsTask {
    enum class BufferType : uint8_t { Null, TcpConnectionId, UdpConnectionId, CompletionMessage, Static, Dynamic };
    int64_t m_timeOffsetMilliseconds = 0;
    RIO_BUFFERID m_rioBufferid = nullptr;
    char* m_buffer = nullptr;
    uint32_t m_bufferLength = 0;
    uint32_t m_bufferOffset = 0;
    uint32_t m_expectedPatternOffset = 0;
    ctsTaskAction m_ioAction = ctsTaskAction::None;
    BufferType m_bufferType = BufferType::Null;
    bool m_trackIo = false;
};
struct ctsConfigSettings { bool ShouldVerifyBuffers = true; };
extern ctsConfigSettings* g_configSettings;
namespace ctsConfig {
uint32_t GetMaxBufferSize();
template <typename... A> void PrintErrorInfo(const wchar_t*, A...) {}
}
class ctsIoPattern {
public:
    static bool VerifyBuffer(const ctsTask& originalTask, uint32_t transferredBytes) noexcept;
};
extern char* g_senderSharedBuffer;
extern uint32_t g_maximumBufferSize;
extern const char* g_recvDeviceView;
extern const char* g_recvHostView;
#include "cts_pattern.h"
extern cts_engine* g_ctsEngine;
"""

# first line of each block -> drop the block's own `static cts_engine* g_ctsEngine` (the prelude declares it)
BLOCKS = {
    "level1_sender_buffer": "// ctsIOPattern.cpp — inside InitOnceIoPatternCallback",
    "level1_verify": "bool ctsIoPattern::VerifyBuffer(const ctsTask& originalTask, uint32_t transferredBytes) noexcept",
    "level2_adapter": "// ctsIOPatternGpu.h (new file in ctsTraffic/)",
    "zero_copy_verify": "bool ctsIoPattern::VerifyBuffer(const ctsTask& task, uint32_t transferred) noexcept",
}


def _blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8").read()
    return [code for lang, code in re.findall(r"```(\w*)\n(.*?)```", text, re.S) if lang == "cpp"]


@pytest.mark.parametrize("name", sorted(BLOCKS))
def test_integration_snippet_compiles(name):
    found = [c for c in _blocks() if c.startswith(BLOCKS[name])]
    assert len(found) == 1, "INTEGRATION.md lost the %s block" % name
    code = found[0].replace("static cts_engine* g_ctsEngine = nullptr;", "")
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, name + ".cpp")
        with open(src, "w", encoding="utf-8") as f:
            f.write(PRELUDE + "\n" + code)
        r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wno-unused-function",
                            "-I", os.path.join(ROOT, "include"), src], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]


# statement fragments: first line -> the parameters that declare their free variables
FRAGMENTS = {
    "device_resident": ("cts_engine* e;  cts_engine_create(dev, &e);",
                        "int dev, const void* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n, "
                        "cts_verify_result* results, uint32_t* conn_first_fail, uint32_t n_conns, hipStream_t stream"),
    "node_counters_prepare": ("// ctsTraffic.cpp, after the engines are created (one per GPU)",
                              "cts_engine** engines, uint32_t gpu_count"),
    "node_counters": ("// ctsConfig.cpp, where the status line reads g_configSettings->TcpStatusDetails",
                      "cts_engine* const* engines, const void* const* blocks, void* const* streams, uint32_t gpu_count, "
                      "bool rccl"),
    "media_stream_records": ("// descs[i] = {byte_offset of datagram i in the recv arena, completed bytes, 0, 0, 0}",
                             "const void* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n, "
                             "cts_datagram_record* records, cts_verify_result* results, void* counters, "
                             "hipStream_t stream, cts_media_stream_client* client, int64_t qpc_now, int64_t qpf"),
    "media_stream_statuses": ("// receive ring of n datagram slots of `stride` bytes",
                              "const void* dev_ring, uint64_t ring_bytes, uint32_t stride, const uint32_t* dev_lengths, "
                              "uint32_t n, cts_datagram_status* dev_status, void* dev_counters, hipStream_t stream, "
                              "cts_datagram_status* host_status, cts_media_stream_client* client, LARGE_INTEGER qpc, "
                              "int64_t qpf"),
    "media_stream_frames": ("cts_frame_window w;",
                            "const void* dev_ring, uint64_t ring_bytes, uint32_t stride, const uint32_t* dev_lengths, "
                            "uint32_t n, void* dev_totals, uint64_t* dev_frame_bytes, void* dev_counters, "
                            "hipStream_t stream, void* host_totals, uint64_t* host_frame_bytes, "
                            "cts_datagram_status* dev_status, cts_datagram_status* host_status, "
                            "cts_media_stream_client* client, LARGE_INTEGER qpc, int64_t qpf, uint32_t consumed"),
}

FRAGMENT_PRELUDE = r"""
#include <hip/hip_runtime_api.h>
#include "cts_engine.h"
#include "cts_media_stream.h"
typedef struct { int64_t QuadPart; } LARGE_INTEGER;
// ctsStatsTracking (ctsStatistics.hpp:87-198), ctsTcpStatistics / ctsConnectionStatistics and the two members of
// ctsConfigSettings the status line reads (ctsConfig.h:415-416): declared by shape only
struct ctsStatsTracking { void Add(int64_t) noexcept; void Increment() noexcept; int64_t GetValue() const noexcept; };
struct ctsTcpStatistics { ctsStatsTracking m_bytesSent, m_bytesRecv; };
struct ctsConnectionStatistics {
    ctsStatsTracking m_activeConnectionCount, m_successfulCompletionCount, m_connectionErrorCount, m_protocolErrorCount;
};
struct ctsConfigSettings { ctsConnectionStatistics ConnectionStatusDetails; ctsTcpStatistics TcpStatusDetails; };
extern ctsConfigSettings* g_configSettings;
extern cts_engine* g_ctsEngine;
"""


def _all_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8").read()
    return [code for lang, code in re.findall(r"```(\w*)\n(.*?)```", text, re.S) if lang in ("c", "cpp")]


@pytest.mark.parametrize("name", sorted(FRAGMENTS))
def test_integration_fragment_compiles(name):
    first, params = FRAGMENTS[name]
    found = [c for c in _all_blocks() if c.startswith(first)]
    assert len(found) == 1, "INTEGRATION.md lost the %s block" % name
    body = "\n".join(l for l in found[0].splitlines() if l.strip() != "...")  # an elision line, not code
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, name + ".cpp")
        with open(src, "w", encoding="utf-8") as f:
            f.write(FRAGMENT_PRELUDE + "\nvoid snippet(" + params + ")\n{\n" + body + "\n}\n")
        r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
                            "-I", os.path.join(ROOT, "include"), src], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
