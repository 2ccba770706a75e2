// pattern_replay.cpp — the C ABI used from C++ the way the reference's own MSTest
// drives ctsIoPattern (MSTest/ctsIOPatternUnitTest_Server/ctsIOPatternUnitTest_Server.cpp:
// TestBaseClass_SingleSuccessfulRecv_Server :280-312, TestBaseClass_InvalidBytesOnRecv
// :449-467), with the oracle's C verifier standing in for the GPU (no device here).
// Built and run by tests/test_cpp_abi.py; exits non-zero on the first failed check.
#include <cstdio>
#include <cstring>
#include <vector>

#include "cts_media_stream.h"
#include "cts_pattern.h"
#include "cts_status.h"

extern "C" int ora_batch_verifier(void*, const uint8_t*, uint64_t, const cts_buf_desc*, uint32_t, cts_verify_result*);
extern "C" void ora_build_sender_buffer(uint8_t* dst, uint32_t max_buffer_size);

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                     \
        }                                                                 \
    } while (0)

static cts_pattern_config server_defaults()
{
    cts_pattern_config c{};
    c.io_pattern = CTS_PATTERN_PUSH;
    c.protocol = CTS_PROTOCOL_TCP;
    c.listening = 1;
    c.verify_buffers = 1;
    c.pre_post_recvs = 1;
    c.pre_post_sends = 1;
    c.buffer_size_low = 1024;
    c.tcp_shutdown = CTS_SHUTDOWN_GRACEFUL;
    c.transfer_size = 10;
    return c;
}

static int single_recv(bool corrupt, uint32_t mode)
{
    cts_pattern_config cfg = server_defaults();
    cfg.verify_mode = mode;
    cts_io_pattern* p = nullptr;
    CHECK(cts_io_pattern_create(&cfg, nullptr, &p) == CTS_OK);
    CHECK(cts_io_pattern_set_verifier(p, ora_batch_verifier, nullptr) == CTS_OK);
    cts_task t{};
    CHECK(cts_io_pattern_initiate_io(p, &t) == CTS_OK);
    CHECK(t.buffer_length == CTS_CONNECTION_ID_LENGTH && t.io_action == CTS_TASK_SEND);
    CHECK(cts_io_pattern_complete_io(p, &t, CTS_CONNECTION_ID_LENGTH, 0) == CTS_IO_CONTINUE);
    CHECK(cts_io_pattern_initiate_io(p, &t) == CTS_OK);
    CHECK(t.buffer_length == 10 && t.io_action == CTS_TASK_RECV);
    if (corrupt) {
        std::memset(t.buffer, 0, t.buffer_length);  // ::ZeroMemory(test_task.m_buffer, ...)
        CHECK(cts_io_pattern_complete_io(p, &t, 10, 0) == CTS_IO_FAILED);
        CHECK(cts_io_pattern_last_error(p) == CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN);
        char msg[512];
        CHECK(cts_io_pattern_failure_message(p, msg, sizeof(msg)) > 0);
        CHECK(std::strstr(msg, "offset (2)") != nullptr);
    } else {
        // "recv" the correct bytes: memcpy(m_buffer, AccessSharedBuffer() + m_expectedPatternOffset, len)
        std::memcpy(t.buffer, cts_shared_buffer() + t.expected_pattern_offset, t.buffer_length);
        CHECK(cts_io_pattern_complete_io(p, &t, 10, 0) == CTS_IO_CONTINUE);
        CHECK(cts_io_pattern_initiate_io(p, &t) == CTS_OK);
        CHECK(t.io_action == CTS_TASK_SEND && t.buffer_length == CTS_COMPLETION_MESSAGE_SIZE);
        CHECK(std::memcmp(t.buffer, "DONE", 4) == 0);
        CHECK(cts_io_pattern_complete_io(p, &t, 4, 0) == CTS_IO_CONTINUE);
        CHECK(cts_io_pattern_initiate_io(p, &t) == CTS_OK);
        CHECK(t.io_action == CTS_TASK_RECV);
        CHECK(cts_io_pattern_complete_io(p, &t, 0, 0) == CTS_IO_COMPLETED);
        CHECK(cts_io_pattern_last_error(p) == 0);
    }
    cts_io_pattern_destroy(p);
    return 0;
}

int main()
{
    std::vector<uint8_t> sender(2 * 65536);
    ora_build_sender_buffer(sender.data(), 65536);
    CHECK(cts_shared_buffer_attach(sender.data(), sender.size()) == CTS_OK);
    for (uint32_t mode : {(uint32_t)CTS_VERIFY_SYNC, (uint32_t)CTS_VERIFY_DEFERRED}) {
        if (single_recv(false, mode)) return 1;
        if (single_recv(true, mode)) return 1;
    }
    uint32_t lens[4];
    CHECK(cts_media_stream_split(1401, 1400, lens, 4) == 2 && lens[0] + lens[1] == 1401);
    char line[256];
    CHECK(cts_status_tcp_header(CTS_STATUS_CSV, line, sizeof(line)) > 0);
    CHECK(std::strcmp(line, "TimeSlice,SendBps,RecvBps,In-Flight,Completed,NetError,DataError\r\n") == 0);
    cts_shared_buffer_release();
    std::puts("pattern_replay: ok");
    return 0;
}
