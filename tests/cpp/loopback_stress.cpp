// loopback_stress.cpp — whole loopback connections (include/cts_loopback.h) for every TCP
// pattern and both functors, SYNC and DEFERRED verify, clean and with one flipped byte on the
// wire, with the oracle's C verifier as the pattern hook. Built by tests/test_host_sanitizers.py
// against the host sources under ASan/UBSan and under TSan (the async functor's send and recv
// threads share a pattern under the connection lock; TSan checks that every access is ordered).
#include <cstdio>
#include <vector>

#include "cts_loopback.h"
#include "cts_pattern.h"

extern "C" int ora_batch_verifier(void*, const uint8_t*, uint64_t, const cts_buf_desc*, uint32_t, cts_verify_result*);
extern "C" void ora_build_sender_buffer(uint8_t* dst, uint32_t max_buffer_size);

#define CHECK(c)                                                                        \
    do {                                                                                \
        if (!(c)) {                                                                     \
            std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

static int run(uint32_t pattern, uint32_t functor, uint32_t mode, bool corrupt)
{
    cts_loopback_config c{};
    c.connections = 3;
    c.io_pattern = pattern;
    c.buffer_size = 16384;
    c.verify_buffers = 1;
    c.transfer_size = 1024 * 1024 + 11;
    c.verify_mode = mode;
    c.batch_buffers = 8;
    c.corrupt_connection = corrupt ? 1u : ~0u;
    c.corrupt_send_index = 13;
    c.push_bytes = 40001;
    c.pull_bytes = 16385;
    c.functor = functor;
    cts_loopback_result r{};
    CHECK(cts_loopback_run(&c, nullptr, ora_batch_verifier, nullptr, &r) == CTS_OK);
    if (corrupt) {
        CHECK(r.data_errors == 1 && r.connections_ok == 2 && r.connections_failed == 1);
    } else {
        CHECK(r.data_errors == 0 && r.connections_ok == 3 && r.connections_failed == 0);
        // Duplex rounds an odd transfer up to even (ctsIoPatternDuplex ctor, ctsIOPattern.cpp:1000-1009)
        const uint64_t xfer = pattern == CTS_PATTERN_DUPLEX ? (c.transfer_size + 1) & ~1ull : c.transfer_size;
        CHECK(r.bytes_recv == 3ull * (xfer + CTS_CONNECTION_ID_LENGTH + 4));
    }
    return 0;
}

int main()
{
    std::vector<uint8_t> sender(CTS_PATTERN_PERIOD + 65536);
    ora_build_sender_buffer(sender.data(), 65536);
    CHECK(cts_shared_buffer_attach(sender.data(), sender.size()) == CTS_OK);
    const uint32_t patterns[] = {CTS_PATTERN_PUSH, CTS_PATTERN_PULL, CTS_PATTERN_PUSHPULL, CTS_PATTERN_DUPLEX};
    for (uint32_t pat : patterns)
        for (uint32_t functor : {CTS_LOOPBACK_FUNCTOR_SYNC, CTS_LOOPBACK_FUNCTOR_ASYNC})
            for (uint32_t mode : {CTS_VERIFY_SYNC, CTS_VERIFY_DEFERRED})
                for (bool corrupt : {false, true}) {
                    if (pat == CTS_PATTERN_DUPLEX && functor == CTS_LOOPBACK_FUNCTOR_SYNC) continue;
                    if (run(pat, functor, mode, corrupt) != 0) {
                        std::fprintf(stderr, "pattern %u functor %u mode %u corrupt %d\n", pat, functor, mode,
                                     (int)corrupt);
                        return 1;
                    }
                }
    std::printf("loopback_stress: ok\n");
    return 0;
}
