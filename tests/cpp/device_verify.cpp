// device_verify.cpp — the headline path from C++ with no Python in the process: a maintainer's
// device-resident use of the C ABI (INTEGRATION.md "Device-resident use"). hipMalloc'd arena,
// descriptors built on the host, cts_fill as the sender, one flipped byte per corrupted buffer,
// cts_verify with results + counters + per-connection first failure, checked against the known
// corruption plan. Built by `make` (ctstraffic_amd/build/device_verify) and run by
// tests/test_cpp_abi.py::test_cpp_device_verify on the GPU box. Exits non-zero on a failed check.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "cts_engine.h"

#define CHECK(c)                                                                        \
    do {                                                                                \
        if (!(c)) {                                                                     \
            std::fprintf(stderr, "%s:%d CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

int main()
{
    cts_engine* e = nullptr;
    CHECK(cts_engine_create(0, &e) == CTS_OK);
    void* stream = nullptr;
    CHECK(cts_engine_stream_create(e, &stream) == CTS_OK);
    hipStream_t s = static_cast<hipStream_t>(stream);

    // 64 connections x 16 buffers of ragged lengths, packed connection-major at 16-byte-aligned
    // slots; expected offsets = per-connection prefix sums mod 65536 (ctsIOPattern.cpp:491-492)
    const uint32_t conns = 64, per = 16, n = conns * per;
    std::vector<cts_buf_desc> d(n);
    uint64_t off = 0;
    for (uint32_t c = 0; c < conns; ++c) {
        uint32_t stream_off = 0;
        for (uint32_t k = 0; k < per; ++k) {
            const uint32_t i = c * per + k;
            const uint32_t len = 1 + (i * 2654435761u) % 70000u;
            d[i] = cts_buf_desc{off, len, stream_off, c, 0};
            stream_off = (stream_off + len) % CTS_PATTERN_PERIOD;
            off += (len + 15u) & ~15u;
        }
    }
    const uint64_t arena_bytes = off;
    void *arena = nullptr, *descs = nullptr, *results = nullptr, *ctr = nullptr, *cff = nullptr;
    CHECK(hipMalloc(&arena, arena_bytes) == hipSuccess);
    CHECK(hipMalloc(&descs, n * sizeof(cts_buf_desc)) == hipSuccess);
    CHECK(hipMalloc(&results, n * sizeof(cts_verify_result)) == hipSuccess);
    CHECK(hipMalloc(&ctr, cts_counters_device_bytes()) == hipSuccess);
    CHECK(hipMalloc(&cff, conns * sizeof(uint32_t)) == hipSuccess);
    CHECK(hipMemcpyAsync(descs, d.data(), n * sizeof(cts_buf_desc), hipMemcpyHostToDevice, s) == hipSuccess);
    CHECK(hipMemsetAsync(cff, 0xFF, conns * sizeof(uint32_t), s) == hipSuccess);
    CHECK(cts_counters_reset(e, ctr, stream) == CTS_OK);
    CHECK(cts_fill(e, arena, arena_bytes, static_cast<cts_buf_desc*>(descs), n, 0, stream) == CTS_OK);

    // corrupt one byte in every 7th buffer, at a buffer-dependent position
    std::vector<uint32_t> bad_at(n, ~0u);
    uint64_t bad_bytes = 0, bad_buffers = 0;
    for (uint32_t i = 0; i < n; i += 7) {
        const uint32_t p = (i * 40503u) % d[i].length;
        uint8_t* b = static_cast<uint8_t*>(arena) + d[i].byte_offset + p;
        uint8_t v = 0;
        CHECK(hipMemcpyAsync(&v, b, 1, hipMemcpyDeviceToHost, s) == hipSuccess);
        CHECK(hipStreamSynchronize(s) == hipSuccess);
        CHECK(v == cts_pattern_byte(d[i].expected_pattern_offset + p));  // the fill wrote the pattern
        v ^= 0xA5;
        CHECK(hipMemcpyAsync(b, &v, 1, hipMemcpyHostToDevice, s) == hipSuccess);
        bad_at[i] = p;
        ++bad_buffers;
        bad_bytes += d[i].length;
    }
    CHECK(cts_verify(e, arena, arena_bytes, static_cast<cts_buf_desc*>(descs), n, 65536,
                     static_cast<cts_verify_result*>(results), ctr, static_cast<uint32_t*>(cff), conns, stream) == CTS_OK);
    std::vector<cts_verify_result> r(n);
    std::vector<uint32_t> first_fail(conns);
    CHECK(hipMemcpyAsync(r.data(), results, n * sizeof(cts_verify_result), hipMemcpyDeviceToHost, s) == hipSuccess);
    CHECK(hipMemcpyAsync(first_fail.data(), cff, conns * sizeof(uint32_t), hipMemcpyDeviceToHost, s) == hipSuccess);
    cts_counters c{};
    CHECK(cts_counters_read(e, ctr, &c, stream) == CTS_OK);  // synchronises the stream

    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        total += d[i].length;
        if (bad_at[i] == ~0u) {
            CHECK(r[i].pass == 1 && r[i].first_mismatch == d[i].length && r[i].mismatch_bytes == 0);
        } else {
            const uint32_t p = bad_at[i];
            const uint8_t exp = cts_pattern_byte(d[i].expected_pattern_offset + p);
            CHECK(r[i].pass == 0 && r[i].first_mismatch == p && r[i].mismatch_bytes == 1);
            CHECK(r[i].expected == exp && r[i].actual == (uint8_t)(exp ^ 0xA5));
        }
    }
    for (uint32_t cc = 0; cc < conns; ++cc) {
        uint32_t want = ~0u;
        for (uint32_t k = 0; k < per && want == ~0u; ++k)
            if (bad_at[cc * per + k] != ~0u) want = cc * per + k;
        CHECK(first_fail[cc] == want);
    }
    CHECK(c.bytes_checked == total && c.buffers_checked == n && c.buffers_failed == bad_buffers);
    CHECK(c.bytes_ok == total - bad_bytes && c.mismatched_bytes == bad_buffers);

    // the node's counters as ctsTraffic's one-process host reads them (ctsConfig.h:415-417): the host fold and the
    // RCCL all-reduce over every engine's device (one here), both through the C ABI
    cts_engine* const engines[1] = {e};
    const void* const blocks[1] = {ctr};
    void* const streams[1] = {stream};
    // the RCCL clique built first, as ctsTraffic's start-up would (the status timer reads at t = 0)
    CHECK(cts_counters_allreduce_prepare(engines, 1) == CTS_OK);
    cts_allreduce_setup st{};
    CHECK(cts_counters_allreduce_setup_times(&st) == CTS_OK && st.prepared == 1 && st.devices == 1);
    cts_counters folded{}, reduced{};
    CHECK(cts_counters_read_multi(engines, blocks, streams, 1, &folded) == CTS_OK);
    const int ar = cts_counters_allreduce(engines, blocks, streams, 1, &reduced);
    CHECK(ar == CTS_OK);
    CHECK(std::memcmp(&folded, &c, sizeof(c)) == 0 && std::memcmp(&reduced, &c, sizeof(c)) == 0);
    // with the DataError count: one per connection holding a corrupted buffer (ctsSocketState.cpp:221-228)
    uint64_t failed_conns = 0;
    for (uint32_t cc = 0; cc < conns; ++cc) failed_conns += first_fail[cc] != ~0u;
    cts_counters_ex cx{}, fx{}, rx{};
    CHECK(cts_counters_read_ex(e, ctr, &cx, stream) == CTS_OK);
    CHECK(cts_counters_read_multi_ex(engines, blocks, streams, 1, &fx) == CTS_OK);
    CHECK(cts_counters_allreduce_ex(engines, blocks, streams, 1, &rx) == CTS_OK);
    CHECK(failed_conns > 0 && cx.connections_failed == failed_conns);
    CHECK(std::memcmp(&cx, &fx, sizeof(cx)) == 0 && std::memcmp(&cx, &rx, sizeof(cx)) == 0);
    CHECK(cx.bytes_checked == c.bytes_checked && cx.buffers_failed == c.buffers_failed);
    CHECK(cts_counters_allreduce_release() == CTS_OK);

    CHECK(hipFree(arena) == hipSuccess && hipFree(descs) == hipSuccess && hipFree(results) == hipSuccess);
    CHECK(hipFree(ctr) == hipSuccess && hipFree(cff) == hipSuccess);
    CHECK(cts_engine_stream_destroy(e, stream) == CTS_OK);
    CHECK(cts_engine_destroy(e) == CTS_OK);
    std::printf("device_verify: ok (%u buffers, %llu bytes, %llu corrupted, %llu connections failed)\n", n,
                (unsigned long long)total, (unsigned long long)bad_buffers, (unsigned long long)failed_conns);
    return 0;
}
