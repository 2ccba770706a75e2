// cts_host_util.cpp — the pure host helpers of the C ABI (include/cts_engine.h): no HIP calls,
// so the host-side sanitizer builds (tests/test_host_sanitizers.py) link them as they are.
#include <stdint.h>

#include "cts_engine.h"

extern "C" {

uint8_t cts_pattern_byte(uint64_t stream_offset)
{
    const uint32_t j = (uint32_t)(stream_offset & 0xFFFFu);
    return (uint8_t)((j & 1u) ? (j >> 9) : ((j >> 1) & 0xFFu));
}

uint64_t cts_sender_buffer_size(uint32_t max_buffer_size) { return (uint64_t)CTS_PATTERN_PERIOD + max_buffer_size; }

uint32_t cts_shard_of(uint32_t x, uint32_t n_shards)
{
    if (n_shards <= 1) return 0;
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x % n_shards;
}

// ctsStatsTracking summed over the node's GPUs (ctsStatistics.hpp:87-198): one process drives one engine per
// GPU (the reference is one process per host, ctsSocketBroker), so the process-wide counters are the host-side
// sum of every engine's device block. Each block is read on its engine's device (cts_counters_read_ex).
int cts_counters_read_multi_ex(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                               uint32_t n, cts_counters_ex* out)
{
    if (out == nullptr || (n > 0 && (engines == nullptr || dev_counters == nullptr))) return CTS_E_INVALID;
    cts_counters_ex sum{0, 0, 0, 0, 0, 0};
    for (uint32_t i = 0; i < n; ++i) {
        if (engines[i] == nullptr || dev_counters[i] == nullptr) return CTS_E_INVALID;
        cts_counters_ex c{};
        const int rc = cts_counters_read_ex(engines[i], dev_counters[i], &c, streams ? streams[i] : nullptr);
        if (rc != CTS_OK) return rc;
        sum.bytes_checked += c.bytes_checked;
        sum.bytes_ok += c.bytes_ok;
        sum.buffers_checked += c.buffers_checked;
        sum.buffers_failed += c.buffers_failed;
        sum.mismatched_bytes += c.mismatched_bytes;
        sum.connections_failed += c.connections_failed;
    }
    *out = sum;
    return CTS_OK;
}

int cts_counters_read_multi(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                            uint32_t n, cts_counters* out)
{
    if (out == nullptr) return CTS_E_INVALID;
    cts_counters_ex x{};
    const int rc = cts_counters_read_multi_ex(engines, dev_counters, streams, n, &x);
    if (rc == CTS_OK)
        *out = cts_counters{x.bytes_checked, x.bytes_ok, x.buffers_checked, x.buffers_failed, x.mismatched_bytes};
    return rc;
}

}  // extern "C"
