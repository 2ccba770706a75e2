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

}  // extern "C"
