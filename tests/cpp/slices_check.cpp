// slices_check.cpp — cts_slices.hpp (one buffer verified as slices, results folded back) against the
// oracle's whole-buffer VerifyBuffer (ctsIOPattern.cpp:745-775): the oracle stands in for the kernel
// on every slice, and the folded result must equal the whole-buffer result field by field. Random
// lengths (0, below/at/above the slice minimum, ragged, up to 2^17), expected offsets and 0..3
// corrupted bytes (first / last byte of the buffer and slice edges included). Run by
// tests/test_host_sanitizers.py under ASan+UBSan and TSan; prints "slices: ok".
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "cts_oracle.h"
#include "cts_slices.hpp"

static_assert(sizeof(ora_desc) == sizeof(cts_buf_desc), "descriptor layouts differ");
static_assert(sizeof(ora_result) == sizeof(cts_verify_result), "result layouts differ");

static int verify(const std::vector<uint8_t>& arena, const cts_buf_desc* d, uint32_t n, cts_verify_result* r)
{
    return ora_verify_batch(arena.data(), arena.size(), reinterpret_cast<const ora_desc*>(d), n,
                            reinterpret_cast<ora_result*>(r), nullptr, nullptr, 0, 1);
}

int main()
{
    std::mt19937_64 rng(0x511CE5);
    const uint32_t lens[] = {0, 1, 15, 1023, 1024, 1025, 4096, 65535, 65536, 65537, 100000, 131072};
    const uint64_t base = 48;  // buffer not at arena offset 0
    int cases = 0;
    for (int it = 0; it < 3000; ++it) {
        const uint32_t len = it < 12 * 8 ? lens[it % 12] : (uint32_t)(rng() % 131073);
        const uint32_t expected = (uint32_t)(rng() % CTS_PATTERN_PERIOD);
        std::vector<uint8_t> arena(base + len + 64, 0xEE);
        cts_buf_desc whole{base, len, expected, 7, 0};
        ora_fill(arena.data(), arena.size(), reinterpret_cast<const ora_desc*>(&whole), 1);
        uint32_t slice_len = 0;
        cts_buf_desc sd[cts::kSliceMax];
        const uint32_t ns = cts::slice_plan(base, len, expected, 7, sd, &slice_len);
        if (ns < 1 || ns > cts::kSliceMax || (len > 0 && (uint64_t)(ns - 1) * slice_len >= len) ||
            (uint64_t)ns * slice_len < len || slice_len % 16 != 0) {
            std::fprintf(stderr, "bad plan: len %u -> %u x %u\n", len, ns, slice_len);
            return 1;
        }
        if (len) {
            const uint32_t nbad = (uint32_t)(rng() % 4);
            for (uint32_t k = 0; k < nbad; ++k) {
                uint32_t at;
                switch (rng() % 4) {
                    case 0: at = 0; break;
                    case 1: at = len - 1; break;
                    case 2: at = (uint32_t)((rng() % ns) * slice_len); at = at < len ? at : len - 1; break;
                    default: at = (uint32_t)(rng() % len);
                }
                arena[base + at] ^= (uint8_t)(1 + rng() % 255);
            }
        }
        cts_verify_result want{}, got_slices[cts::kSliceMax] = {};
        if (verify(arena, &whole, 1, &want) != 0 || verify(arena, sd, ns, got_slices) != 0) return 1;
        const cts_verify_result got = cts::slice_merge(got_slices, ns, slice_len, len);
        if (std::memcmp(&got, &want, sizeof(got)) != 0) {
            std::fprintf(stderr, "len %u exp %u: merged {%u %u %u %u %u %u} vs whole {%u %u %u %u %u %u}\n", len,
                         expected, got.first_mismatch, got.mismatch_bytes, got.expected, got.actual, got.pass,
                         got.flags, want.first_mismatch, want.mismatch_bytes, want.expected, want.actual, want.pass,
                         want.flags);
            return 1;
        }
        ++cases;
    }
    std::printf("slices: ok (%d cases)\n", cases);
    return 0;
}
