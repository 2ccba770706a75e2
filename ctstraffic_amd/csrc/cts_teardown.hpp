// cts_teardown.hpp — how the loopback feeders end their patterns (cts_loopback.cpp, cts_loopback_udp.cpp).
#pragma once

#include <vector>

#include "cts_pattern.h"

namespace cts {

// cts_io_pattern_destroy, called again while it answers CTS_E_TIMEOUT (a kernel still reads the pattern's buffers;
// each call waits at most CTS_PATTERN_DESTROY_WAIT_MS), at most `tries` calls. Returns destroy's last status; a
// pattern still CTS_E_TIMEOUT after the last call stays allocated (left to the process rather than freed under the
// GPU's reads), and the caller reports the status.
inline int destroy_pattern(cts_io_pattern* p, int tries = 5)
{
    if (p == nullptr) return CTS_OK;
    int rc = CTS_E_TIMEOUT;
    for (int k = 0; k < tries && rc == CTS_E_TIMEOUT; ++k) rc = cts_io_pattern_destroy(p);
    return rc;
}

// Every pattern of a run, each destroyed whatever the others answered; the first failure is returned.
inline int destroy_patterns(const std::vector<cts_io_pattern*>& pats)
{
    int first = CTS_OK;
    for (cts_io_pattern* p : pats) {
        const int rc = destroy_pattern(p);
        if (first == CTS_OK && rc != CTS_OK) first = rc;
    }
    return first;
}

}  // namespace cts
