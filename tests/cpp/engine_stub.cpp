// engine_stub.cpp — link-time fakes for the device half of libcts_engine.so, so the host C++
// (cts_pattern.cpp, cts_media_stream.cpp, cts_status.cpp, cts_loopback.cpp) can be built with
// g++ under AddressSanitizer/UBSan/ThreadSanitizer on a machine without a GPU. This is how the
// reference's own MSTest projects replace ctsConfig (link-time fakes, no mocks).
// Every device entry point fails with CTS_E_NO_DEVICE; host allocations come from malloc.
// Used only by tests/test_host_sanitizers.py.
#include <cstdint>
#include <cstdlib>

#include <hip/hip_runtime_api.h>

#include "cts_engine.h"

extern "C" {

int cts_host_alloc(cts_engine*, uint64_t bytes, void** host_ptr, void** dev_view)
{
    if (host_ptr == nullptr || bytes == 0) return CTS_E_INVALID;
    void* p = std::aligned_alloc(64, (bytes + 63) & ~(uint64_t)63);
    if (p == nullptr) return CTS_E_NOMEM;
    *host_ptr = p;
    if (dev_view != nullptr) *dev_view = p;
    return CTS_OK;
}

int cts_host_free(cts_engine*, void* host_ptr)
{
    std::free(host_ptr);
    return CTS_OK;
}

int cts_sender_buffer_fill(cts_engine*, void*, uint32_t, void*) { return CTS_E_NO_DEVICE; }

int cts_verify(cts_engine*, const void*, uint64_t, const cts_buf_desc*, uint32_t, uint32_t, cts_verify_result*, void*,
               uint32_t*, uint32_t, void*)
{
    return CTS_E_NO_DEVICE;
}

int cts_verify_host(cts_engine*, const void*, uint32_t, uint32_t, cts_verify_result*) { return CTS_E_NO_DEVICE; }
int cts_verify_mapped(cts_engine*, const void*, uint32_t, uint32_t, cts_verify_result*) { return CTS_E_NO_DEVICE; }
int cts_engine_get_attr(const cts_engine*, int, int*) { return CTS_E_NO_DEVICE; }

int cts_engine_stream_create(cts_engine*, void**) { return CTS_E_NO_DEVICE; }
int cts_engine_stream_destroy(cts_engine*, void*) { return CTS_E_NO_DEVICE; }

hipError_t hipStreamSynchronize(hipStream_t) { return hipErrorNoDevice; }

}  // extern "C"
