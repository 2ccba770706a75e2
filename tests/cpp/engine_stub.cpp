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
#include "cts_internal.hpp"
#include "cts_media_stream.h"

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

int cts_media_stream_verify_frames(cts_engine*, const void*, uint64_t, const cts_buf_desc*, uint32_t,
                                   const cts_frame_window*, void*, uint64_t*, void*, void*)
{
    return CTS_E_NO_DEVICE;
}
int cts_media_stream_verify_status(cts_engine*, const void*, uint64_t, const cts_buf_desc*, uint32_t,
                                   cts_datagram_status*, void*, void*)
{
    return CTS_E_NO_DEVICE;
}

int cts_verify_host(cts_engine*, const void*, uint32_t, uint32_t, cts_verify_result*) { return CTS_E_NO_DEVICE; }
int cts_verify_mapped(cts_engine*, const void*, uint32_t, uint32_t, cts_verify_result*) { return CTS_E_NO_DEVICE; }
uint64_t cts_mailbox_launches(const cts_engine*) { return 0; }
int cts_engine_get_attr(const cts_engine*, int, int*) { return CTS_E_NO_DEVICE; }

int cts_engine_stream_create(cts_engine*, void**) { return CTS_E_NO_DEVICE; }
int cts_engine_stream_destroy(cts_engine*, void*) { return CTS_E_NO_DEVICE; }

// The HIP runtime calls the host code makes, all failing. Weak: a driver that needs a working fake device
// (counters_fold.cpp: host memory standing in for device memory) defines its own.
#define CTS_STUB __attribute__((weak))
CTS_STUB hipError_t hipStreamSynchronize(hipStream_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipMallocAsync(void**, size_t, hipStream_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipMemsetAsync(void*, int, size_t, hipStream_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipFreeAsync(void*, hipStream_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipMemcpyAsync(void*, const void*, size_t, hipMemcpyKind, hipStream_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipEventCreateWithFlags(hipEvent_t*, unsigned) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipEventQuery(hipEvent_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipEventSynchronize(hipEvent_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipEventDestroy(hipEvent_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipMalloc(void**, size_t) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipFree(void*) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipGetDevice(int*) { return hipErrorNoDevice; }
CTS_STUB hipError_t hipSetDevice(int) { return hipErrorNoDevice; }
CTS_STUB int cts_engine_device(const cts_engine*) { return CTS_E_NO_DEVICE; }

// A "device" counter block here is host memory with the device layout (CTS_COUNTER_SHARDS shards of 8 u64,
// the first kCounterCount used), so the host-side fold of cts_counters_read_multi can be driven without a GPU.
int cts_counters_read_ex(cts_engine* e, const void* dev_counters, cts_counters_ex* out, void*)
{
    if (e == nullptr || dev_counters == nullptr || out == nullptr) return CTS_E_INVALID;
    const uint64_t* h = static_cast<const uint64_t*>(dev_counters);
    uint64_t v[cts::kCounterCount] = {};
    for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh)
        for (int k = 0; k < cts::kCounterCount; ++k) v[k] += h[sh * 8 + k];
    *out = cts::counters_ex_of(v);
    return CTS_OK;
}
int cts_counters_read(cts_engine* e, const void* dev_counters, cts_counters* out, void* s)
{
    if (out == nullptr) return CTS_E_INVALID;
    cts_counters_ex x{};
    const int rc = cts_counters_read_ex(e, dev_counters, &x, s);
    if (rc == CTS_OK) *out = cts::counters_of(x);
    return rc;
}

}  // extern "C"

namespace cts {
// the device fold of cts_counters_allreduce (cts_collective.cpp); counters_fold.cpp defines a host one
CTS_STUB hipError_t launch_counters_fold(const void*, uint64_t*, bool, hipStream_t) { return hipErrorNoDevice; }
}  // namespace cts
