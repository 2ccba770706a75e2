// cts_engine.cpp — the C ABI (include/cts_engine.h) over the gfx950 kernels.
//
// Every entry point is noexcept and returns a cts_status, mirroring the
// reference's noexcept IO surface (ctsIOPattern.h:143-144) while replacing its
// FAIL_FAST process aborts with error codes a foreign caller can handle.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "cts_engine.h"
#include "cts_internal.hpp"
#include "cts_slices.hpp"

struct cts_engine {
    int device = 0;
    cts::LaunchGeometry geo;
    std::mutex host_mu;  // serialises the single-buffer host path (shared staging)
    hipStream_t stream = nullptr;
    // single-buffer host staging: pinned, device-mapped (zero-copy reads over PCIe)
    uint8_t* stage = nullptr;
    size_t stage_cap = 0;
    cts_buf_desc* stage_desc = nullptr;       // pinned, device-mapped
    cts_verify_result* stage_res = nullptr;   // pinned, device-mapped
    // cts_verify_host_batch staging (pinned, device-mapped), grown on demand and kept
    void* batch_desc = nullptr;
    size_t batch_desc_cap = 0;
    void* batch_res = nullptr;
    size_t batch_res_cap = 0;
    void* batch_ctr = nullptr;
    // cts_verify_mapped: concurrent SYNC verifies combined into one launch (flat combining)
    std::mutex comb_mu;
    std::condition_variable comb_cv;
    std::vector<struct cts_sync_req*> comb_q;  // waiting for the next launch
    bool comb_busy = false;
    int sync_coalesce = 0;  // CTS_ATTR_SYNC_COALESCE (read by cts_pattern's SYNC verify)
    // a leader owns comb_stream and the comb_* staging
    hipStream_t comb_stream = nullptr;
    void* comb_desc = nullptr;
    size_t comb_desc_cap = 0;
    void* comb_res = nullptr;
    size_t comb_res_cap = 0;
};

// One caller of cts_verify_mapped: its buffer, and its answer once `done`.
struct cts_sync_req {
    const uint8_t* dev;
    uint32_t len;
    uint32_t expected;
    cts_verify_result out;
    int rc;
    bool done;
};

namespace {

int env_int(const char* name, int dflt)
{
    const char* v = std::getenv(name);
    if (v == nullptr || *v == 0) return dflt;
    return std::atoi(v);
}

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = (prev == dev) || (hipSetDevice(dev) == hipSuccess);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

inline int hip_status(hipError_t e) { return e == hipSuccess ? CTS_OK : CTS_E_HIP; }

// Pinned host memory that the device reads directly (hipHostMalloc memory is
// mapped into the device address space).
int host_alloc_mapped(size_t bytes, void** out)
{
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return CTS_E_NOMEM;
    *out = p;
    return CTS_OK;
}

template <typename T>
T* device_view(T* host)
{
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) return nullptr;
    return static_cast<T*>(d);
}

// Grow a pinned, device-mapped staging area to >= bytes (powers of two from `floor`).
int ensure_pinned(void** p, size_t* cap, size_t bytes, size_t floor)
{
    if (*cap >= bytes && *p != nullptr) return CTS_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    size_t c = floor;
    while (c < bytes) c <<= 1;
    const int rc = host_alloc_mapped(c, p);
    if (rc != CTS_OK) return rc;
    *cap = c;
    return CTS_OK;
}

int ensure_stage(cts_engine* e, size_t bytes)
{
    void* p = e->stage;
    const int rc = ensure_pinned(&p, &e->stage_cap, bytes, 1u << 20);
    e->stage = static_cast<uint8_t*>(p);
    return rc;
}

// The leader's half of cts_verify_mapped: every request of `batch` as slices of one launch.
// Descriptors address the group relative to its lowest buffer (one flat device address range:
// mapped pinned host memory and HBM share the GPU's virtual address space; only the described
// bytes are read). Per-request verdicts fold back with slice_merge, so each caller gets exactly
// what a launch of its own would have returned (ctsIOPattern.cpp:745-775).
void run_sync_group(cts_engine* e, const std::vector<cts_sync_req*>& batch)
{
    int rc = CTS_OK;
    DeviceGuard g(e->device);
    if (!g.ok) rc = CTS_E_HIP;
    if (rc == CTS_OK && e->comb_stream == nullptr &&
        hipStreamCreateWithFlags(&e->comb_stream, hipStreamNonBlocking) != hipSuccess) {
        e->comb_stream = nullptr;
        rc = CTS_E_HIP;
    }
    const size_t maxd = (size_t)cts::kSliceMax * batch.size();
    if (rc == CTS_OK) rc = ensure_pinned(&e->comb_desc, &e->comb_desc_cap, maxd * sizeof(cts_buf_desc), 4096);
    if (rc == CTS_OK) rc = ensure_pinned(&e->comb_res, &e->comb_res_cap, maxd * sizeof(cts_verify_result), 4096);
    std::vector<uint32_t> first(batch.size()), count(batch.size()), slen(batch.size());
    if (rc == CTS_OK) {
        const uint8_t* base = batch[0]->dev;
        const uint8_t* end = batch[0]->dev + batch[0]->len;
        for (const cts_sync_req* r : batch) {
            base = std::min(base, r->dev);
            end = std::max(end, r->dev + r->len);
        }
        base -= reinterpret_cast<uintptr_t>(base) & 15u;  // the kernels align loads from a 16-B arena base
        auto* hd = static_cast<cts_buf_desc*>(e->comb_desc);
        uint32_t nd = 0, maxsl = 0;
        for (size_t i = 0; i < batch.size(); ++i) {
            first[i] = nd;
            count[i] = cts::slice_plan((uint64_t)(batch[i]->dev - base), batch[i]->len, batch[i]->expected,
                                       (uint32_t)i, hd + nd, &slen[i]);
            nd += count[i];
            maxsl = std::max(maxsl, slen[i]);
        }
        const cts_buf_desc* dd = device_view(hd);
        cts_verify_result* dr = device_view(static_cast<cts_verify_result*>(e->comb_res));
        hipError_t err = (dd && dr) ? cts::launch_verify(base, (uint64_t)(end - base), dd, nd, maxsl, dr, nullptr,
                                                         nullptr, 0, e->comb_stream, e->geo)
                                    : hipErrorInvalidValue;
        if (err == hipSuccess) err = hipStreamSynchronize(e->comb_stream);
        if (err != hipSuccess) rc = CTS_E_HIP;
    }
    const auto* res = static_cast<const cts_verify_result*>(e->comb_res);
    for (size_t i = 0; i < batch.size(); ++i) {
        batch[i]->rc = rc;
        if (rc == CTS_OK) batch[i]->out = cts::slice_merge(res + first[i], count[i], slen[i], batch[i]->len);
    }
}

}  // namespace

extern "C" {

#if CTS_TUNING
#define cts_variant_count(k) cts::k
const char* cts_version(void) { return "ctstraffic_amd 0.2.0 (gfx950, tuning build: every launch variant)"; }
#else
#define cts_variant_count(k) 0
const char* cts_version(void) { return "ctstraffic_amd 0.2.0 (gfx950)"; }
#endif

const char* cts_status_string(int status)
{
    switch (status) {
    case CTS_OK: return "ok";
    case CTS_E_INVALID: return "invalid argument";
    case CTS_E_HIP: return "HIP runtime error";
    case CTS_E_NOMEM: return "out of memory";
    case CTS_E_NO_DEVICE: return "no such HIP device";
    default: return "unknown status";
    }
}

int cts_engine_create(int device, cts_engine** out)
{
    if (out == nullptr) return CTS_E_INVALID;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return CTS_E_NO_DEVICE;
    if (device < 0 || device >= count) return CTS_E_NO_DEVICE;
    DeviceGuard g(device);
    if (!g.ok) return CTS_E_HIP;
    cts_engine* e = new (std::nothrow) cts_engine();
    if (e == nullptr) return CTS_E_NOMEM;
    e->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
        e->geo.num_cus = cus;
    e->geo.blocks_per_cu = env_int("CTS_BLOCKS_PER_CU", e->geo.blocks_per_cu);
    e->geo.nontemporal = env_int("CTS_NT_LOADS", e->geo.nontemporal);
    e->geo.small_threshold = env_int("CTS_SMALL_THRESHOLD", e->geo.small_threshold);
    e->geo.verify_variant = env_int("CTS_VERIFY_VARIANT", e->geo.verify_variant);
    e->geo.small_blocks_per_cu = env_int("CTS_SMALL_BLOCKS_PER_CU", e->geo.small_blocks_per_cu);
    e->geo.small_variant = env_int("CTS_SMALL_VARIANT", e->geo.small_variant);
    e->geo.fill_blocks_per_cu = env_int("CTS_FILL_BLOCKS_PER_CU", e->geo.fill_blocks_per_cu);
    e->geo.ms_variant = env_int("CTS_MS_VARIANT", e->geo.ms_variant);
    e->geo.small_chunk = env_int("CTS_SMALL_CHUNK", e->geo.small_chunk);
    e->geo.fill_nt = env_int("CTS_FILL_NT", e->geo.fill_nt);
    // a variant this build does not compile falls back to the default (the product build has one per path)
    if (!cts::variant_ok(e->geo.verify_variant, cts::kDefaultVerifyVariant, cts_variant_count(kVerifyVariants)))
        e->geo.verify_variant = cts::kDefaultVerifyVariant;
    if (!cts::variant_ok(e->geo.small_variant, cts::kDefaultSmallVariant, cts_variant_count(kSmallVariants)))
        e->geo.small_variant = cts::kDefaultSmallVariant;
    if (!cts::variant_ok(e->geo.ms_variant, cts::kDefaultMediaStreamVariant, cts_variant_count(kMediaStreamVariants)))
        e->geo.ms_variant = cts::kDefaultMediaStreamVariant;
    e->sync_coalesce = env_int("CTS_SYNC_COALESCE", e->sync_coalesce) ? 1 : 0;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return CTS_E_HIP;
    }
    void* p = nullptr;
    if (host_alloc_mapped(cts::kSliceMax * sizeof(cts_buf_desc), &p) != CTS_OK) {
        cts_engine_destroy(e);
        return CTS_E_NOMEM;
    }
    e->stage_desc = static_cast<cts_buf_desc*>(p);
    if (host_alloc_mapped(cts::kSliceMax * sizeof(cts_verify_result), &p) != CTS_OK) {
        cts_engine_destroy(e);
        return CTS_E_NOMEM;
    }
    e->stage_res = static_cast<cts_verify_result*>(p);
    *out = e;
    return CTS_OK;
}

int cts_engine_destroy(cts_engine* e)
{
    if (e == nullptr) return CTS_E_INVALID;
    {
        DeviceGuard g(e->device);
        if (e->stream) {
            (void)hipStreamSynchronize(e->stream);
            (void)hipStreamDestroy(e->stream);
        }
        if (e->stage) (void)hipHostFree(e->stage);
        if (e->stage_desc) (void)hipHostFree(e->stage_desc);
        if (e->stage_res) (void)hipHostFree(e->stage_res);
        if (e->batch_desc) (void)hipHostFree(e->batch_desc);
        if (e->batch_res) (void)hipHostFree(e->batch_res);
        if (e->batch_ctr) (void)hipHostFree(e->batch_ctr);
        if (e->comb_stream) {
            (void)hipStreamSynchronize(e->comb_stream);
            (void)hipStreamDestroy(e->comb_stream);
        }
        if (e->comb_desc) (void)hipHostFree(e->comb_desc);
        if (e->comb_res) (void)hipHostFree(e->comb_res);
    }
    delete e;
    return CTS_OK;
}

int cts_engine_device(const cts_engine* e) { return e ? e->device : CTS_E_INVALID; }

int cts_engine_stream_create(cts_engine* e, void** stream)
{
    if (e == nullptr || stream == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return CTS_E_HIP;
    *stream = s;
    return CTS_OK;
}

int cts_engine_stream_destroy(cts_engine* e, void* stream)
{
    if (e == nullptr || stream == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    return hip_status(hipStreamDestroy(static_cast<hipStream_t>(stream)));
}

int cts_engine_set_attr(cts_engine* e, int attr, int value)
{
    if (e == nullptr) return CTS_E_INVALID;
    switch (attr) {
    case CTS_ATTR_BLOCKS_PER_CU:
        if (value < 1 || value > 64) return CTS_E_INVALID;
        e->geo.blocks_per_cu = value;
        return CTS_OK;
    case CTS_ATTR_NT_LOADS: e->geo.nontemporal = value ? 1 : 0; return CTS_OK;
    case CTS_ATTR_SMALL_THRESHOLD:
        if (value < 0) return CTS_E_INVALID;
        e->geo.small_threshold = value;
        return CTS_OK;
    case CTS_ATTR_VERIFY_VARIANT:
        if (!cts::variant_ok(value, cts::kDefaultVerifyVariant, cts_variant_count(kVerifyVariants))) return CTS_E_INVALID;
        e->geo.verify_variant = value;
        return CTS_OK;
    case CTS_ATTR_SMALL_BLOCKS_PER_CU:
        if (value < 1 || value > 256) return CTS_E_INVALID;
        e->geo.small_blocks_per_cu = value;
        return CTS_OK;
    case CTS_ATTR_SMALL_VARIANT:
        if (!cts::variant_ok(value, cts::kDefaultSmallVariant, cts_variant_count(kSmallVariants))) return CTS_E_INVALID;
        e->geo.small_variant = value;
        return CTS_OK;
    case CTS_ATTR_FILL_BLOCKS_PER_CU:
        if (value < 1 || value > 64) return CTS_E_INVALID;
        e->geo.fill_blocks_per_cu = value;
        return CTS_OK;
    case CTS_ATTR_MS_VARIANT:
        if (!cts::variant_ok(value, cts::kDefaultMediaStreamVariant, cts_variant_count(kMediaStreamVariants)))
            return CTS_E_INVALID;
        e->geo.ms_variant = value;
        return CTS_OK;
    case CTS_ATTR_SMALL_CHUNK:
        if (value < 0 || value > (1 << 24)) return CTS_E_INVALID;
        e->geo.small_chunk = value;
        return CTS_OK;
    case CTS_ATTR_SYNC_COALESCE: e->sync_coalesce = value ? 1 : 0; return CTS_OK;
    case CTS_ATTR_FILL_NT:
        if (value < 0 || value > 2) return CTS_E_INVALID;
        e->geo.fill_nt = value;
        return CTS_OK;
    default: return CTS_E_INVALID;
    }
}

int cts_engine_get_attr(const cts_engine* e, int attr, int* value)
{
    if (e == nullptr || value == nullptr) return CTS_E_INVALID;
    switch (attr) {
    case CTS_ATTR_BLOCKS_PER_CU: *value = e->geo.blocks_per_cu; return CTS_OK;
    case CTS_ATTR_NT_LOADS: *value = e->geo.nontemporal; return CTS_OK;
    case CTS_ATTR_SMALL_THRESHOLD: *value = e->geo.small_threshold; return CTS_OK;
    case CTS_ATTR_VERIFY_VARIANT: *value = e->geo.verify_variant; return CTS_OK;
    case CTS_ATTR_SMALL_BLOCKS_PER_CU: *value = e->geo.small_blocks_per_cu; return CTS_OK;
    case CTS_ATTR_SMALL_VARIANT: *value = e->geo.small_variant; return CTS_OK;
    case CTS_ATTR_FILL_BLOCKS_PER_CU: *value = e->geo.fill_blocks_per_cu; return CTS_OK;
    case CTS_ATTR_MS_VARIANT: *value = e->geo.ms_variant; return CTS_OK;
    case CTS_ATTR_SMALL_CHUNK: *value = e->geo.small_chunk; return CTS_OK;
    case CTS_ATTR_FILL_NT: *value = e->geo.fill_nt; return CTS_OK;
    case CTS_ATTR_SYNC_COALESCE: *value = e->sync_coalesce; return CTS_OK;
    default: return CTS_E_INVALID;
    }
}

int cts_sender_buffer_fill(cts_engine* e, void* dev_dst, uint32_t max_buffer_size, void* stream)
{
    if (e == nullptr || dev_dst == nullptr || ((uintptr_t)dev_dst & 15u) != 0) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_fill_span(static_cast<uint8_t*>(dev_dst), cts_sender_buffer_size(max_buffer_size), 0,
                                            static_cast<hipStream_t>(stream), e->geo));
}

int cts_fill(cts_engine* e, void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs, uint32_t n,
             uint32_t max_length_hint, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || ((uintptr_t)dev_arena & 15u) != 0) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_fill(static_cast<uint8_t*>(dev_arena), arena_bytes, dev_descs, n, max_length_hint,
                                       static_cast<hipStream_t>(stream), e->geo));
}

int cts_verify(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs, uint32_t n,
               uint32_t max_length_hint, cts_verify_result* dev_results, void* dev_counters,
               uint32_t* dev_conn_first_fail, uint32_t n_conns, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || ((uintptr_t)dev_arena & 15u) != 0) return CTS_E_INVALID;
    if (dev_conn_first_fail == nullptr && n_conns != 0) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_verify(static_cast<const uint8_t*>(dev_arena), arena_bytes, dev_descs, n,
                                         max_length_hint, dev_results, static_cast<uint64_t*>(dev_counters),
                                         dev_conn_first_fail, n_conns, static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_fill(cts_engine* e, void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs,
                          const cts_datagram_header* dev_headers, uint32_t n, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || dev_headers == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_fill(static_cast<uint8_t*>(dev_arena), arena_bytes, dev_descs,
                                                    dev_headers, n, static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_verify(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs,
                            uint32_t n, cts_datagram_record* dev_records, cts_verify_result* dev_results,
                            void* dev_counters, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || ((uintptr_t)dev_arena & 15u) != 0) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_verify(static_cast<const uint8_t*>(dev_arena), arena_bytes, dev_descs,
                                                      n, dev_records, dev_results,
                                                      static_cast<uint64_t*>(dev_counters),
                                                      static_cast<hipStream_t>(stream), e->geo));
}

size_t cts_counters_device_bytes(void) { return (size_t)CTS_COUNTER_SHARDS * cts::kCounterSlots * sizeof(uint64_t); }

int cts_counters_reset(cts_engine* e, void* dev_counters, void* stream)
{
    if (e == nullptr || dev_counters == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(hipMemsetAsync(dev_counters, 0, cts_counters_device_bytes(), static_cast<hipStream_t>(stream)));
}

int cts_counters_read(cts_engine* e, const void* dev_counters, cts_counters* out, void* stream)
{
    if (e == nullptr || dev_counters == nullptr || out == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    std::vector<uint64_t> h(CTS_COUNTER_SHARDS * cts::kCounterSlots);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (hipMemcpyAsync(h.data(), dev_counters, cts_counters_device_bytes(), hipMemcpyDeviceToHost, s) != hipSuccess)
        return CTS_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return CTS_E_HIP;
    uint64_t v[5] = {0, 0, 0, 0, 0};
    for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh)
        for (int k = 0; k < 5; ++k) v[k] += h[sh * cts::kCounterSlots + k];
    out->bytes_checked = v[cts::kBytesChecked];
    out->bytes_ok = v[cts::kBytesOk];
    out->buffers_checked = v[cts::kBuffersChecked];
    out->buffers_failed = v[cts::kBuffersFailed];
    out->mismatched_bytes = v[cts::kMismatchedBytes];
    return CTS_OK;
}

int cts_host_alloc(cts_engine* e, uint64_t bytes, void** host_ptr, void** dev_view)
{
    if (e == nullptr || host_ptr == nullptr || bytes == 0) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    void* p = nullptr;
    const int rc = host_alloc_mapped((size_t)((bytes + 15u) & ~(uint64_t)15u), &p);
    if (rc != CTS_OK) return rc;
    *host_ptr = p;
    if (dev_view != nullptr) {
        void* d = nullptr;
        if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
            (void)hipHostFree(p);
            *host_ptr = nullptr;
            return CTS_E_HIP;
        }
        *dev_view = d;
    }
    return CTS_OK;
}

int cts_host_free(cts_engine* e, void* host_ptr)
{
    if (e == nullptr || host_ptr == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    return hip_status(hipHostFree(host_ptr));
}

int cts_host_device_pointer(void* host_ptr, void** dev_view)
{
    if (host_ptr == nullptr || dev_view == nullptr) return CTS_E_INVALID;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, host_ptr, 0) != hipSuccess) return CTS_E_INVALID;
    *dev_view = d;
    return CTS_OK;
}

int cts_verify_host(cts_engine* e, const void* host_buf, uint32_t len, uint32_t expected_offset, cts_verify_result* out)
{
    if (e == nullptr || out == nullptr || (host_buf == nullptr && len != 0)) return CTS_E_INVALID;
    if (expected_offset >= CTS_PATTERN_PERIOD) return CTS_E_INVALID;
    std::lock_guard<std::mutex> lk(e->host_mu);
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    int rc = ensure_stage(e, (size_t)len + 16);
    if (rc != CTS_OK) return rc;
    if (len) std::memcpy(e->stage, host_buf, len);
    // latency-bound single buffer: verified as up to cts::kSliceMax slices read at once (cts_slices.hpp)
    uint32_t slice_len = 0;
    const uint32_t ns = cts::slice_plan(0, len, expected_offset, 0, e->stage_desc, &slice_len);
    const uint8_t* arena = device_view(e->stage);
    const cts_buf_desc* dd = device_view(e->stage_desc);
    cts_verify_result* dr = device_view(e->stage_res);
    if (!arena || !dd || !dr) return CTS_E_HIP;
    hipError_t err = cts::launch_verify(arena, e->stage_cap, dd, ns, slice_len, dr, nullptr, nullptr, 0, e->stream,
                                        e->geo);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return CTS_E_HIP;
    *out = cts::slice_merge(e->stage_res, ns, slice_len, len);
    return CTS_OK;
}

int cts_verify_host_batch(cts_engine* e, const void* const* bufs, const uint32_t* lens, const uint32_t* expected,
                          const uint32_t* skip_heads, uint32_t n, cts_verify_result* results, cts_counters* counters)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (bufs == nullptr || lens == nullptr || expected == nullptr || results == nullptr) return CTS_E_INVALID;
    std::lock_guard<std::mutex> lk(e->host_mu);
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    // Stage every buffer into one pinned, device-mapped arena (16-byte aligned
    // slots), describe it, verify it in place over PCIe, read results.
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (bufs[i] == nullptr && lens[i] != 0) return CTS_E_INVALID;
        total += ((uint64_t)lens[i] + 15u) & ~(uint64_t)15u;
    }
    int rc = ensure_stage(e, (size_t)total + 16);
    if (rc != CTS_OK) return rc;
    if ((rc = ensure_pinned(&e->batch_desc, &e->batch_desc_cap, sizeof(cts_buf_desc) * n, 4096)) != CTS_OK) return rc;
    if ((rc = ensure_pinned(&e->batch_res, &e->batch_res_cap, sizeof(cts_verify_result) * n, 4096)) != CTS_OK) return rc;
    if (counters && e->batch_ctr == nullptr &&
        (rc = host_alloc_mapped(cts_counters_device_bytes(), &e->batch_ctr)) != CTS_OK)
        return rc;
    void* const pres = e->batch_res;
    void* const pctr = counters ? e->batch_ctr : nullptr;
    cts_buf_desc* hd = static_cast<cts_buf_desc*>(e->batch_desc);
    uint64_t off = 0;
    uint32_t maxlen = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (lens[i]) std::memcpy(e->stage + off, bufs[i], lens[i]);
        hd[i].byte_offset = off;
        hd[i].length = lens[i];
        hd[i].expected_pattern_offset = expected[i];
        hd[i].conn_index = i;
        hd[i].skip_head = skip_heads ? skip_heads[i] : 0u;
        maxlen = lens[i] > maxlen ? lens[i] : maxlen;
        off += ((uint64_t)lens[i] + 15u) & ~(uint64_t)15u;
    }
    if (pctr) std::memset(pctr, 0, cts_counters_device_bytes());
    hipError_t err = cts::launch_verify(device_view(e->stage), e->stage_cap, device_view(hd), n, maxlen,
                                        device_view(static_cast<cts_verify_result*>(pres)),
                                        pctr ? device_view(static_cast<uint64_t*>(pctr)) : nullptr, nullptr, 0,
                                        e->stream, e->geo);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err == hipSuccess) {
        std::memcpy(results, pres, sizeof(cts_verify_result) * n);
        if (counters) {
            const uint64_t* h = static_cast<const uint64_t*>(pctr);
            for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh) {
                counters->bytes_checked += h[sh * cts::kCounterSlots + cts::kBytesChecked];
                counters->bytes_ok += h[sh * cts::kCounterSlots + cts::kBytesOk];
                counters->buffers_checked += h[sh * cts::kCounterSlots + cts::kBuffersChecked];
                counters->buffers_failed += h[sh * cts::kCounterSlots + cts::kBuffersFailed];
                counters->mismatched_bytes += h[sh * cts::kCounterSlots + cts::kMismatchedBytes];
            }
        }
    }
    return err == hipSuccess ? CTS_OK : CTS_E_HIP;
}

int cts_verify_mapped(cts_engine* e, const void* dev_buf, uint32_t len, uint32_t expected_offset,
                      cts_verify_result* out)
{
    if (e == nullptr || out == nullptr || (dev_buf == nullptr && len != 0)) return CTS_E_INVALID;
    if (expected_offset >= CTS_PATTERN_PERIOD) return CTS_E_INVALID;
    cts_sync_req me{static_cast<const uint8_t*>(dev_buf), len, expected_offset, cts_verify_result{}, CTS_OK, false};
    std::unique_lock<std::mutex> lk(e->comb_mu);
    e->comb_q.push_back(&me);
    while (!me.done) {
        if (e->comb_busy) {
            e->comb_cv.wait(lk);
            continue;
        }
        // leader: take everyone queued so far (callers that arrive during this launch form the next one)
        e->comb_busy = true;
        std::vector<cts_sync_req*> batch;
        batch.swap(e->comb_q);
        lk.unlock();
        run_sync_group(e, batch);
        lk.lock();
        for (cts_sync_req* r : batch) r->done = true;
        e->comb_busy = false;
        e->comb_cv.notify_all();
    }
    *out = me.out;
    return me.rc;
}

}  // extern "C"
