// engine_devices.cpp — the engine's C ABI (cts_engine.cpp) on a fake eight-device HIP runtime, built with g++ under
// the host sanitizers (tests/test_host_sanitizers.py). The test box has one GPU, so every engine on device g > 0
// runs only here: each entry point must make the engine's device current for every HIP call and launch it makes
// (DeviceGuard) and give the caller its own device back, on the caller's thread, the watchdog thread and
// concurrent callers alike.
//
// The fake runtime keeps a current device per thread, gives every stream and event the device current at its
// creation, and counts a violation whenever a stream-ordered call (launch, memset, copy, event record, stream
// synchronize or destroy) runs with another device current. The SYNC mailbox's resident grid
// (cts::launch_mailbox) is emulated by a host thread that polls the slot rings exactly as mailbox_kernel does
// (tags, no-op jobs, stop jobs, the idle exit; on demand a job left unanswered) and verifies each job; the event
// recorded after it completes when that thread has left, and hipHostFree counts a violation when it would wait
// on a running grid (the reason Pause exists). The verify and fill launches compute what the kernels do with the
// oracle (oracle/cts_oracle.c), so verdicts are checked as well as devices, and whole loopback TCP connections
// (cts_loopback_run_multi, SYNC and DEFERRED patterns, clean and corrupt) run over eight engines: their IO threads
// start on device 0, as new threads do, and drive patterns on every device, and MediaStream connections (SYNC, and
// DEFERRED through an emulated frame-sum pass) with their client timer threads on device 0. cts_counters_allreduce
// (cts_collective.cpp) then reduces nine engines' counter blocks over a stub RCCL (argv[1]), and bench.py's
// single-process leg (tools/bench_multi.cpp) runs one native launch thread per engine on eight devices.
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "cts_engine.h"
#include "cts_internal.hpp"
#include "cts_loopback.h"
#include "cts_media_stream.h"
#include "cts_oracle.h"
#include "cts_pattern.h"

namespace {

constexpr int kDevices = 8;
thread_local int t_cur = 0;

std::atomic<int> g_violations{0};
std::atomic<int> g_launches[kDevices];
std::atomic<int> g_grids{0};  // emulated mailbox grids started
std::atomic<int> g_drop_jobs{0};  // the emulated grids leave this many verify jobs unanswered (a lost job)
std::atomic<int> g_async_us{0};
std::atomic<int> g_not_ready{0};  // event queries that found work still in flight   // > 0: a verify launch completes this long after it was enqueued, on its own thread
std::mutex g_grid_mu;
std::vector<std::shared_ptr<std::atomic<bool>>> g_grid_done;  // every grid's done flag, in launch order

void violation(const char* what, int want, int have)
{
    std::fprintf(stderr, "violation: %s on device %d with device %d current\n", what, want, have);
    g_violations.fetch_add(1);
}

}  // namespace

// The runtime's opaque handles, defined by the fake. A stream runs its asynchronous work (an emulated mailbox grid,
// a verify launch while g_async_us > 0) each on a thread of its own that first waits for every earlier item of the
// stream, so the stream stays in order; its synchronous operations wait for the items before them.
using Done = std::shared_ptr<std::atomic<bool>>;
struct ihipStream_t {
    int device;
    std::mutex mu;
    std::vector<std::pair<Done, std::thread>> items;  // enqueued work, oldest first (finished ones reaped)
};
struct ihipEvent_t {
    int device;
    std::mutex mu;
    std::vector<Done> waits;  // the stream's work when recorded
};

namespace {

std::mutex g_mu;                 // guards g_streams, g_pinned and every null stream
std::set<ihipStream_t*> g_streams;
std::set<void*> g_pinned;
ihipStream_t g_null[kDevices];   // the null stream of each device
const bool g_null_init = [] {
    for (int d = 0; d < kDevices; ++d) g_null[d].device = d;
    return true;
}();

ihipStream_t* stream_of(hipStream_t s) { return s ? s : &g_null[t_cur]; }

void check_stream(const char* what, hipStream_t s)
{
    const ihipStream_t* st = stream_of(s);
    if (st->device != t_cur) violation(what, st->device, t_cur);
}

// an emulated grid still running on a stream of `dev` (what hipDeviceSynchronize of `dev` would wait for); -1: any
bool grid_running(int dev)
{
    std::lock_guard<std::mutex> lk(g_mu);
    auto busy = [](ihipStream_t* st) {
        std::lock_guard<std::mutex> l2(st->mu);
        for (auto& w : st->items)
            if (!w.first->load(std::memory_order_acquire)) return true;
        return false;
    };
    for (ihipStream_t* st : g_streams)
        if ((dev < 0 || st->device == dev) && busy(st)) return true;
    for (int d = 0; d < kDevices; ++d)
        if ((dev < 0 || d == dev) && busy(&g_null[d])) return true;
    return false;
}

void join_stream(ihipStream_t* st)
{
    std::vector<std::pair<Done, std::thread>> items;
    {
        std::lock_guard<std::mutex> lk(st->mu);
        items.swap(st->items);
    }
    for (auto& w : items) w.second.join();
}

std::vector<Done> pending(ihipStream_t* st)
{
    std::vector<Done> w;
    std::lock_guard<std::mutex> lk(st->mu);
    for (auto& x : st->items)
        if (!x.first->load(std::memory_order_acquire)) w.push_back(x.first);
    return w;
}

void wait_for(const std::vector<Done>& w)
{
    for (auto& d : w)
        while (!d->load(std::memory_order_acquire)) std::this_thread::sleep_for(std::chrono::microseconds(10));
}

// a synchronous operation on a stream: after everything enqueued before it
void in_order(hipStream_t s) { wait_for(pending(stream_of(s))); }

// asynchronous work on a stream: runs after everything enqueued before it
template <typename F>
Done enqueue(ihipStream_t* st, F body)
{
    auto done = std::make_shared<std::atomic<bool>>(false);
    std::lock_guard<std::mutex> lk(st->mu);
    std::vector<Done> before;
    for (auto it = st->items.begin(); it != st->items.end();) {
        if (it->first->load(std::memory_order_acquire)) {  // finished: reap
            it->second.join();
            it = st->items.erase(it);
        } else {
            before.push_back(it->first);
            ++it;
        }
    }
    std::thread t([before, body, done]() mutable {
        wait_for(before);
        body();
        done->store(true, std::memory_order_release);
    });
    st->items.emplace_back(done, std::move(t));
    return done;
}

}  // namespace

extern "C" {

hipError_t hipGetDeviceCount(int* count)
{
    *count = kDevices;
    return hipSuccess;
}
hipError_t hipGetDevice(int* d)
{
    *d = t_cur;
    return hipSuccess;
}
hipError_t hipSetDevice(int d)
{
    if (d < 0 || d >= kDevices) return hipErrorInvalidDevice;
    t_cur = d;
    return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t attr, int dev)
{
    if (dev < 0 || dev >= kDevices) return hipErrorInvalidDevice;
    *v = attr == hipDeviceAttributeMultiprocessorCount ? 256 : 0;
    return hipSuccess;
}
hipError_t hipDeviceGetPCIBusId(char* bus, int len, int dev)
{
    if (dev < 0 || dev >= kDevices) return hipErrorInvalidDevice;
    std::snprintf(bus, (size_t)len, "0000:FF:%02X.0", dev);  // no such PCI device: numa node -1
    return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int)
{
    ihipStream_t* st = new ihipStream_t();
    st->device = t_cur;
    std::lock_guard<std::mutex> lk(g_mu);
    g_streams.insert(st);
    *s = st;
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s)
{
    if (s == nullptr) return hipErrorInvalidHandle;
    check_stream("hipStreamDestroy", s);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_streams.erase(s) == 0) return hipErrorInvalidHandle;
    }
    join_stream(s);
    delete s;
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s)
{
    check_stream("hipStreamSynchronize", s);
    join_stream(stream_of(s));
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned)
{
    ihipEvent_t* ev = new ihipEvent_t();
    ev->device = t_cur;
    *e = ev;
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s)
{
    check_stream("hipEventRecord", s);
    ihipStream_t* st = stream_of(s);
    if (st->device != e->device) violation("hipEventRecord (event of another device)", e->device, st->device);
    std::vector<Done> w = pending(st);
    std::lock_guard<std::mutex> lk(e->mu);
    e->waits.swap(w);
    return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e)
{
    std::lock_guard<std::mutex> lk(e->mu);
    for (auto& w : e->waits)
        if (!w->load(std::memory_order_acquire)) {
            g_not_ready.fetch_add(1);
            return hipErrorNotReady;
        }
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e)
{
    delete e;
    return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t bytes, unsigned int)
{
    *p = std::aligned_alloc(64, (bytes + 63) & ~(size_t)63);
    if (*p == nullptr) return hipErrorOutOfMemory;
    std::memset(*p, 0, bytes);
    std::lock_guard<std::mutex> lk(g_mu);
    g_pinned.insert(*p);
    return hipSuccess;
}
hipError_t hipHostFree(void* p)
{
    // the runtime's free is an implicit hipDeviceSynchronize of the current device: a resident grid still polling
    // there would hold it up for as long as that grid's callers keep posting
    if (grid_running(t_cur)) violation("hipHostFree while a mailbox grid runs on the current device", t_cur, t_cur);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_pinned.erase(p) == 0) return hipErrorInvalidValue;
    }
    std::free(p);
    return hipSuccess;
}
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int)
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (void* b : g_pinned)  // (a handful of allocations: a scan is fine)
        if (b == h) {
            *d = h;  // portable mapped memory: the same address on every device
            return hipSuccess;
        }
    return hipErrorInvalidValue;
}
hipError_t hipMemsetAsync(void* dst, int v, size_t bytes, hipStream_t s)
{
    check_stream("hipMemsetAsync", s);
    in_order(s);
    std::memset(dst, v, bytes);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t bytes, hipMemcpyKind, hipStream_t s)
{
    check_stream("hipMemcpyAsync", s);
    in_order(s);
    std::memcpy(dst, src, bytes);
    return hipSuccess;
}
hipError_t hipMallocAsync(void** p, size_t bytes, hipStream_t s)
{
    check_stream("hipMallocAsync", s);
    *p = std::calloc(1, bytes);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFreeAsync(void* p, hipStream_t s)
{
    check_stream("hipFreeAsync", s);
    in_order(s);
    std::free(p);
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e)
{
    while (hipEventQuery(e) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(20));
    return hipSuccess;
}

// std::condition_variable::wait_for (the mailbox watchdog) waits in pthread_cond_clockwait, which this
// toolchain's ThreadSanitizer does not intercept: it would miss the wait's unlock and report a double lock. The
// driver routes it to pthread_cond_timedwait (intercepted) with the same deadline.
int pthread_cond_clockwait(pthread_cond_t* c, pthread_mutex_t* m, clockid_t clk, const struct timespec* abs)
{
    struct timespec now_c, now_r;
    clock_gettime(clk, &now_c);
    clock_gettime(CLOCK_REALTIME, &now_r);
    int64_t left = (int64_t)(abs->tv_sec - now_c.tv_sec) * 1000000000 + (abs->tv_nsec - now_c.tv_nsec);
    if (left < 0) left = 0;
    const int64_t t = (int64_t)now_r.tv_sec * 1000000000 + now_r.tv_nsec + left;
    struct timespec dl;
    dl.tv_sec = t / 1000000000;
    dl.tv_nsec = t % 1000000000;
    return pthread_cond_timedwait(c, m, &dl);
}

}  // extern "C"

// ---- the launchers: record the device, write clean records ---------------------------------------------------
namespace cts {
namespace {

// a launch: counted on its stream's device; the synchronous fakes run after the stream's earlier work
void launched(const char* what, hipStream_t s, bool sync = true)
{
    check_stream(what, s);
    g_launches[stream_of(s)->device].fetch_add(1);
    if (sync) in_order(s);
}

static_assert(sizeof(ora_desc) == sizeof(cts_buf_desc) && sizeof(ora_result) == sizeof(cts_verify_result),
              "the oracle's records are the ABI's");

}  // namespace

hipError_t launch_fill(uint8_t* arena, uint64_t bytes, const cts_buf_desc* d, uint32_t n, uint32_t, hipStream_t s,
                       const LaunchGeometry&)
{
    launched("launch_fill", s);
    ora_fill(arena, bytes, reinterpret_cast<const ora_desc*>(d), n);
    return hipSuccess;
}
hipError_t launch_fill_span(uint8_t* dst, uint64_t bytes, uint32_t pattern_offset, hipStream_t s, const LaunchGeometry&)
{
    launched("launch_fill_span", s);
    for (uint64_t i = 0; i < bytes; ++i) dst[i] = ora_pattern_byte(pattern_offset + i);
    return hipSuccess;
}
hipError_t launch_verify(const uint8_t* arena, uint64_t bytes, const cts_buf_desc* d, uint32_t n, uint32_t,
                         cts_verify_result* r, uint64_t* counters, uint32_t* first_fail, uint32_t n_conns,
                         hipStream_t s, const LaunchGeometry&)
{
    const int async_us = g_async_us.load();
    launched("launch_verify", s, async_us == 0);
    auto body = [=] {
        if (async_us > 0) {  // 0.5-1.5 x async_us: launches on different streams finish in any order
            thread_local uint32_t x = 0x9E3779B9u ^ (uint32_t)(uintptr_t)&x;
            x ^= x << 13;
            x ^= x >> 17;
            x ^= x << 5;
            std::this_thread::sleep_for(std::chrono::microseconds(async_us / 2 + x % (uint32_t)(async_us + 1)));
        }
        ora_counters c{};
        // the launch's own first failures, then merged into the caller's slots by an atomic min per connection as
        // the kernels do: a min that found the slot empty is the connection's first failure (kConnectionsFailed)
        std::vector<uint32_t> own(first_fail != nullptr ? n_conns : 0u, 0xFFFFFFFFu);
        (void)ora_verify_batch(arena, bytes, reinterpret_cast<const ora_desc*>(d), n, reinterpret_cast<ora_result*>(r),
                               &c, own.empty() ? nullptr : own.data(), (uint32_t)own.size(), 1);
        uint64_t conns = 0;
        for (uint32_t k = 0; k < own.size(); ++k) {
            if (own[k] == 0xFFFFFFFFu) continue;
            uint32_t cur = __atomic_load_n(&first_fail[k], __ATOMIC_RELAXED);
            const uint32_t old = cur;
            while (own[k] < cur &&
                   !__atomic_compare_exchange_n(&first_fail[k], &cur, own[k], false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
            }
            if (old == 0xFFFFFFFFu && cur == 0xFFFFFFFFu) ++conns;  // (cur holds the value the exchange replaced)
        }
        if (counters != nullptr) {  // (shard 0 of the device block; atomics, as the kernels': streams run at once)
            __atomic_fetch_add(&counters[kBytesChecked], c.bytes_checked, __ATOMIC_RELAXED);
            __atomic_fetch_add(&counters[kBytesOk], c.bytes_ok, __ATOMIC_RELAXED);
            __atomic_fetch_add(&counters[kBuffersChecked], c.buffers_checked, __ATOMIC_RELAXED);
            __atomic_fetch_add(&counters[kBuffersFailed], c.buffers_failed, __ATOMIC_RELAXED);
            __atomic_fetch_add(&counters[kMismatchedBytes], c.mismatched_bytes, __ATOMIC_RELAXED);
            __atomic_fetch_add(&counters[kConnectionsFailed], conns, __ATOMIC_RELAXED);
        }
    };
    if (d == nullptr && n != 0) return hipErrorInvalidValue;
    if (async_us > 0) enqueue(stream_of(s), body);  // done later, behind the stream's earlier work
    else body();
    return hipSuccess;
}
hipError_t launch_verify_strided(const uint8_t*, uint64_t, uint32_t, const uint32_t*, uint32_t, uint32_t, uint32_t,
                                 uint32_t, cts_verify_result*, uint64_t*, uint32_t*, uint32_t, hipStream_t s,
                                 const LaunchGeometry&)
{
    launched("launch_verify_strided", s);
    return hipSuccess;
}
hipError_t launch_media_stream_fill(uint8_t*, uint64_t, const cts_buf_desc*, const cts_datagram_header*, uint32_t,
                                    hipStream_t s, const LaunchGeometry&)
{
    launched("launch_media_stream_fill", s);
    return hipSuccess;
}
hipError_t launch_media_stream_fill_strided(uint8_t*, uint64_t, uint32_t, const uint32_t*, const cts_datagram_header*,
                                            uint32_t, hipStream_t s, const LaunchGeometry&)
{
    launched("launch_media_stream_fill_strided", s);
    return hipSuccess;
}
hipError_t launch_media_stream_verify(const uint8_t*, uint64_t, const cts_buf_desc*, uint32_t, cts_datagram_record*,
                                      cts_verify_result*, uint64_t*, hipStream_t s, const LaunchGeometry&)
{
    launched("launch_media_stream_verify", s);
    return hipSuccess;
}
hipError_t launch_media_stream_verify_strided(const uint8_t*, uint64_t, uint32_t, const uint32_t*, uint32_t,
                                              cts_datagram_record*, cts_verify_result*, uint64_t*, hipStream_t s,
                                              const LaunchGeometry&)
{
    launched("launch_media_stream_verify_strided", s);
    return hipSuccess;
}
// One received datagram as media_stream_verify_quad_kernel reads it (ValidateBufferLengthFromTask, the payload
// verify after the 26-byte header at pattern offset 0).
struct MsDatagram {
    uint32_t kind = CTS_DGRAM_BAD_DESC, completed = 0;
    uint16_t flag = 0;
    int64_t seq = 0;
    bool clean = false;
};
MsDatagram ms_read(const uint8_t* arena, uint64_t bytes, const cts_buf_desc* descs, const uint32_t* lengths,
                   uint32_t stride, uint32_t i)
{
    MsDatagram m;
    const uint64_t off = descs ? descs[i].byte_offset : (uint64_t)i * stride;
    m.completed = descs ? descs[i].length : lengths[i];
    if (off > bytes || bytes - off < m.completed || (!descs && m.completed > stride)) return m;
    const uint8_t* b = arena + off;
    if (m.completed == 0) {
        m.kind = CTS_DGRAM_ZERO;
    } else if (m.completed < CTS_UDP_FLAG_LENGTH) {
        m.kind = CTS_DGRAM_SHORT;
    } else {
        std::memcpy(&m.flag, b, 2);
        if (m.flag == CTS_UDP_FLAG_DATA)
            m.kind = m.completed < CTS_UDP_DATA_HEADER_LENGTH ? CTS_DGRAM_SHORT : CTS_DGRAM_DATA;
        else if (m.flag == CTS_UDP_FLAG_ID)
            m.kind = m.completed < CTS_UDP_CONNECTION_ID_HEADER_LENGTH ? CTS_DGRAM_SHORT : CTS_DGRAM_ID;
        else
            m.kind = CTS_DGRAM_UNKNOWN;
    }
    if (m.kind == CTS_DGRAM_DATA) {
        std::memcpy(&m.seq, b + 2, 8);
        m.clean = true;
        for (uint32_t x = CTS_UDP_DATA_HEADER_LENGTH; x < m.completed && m.clean; ++x)
            m.clean = b[x] == ora_pattern_byte(x - CTS_UDP_DATA_HEADER_LENGTH);
    }
    return m;
}

hipError_t launch_media_stream_status(const uint8_t* arena, uint64_t bytes, const cts_buf_desc* descs,
                                      const uint32_t* lengths, uint32_t stride, uint32_t n, cts_datagram_status* st,
                                      uint64_t*, hipStream_t s, const LaunchGeometry&)
{
    launched("launch_media_stream_status", s);
    for (uint32_t i = 0; st != nullptr && i < n; ++i) {
        const MsDatagram m = ms_read(arena, bytes, descs, lengths, stride, i);
        st[i] = cts_datagram_status{m.kind == CTS_DGRAM_DATA ? m.seq : 0, m.completed, m.flag, (uint8_t)m.kind,
                                    (uint8_t)(m.clean ? 1 : 0)};
    }
    return hipSuccess;
}
// the frame sums of media_stream_verify_quad_kernel<FRAMES>, all in shard 0
hipError_t launch_media_stream_frames(const uint8_t* arena, uint64_t bytes, const cts_buf_desc* descs,
                                      const uint32_t* lengths, uint32_t stride, uint32_t n, const cts_frame_window& w,
                                      uint64_t* totals, uint64_t* frame_bytes, uint64_t*, hipStream_t s,
                                      const LaunchGeometry&)
{
    launched("launch_media_stream_frames", s);
    std::memset(totals, 0, cts_frame_totals_device_bytes());
    if (w.frames) std::memset(frame_bytes, 0, sizeof(uint64_t) * w.frames);
    uint32_t inv_first = 0, exc = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const MsDatagram m = ms_read(arena, bytes, descs, lengths, stride, i);
        if (m.kind == CTS_DGRAM_DATA && m.clean) {
            totals[0] += (uint64_t)m.completed * 8u;
            totals[2] += 1;
            const uint64_t k = (uint64_t)m.seq - (uint64_t)w.head_sequence_number;
            if (m.seq > w.final_frame || m.seq < w.head_sequence_number || k >= w.frames) totals[1] += 1;
            else frame_bytes[k] += m.completed;
        } else if (!(m.kind == CTS_DGRAM_ZERO && w.finished)) {
            ++exc;
            inv_first = std::max(inv_first, ~i);
        }
    }
    totals[3] = (uint64_t)inv_first | ((uint64_t)exc << 32);
    return hipSuccess;
}

// counters_fold_kernel: the 64 shards' kCounterCount sums into out (accumulating), after the stream's earlier work
hipError_t launch_counters_fold(const void* block, uint64_t* out, bool accumulate, hipStream_t s)
{
    launched("launch_counters_fold", s);
    const uint64_t* h = static_cast<const uint64_t*>(block);
    for (int k = 0; k < kCounterCount; ++k) {
        uint64_t v = accumulate ? out[k] : 0;
        for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh) v += h[sh * kCounterSlots + k];
        out[k] = v;
    }
    return hipSuccess;
}

// The resident grid, emulated: group g polls slot g * per_group + j % per_group for the tag j + 1 from
// starts.j[g] on, as mailbox_kernel does; every piece of a job is answered clean; a stop job (len 0) is answered
// by every workgroup of the group and ends it; a group that waits idle_ticks (100 MHz) for a job leaves.
hipError_t launch_mailbox(const MailSlot* slots, MailPart* parts, uint32_t per_group, const MailStarts& starts,
                          uint32_t groups, uint64_t idle_ticks, hipStream_t s, uint64_t)
{
    launched("launch_mailbox", s, false);
    ihipStream_t* st = stream_of(s);
    const MailStarts js = starts;
    MailSlot* ring = const_cast<MailSlot*>(slots);
    const Done done = enqueue(st, [=] {
        using clock = std::chrono::steady_clock;
        const auto idle = std::chrono::nanoseconds(idle_ticks * 10);
        std::vector<uint64_t> j(js.j, js.j + groups);
        std::vector<bool> live(groups, true);
        std::vector<clock::time_point> since(groups, clock::now());
        uint32_t nlive = groups;
        while (nlive != 0) {
            bool progress = false;
            for (uint32_t g = 0; g < groups; ++g) {
                if (!live[g]) continue;
                const uint32_t k = g * per_group + (uint32_t)(j[g] % per_group);
                const uint32_t tag = (uint32_t)(j[g] + 1);
                const uint64_t ls = __atomic_load_n(&ring[k].len_seq, __ATOMIC_ACQUIRE);
                const uint32_t have = (uint32_t)(ls >> 32);
                if (have == tag) {
                    const uint64_t pe = __atomic_load_n(&ring[k].ptr_exp, __ATOMIC_RELAXED);
                    const uint32_t len = (uint32_t)ls;
                    ++j[g];
                    progress = true;
                    since[g] = clock::now();
                    if (len == kMailSkip) continue;
                    if (len != 0) {
                        int d = g_drop_jobs.load();
                        if (d > 0 && g_drop_jobs.compare_exchange_strong(d, d - 1)) continue;  // never answered
                    }
                    const uint64_t ptr = pe & 0xFFFFFFFFFFFFull;
                    const uint32_t np = mail_parts(ptr, len);
                    // the job verified whole; part 0 carries its first mismatch and count, the others answer clean
                    uint32_t first = 0xFFFFFFFFu, count = 0, actual = 0;
                    const uint8_t* b = reinterpret_cast<const uint8_t*>(ptr);
                    for (uint32_t x = 0; len != 0 && x < len; ++x)
                        if (b[x] != ora_pattern_byte((pe >> 48) + x)) {
                            if (first == 0xFFFFFFFFu) {
                                first = x;
                                actual = b[x];
                            }
                            ++count;
                        }
                    for (uint32_t i = 0; i < np; ++i) {
                        MailPart* p = parts + (size_t)k * kMailGroup + i;
                        const bool mine = i == 0 && count != 0;
                        __atomic_store_n(&p->g0, (mine ? first : 0xFFFFFFFFull) | ((uint64_t)tag << 32),
                                         __ATOMIC_RELEASE);
                        __atomic_store_n(&p->g1,
                                         (mine ? (uint64_t)count | ((uint64_t)actual << 32) : 0) |
                                             ((uint64_t)(tag & 0xFFFFFFu) << 40),
                                         __ATOMIC_RELEASE);
                    }
                    if (len == 0) {
                        live[g] = false;
                        --nlive;
                    }
                } else if ((int32_t)(have - tag) > 0) {  // a later job holds the slot: this one is a no-op
                    ++j[g];
                    progress = true;
                } else if (clock::now() - since[g] > idle) {
                    live[g] = false;
                    --nlive;
                }
            }
            if (!progress) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    });
    {
        std::lock_guard<std::mutex> lk(g_grid_mu);
        g_grid_done.push_back(done);
    }
    g_grids.fetch_add(1);
    return hipSuccess;
}

}  // namespace cts

// ---- the driver --------------------------------------------------------------------------------------------
// tools/bench_multi.cpp (bench.py's single-process leg): one native launch thread per GPU
extern "C" {
struct cts_bench_gpu {  // as declared in tools/bench_multi.cpp (and bench.py's _BenchGpu)
    cts_engine* engine;
    int device;
    uint32_t arenas;
    const void* const* arena;
    uint64_t arena_bytes;
    const cts_buf_desc* descs;
    uint32_t n;
    uint32_t max_length_hint;
    cts_verify_result* const* results;
    void* counters;
    uint32_t* const* conn_first_fail;
    uint32_t n_conns;
    void* const* streams;
    uint32_t nstreams;
};
int cts_bench_run_multi(const cts_bench_gpu* gpus, uint32_t G, uint32_t launches, double* t0, double* t1,
                        double* t_start, int sync);
}

namespace {

int g_fail = 0;
std::vector<uint8_t> g_S;  // g_senderSharedBuffer for 1 MiB buffers: S[k + b] is the pattern byte at offset k + b
#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                          \
        }                                                                      \
    } while (0)

// One engine's every device entry point from a thread whose own device is `home`; the launches counted on the
// engine's device must grow by exactly the entry points that launch, and `home` must be current afterwards.
void drive(cts_engine* e, int dev, int home, int rounds)
{
    CHECK(hipSetDevice(home) == hipSuccess);
    alignas(64) static thread_local uint8_t arena[1 << 18];
    alignas(64) static thread_local uint64_t block[CTS_COUNTER_SHARDS * 8];
    alignas(64) static thread_local uint8_t bad[70000];
    const uint8_t* const S = g_S.data();
    cts_buf_desc d[2] = {{0, 4096, 0, 0, 0}, {4096, 1472, 7, 1, 0}};
    cts_verify_result r[2];
    uint32_t lens[2] = {1472, 1472}, first_fail[2] = {0, 0};
    cts_datagram_header hd[2] = {{1, 2, 3}, {2, 2, 3}};
    cts_datagram_record rec[2];
    cts_datagram_status sts[2];
    cts_frame_window w{0, 100, 4, 0};
    alignas(8) static thread_local uint8_t totals[4096];
    uint64_t frame_bytes[4];
    cts_counters c{};
    void* s = nullptr;
    int cur = -1;
    auto here = [&](const char* what) {
        (void)hipGetDevice(&cur);
        if (cur != home) {
            std::fprintf(stderr, "%s left device %d current (caller's %d, engine's %d)\n", what, cur, home, dev);
            ++g_fail;
            (void)hipSetDevice(home);
        }
    };
    CHECK(cts_engine_stream_create(e, &s) == CTS_OK);
    here("stream_create");
    CHECK(s != nullptr && static_cast<ihipStream_t*>(s)->device == dev);
    for (int it = 0; it < rounds; ++it) {
        const int before = g_launches[dev].load();
        CHECK(cts_counters_reset(e, block, s) == CTS_OK);
        here("counters_reset");
        CHECK(cts_fill(e, arena, sizeof(arena), d, 2, 4096, s) == CTS_OK);
        here("fill");
        CHECK(cts_sender_buffer_fill(e, arena + (1 << 17), 1024, s) == CTS_OK);
        here("sender_buffer_fill");
        CHECK(std::memcmp(arena + (1 << 17), S, 65536 + 1024) == 0);
        CHECK(cts_verify(e, arena, sizeof(arena), d, 2, 4096, r, block, first_fail, 2, s) == CTS_OK);
        here("verify");
        CHECK(r[0].pass == 1 && r[1].pass == 1 && r[1].first_mismatch == 1472);
        arena[4096 + 1000] ^= 0x40;
        CHECK(cts_verify(e, arena, sizeof(arena), d, 2, 4096, r, block, first_fail, 2, nullptr) == CTS_OK);  // null stream
        here("verify (null stream)");
        CHECK(r[0].pass == 1 && r[1].pass == 0 && r[1].first_mismatch == 1000 && r[1].mismatch_bytes == 1);
        CHECK(cts_verify_strided(e, arena, sizeof(arena), 2048, lens, 2, 0, 0, 0, r, block, first_fail, 2, s) == CTS_OK);
        here("verify_strided");
        CHECK(cts_media_stream_fill(e, arena, sizeof(arena), d, hd, 2, s) == CTS_OK);
        here("media_stream_fill");
        CHECK(cts_media_stream_fill_strided(e, arena, sizeof(arena), 2048, lens, hd, 2, s) == CTS_OK);
        here("media_stream_fill_strided");
        CHECK(cts_media_stream_verify(e, arena, sizeof(arena), d, 2, rec, r, block, s) == CTS_OK);
        here("media_stream_verify");
        CHECK(cts_media_stream_verify_strided(e, arena, sizeof(arena), 2048, lens, 2, rec, r, block, s) == CTS_OK);
        here("media_stream_verify_strided");
        CHECK(cts_media_stream_verify_status(e, arena, sizeof(arena), d, 2, sts, block, s) == CTS_OK);
        here("media_stream_verify_status");
        CHECK(cts_media_stream_verify_strided_status(e, arena, sizeof(arena), 2048, lens, 2, sts, block, s) == CTS_OK);
        here("media_stream_verify_strided_status");
        CHECK(cts_media_stream_verify_frames(e, arena, sizeof(arena), d, 2, &w, totals, frame_bytes, block, s) == CTS_OK);
        here("media_stream_verify_frames");
        CHECK(cts_media_stream_verify_strided_frames(e, arena, sizeof(arena), 2048, lens, 2, &w, totals, frame_bytes,
                                                     block, s) == CTS_OK);
        here("media_stream_verify_strided_frames");
        CHECK(g_launches[dev].load() - before >= 13);
        CHECK(cts_counters_read(e, block, &c, s) == CTS_OK);
        here("counters_read");
        CHECK(c.buffers_checked == 4 && c.buffers_failed == 1 && c.mismatched_bytes == 1);
        // the host paths: one-buffer verifies (the mailbox, and the launch path), a batch, pinned memory
        for (int k = 0; k < 4; ++k) {
            cts_verify_result hr{};
            const uint32_t len = k == 3 ? 70000u : 1024u << k;
            CHECK(cts_verify_host(e, S + k, len, (uint32_t)k, &hr) == CTS_OK);
            here("verify_host");
            CHECK(hr.pass == 1 && hr.first_mismatch == len);
            std::memcpy(bad, S + k, len);
            bad[len - 1 - (uint32_t)it] ^= 0x01;
            CHECK(cts_verify_host(e, bad, len, (uint32_t)k, &hr) == CTS_OK);
            here("verify_host (corrupt)");
            CHECK(hr.pass == 0 && hr.first_mismatch == len - 1 - (uint32_t)it && hr.mismatch_bytes == 1 &&
                  hr.actual == (S[k + len - 1 - it] ^ 0x01) && hr.expected == S[k + len - 1 - it]);
        }
        void* hp = nullptr;
        void* dv = nullptr;
        CHECK(cts_host_alloc(e, 4096, &hp, &dv) == CTS_OK);
        here("host_alloc");
        if (hp != nullptr) std::memcpy(hp, S + 5, 4000);
        cts_verify_result mr{};
        CHECK(cts_verify_mapped(e, dv, 4000, 5, &mr) == CTS_OK && mr.pass == 1);
        here("verify_mapped");
        CHECK(cts_host_free(e, hp) == CTS_OK);  // stops this engine's grid first
        here("host_free");
        const void* bufs[2] = {S, S + 100};
        const uint32_t blens[2] = {100, 3000}, exp[2] = {0, 100};
        cts_verify_result br[2];
        cts_counters bc{};
        CHECK(cts_verify_host_batch(e, bufs, blens, exp, nullptr, 2, br, &bc) == CTS_OK);
        here("verify_host_batch");
        CHECK(br[0].pass == 1 && br[1].pass == 1 && bc.buffers_checked == 2 && bc.bytes_ok == 3100);
        int prev = cts_engine_set_attr(e, CTS_ATTR_SYNC_MAILBOX, 0);
        CHECK(prev == CTS_OK);
        cts_verify_result lr{};
        CHECK(cts_verify_host(e, S + 3, 9000, 3, &lr) == CTS_OK);
        here("verify_host (launch path)");
        CHECK(lr.pass == 1 && lr.first_mismatch == 9000);
        CHECK(cts_engine_set_attr(e, CTS_ATTR_SYNC_MAILBOX, 1) == CTS_OK);
    }
    CHECK(cts_engine_numa_node(e) == -1);
    here("numa_node");
    CHECK(cts_engine_stream_destroy(e, s) == CTS_OK);
    here("stream_destroy");
}

}  // namespace

int main(int argc, char** argv)
{
    // argv[1]: the stub RCCL (tests/cpp/rccl_stub.cpp) for cts_counters_allreduce; without it that phase is skipped
    if (argc > 1) setenv("CTS_RCCL_LIBRARY", argv[1], 1);
    std::setvbuf(stdout, nullptr, _IONBF, 0);
    g_S.resize(ora_sender_buffer_size(1u << 20));
    ora_build_sender_buffer(g_S.data(), 1u << 20);
    // grids stay up between posts (no watchdog stop for 10 s): every pinned free below meets running grids
    setenv("CTS_MAILBOX_IDLE_MS", "10000", 1);
    // engines on every device, created from a thread whose device is 3
    CHECK(hipSetDevice(3) == hipSuccess);
    cts_engine* eng[kDevices + 1] = {};
    for (int g = 0; g < kDevices; ++g) {
        CHECK(cts_engine_create(g, &eng[g]) == CTS_OK);
        CHECK(eng[g] != nullptr && cts_engine_device(eng[g]) == g);
    }
    CHECK(cts_engine_create(5, &eng[kDevices]) == CTS_OK);  // a second engine on one device
    cts_engine* bad = nullptr;
    CHECK(cts_engine_create(kDevices, &bad) == CTS_E_NO_DEVICE && bad == nullptr);
    int cur = -1;
    (void)hipGetDevice(&cur);
    CHECK(cur == 3);

    // every engine from the main thread (device 3 current), one after the other
    for (int g = 0; g <= kDevices; ++g) drive(eng[g], cts_engine_device(eng[g]), 3, 2);
    std::printf("sequential: %d grids, violations %d\n", g_grids.load(), g_violations.load());

    // a staging buffer that grows on engine 2 from a thread whose device (1) runs engine 1's grid: the old
    // buffer's free must happen on device 2, with device 2's grids stopped, not on the caller's device
    {
        cts_verify_result r{};
        CHECK(cts_verify_mapped(eng[1], eng[1] ? (const void*)g_S.data() : nullptr, 4096, 0, &r) == CTS_OK);  // device 1 busy
        CHECK(hipSetDevice(1) == hipSuccess);
        CHECK(cts_verify_host(eng[2], g_S.data() + 9, (1u << 20) - 64, 9, &r) == CTS_OK && r.pass == 1);
        (void)hipGetDevice(&cur);
        CHECK(cur == 1);
        CHECK(hipSetDevice(3) == hipSuccess);
    }
    std::printf("growth: violations %d\n", g_violations.load());

    // one thread per engine at once, each starting from another device than its engine's
    std::vector<std::thread> ts;
    for (int g = 0; g <= kDevices; ++g)
        ts.emplace_back([&, g] { drive(eng[g], cts_engine_device(eng[g]), (g + 1) % kDevices, 3); });
    for (auto& t : ts) t.join();
    std::printf("threads: %d grids, violations %d\n", g_grids.load(), g_violations.load());

    // whole loopback TCP connections over the eight engines (connection i on engine cts_shard_of(i, 8)): the feeder's
    // side threads start on device 0 and drive SYNC (the mailbox) and DEFERRED (batches, events) patterns on every
    // device; the wire corruption of one connection must fail exactly that connection. Verify launches complete
    // 150-450 us after they are enqueued, so DEFERRED batches are really in flight when the pattern polls their events.
    g_async_us.store(300);
    struct Run {
        uint32_t pattern, mode, corrupt;
        uint32_t buffer_high = 0, recv_whole = 1, depth = 2, batch = 8;  // -Buffer:[64 KiB, high], partial recvs, DEFERRED
    };
    const Run runs[] = {
        {CTS_PATTERN_PUSH, CTS_VERIFY_DEFERRED, 0},
        {CTS_PATTERN_PULL, CTS_VERIFY_SYNC, 0},
        {CTS_PATTERN_PUSH, CTS_VERIFY_SYNC, 1},
        {CTS_PATTERN_PULL, CTS_VERIFY_DEFERRED, 1},
        {CTS_PATTERN_PUSHPULL, CTS_VERIFY_DEFERRED, 0},
        {CTS_PATTERN_DUPLEX, CTS_VERIFY_DEFERRED, 0},
        {CTS_PATTERN_DUPLEX, CTS_VERIFY_SYNC, 1},
        // random buffer sizes, partial completions, other DEFERRED depths and batches
        {CTS_PATTERN_PUSH, CTS_VERIFY_DEFERRED, 0, 200000u, 0u, 3u, 16u},
        {CTS_PATTERN_PULL, CTS_VERIFY_DEFERRED, 1, 0u, 0u, 1u, 8u},
        {CTS_PATTERN_PUSHPULL, CTS_VERIFY_SYNC, 0, 150000u, 0u, 2u, 8u},
        {CTS_PATTERN_DUPLEX, CTS_VERIFY_DEFERRED, 1, 100000u, 0u, 2u, 12u},
    };
    for (const Run& run : runs) {
        char depth[8];
        std::snprintf(depth, sizeof(depth), "%u", run.depth);
        setenv("CTS_DEFERRED_DEPTH", depth, 1);
        cts_loopback_config cfg{};
        cfg.connections = 16;
        cfg.io_pattern = run.pattern;
        cfg.buffer_size = 65536;
        cfg.buffer_size_high = run.buffer_high;
        cfg.random_seed = 7;
        cfg.verify_buffers = 1;
        cfg.transfer_size = (2u << 20) + 12345;
        cfg.verify_mode = run.mode;
        cfg.batch_buffers = run.batch;
        cfg.corrupt_connection = run.corrupt ? 5u : ~0u;
        cfg.corrupt_send_index = 11;
        cfg.recv_whole = run.recv_whole;
        cts_loopback_result out{};
        CHECK(cts_loopback_run_multi(&cfg, eng, kDevices, nullptr, nullptr, &out) == CTS_OK);
        (void)hipGetDevice(&cur);
        CHECK(cur == 3);
        if (run.corrupt)
            CHECK(out.connections_ok == 15 && out.connections_failed == 1 && out.data_errors == 1);
        else
            CHECK(out.connections_ok == 16 && out.connections_failed == 0 && out.data_errors == 0 &&
                  out.buffers_verified >= (run.recv_whole && !run.buffer_high ? 16u * 33u : 16u));
        std::printf("loopback pattern %u mode %u corrupt %u buffers [65536, %u] whole %u depth %u batch %u: ok %u "
                    "failed %u data errors %u verified %llu\n",
                    run.pattern, run.mode, run.corrupt, run.buffer_high, run.recv_whole, run.depth, run.batch,
                    out.connections_ok, out.connections_failed, out.data_errors,
                    (unsigned long long)out.buffers_verified);
    }
    unsetenv("CTS_DEFERRED_DEPTH");
    // MediaStream over loopback UDP on engine 6, SYNC (one verify per datagram) and DEFERRED (the frame-sum pass
    // flushed at every render tick): the client's timer thread starts on device 0 and flushes through the pattern
    for (uint32_t run = 0; run < 4; ++run) {
        const uint32_t corrupt = run & 1u, mode = run < 2 ? CTS_VERIFY_SYNC : CTS_VERIFY_DEFERRED;
        cts_media_stream_loopback_config mc{};
        mc.connections = 2;
        mc.frame_size_bytes = 3000;
        mc.frames_per_second = 100;
        mc.stream_length_frames = 30;
        mc.buffered_frames = 15;
        mc.verify_buffers = 1;
        mc.corrupt_connection = corrupt ? 1u : ~0u;
        mc.corrupt_datagram = 20;
        mc.verify_mode = mode;
        mc.batch_buffers = 16;
        cts_media_stream_loopback_result mo{};
        CHECK(cts_loopback_media_stream_run(&mc, eng[6], nullptr, nullptr, &mo) == CTS_OK);
        (void)hipGetDevice(&cur);
        CHECK(cur == 3);
        if (corrupt)
            CHECK(mo.connections_ok == 1 && mo.connections_failed == 1 && mo.data_errors == 1);
        else
            CHECK(mo.connections_ok == 2 && mo.connections_failed == 0 && mo.data_errors == 0);
        std::printf("media stream mode %u corrupt %u: ok %u failed %u data errors %u datagrams %llu\n", mode, corrupt,
                    mo.connections_ok, mo.connections_failed, mo.data_errors,
                    (unsigned long long)mo.datagrams_received);
    }
    cts_shared_buffer_release();
    g_async_us.store(0);
    CHECK(g_not_ready.load() > 0);  // DEFERRED polled batches still in flight
    std::printf("loopback: %d grids, %d event queries in flight, violations %d\n", g_grids.load(), g_not_ready.load(),
                g_violations.load());

    // the node's counters: every engine verifies a batch with a few corrupt buffers on a stream of its own (launches
    // still in flight), then cts_counters_allreduce (each block folded on its device, one all-reduce per device over
    // the stub RCCL; engines 5 and 5b share device 5) from a thread on device 3 must equal cts_counters_read_multi
    // and the oracle's sums, with device 3 current afterwards
    if (argc > 1) {
        g_async_us.store(300);
        constexpr uint32_t kN = kDevices + 1, kBufs = 32;
        std::vector<std::vector<uint8_t>> arenas(kN, std::vector<uint8_t>((size_t)kBufs * 4096 + 64));
        std::vector<std::vector<uint64_t>> blocks(kN, std::vector<uint64_t>(CTS_COUNTER_SHARDS * 8));
        std::vector<std::vector<cts_buf_desc>> descs(kN);
        std::vector<std::vector<cts_verify_result>> res(kN, std::vector<cts_verify_result>(kBufs));
        std::vector<void*> streams(kN);
        std::vector<const void*> bptr(kN);
        std::vector<std::vector<uint32_t>> first_fail(kN, std::vector<uint32_t>(5, 0xFFFFFFFFu));  // the live slots
        std::vector<std::vector<uint32_t>> want_ff(kN, std::vector<uint32_t>(5, 0xFFFFFFFFu));
        uint64_t want[cts::kCounterCount] = {};
        for (uint32_t g = 0; g < kN; ++g) {
            uint8_t* a = reinterpret_cast<uint8_t*>(((uintptr_t)arenas[g].data() + 15u) & ~(uintptr_t)15u);
            for (uint32_t b = 0; b < kBufs; ++b) {
                const uint32_t len = 1000u + 97u * b + g, e = (7919u * b + 31u * g) & 0xFFFFu;
                descs[g].push_back(cts_buf_desc{(uint64_t)b * 4096u, len, e, b % 5u, 0u});
                for (uint32_t k = 0; k < len; ++k) a[(size_t)b * 4096u + k] = ora_pattern_byte(e + k);
                want[cts::kBytesChecked] += len;
                want[cts::kBuffersChecked] += 1;
                if ((b + g) % 7u == 3u) {  // one corrupt byte
                    a[(size_t)b * 4096u + len / 2] ^= 0x10;
                    want[cts::kBuffersFailed] += 1;
                    want[cts::kMismatchedBytes] += 1;
                    if (want_ff[g][b % 5u] == 0xFFFFFFFFu) want[cts::kConnectionsFailed] += 1;
                    want_ff[g][b % 5u] = std::min(want_ff[g][b % 5u], b);
                } else {
                    want[cts::kBytesOk] += len;
                }
            }
            CHECK(cts_engine_stream_create(eng[g], &streams[g]) == CTS_OK);
            CHECK(cts_counters_reset(eng[g], blocks[g].data(), streams[g]) == CTS_OK);
            CHECK(cts_verify(eng[g], a, (uint64_t)kBufs * 4096u, descs[g].data(), kBufs, 4096u, res[g].data(),
                             blocks[g].data(), first_fail[g].data(), 5, streams[g]) == CTS_OK);
            bptr[g] = blocks[g].data();
        }
        // the clique set up before the status timer's first read (from the same thread, device 3 current)
        CHECK(cts_counters_allreduce_prepare(eng, kN) == CTS_OK);
        (void)hipGetDevice(&cur);
        CHECK(cur == 3);
        cts_allreduce_setup st{};
        CHECK(cts_counters_allreduce_setup_times(&st) == CTS_OK && st.prepared == 1 && st.devices == kDevices);
        cts_counters_ex all{}, fold{};
        CHECK(cts_counters_allreduce_ex(eng, bptr.data(), streams.data(), kN, &all) == CTS_OK);
        CHECK(cts_counters_read_multi_ex(eng, bptr.data(), streams.data(), kN, &fold) == CTS_OK);
        (void)hipGetDevice(&cur);
        CHECK(cur == 3);
        const uint64_t got[cts::kCounterCount] = {all.bytes_checked, all.bytes_ok, all.buffers_checked, all.buffers_failed,
                                             all.mismatched_bytes, all.connections_failed};
        const uint64_t gotf[cts::kCounterCount] = {fold.bytes_checked, fold.bytes_ok, fold.buffers_checked,
                                              fold.buffers_failed, fold.mismatched_bytes, fold.connections_failed};
        for (int k = 0; k < cts::kCounterCount; ++k) CHECK(got[k] == want[k] && gotf[k] == want[k]);
        CHECK(want[cts::kConnectionsFailed] > 0);
        for (uint32_t g = 0; g < kN; ++g) CHECK(first_fail[g] == want_ff[g]);  // (the reads synchronised the streams)
        for (uint32_t g = 0; g < kN; ++g) CHECK(cts_engine_stream_destroy(eng[g], streams[g]) == CTS_OK);
        CHECK(cts_counters_allreduce_release() == CTS_OK);
        g_async_us.store(0);
        std::printf("allreduce: %llu buffers, %llu failed, %llu connections failed, equal to the host fold and the "
                    "oracle\n",
                    (unsigned long long)all.buffers_checked, (unsigned long long)all.buffers_failed,
                    (unsigned long long)all.connections_failed);
    } else {
        std::printf("allreduce: skipped (no stub RCCL)\n");
    }

    // bench.py's single-process leg at eight GPUs: one native thread per engine sets its device and issues its
    // launches round robin over 2 arenas and 2 streams (launches in flight), then synchronises its streams
    {
        g_async_us.store(200);
        constexpr uint32_t kG = kDevices, kR = 2, kS = 2, kBufs = 16, kLaunches = 6;
        struct Gpu {
            std::vector<uint8_t> mem[kR];
            const void* arena[kR];
            std::vector<cts_verify_result> res[kR];
            cts_verify_result* resp[kR];
            std::vector<uint32_t> cff[kR];
            uint32_t* cffp[kR];
            std::vector<uint64_t> block;
            void* streams[kS];
        };
        std::vector<Gpu> gp(kG);
        std::vector<cts_buf_desc> dd;
        for (uint32_t b = 0; b < kBufs; ++b) dd.push_back(cts_buf_desc{(uint64_t)b * 4096u, 4096u, (1237u * b) & 0xFFFFu, b % 4u, 0u});
        std::vector<cts_bench_gpu> work(kG);
        for (uint32_t g = 0; g < kG; ++g) {
            Gpu& G = gp[g];
            for (uint32_t a = 0; a < kR; ++a) {
                G.mem[a].assign((size_t)kBufs * 4096u + 16, 0);
                uint8_t* base = reinterpret_cast<uint8_t*>(((uintptr_t)G.mem[a].data() + 15u) & ~(uintptr_t)15u);
                for (uint32_t b = 0; b < kBufs; ++b)
                    for (uint32_t k = 0; k < 4096u; ++k) base[(size_t)b * 4096u + k] = ora_pattern_byte(dd[b].expected_pattern_offset + k);
                if (a == 1) base[(size_t)(g % kBufs) * 4096u + 100u] ^= 0x01;  // arena 1: buffer g % 16 corrupt
                G.arena[a] = base;
                G.res[a].assign(kBufs, cts_verify_result{});
                G.resp[a] = G.res[a].data();
                G.cff[a].assign(4, 0xFFFFFFFFu);
                G.cffp[a] = G.cff[a].data();
            }
            G.block.assign(CTS_COUNTER_SHARDS * 8, 0);
            for (uint32_t k = 0; k < kS; ++k) CHECK(cts_engine_stream_create(eng[g], &G.streams[k]) == CTS_OK);
            work[g] = cts_bench_gpu{eng[g], (int)g, kR, G.arena, (uint64_t)kBufs * 4096u, dd.data(), kBufs, 4096u,
                                    G.resp, G.block.data(), G.cffp, 4u, G.streams, kS};
        }
        double t0[kG], t1[kG], ts = 0;
        CHECK(cts_bench_run_multi(work.data(), kG, kLaunches, t0, t1, &ts, 1) == CTS_OK);
        (void)hipGetDevice(&cur);
        CHECK(cur == 3);
        for (uint32_t g = 0; g < kG; ++g) {
            cts_counters c{};
            CHECK(cts_counters_read(eng[g], gp[g].block.data(), &c, gp[g].streams[0]) == CTS_OK);
            CHECK(c.buffers_checked == (uint64_t)kLaunches * kBufs && c.buffers_failed == kLaunches / kR &&
                  c.mismatched_bytes == kLaunches / kR);
            for (uint32_t b = 0; b < kBufs; ++b) {
                CHECK(gp[g].res[0][b].pass == 1);
                CHECK(gp[g].res[1][b].pass == (b == g % kBufs ? 0 : 1));
            }
            CHECK(gp[g].res[1][g % kBufs].first_mismatch == 100u);
            CHECK(gp[g].cff[1][(g % kBufs) % 4u] == g % kBufs && gp[g].cff[0][0] == 0xFFFFFFFFu);
            for (uint32_t k = 0; k < kS; ++k) CHECK(cts_engine_stream_destroy(eng[g], gp[g].streams[k]) == CTS_OK);
        }
        g_async_us.store(0);
        std::printf("bench_multi: %u GPUs x %u launches, records, first failures and counters as planned\n", kG,
                    kLaunches);
    }

    // a DEFERRED pattern on engine 7 whose batch launch does not finish in time (a hung kernel, emulated: it completes
    // late, 0.5-1.5 s): cts_io_pattern_destroy gives up within its bound (CTS_PATTERN_DESTROY_WAIT_MS) with
    // CTS_E_TIMEOUT and leaves the pattern allocated under the running launch; once the launch has finished a second
    // destroy succeeds. Then the same with nothing in flight when destroy starts: the late kernel is the filling
    // batch destroy launches itself (its flush waits are bounded too)
    {
        std::vector<uint8_t> sender(ora_sender_buffer_size(4096));
        ora_build_sender_buffer(sender.data(), 4096);
        CHECK(cts_shared_buffer_attach(sender.data(), sender.size()) == CTS_OK);
        setenv("CTS_PATTERN_DESTROY_WAIT_MS", "300", 1);
        cts_pattern_config pc{};
        pc.io_pattern = CTS_PATTERN_PUSH;
        pc.protocol = CTS_PROTOCOL_TCP;
        pc.listening = 1;
        pc.verify_buffers = 1;
        pc.pre_post_recvs = 1;
        pc.pre_post_sends = 1;
        pc.buffer_size_low = 4096;
        pc.tcp_shutdown = CTS_SHUTDOWN_GRACEFUL;
        pc.transfer_size = 64u * 4096u;
        pc.verify_mode = CTS_VERIFY_DEFERRED;
        pc.batch_buffers = 12;  // launches of 4 (depth 2)
        cts_io_pattern* pat = nullptr;
        CHECK(cts_io_pattern_create(&pc, eng[7], &pat) == CTS_OK);
        if (pat != nullptr) {
            cts_task t{};
            CHECK(cts_io_pattern_initiate_io(pat, &t) == CTS_OK && t.io_action == CTS_TASK_SEND);
            CHECK(cts_io_pattern_complete_io(pat, &t, t.buffer_length, 0) == CTS_IO_CONTINUE);
            g_async_us.store(1000000);  // 0.5-1.5 s (the fake's jitter is 0.5-1.5 x): past the 0.3 s bound
            for (int k = 0; k < 6; ++k) {  // one launch of 4 in flight, 2 completions queued
                CHECK(cts_io_pattern_initiate_io(pat, &t) == CTS_OK && t.io_action == CTS_TASK_RECV);
                std::memcpy(t.buffer + t.buffer_offset, cts_shared_buffer() + t.expected_pattern_offset, t.buffer_length);
                CHECK(cts_io_pattern_complete_io(pat, &t, t.buffer_length, 0) == CTS_IO_CONTINUE);
            }
            const auto t0 = std::chrono::steady_clock::now();
            const int rc1 = cts_io_pattern_destroy(pat);
            const double s1 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            CHECK(rc1 == CTS_E_TIMEOUT && s1 < 0.9);
            (void)hipGetDevice(&cur);
            CHECK(cur == 3);
            g_async_us.store(0);
            std::this_thread::sleep_for(std::chrono::milliseconds(1700));  // the hung launch ends
            const int rc2 = cts_io_pattern_destroy(pat);
            CHECK(rc2 == CTS_OK);
            std::printf("destroy under a hung launch: CTS_E_TIMEOUT after %.3f s, then ok\n", s1);
        }
        pat = nullptr;
        CHECK(cts_io_pattern_create(&pc, eng[7], &pat) == CTS_OK);
        if (pat != nullptr) {
            cts_task t{};
            CHECK(cts_io_pattern_initiate_io(pat, &t) == CTS_OK && t.io_action == CTS_TASK_SEND);
            CHECK(cts_io_pattern_complete_io(pat, &t, t.buffer_length, 0) == CTS_IO_CONTINUE);
            for (int k = 0; k < 2; ++k) {  // two completions queued, fewer than a launch: nothing in flight
                CHECK(cts_io_pattern_initiate_io(pat, &t) == CTS_OK && t.io_action == CTS_TASK_RECV);
                std::memcpy(t.buffer + t.buffer_offset, cts_shared_buffer() + t.expected_pattern_offset, t.buffer_length);
                CHECK(cts_io_pattern_complete_io(pat, &t, t.buffer_length, 0) == CTS_IO_CONTINUE);
            }
            g_async_us.store(1000000);  // the batch destroy launches finishes late
            const auto t0 = std::chrono::steady_clock::now();
            const int rc1 = cts_io_pattern_destroy(pat);
            const double s1 = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            CHECK(rc1 == CTS_E_TIMEOUT && s1 < 0.9);
            g_async_us.store(0);
            std::this_thread::sleep_for(std::chrono::milliseconds(1700));
            CHECK(cts_io_pattern_destroy(pat) == CTS_OK);
            std::printf("destroy whose own flush is late: CTS_E_TIMEOUT after %.3f s, then ok\n", s1);
        }
        unsetenv("CTS_PATTERN_DESTROY_WAIT_MS");
        cts_shared_buffer_release();
    }

    // an idle engine's watchdog stops its grid from its own thread (no device current there but its own guard)
    setenv("CTS_MAILBOX_IDLE_MS", "20", 1);
    cts_engine* idle = nullptr;
    CHECK(cts_engine_create(6, &idle) == CTS_OK);
    {
        cts_verify_result r{};
        CHECK(cts_verify_mapped(idle, idle ? (const void*)(g_S.data() + 1) : nullptr, 8192, 1, &r) == CTS_OK &&
              r.pass == 1);
        std::shared_ptr<std::atomic<bool>> last;
        {
            std::lock_guard<std::mutex> lk(g_grid_mu);
            last = g_grid_done.back();
        }
        for (int i = 0; i < 200 && !last->load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
        CHECK(last->load());
        CHECK(cts_mailbox_launches(idle) == 1);
    }
    CHECK(cts_engine_destroy(idle) == CTS_OK);

    // a grid that left on its own (its idle exit, CTS_MAILBOX_EXIT_MS, before the watchdog's stop): a free stops
    // nothing and does not wait for stop jobs no workgroup will answer (CTS_MAILBOX_TIMEOUT_MS), and the next post
    // relaunches
    setenv("CTS_MAILBOX_IDLE_MS", "10000", 1);
    setenv("CTS_MAILBOX_EXIT_MS", "40", 1);
    cts_engine* lone = nullptr;
    CHECK(cts_engine_create(2, &lone) == CTS_OK);
    {
        cts_verify_result r{};
        CHECK(cts_verify_mapped(lone, lone ? (const void*)(g_S.data() + 7) : nullptr, 5000, 7, &r) == CTS_OK &&
              r.pass == 1);
        std::shared_ptr<std::atomic<bool>> last;
        {
            std::lock_guard<std::mutex> lk(g_grid_mu);
            last = g_grid_done.back();
        }
        for (int i = 0; i < 200 && !last->load(); ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
        CHECK(last->load());
        void *hp = nullptr, *dv = nullptr;
        CHECK(cts_host_alloc(lone, 4096, &hp, &dv) == CTS_OK);
        const auto t0 = std::chrono::steady_clock::now();
        CHECK(cts_host_free(lone, hp) == CTS_OK);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CHECK(s < 0.5);
        CHECK(cts_verify_mapped(lone, lone ? (const void*)(g_S.data() + 7) : nullptr, 5000, 7, &r) == CTS_OK &&
              r.pass == 1);
        CHECK(cts_mailbox_launches(lone) == 2);
        std::printf("grid gone on its own: free %.3f s\n", s);
    }
    CHECK(cts_engine_destroy(lone) == CTS_OK);

    // a job the grid never answers: the caller gives up after CTS_MAILBOX_TIMEOUT_MS and verifies with a launch (the
    // answer stays exact), the mailbox is broken until its grid has drained (the idle exit), then starts over
    setenv("CTS_MAILBOX_TIMEOUT_MS", "200", 1);
    cts_engine* flaky = nullptr;
    CHECK(cts_engine_create(4, &flaky) == CTS_OK);
    {
        static uint8_t buf[20000];
        std::memcpy(buf, g_S.data() + 11, sizeof(buf));
        buf[12345] ^= 0x80;
        cts_verify_result r{};
        CHECK(cts_verify_mapped(flaky, flaky ? (const void*)buf : nullptr, sizeof(buf), 11, &r) == CTS_OK &&
              r.pass == 0 && r.first_mismatch == 12345);
        g_drop_jobs.store(1);
        const auto t0 = std::chrono::steady_clock::now();
        r = cts_verify_result{};
        CHECK(cts_verify_mapped(flaky, flaky ? (const void*)buf : nullptr, sizeof(buf), 11, &r) == CTS_OK &&
              r.pass == 0 && r.first_mismatch == 12345 && r.mismatch_bytes == 1);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CHECK(s >= 0.2 && g_drop_jobs.load() == 0);
        std::this_thread::sleep_for(std::chrono::milliseconds(300));  // the grid's idle exit (40 ms)
        for (int k = 0; k < 3; ++k) {
            r = cts_verify_result{};
            CHECK(cts_verify_mapped(flaky, flaky ? (const void*)buf : nullptr, sizeof(buf), 11, &r) == CTS_OK &&
                  r.pass == 0 && r.first_mismatch == 12345);
        }
        CHECK(cts_mailbox_launches(flaky) == 2);
        std::printf("lost job: answered by a launch after %.3f s, mailbox relaunched\n", s);
    }
    CHECK(cts_engine_destroy(flaky) == CTS_OK);
    unsetenv("CTS_MAILBOX_TIMEOUT_MS");
    unsetenv("CTS_MAILBOX_EXIT_MS");

    for (int g = 0; g <= kDevices; ++g) CHECK(cts_engine_destroy(eng[g]) == CTS_OK);
    (void)hipGetDevice(&cur);
    CHECK(cur == 3);
    for (int g = 0; g < kDevices; ++g) CHECK(g_launches[g].load() > 0);
    CHECK(g_grids.load() >= kDevices + 1);
    CHECK(g_violations.load() == 0);
    CHECK(!grid_running(-1));
    for (int g = 0; g < kDevices; ++g) join_stream(&g_null[g]);
    if (g_fail != 0) {
        std::fprintf(stderr, "engine_devices: %d failures\n", g_fail);
        return 1;
    }
    std::printf("engine_devices: ok (%d engines on %d devices, %d mailbox grids)\n", kDevices + 2, kDevices,
                g_grids.load());
    return 0;
}
