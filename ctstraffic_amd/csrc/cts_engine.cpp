// cts_engine.cpp — the C ABI (include/cts_engine.h) over the gfx950 kernels.
//
// Every entry point is noexcept and returns a cts_status, mirroring the
// reference's noexcept IO surface (ctsIOPattern.h:143-144) while replacing its
// FAIL_FAST process aborts with error codes a foreign caller can handle.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "cts_engine.h"
#include "cts_internal.hpp"
#include "cts_slices.hpp"

struct Mailbox;

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
    int sync_mailbox = 1;  // CTS_ATTR_SYNC_MAILBOX (read by cts_pattern's SYNC verify and cts_verify_host)
    // cts_verify_host through the mailbox: pinned, device-mapped staging buffers, one per concurrent caller
    struct HostStage {
        void* p = nullptr;
        size_t cap = 0;
    };
    std::mutex stage_pool_mu;
    std::vector<HostStage> stage_pool;  // idle stages
    std::unique_ptr<Mailbox> mail;  // cts_verify_mapped's resident grid, started on first use
    std::mutex mail_init_mu;
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

// hipHostFree with the engine's mailbox grid stopped first (defined after Mailbox)
void pinned_free(cts_engine* e, void* p);

// Grow a pinned, device-mapped staging area to >= bytes (powers of two from `floor`).
int ensure_pinned(cts_engine* e, void** p, size_t* cap, size_t bytes, size_t floor)
{
    if (*cap >= bytes && *p != nullptr) return CTS_OK;
    if (*p) pinned_free(e, *p);
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
    const int rc = ensure_pinned(e, &p, &e->stage_cap, bytes, 1u << 20);
    e->stage = static_cast<uint8_t*>(p);
    return rc;
}

}  // namespace

// ---- cts_verify_mapped: the SYNC mailbox -------------------------------------------------------
// A resident grid (cts::launch_mailbox) answers one-buffer verifies posted through host-coherent
// pinned slots, so a SYNC completion pays PCIe round trips instead of a launch + synchronize; the
// caller folds the grid's per-piece part records into the RtlCompareMemory record itself.
// Jobs are claimed under `mu`, in the group with the fewest outstanding; group g's job j uses slot
// g * per_group + j % per_group once its previous user (j - per_group) has read its answer (free_at).
// The grid is (re)launched by the first post after it stopped, at every group's next job number, and a
// watchdog thread stops it with one stop job per group after `idle_ms` without posts, so an idle engine
// neither holds workgroups nor polls PCIe. The grid's own exit bound (a group leaves after exit_ms
// without a job, far longer) is a safety net: while posts keep coming, the watchdog gives every group
// that has had no job for exit_ms / 4 a no-op job (kMailSkip: nobody answers it, its slot is free again
// at once), whatever the post rate and the number of groups; a caller's job also goes to such a group
// first; and a post after exit_ms / 2 of silence checks whether the grid already left (a starved watchdog).
// A workgroup that fell a whole ring behind (a late poller) takes the jobs whose slots hold later jobs as
// no-ops (mailbox_kernel). A job unanswered after timeout_s marks the mailbox broken: callers then verify
// with a launch per call (cts_verify_mapped), and the first post after the grid has drained resets the
// rings and starts over. Freeing pinned memory (cts_host_free, a growing staging buffer, teardown) first makes
// the engine's device current and stops every engine's grid on it (DeviceQuiesce, Pause): a free waits for
// every kernel on the current device, and a resident grid would keep it waiting for as long as threads post.
struct Mailbox {
    cts_engine* e = nullptr;
    // groups x cts::kMailGroup workgroups: 8 groups measured best for 8-16 concurrent callers (with 16
    // workgroups per group: 18.7 / 25.3 us per 64 KiB verify at 8 / 16 threads against 19.6-32.6 for 1-4
    // groups, profiles/r02/sync_probe_groups.jsonl; with 4: 8 and 16 groups alike, mailbox_group_ab.jsonl).
    // A job goes to the group with the fewest outstanding, so one caller keeps one group hot and the idle
    // ones back off.
    uint32_t nslots = 1024, groups = 8, per_group = 128;
    int exit_ms = 1000;                  // the grid's own per-group idle exit (CTS_MAILBOX_EXIT_MS)
    uint64_t idle_ticks = 100000000ull;  // exit_ms at 100 MHz (s_memrealtime)
    int idle_ms = 50;
    double timeout_s = 2.0;              // CTS_MAILBOX_TIMEOUT_MS
    uint64_t delay_ticks = 0;            // CTS_MAILBOX_DELAY_MS (test hook: a late poller in the first launch)
    cts::MailSlot* slots = nullptr;      // host view (coherent, pinned)
    cts::MailSlot* dslots = nullptr;     // device view
    cts::MailPart* parts = nullptr;      // nslots x kMailGroup part records, host view (coherent, pinned)
    cts::MailPart* dparts = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t grid_done = nullptr;      // recorded after each launch: hipStreamQuery cannot see a kernel end
                                         // it was not asked about before (no completion signal), an event can
    std::unique_ptr<std::atomic<uint64_t>[]> free_at;
    std::mutex mu;
    bool running = false, broken = false, quit = false;
    uint32_t paused = 0;                 // Pause() callers: no (re)launch, posts fall back to a launch
    uint64_t next[cts::kMailMaxGroups] = {};       // each group's next job number
    uint32_t busy[cts::kMailMaxGroups] = {};       // each group's jobs outstanding
    uint32_t outstanding = 0;
    std::chrono::steady_clock::time_point last_post;
    std::chrono::steady_clock::time_point last_used[cts::kMailMaxGroups];  // each group's latest job
    std::condition_variable cv;
    std::thread watchdog;
    std::atomic<uint64_t> launches{0};
    std::atomic<bool> broken_flag{false};  // `broken`, readable without mu

    ~Mailbox();  // (after DeviceQuiesce)

    int Init(cts_engine* eng)
    {
        e = eng;
        nslots = (uint32_t)std::max(16, env_int("CTS_MAILBOX_SLOTS", (int)nslots));
        groups = (uint32_t)std::min((int)cts::kMailMaxGroups, std::max(1, env_int("CTS_MAILBOX_GROUPS", (int)groups)));
        idle_ms = std::max(1, env_int("CTS_MAILBOX_IDLE_MS", idle_ms));
        exit_ms = std::max(40, env_int("CTS_MAILBOX_EXIT_MS", exit_ms));
        idle_ticks = (uint64_t)exit_ms * 100000ull;
        timeout_s = std::max(1, env_int("CTS_MAILBOX_TIMEOUT_MS", (int)(timeout_s * 1000))) / 1000.0;
        delay_ticks = (uint64_t)std::max(0, env_int("CTS_MAILBOX_DELAY_MS", 0)) * 100000ull;
        DeviceGuard g(e->device);
        if (!g.ok) return CTS_E_HIP;
        void* p = nullptr;
        per_group = (nslots + groups - 1) / groups;
        nslots = per_group * groups;
        if (hipHostMalloc(&p, sizeof(cts::MailSlot) * nslots,
                          hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess)
            return CTS_E_NOMEM;
        slots = static_cast<cts::MailSlot*>(p);
        std::memset(slots, 0, sizeof(cts::MailSlot) * nslots);
        if ((dslots = device_view(slots)) == nullptr) return CTS_E_HIP;
        const size_t pbytes = sizeof(cts::MailPart) * nslots * cts::kMailGroup;
        if (hipHostMalloc(&p, pbytes, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) !=
            hipSuccess)
            return CTS_E_NOMEM;
        parts = static_cast<cts::MailPart*>(p);
        std::memset(parts, 0, pbytes);
        if ((dparts = device_view(parts)) == nullptr) return CTS_E_HIP;
        if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) {
            stream = nullptr;
            return CTS_E_HIP;
        }
        if (hipEventCreateWithFlags(&grid_done, hipEventDisableTiming) != hipSuccess) {
            grid_done = nullptr;
            return CTS_E_HIP;
        }
        free_at.reset(new (std::nothrow) std::atomic<uint64_t>[nslots]);
        if (!free_at) return CTS_E_NOMEM;
        ResetRings();
        last_post = std::chrono::steady_clock::now();
        try {  // nothing may cross the C ABI: a thread that cannot start leaves the engine on the launch path
            watchdog = std::thread([this] { Watch(); });
        } catch (const std::system_error&) {
            return CTS_E_NOMEM;
        }
        return CTS_OK;
    }

    // no grid runs (or Init): every slot and part record empty, group g's job numbers from 0 again
    void ResetRings()
    {
        std::memset(slots, 0, sizeof(cts::MailSlot) * nslots);
        std::memset(parts, 0, sizeof(cts::MailPart) * nslots * cts::kMailGroup);
        for (uint32_t i = 0; i < nslots; ++i) free_at[i].store(i % per_group, std::memory_order_relaxed);  // job j of its group
        for (uint32_t i = 0; i < cts::kMailMaxGroups; ++i) next[i] = busy[i] = 0;
    }

    // under mu: the grid's last launch has ended (or there was none)
    bool DrainedLocked()
    {
        if (launches.load(std::memory_order_relaxed) == 0) return true;
        DeviceGuard g(e->device);
        return hipEventQuery(grid_done) == hipSuccess;
    }

    // under mu: start the grid at every group's next job (after any grid still draining, same stream)
    int LaunchLocked()
    {
        DeviceGuard g(e->device);
        if (!g.ok) return CTS_E_HIP;
        cts::MailStarts starts{};
        for (uint32_t i = 0; i < groups; ++i) starts.j[i] = next[i];
        const uint64_t delay = launches.load(std::memory_order_relaxed) == 0 ? delay_ticks : 0;
        if (cts::launch_mailbox(dslots, dparts, per_group, starts, groups, idle_ticks, stream, delay) != hipSuccess ||
            hipEventRecord(grid_done, stream) != hipSuccess)
            return CTS_E_HIP;
        running = true;
        launches.fetch_add(1, std::memory_order_relaxed);
        const auto now = std::chrono::steady_clock::now();
        for (uint32_t i = 0; i < groups; ++i) last_used[i] = now;
        return CTS_OK;
    }

    // Claim a job number in the least busy group (launching the grid if needed), write the job, wait
    // for the answer. Verify [ptr, ptr + len) (len > 0), or stop the grid (len == 0: one stop job per
    // group, so every group leaves; only_if_idle: not while another job is outstanding).
    int Post(uint64_t ptr, uint32_t len, uint32_t expected, cts_verify_result* out, bool only_if_idle)
    {
        uint64_t js[cts::kMailMaxGroups];
        uint32_t g0 = 0, n = 1;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (broken) {
                // a job timed out: start over once nothing is outstanding and the grid has ended
                if (len == 0 || outstanding != 0 || !DrainedLocked()) return CTS_E_HIP;
                ResetRings();
                broken = false;
                broken_flag.store(false, std::memory_order_release);
            }
            if (len != 0 && paused != 0) return CTS_E_HIP;  // a free is waiting for the grid to end
            if (len == 0) {
                if (!running || (only_if_idle && outstanding != 0)) return CTS_OK;
                running = false;
                // a grid that already left on its own (idle exit) answers no stop job
                if (outstanding == 0 && DrainedLocked()) return CTS_OK;
                n = groups;
            } else {
                const auto now = std::chrono::steady_clock::now();
                if (running && now - last_post > std::chrono::milliseconds(exit_ms / 2)) {
                    // silent long enough that the grid may have left on its own (the watchdog was starved)
                    DeviceGuard g(e->device);
                    if (hipEventQuery(grid_done) == hipSuccess) running = false;
                }
                if (!running) {
                    const int rc = LaunchLocked();
                    if (rc != CTS_OK) return rc;
                }
                for (uint32_t i = 1; i < groups; ++i)
                    if (busy[i] < busy[g0]) g0 = i;
                // keep every group inside its idle exit: one that has waited exit_ms / 4 takes this job
                for (uint32_t i = 0; i < groups; ++i)
                    if (busy[i] == 0 && now - last_used[i] > std::chrono::milliseconds(exit_ms / 4)) {
                        g0 = i;
                        break;
                    }
                last_used[g0] = now;
            }
            for (uint32_t i = 0; i < n; ++i) {
                js[i] = next[g0 + i]++;
                ++busy[g0 + i];
            }
            ++outstanding;
            last_post = std::chrono::steady_clock::now();
        }
        int rc = CTS_OK;
        for (uint32_t i = 0; i < n && rc == CTS_OK; ++i) rc = Run(g0 + i, js[i], ptr, len, expected, out);
        std::lock_guard<std::mutex> lk(mu);
        if (rc != CTS_OK) {
            broken = true;  // a straggler may still read or answer the slot: never reuse it
            broken_flag.store(true, std::memory_order_release);
            running = false;
        }
        for (uint32_t i = 0; i < n; ++i) --busy[g0 + i];
        --outstanding;
        return rc;
    }

    // Group g's job j: wait for its slot, write the job, fold the part records.
    int Run(uint32_t g, uint64_t j, uint64_t ptr, uint32_t len, uint32_t expected, cts_verify_result* out)
    {
        const uint32_t k = g * per_group + (uint32_t)(j % per_group);
        const uint64_t t = j;
        while (free_at[k].load(std::memory_order_acquire) != t) {
            // the slot's previous ticket timed out: it is never freed, and the mailbox is broken
            if (broken_flag.load(std::memory_order_acquire)) return CTS_E_HIP;
            std::this_thread::yield();
        }
        const uint32_t tag = (uint32_t)(t + 1);
        // the job half first, then the tagged half: the grid's one 16-B read of a copy sees a new tag only
        // with the new job
        cts::mail_write(slots + k, (ptr & 0xFFFFFFFFFFFFull) | ((uint64_t)expected << 48), (uint64_t)len | ((uint64_t)tag << 32));
        const uint32_t np = cts::mail_parts(ptr, len);
        const cts::MailPart* const pr = parts + (size_t)k * cts::kMailGroup;
        const auto t_start = std::chrono::steady_clock::now();
        uint32_t first = 0xFFFFFFFFu, actual = 0;
        uint64_t count = 0;
        for (uint32_t i = 0; i < np; ++i) {
            uint64_t g0, g1;
            for (uint32_t spin = 0;; ++spin) {
                g0 = __atomic_load_n(&pr[i].g0, __ATOMIC_ACQUIRE);
                g1 = __atomic_load_n(&pr[i].g1, __ATOMIC_ACQUIRE);
                if ((uint32_t)(g0 >> 32) == tag && (uint32_t)(g1 >> 40) == (tag & 0xFFFFFFu)) break;
                if ((spin & 255u) == 255u) {
                    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > timeout_s)
                        return CTS_E_HIP;
                    std::this_thread::yield();
                }
            }
            if ((uint32_t)g0 < first) {
                first = (uint32_t)g0;
                actual = (uint32_t)(g1 >> 32) & 0xFFu;
            }
            count += (uint32_t)g1;
        }
        free_at[k].store(t + per_group, std::memory_order_release);
        if (out != nullptr && len != 0) {
            // RtlCompareMemory of the whole buffer (ctsIOPattern.cpp:753-774): the smallest first
            // difference over the pieces; expected/actual are the two bytes the reference prints
            const bool pass = first == 0xFFFFFFFFu;
            out->first_mismatch = pass ? len : first;
            out->mismatch_bytes = (uint32_t)count;
            out->expected = pass ? 0 : cts_pattern_byte((uint64_t)expected + first);
            out->actual = pass ? 0 : (uint8_t)actual;
            out->pass = pass ? 1 : 0;
            out->flags = 0;
        }
        return CTS_OK;
    }

    int Stop(bool only_if_idle) { return Post(0, 0, 0, nullptr, only_if_idle); }

    // Stop the grid and wait (bounded) until it has ended; posts fall back to a launch until Resume.
    void Pause()
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            ++paused;
        }
        (void)Stop(false);
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            {
                std::lock_guard<std::mutex> lk(mu);
                if (DrainedLocked()) return;
            }
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) return;
            std::this_thread::yield();
        }
    }
    void Resume()
    {
        std::lock_guard<std::mutex> lk(mu);
        --paused;
    }

    // under mu: a no-op job for every group that has had none for exit_ms / 4, so no group reaches its idle exit
    // while the grid is meant to run. The slot of a no-op is free again at once (no workgroup answers it).
    void KeepaliveLocked(std::chrono::steady_clock::time_point now)
    {
        for (uint32_t g = 0; g < groups; ++g) {
            if (busy[g] != 0 || now - last_used[g] <= std::chrono::milliseconds(exit_ms / 4)) continue;
            const uint64_t t = next[g];
            const uint32_t k = g * per_group + (uint32_t)(t % per_group);
            if (free_at[k].load(std::memory_order_acquire) != t) continue;  // (busy == 0: always free)
            ++next[g];
            cts::mail_write(slots + k, 0, (uint64_t)cts::kMailSkip | ((uint64_t)(uint32_t)(t + 1) << 32));
            free_at[k].store(t + per_group, std::memory_order_release);
            last_used[g] = now;
        }
    }

    void Watch()
    {
        std::unique_lock<std::mutex> lk(mu);
        while (!quit) {
            cv.wait_for(lk, std::chrono::milliseconds(std::max(1, std::min(idle_ms / 2, exit_ms / 8))));
            if (quit || !running || broken) continue;
            const auto now = std::chrono::steady_clock::now();
            // keep the groups alive while posts keep coming; after exit_ms / 2 of silence the grid may leave on
            // its own (the next post sees it ended and relaunches)
            if (now - last_post < std::chrono::milliseconds(exit_ms / 2)) KeepaliveLocked(now);
            if (outstanding != 0) continue;
            if (now - last_post < std::chrono::milliseconds(idle_ms)) continue;
            lk.unlock();
            (void)Stop(true);
            lk.lock();
        }
    }
};

namespace {

// Every engine's mailbox, whatever its device. hipHostFree is an implicit hipDeviceSynchronize of the current
// device: a resident grid on that device, any engine's, would hold a free up for as long as its callers keep
// posting. A pinned free therefore makes its engine's device current and stops every grid on it first
// (DeviceQuiesce); the grids relaunch on their next post.
std::mutex g_mail_reg_mu;  // guards g_mail_reg; held while a free pauses grids (lock order: before any Mailbox::mu)
std::vector<Mailbox*> g_mail_reg;

class DeviceQuiesce {
public:
    explicit DeviceQuiesce(int device) : dev_(device), guard_(device), lk_(g_mail_reg_mu)
    {
        for (Mailbox* m : g_mail_reg)
            if (m->e->device == dev_) m->Pause();
    }
    ~DeviceQuiesce()
    {
        for (Mailbox* m : g_mail_reg)
            if (m->e->device == dev_) m->Resume();
    }
    DeviceQuiesce(const DeviceQuiesce&) = delete;
    DeviceQuiesce& operator=(const DeviceQuiesce&) = delete;

private:
    int dev_;
    DeviceGuard guard_;
    std::unique_lock<std::mutex> lk_;
};

int pinned_free_on(int device, void* p)
{
    DeviceQuiesce q(device);
    return hip_status(hipHostFree(p));
}

void pinned_free(cts_engine* e, void* p) { (void)pinned_free_on(e->device, p); }

int mailbox_of(cts_engine* e, Mailbox** out)
{
    std::lock_guard<std::mutex> lk(e->mail_init_mu);
    if (!e->mail) {
        std::unique_ptr<Mailbox> m(new (std::nothrow) Mailbox());
        if (!m) return CTS_E_NOMEM;
        const int rc = m->Init(e);
        if (rc != CTS_OK) return rc;
        {
            std::lock_guard<std::mutex> lk(g_mail_reg_mu);
            try {
                g_mail_reg.push_back(m.get());
            } catch (const std::bad_alloc&) {  // nothing may cross the C ABI
                return CTS_E_NOMEM;
            }
        }
        e->mail = std::move(m);
    }
    *out = e->mail.get();
    return CTS_OK;
}

}  // namespace

Mailbox::~Mailbox()
{
    if (e == nullptr) return;
    {
        std::lock_guard<std::mutex> lk(g_mail_reg_mu);  // no free pauses this mailbox from here on
        g_mail_reg.erase(std::remove(g_mail_reg.begin(), g_mail_reg.end(), this), g_mail_reg.end());
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        quit = true;
    }
    cv.notify_all();
    if (watchdog.joinable()) watchdog.join();
    (void)Stop(false);
    {
        DeviceGuard g(e->device);
        if (stream) {
            (void)hipStreamSynchronize(stream);
            (void)hipStreamDestroy(stream);
        }
        if (grid_done) (void)hipEventDestroy(grid_done);
    }
    if (parts == nullptr && slots == nullptr) return;
    DeviceQuiesce q(e->device);  // the other engines' grids on this device
    if (parts) (void)hipHostFree(parts);
    if (slots) (void)hipHostFree(slots);
}

extern "C" {

const char* cts_version(void) { return "ctstraffic_amd 0.3.0 (gfx950)"; }

const char* cts_status_string(int status)
{
    switch (status) {
    case CTS_OK: return "ok";
    case CTS_E_INVALID: return "invalid argument";
    case CTS_E_HIP: return "HIP runtime error";
    case CTS_E_NOMEM: return "out of memory";
    case CTS_E_NO_DEVICE: return "no such HIP device";
    case CTS_E_UNAVAILABLE: return "runtime library unavailable (RCCL)";
    case CTS_E_TIMEOUT: return "timed out (nothing freed; retry)";
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
    e->geo.small_blocks_per_cu = env_int("CTS_SMALL_BLOCKS_PER_CU", e->geo.small_blocks_per_cu);
    e->geo.fill_blocks_per_cu = env_int("CTS_FILL_BLOCKS_PER_CU", e->geo.fill_blocks_per_cu);
    e->geo.small_chunk = env_int("CTS_SMALL_CHUNK", e->geo.small_chunk);
    e->geo.fill_nt = env_int("CTS_FILL_NT", e->geo.fill_nt);
    e->geo.ring_fill_blocks_per_cu = env_int("CTS_RING_FILL_BLOCKS_PER_CU", e->geo.ring_fill_blocks_per_cu);
    e->sync_mailbox = env_int("CTS_SYNC_MAILBOX", e->sync_mailbox) ? 1 : 0;
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
    e->mail.reset();  // stops the resident grid (kMailStop) and joins its watchdog
    {
        DeviceGuard g(e->device);
        if (e->stream) {
            (void)hipStreamSynchronize(e->stream);
            (void)hipStreamDestroy(e->stream);
        }
    }
    {
        DeviceQuiesce q(e->device);  // the other engines' grids on this device
        for (auto& st : e->stage_pool) (void)hipHostFree(st.p);
        e->stage_pool.clear();
        if (e->stage) (void)hipHostFree(e->stage);
        if (e->stage_desc) (void)hipHostFree(e->stage_desc);
        if (e->stage_res) (void)hipHostFree(e->stage_res);
        if (e->batch_desc) (void)hipHostFree(e->batch_desc);
        if (e->batch_res) (void)hipHostFree(e->batch_res);
        if (e->batch_ctr) (void)hipHostFree(e->batch_ctr);
    }
    delete e;
    return CTS_OK;
}

int cts_engine_device(const cts_engine* e) { return e ? e->device : CTS_E_INVALID; }

int cts_engine_numa_node(const cts_engine* e)
{
    if (e == nullptr) return -1;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), e->device) != hipSuccess) return -1;
    std::string path = "/sys/bus/pci/devices/";
    for (const char* c = bus; *c; ++c) path += (char)std::tolower((unsigned char)*c);
    path += "/numa_node";
    FILE* f = std::fopen(path.c_str(), "r");
    if (f == nullptr) return -1;
    int node = -1;
    if (std::fscanf(f, "%d", &node) != 1) node = -1;
    std::fclose(f);
    return node;
}

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
    // the kernel of each path is fixed: its id is accepted, nothing else
    case CTS_ATTR_VERIFY_VARIANT: return value == cts::kVerifyKernelId ? CTS_OK : CTS_E_INVALID;
    case CTS_ATTR_SMALL_VARIANT: return value == cts::kSmallKernelId ? CTS_OK : CTS_E_INVALID;
    case CTS_ATTR_MS_VARIANT: return value == cts::kMediaStreamKernelId ? CTS_OK : CTS_E_INVALID;
    case CTS_ATTR_SMALL_BLOCKS_PER_CU:
        if (value < 1 || value > 256) return CTS_E_INVALID;
        e->geo.small_blocks_per_cu = value;
        return CTS_OK;
    case CTS_ATTR_FILL_BLOCKS_PER_CU:
        if (value < 1 || value > 64) return CTS_E_INVALID;
        e->geo.fill_blocks_per_cu = value;
        return CTS_OK;
    case CTS_ATTR_SMALL_CHUNK:
        if (value < 0 || value > (1 << 24)) return CTS_E_INVALID;
        e->geo.small_chunk = value;
        return CTS_OK;
    case CTS_ATTR_SYNC_MAILBOX: e->sync_mailbox = value ? 1 : 0; return CTS_OK;
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
    case CTS_ATTR_VERIFY_VARIANT: *value = cts::kVerifyKernelId; return CTS_OK;
    case CTS_ATTR_SMALL_BLOCKS_PER_CU: *value = e->geo.small_blocks_per_cu; return CTS_OK;
    case CTS_ATTR_SMALL_VARIANT: *value = cts::kSmallKernelId; return CTS_OK;
    case CTS_ATTR_FILL_BLOCKS_PER_CU: *value = e->geo.fill_blocks_per_cu; return CTS_OK;
    case CTS_ATTR_MS_VARIANT: *value = cts::kMediaStreamKernelId; return CTS_OK;
    case CTS_ATTR_SMALL_CHUNK: *value = e->geo.small_chunk; return CTS_OK;
    case CTS_ATTR_FILL_NT: *value = e->geo.fill_nt; return CTS_OK;
    case CTS_ATTR_SYNC_MAILBOX: *value = e->sync_mailbox; return CTS_OK;
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

// The kernels write 12-byte records and DataError slots as dwords and add to the counter block with 64-bit
// atomics: a misaligned output would fault on the device, so it is refused here.
static bool outputs_misaligned(const void* results, const void* counters, const void* conn_first_fail = nullptr)
{
    return ((uintptr_t)results & 3u) != 0 || ((uintptr_t)counters & 7u) != 0 || ((uintptr_t)conn_first_fail & 3u) != 0;
}

int cts_verify(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs, uint32_t n,
               uint32_t max_length_hint, cts_verify_result* dev_results, void* dev_counters,
               uint32_t* dev_conn_first_fail, uint32_t n_conns, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || ((uintptr_t)dev_arena & 15u) != 0) return CTS_E_INVALID;
    if (dev_conn_first_fail == nullptr && n_conns != 0) return CTS_E_INVALID;
    if (outputs_misaligned(dev_results, dev_counters, dev_conn_first_fail)) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_verify(static_cast<const uint8_t*>(dev_arena), arena_bytes, dev_descs, n,
                                         max_length_hint, dev_results, static_cast<uint64_t*>(dev_counters),
                                         dev_conn_first_fail, n_conns, static_cast<hipStream_t>(stream), e->geo));
}

int cts_verify_strided(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                       const uint32_t* dev_lengths, uint32_t n, uint32_t skip_head, uint32_t expected_offset,
                       uint32_t conn_index, cts_verify_result* dev_results, void* dev_counters,
                       uint32_t* dev_conn_first_fail, uint32_t n_conns, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_lengths == nullptr || stride == 0 || arena_bytes < 16 ||
        ((uintptr_t)dev_arena & 15u) != 0 || ((uintptr_t)dev_lengths & 3u) != 0)
        return CTS_E_INVALID;
    if (expected_offset >= CTS_PATTERN_PERIOD) return CTS_E_INVALID;
    if (dev_conn_first_fail == nullptr && n_conns != 0) return CTS_E_INVALID;
    if (outputs_misaligned(dev_results, dev_counters, dev_conn_first_fail)) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_verify_strided(static_cast<const uint8_t*>(dev_arena), arena_bytes, stride, dev_lengths, n,
                                                 skip_head, expected_offset, conn_index, dev_results,
                                                 static_cast<uint64_t*>(dev_counters), dev_conn_first_fail, n_conns,
                                                 static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_fill(cts_engine* e, void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs,
                          const cts_datagram_header* dev_headers, uint32_t n, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || dev_headers == nullptr ||
        ((uintptr_t)dev_headers & 7u) != 0)
        return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_fill(static_cast<uint8_t*>(dev_arena), arena_bytes, dev_descs,
                                                    dev_headers, n, static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_fill_strided(cts_engine* e, void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                                  const uint32_t* dev_lengths, const cts_datagram_header* dev_headers, uint32_t n,
                                  void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || ((uintptr_t)dev_arena & 15u) != 0 || dev_lengths == nullptr ||
        ((uintptr_t)dev_lengths & 3u) != 0 || dev_headers == nullptr || ((uintptr_t)dev_headers & 7u) != 0 ||
        stride < 32u || (stride & 15u) != 0 || stride > (1u << 20))
        return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_fill_strided(static_cast<uint8_t*>(dev_arena), arena_bytes, stride,
                                                            dev_lengths, dev_headers, n,
                                                            static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_verify(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs,
                            uint32_t n, cts_datagram_record* dev_records, cts_verify_result* dev_results,
                            void* dev_counters, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || ((uintptr_t)dev_arena & 15u) != 0) return CTS_E_INVALID;
    if (outputs_misaligned(dev_results, dev_counters, dev_records)) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_verify(static_cast<const uint8_t*>(dev_arena), arena_bytes, dev_descs,
                                                      n, dev_records, dev_results,
                                                      static_cast<uint64_t*>(dev_counters),
                                                      static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_verify_strided(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                                    const uint32_t* dev_lengths, uint32_t n, cts_datagram_record* dev_records,
                                    cts_verify_result* dev_results, void* dev_counters, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_lengths == nullptr || ((uintptr_t)dev_lengths & 3u) != 0 ||
        ((uintptr_t)dev_arena & 15u) != 0 || arena_bytes < 16u || stride == 0)
        return CTS_E_INVALID;
    if (outputs_misaligned(dev_results, dev_counters, dev_records)) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_verify_strided(static_cast<const uint8_t*>(dev_arena), arena_bytes, stride,
                                                              dev_lengths, n, dev_records, dev_results,
                                                              static_cast<uint64_t*>(dev_counters),
                                                              static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_verify_status(cts_engine* e, const void* dev_arena, uint64_t arena_bytes,
                                   const cts_buf_desc* dev_descs, uint32_t n, cts_datagram_status* dev_status,
                                   void* dev_counters, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_descs == nullptr || ((uintptr_t)dev_descs & 7u) != 0 || ((uintptr_t)dev_arena & 15u) != 0 ||
        outputs_misaligned(dev_status, dev_counters))
        return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_status(static_cast<const uint8_t*>(dev_arena), arena_bytes, dev_descs,
                                                      nullptr, 0u, n, dev_status, static_cast<uint64_t*>(dev_counters),
                                                      static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_verify_strided_status(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                                           const uint32_t* dev_lengths, uint32_t n, cts_datagram_status* dev_status,
                                           void* dev_counters, void* stream)
{
    if (e == nullptr) return CTS_E_INVALID;
    if (n == 0) return CTS_OK;
    if (dev_arena == nullptr || dev_lengths == nullptr || ((uintptr_t)dev_lengths & 3u) != 0 ||
        ((uintptr_t)dev_arena & 15u) != 0 || arena_bytes < 16u || stride == 0 || outputs_misaligned(dev_status, dev_counters))
        return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_status(static_cast<const uint8_t*>(dev_arena), arena_bytes, nullptr,
                                                      dev_lengths, stride, n, dev_status,
                                                      static_cast<uint64_t*>(dev_counters),
                                                      static_cast<hipStream_t>(stream), e->geo));
}

static int media_stream_frames(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, const cts_buf_desc* dev_descs,
                               uint32_t stride, const uint32_t* dev_lengths, uint32_t n, const cts_frame_window* w,
                               void* dev_totals, uint64_t* dev_frame_bytes, void* dev_counters, void* stream)
{
    if (e == nullptr || w == nullptr || dev_totals == nullptr || ((uintptr_t)dev_totals & 7u) != 0 ||
        (w->frames != 0 && (dev_frame_bytes == nullptr || ((uintptr_t)dev_frame_bytes & 7u) != 0)))
        return CTS_E_INVALID;
    if (n != 0 && (dev_arena == nullptr || ((uintptr_t)dev_arena & 15u) != 0 || outputs_misaligned(nullptr, dev_counters)))
        return CTS_E_INVALID;
    if (n != 0 && dev_descs == nullptr &&
        (dev_lengths == nullptr || ((uintptr_t)dev_lengths & 3u) != 0 || arena_bytes < 16u || stride == 0))
        return CTS_E_INVALID;
    if (n != 0 && dev_descs != nullptr && ((uintptr_t)dev_descs & 7u) != 0) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(cts::launch_media_stream_frames(static_cast<const uint8_t*>(dev_arena), arena_bytes, dev_descs,
                                                      dev_lengths, stride, n, *w, static_cast<uint64_t*>(dev_totals),
                                                      dev_frame_bytes, static_cast<uint64_t*>(dev_counters),
                                                      static_cast<hipStream_t>(stream), e->geo));
}

int cts_media_stream_verify_frames(cts_engine* e, const void* dev_arena, uint64_t arena_bytes,
                                   const cts_buf_desc* dev_descs, uint32_t n, const cts_frame_window* window,
                                   void* dev_totals, uint64_t* dev_frame_bytes, void* dev_counters, void* stream)
{
    if (n != 0 && dev_descs == nullptr) return CTS_E_INVALID;
    return media_stream_frames(e, dev_arena, arena_bytes, dev_descs, 0u, nullptr, n, window, dev_totals,
                               dev_frame_bytes, dev_counters, stream);
}

int cts_media_stream_verify_strided_frames(cts_engine* e, const void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                                           const uint32_t* dev_lengths, uint32_t n, const cts_frame_window* window,
                                           void* dev_totals, uint64_t* dev_frame_bytes, void* dev_counters,
                                           void* stream)
{
    if (n != 0 && dev_lengths == nullptr) return CTS_E_INVALID;
    return media_stream_frames(e, dev_arena, arena_bytes, nullptr, stride, dev_lengths, n, window, dev_totals,
                               dev_frame_bytes, dev_counters, stream);
}

size_t cts_counters_device_bytes(void) { return (size_t)CTS_COUNTER_SHARDS * cts::kCounterSlots * sizeof(uint64_t); }

int cts_counters_reset(cts_engine* e, void* dev_counters, void* stream)
{
    if (e == nullptr || dev_counters == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    return hip_status(hipMemsetAsync(dev_counters, 0, cts_counters_device_bytes(), static_cast<hipStream_t>(stream)));
}

int cts_counters_read_ex(cts_engine* e, const void* dev_counters, cts_counters_ex* out, void* stream)
{
    if (e == nullptr || dev_counters == nullptr || out == nullptr) return CTS_E_INVALID;
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    uint64_t h[CTS_COUNTER_SHARDS * cts::kCounterSlots];  // 4 KiB: no allocation on the ABI path
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (hipMemcpyAsync(h, dev_counters, cts_counters_device_bytes(), hipMemcpyDeviceToHost, s) != hipSuccess)
        return CTS_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return CTS_E_HIP;
    uint64_t v[cts::kCounterCount] = {};
    for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh)
        for (int k = 0; k < cts::kCounterCount; ++k) v[k] += h[sh * cts::kCounterSlots + k];
    *out = cts::counters_ex_of(v);
    return CTS_OK;
}

int cts_counters_read(cts_engine* e, const void* dev_counters, cts_counters* out, void* stream)
{
    if (out == nullptr) return CTS_E_INVALID;
    cts_counters_ex x{};
    const int rc = cts_counters_read_ex(e, dev_counters, &x, stream);
    if (rc == CTS_OK) *out = cts::counters_of(x);
    return rc;
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
            (void)pinned_free_on(e->device, p);
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
    // hipHostFree waits for the device's kernels: every resident mailbox grid on the device is stopped first, so a
    // free returns while other threads keep posting (their verifies take the launch path meanwhile)
    return pinned_free_on(e->device, host_ptr);
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
    if (e->sync_mailbox) {
        // copy into a staging buffer of this call's own (concurrent callers do not wait for each other) and
        // post it to the resident mailbox grid: no launch or stream synchronize per call
        cts_engine::HostStage st;
        {
            std::lock_guard<std::mutex> lk(e->stage_pool_mu);
            if (!e->stage_pool.empty()) {
                st = e->stage_pool.back();
                e->stage_pool.pop_back();
            }
        }
        int rc = ensure_pinned(e, &st.p, &st.cap, (size_t)len + 16, 64u << 10);
        const uint8_t* dev = rc == CTS_OK ? device_view(static_cast<uint8_t*>(st.p)) : nullptr;
        if (rc == CTS_OK && dev == nullptr) rc = CTS_E_HIP;
        if (rc == CTS_OK) {
            if (len) std::memcpy(st.p, host_buf, len);
            rc = cts_verify_mapped(e, dev, len, expected_offset, out);
        }
        if (st.p != nullptr) {
            bool pooled = false;
            {
                std::lock_guard<std::mutex> lk(e->stage_pool_mu);
                try {
                    e->stage_pool.push_back(st);
                    pooled = true;
                } catch (const std::bad_alloc&) {  // nothing may cross the C ABI: the stage is freed instead
                }
            }
            if (!pooled) pinned_free(e, st.p);
        }
        return rc;
    }
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
    if ((rc = ensure_pinned(e, &e->batch_desc, &e->batch_desc_cap, sizeof(cts_buf_desc) * n, 4096)) != CTS_OK) return rc;
    if ((rc = ensure_pinned(e, &e->batch_res, &e->batch_res_cap, sizeof(cts_verify_result) * n, 4096)) != CTS_OK) return rc;
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
    if (len == 0) {  // RtlCompareMemory of nothing: a match (no device work)
        *out = cts_verify_result{0, 0, 0, 0, 1, 0};
        return CTS_OK;
    }
    Mailbox* m = nullptr;
    const int rc = mailbox_of(e, &m);
    if (rc != CTS_OK) return rc;
    if (m->Post(reinterpret_cast<uint64_t>(dev_buf), len, expected_offset, out, false) == CTS_OK) return CTS_OK;
    // the mailbox is broken (a job timed out; it starts over once its grid has drained) or paused (a free is
    // waiting for the grid to end): this verify takes one sliced launch + synchronize instead
    std::lock_guard<std::mutex> lk(e->host_mu);
    DeviceGuard g(e->device);
    if (!g.ok) return CTS_E_HIP;
    const uint64_t d = reinterpret_cast<uintptr_t>(dev_buf) & 15u;  // (the arena base must be 16-byte aligned)
    uint32_t slice_len = 0;
    const uint32_t ns = cts::slice_plan(d, len, expected_offset, 0, e->stage_desc, &slice_len);
    const cts_buf_desc* dd = device_view(e->stage_desc);
    cts_verify_result* dr = device_view(e->stage_res);
    if (!dd || !dr) return CTS_E_HIP;
    hipError_t err = cts::launch_verify(static_cast<const uint8_t*>(dev_buf) - d, d + len, dd, ns, slice_len, dr,
                                        nullptr, nullptr, 0, e->stream, e->geo);
    if (err == hipSuccess) err = hipStreamSynchronize(e->stream);
    if (err != hipSuccess) return CTS_E_HIP;
    *out = cts::slice_merge(e->stage_res, ns, slice_len, len);
    return CTS_OK;
}

uint64_t cts_mailbox_launches(const cts_engine* e)
{
    return (e != nullptr && e->mail) ? e->mail->launches.load(std::memory_order_relaxed) : 0;
}

}  // extern "C"
