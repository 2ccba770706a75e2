// mailbox_bisect.hip — the product mailbox kernel (cts_kernels.hip, included verbatim) driven by a bare
// host loop: no engine, no mutex, no ticket bookkeeping. Per 64 KiB verify it reports the mean time from
// writing the job to the first and to the last of the group's part records, so the gap between
// tools/sync_probe (cts_verify_mapped) and tools/mailbox_probe's ping-pong splits into host overhead,
// the kernel's own work, and the spread of the 16 workgroups' poll phases. Diagnostic only.
//   build: make tools/mailbox_bisect     run: tools/mailbox_bisect [iters]
#define CTS_MAILBOX_TRACE 1
#include "../ctstraffic_amd/csrc/cts_kernels.hip"

#include <algorithm>
#include <vector>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename T>
static T* host_coherent(size_t bytes, T** dev)
{
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess)
        return nullptr;
    std::memset(p, 0, bytes);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) return nullptr;
    *dev = static_cast<T*>(d);
    return static_cast<T*>(p);
}

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
    const uint32_t len = 65536, nslots = 1024;
    uint8_t *buf = nullptr, *dbuf = nullptr;
    void* p = nullptr;
    if (hipHostMalloc(&p, len, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) return 1;
    buf = static_cast<uint8_t*>(p);
    if (hipHostGetDevicePointer((void**)&dbuf, buf, 0) != hipSuccess) return 1;
    const uint32_t expected = 1000;
    for (uint32_t b = 0; b < len; ++b) {  // the u16 little-endian ramp, period 64 KiB
        const uint32_t q = (expected + b) & 0xFFFFu;
        buf[b] = (uint8_t)((q >> 1) >> (8u * (q & 1u)));
    }
    const uint32_t polls = 1;
    for (const uint32_t G : {1u, 8u}) {
        cts::MailSlot* dslots = nullptr;
        cts::MailPart* dparts = nullptr;
        cts::MailSlot* slots = host_coherent<cts::MailSlot>(sizeof(cts::MailSlot) * nslots, &dslots);
        cts::MailPart* parts = host_coherent<cts::MailPart>(sizeof(cts::MailPart) * nslots * cts::kMailGroup, &dparts);
        if (!slots || !parts) return 1;
        hipStream_t s;
        (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        const size_t trace_n = 1024u * cts::kMailGroup * 8u;
        uint64_t* trace = nullptr;
        if (hipMalloc((void**)&trace, trace_n * 8) != hipSuccess) return 1;
        (void)hipMemset(trace, 0, trace_n * 8);
        if (hipMemcpyToSymbol(HIP_SYMBOL(cts::cts_mail_trace), &trace, sizeof(trace)) != hipSuccess) return 1;
        (void)hipDeviceSynchronize();
        // every job goes to group 0 (the engine's choice for one caller); the other G - 1 groups idle
        const uint32_t S = nslots / G;
        cts::MailStarts starts{};
        if (cts::launch_mailbox(dslots, dparts, S, starts, G, 100000000ull, s, 0) != hipSuccess) return 1;
        const uint64_t ptr = reinterpret_cast<uint64_t>(dbuf);
        const uint32_t np = cts::mail_parts(ptr, len);
        double sum_first = 0, sum_last = 0, t_begin = 0;
        int bad = 0;
        bool ok = true;
        uint64_t t = 0;
        for (int i = 0; i < iters + 100 && ok; ++i, ++t) {
            if (i == 100) t_begin = now_us();
            const uint32_t k = (uint32_t)(t % S), tag = (uint32_t)(t + 1);
            const double t0 = now_us();
            cts::mail_write(slots + k, (ptr & 0xFFFFFFFFFFFFull) | ((uint64_t)expected << 48), (uint64_t)len | ((uint64_t)tag << 32));
            const cts::MailPart* const pr = parts + (size_t)k * cts::kMailGroup;
            double t_first = 0;
            uint32_t seen = 0, first = 0xFFFFFFFFu;
            uint32_t done[cts::kMailGroup] = {};
            while (seen < np) {
                for (uint32_t j = 0; j < np; ++j) {
                    if (done[j]) continue;
                    const uint64_t g0 = __atomic_load_n(&pr[j].g0, __ATOMIC_ACQUIRE);
                    const uint64_t g1 = __atomic_load_n(&pr[j].g1, __ATOMIC_ACQUIRE);
                    if ((uint32_t)(g0 >> 32) != tag || (uint32_t)(g1 >> 40) != (tag & 0xFFFFFFu)) continue;
                    done[j] = 1;
                    if (seen++ == 0) t_first = now_us();
                    first = (uint32_t)g0 < first ? (uint32_t)g0 : first;
                }
                if (now_us() - t0 > 2e6) {
                    ok = false;
                    break;
                }
            }
            const double t1 = now_us();
            if (first != 0xFFFFFFFFu) ++bad;
            if (i >= 100) {
                sum_first += t_first - t0;
                sum_last += t1 - t0;
            }
        }
        const double total = now_us() - t_begin;
        // stop: one stop job per group (len 0; group 0 at job t, the others at job 0), then let the grid drain
        for (uint32_t g = 0; g < G && ok; ++g) {
            const uint64_t jg = g == 0 ? t : 0;
            cts::mail_write(slots + g * S + (uint32_t)(jg % S), 0ull, (uint64_t)(uint32_t)(jg + 1) << 32);
        }
        (void)hipStreamSynchronize(s);
        // GPU-side split of the last 1024 tickets (s_memrealtime: 10 ns ticks): spread of the 16
        // workgroups' matching polls, poll -> data compared, compared -> part stored, first match -> last store
        {
            std::vector<uint64_t> h(trace_n);
            (void)hipMemcpy(h.data(), trace, trace_n * 8, hipMemcpyDeviceToHost);
            double spread = 0, work = 0, work_max = 0, store = 0, span = 0, wave_spread = 0, last_wave = 0, st_after = 0;
            int nw = 0;
            int n = 0;
            for (uint64_t tt = t - 1023; tt < t; ++tt) {
                const uint64_t* r = h.data() + (tt % 1024u) * cts::kMailGroup * 8u;
                uint64_t dmin = ~0ull, dmax = 0, smax = 0, wmax = 0;
                double wsum = 0, ssum = 0;
                bool okr = true;
                for (uint32_t w = 0; w < np; ++w) {
                    const uint64_t d = r[w * 8], c = r[w * 8 + 1], st = r[w * 8 + 2];
                    uint64_t wlo = ~0ull, whi = 0;
                    for (int x = 4; x < 8; ++x) {
                        wlo = std::min(wlo, r[w * 8 + x]);
                        whi = std::max(whi, r[w * 8 + x]);
                    }
                    if (whi >= d && wlo >= d) {
                        wave_spread += (double)(whi - wlo);
                        last_wave += (double)(whi - d);
                        st_after += st >= whi ? (double)(st - whi) : 0.0;
                        ++nw;
                    }
                    if (!d || !c || !st || c < d || st < c) okr = false;
                    dmin = std::min(dmin, d);
                    dmax = std::max(dmax, d);
                    smax = std::max(smax, st);
                    wmax = std::max(wmax, c - d);
                    wsum += (double)(c - d);
                    ssum += (double)(st - c);
                }
                if (!okr) continue;
                spread += (double)(dmax - dmin);
                work += wsum / np;
                work_max += (double)wmax;
                store += ssum / np;
                span += (double)(smax - dmin);
                ++n;
            }
            if (n)
                std::printf("{\"polls\": %u, \"groups\": %u, \"tickets\": %d, \"us_poll_match_spread\": %.3f, \"us_match_to_compared\": %.3f, "
                            "\"us_match_to_compared_max\": %.3f, \"us_compared_to_stored\": %.3f, \"us_first_match_to_last_store\": %.3f, "
                            "\"us_data_wave_spread\": %.3f, \"us_match_to_last_wave\": %.3f, \"us_last_wave_to_stored\": %.3f}\n",
                            polls, G, n, spread / n / 100, work / n / 100, work_max / n / 100, store / n / 100, span / n / 100,
                            nw ? wave_spread / nw / 100 : 0.0, nw ? last_wave / nw / 100 : 0.0, nw ? st_after / nw / 100 : 0.0);
        }
        (void)hipFree(trace);
        std::printf("{\"polls\": %u, \"groups\": %u, \"iters\": %d, \"us_per_verify\": %.3f, \"us_to_first_part\": %.3f, "
                    "\"us_to_last_part\": %.3f, \"bad\": %d, \"ok\": %d}\n",
                    polls, G, iters, total / iters, sum_first / iters, sum_last / iters, bad, ok ? 1 : 0);
        std::fflush(stdout);
        (void)hipStreamDestroy(s);
        (void)hipHostFree(slots);
        (void)hipHostFree(parts);
        if (!ok) return 2;
    }
    return 0;
}
