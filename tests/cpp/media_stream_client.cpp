// media_stream_client.cpp — the MediaStream client's three feeds (cts_media_stream.cpp) under the sanitizers:
// per-datagram records + results, compact statuses, and per-batch frame sums (what media_stream_verify_quad_kernel
// writes in its FRAMES form, restated here from the statuses), over random streams with drops, duplicates, stale and
// future sequence numbers, datagrams past the final frame, zero-byte / short / ID datagrams and corrupt payloads,
// with render ticks between batches. The three clients must agree at every tick and at the end. Several streams then
// run on threads at once, so TSan sees the process-wide UDP counters (g_udp) fed from every client, and the counters
// must equal the sum of the clients' own statistics; the UDP status line and summary are formatted from them.
// Built with g++ against tests/cpp/engine_stub.cpp; run by tests/test_host_sanitizers.py.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "cts_media_stream.h"
#include "cts_pattern.h"
#include "cts_status.h"

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                \
        }                                                                \
    } while (0)

namespace {

struct Dgram {
    uint8_t kind;
    bool pass;
    uint32_t completed;
    int64_t seq;
};

// a server's stream of n_frames frames as the client receives it: datagrams of each frame in order, some dropped,
// some repeated, a few with a wrong sequence number, a few exceptions (per `exceptions`)
std::vector<Dgram> make_stream(std::mt19937_64& rng, uint32_t frame_size, uint32_t max_dgram, int64_t n_frames,
                               bool exceptions)
{
    std::vector<uint32_t> lens(frame_size);
    const uint64_t per = cts_media_stream_split(frame_size, max_dgram, lens.data(), lens.size());
    CHECK(per > 0 && per <= lens.size());
    std::uniform_real_distribution<double> u(0.0, 1.0);
    std::vector<Dgram> s;
    for (int64_t f = 1; f <= n_frames; ++f) {
        for (uint64_t k = 0; k < per; ++k) {
            const double r = u(rng);
            if (r < 0.03) continue;  // dropped
            int64_t seq = f;
            if (r > 0.985) seq = f + 2 + (int64_t)(rng() % 7);                 // a future (or past-final) frame
            else if (r > 0.975) seq = f > 3 ? f - 3 : f;                         // a stale one
            s.push_back(Dgram{CTS_DGRAM_DATA, true, lens[k], seq});
            if (u(rng) < 0.02) s.push_back(s.back());                           // repeated
        }
    }
    if (exceptions && s.size() > 16) {
        const size_t at = s.size() / 2 + rng() % (s.size() / 4);
        switch (rng() % 4) {
        case 0: s[at].pass = false; break;                                      // corrupt payload
        case 1: s[at] = Dgram{CTS_DGRAM_ZERO, false, 0, 0}; break;              // zero bytes mid-stream
        case 2: s[at] = Dgram{CTS_DGRAM_SHORT, false, 11, 0}; break;
        default: s.insert(s.begin() + (ptrdiff_t)at, Dgram{CTS_DGRAM_ID, false, 39, 0}); break;  // an ID datagram
        }
    }
    return s;
}

// media_stream_verify_quad_kernel's FRAMES sums of statuses st under window w
void sums_of(const cts_datagram_status* st, uint32_t n, const cts_frame_window& w, cts_frame_totals& t,
             std::vector<uint64_t>& fb)
{
    t = cts_frame_totals{};
    t.first_exception = 0xFFFFFFFFu;
    fb.assign(w.frames, 0);
    for (uint32_t i = 0; i < n; ++i) {
        const cts_datagram_status& d = st[i];
        if (d.kind == CTS_DGRAM_DATA && d.pass) {
            t.bits_received += 8ull * d.completed_bytes;
            ++t.datagrams;
            const int64_t k = d.sequence_number - w.head_sequence_number;
            if (d.sequence_number > w.final_frame || k < 0 || k >= (int64_t)w.frames) ++t.error_frames;
            else fb[(size_t)k] += d.completed_bytes;
        } else if (!(d.kind == CTS_DGRAM_ZERO && w.finished)) {
            ++t.exceptions;
            if (i < t.first_exception) t.first_exception = i;
        }
    }
}

bool same_stats(const cts_media_stream_stats& a, const cts_media_stream_stats& b)
{
    return a.bits_received == b.bits_received && a.successful_frames == b.successful_frames &&
           a.dropped_frames == b.dropped_frames && a.duplicate_frames == b.duplicate_frames &&
           a.error_frames == b.error_frames && a.datagrams == b.datagrams && a.last_error == b.last_error &&
           a.finished == b.finished && a.head_sequence_number == b.head_sequence_number &&
           a.has_failure == b.has_failure && a.fail_datagram == b.fail_datagram;
}

// One stream through the three clients in lockstep; returns the (common) final statistics.
cts_media_stream_stats run_stream(uint64_t seed, bool exceptions)
{
    std::mt19937_64 rng(seed);
    const uint32_t frame_size = 4000 + (uint32_t)(rng() % 9000), max_dgram = 1472;
    const uint32_t buffered = 2 + (uint32_t)(rng() % 5);
    const int64_t n_frames = 20 + (int64_t)(rng() % 40);
    const std::vector<Dgram> s = make_stream(rng, frame_size, max_dgram, n_frames, exceptions);
    const cts_media_stream_settings cfg{frame_size, max_dgram, 30, buffered, n_frames};
    cts_media_stream_client *cm = nullptr, *cs = nullptr, *cf = nullptr;
    CHECK(cts_media_stream_client_create(&cfg, &cm) == CTS_OK);
    CHECK(cts_media_stream_client_create(&cfg, &cs) == CTS_OK);
    CHECK(cts_media_stream_client_create(&cfg, &cf) == CTS_OK);
    const uint32_t batch = 1 + (uint32_t)(rng() % 24);
    std::vector<cts_datagram_record> recs;
    std::vector<cts_verify_result> res;
    std::vector<cts_datagram_status> st;
    std::vector<uint64_t> fb;
    size_t i = 0;
    int rc_m = CTS_IO_CONTINUE;
    for (uint32_t tick = 0; tick < 4 * (uint32_t)n_frames + 64; ++tick) {
        const uint32_t n = (uint32_t)std::min<size_t>(batch, s.size() - i);
        recs.assign(n, cts_datagram_record{});
        res.assign(n, cts_verify_result{});
        st.assign(n, cts_datagram_status{});
        for (uint32_t j = 0; j < n; ++j) {
            const Dgram& d = s[i + j];
            recs[j].sequence_number = d.kind == CTS_DGRAM_DATA ? d.seq : 0;
            recs[j].flag = d.kind == CTS_DGRAM_ID ? CTS_UDP_FLAG_ID : 0;
            recs[j].kind = d.kind;
            recs[j].completed_bytes = d.completed;
            res[j].pass = d.kind == CTS_DGRAM_DATA && d.pass ? 1 : 0;
            res[j].flags = d.kind == CTS_DGRAM_DATA ? 0 : CTS_RESULT_FLAG_NOT_DATA;
            st[j] = cts_datagram_status{recs[j].sequence_number, d.completed, recs[j].flag, d.kind,
                                        (uint8_t)res[j].pass};
        }
        i += n;
        uint32_t used_m = 0, used_s = 0;
        rc_m = cts_media_stream_client_complete(cm, recs.data(), res.data(), n, 1000 + tick, 1000000, &used_m);
        const int rc_s = cts_media_stream_client_complete_status(cs, st.data(), n, 1000 + tick, 1000000, &used_s);
        CHECK(rc_m >= 0 && rc_m == rc_s && used_m == used_s);
        cts_frame_window w{};
        CHECK(cts_media_stream_client_window(cf, &w) == CTS_OK);
        cts_frame_totals t{};
        sums_of(st.data(), n, w, t, fb);
        int rc_f = cts_media_stream_client_complete_frames(cf, &w, &t, fb.data(), n, 1000 + tick, 1000000);
        if (rc_f == CTS_MS_FRAMES_REPLAY) {
            uint32_t used_f = 0;
            rc_f = cts_media_stream_client_complete_status(cf, st.data(), n, 1000 + tick, 1000000, &used_f);
        }
        CHECK(rc_f == rc_m);
        // the sums of a batch are only valid for the window they were summed over
        if (w.frames > 1) {
            cts_frame_window moved = w;
            ++moved.head_sequence_number;
            CHECK(cts_media_stream_client_complete_frames(cf, &moved, &t, fb.data(), n, 0, 0) == CTS_E_INVALID);
        }
        if (tick % 2 == 1 || i == s.size()) {
            const int r1 = cts_media_stream_client_render(cm), r2 = cts_media_stream_client_render(cs),
                      r3 = cts_media_stream_client_render(cf);
            CHECK(r1 >= 0 && r1 == r2 && r1 == r3);
        }
        cts_media_stream_stats a{}, b{}, c{};
        CHECK(cts_media_stream_client_stats(cm, &a) == CTS_OK && cts_media_stream_client_stats(cs, &b) == CTS_OK &&
              cts_media_stream_client_stats(cf, &c) == CTS_OK);
        CHECK(same_stats(a, b) && same_stats(a, c));
        if (a.finished != 0 || rc_m == CTS_IO_FAILED) break;
    }
    cts_media_stream_stats a{};
    CHECK(cts_media_stream_client_stats(cm, &a) == CTS_OK);
    CHECK(cts_media_stream_client_destroy(cm) == CTS_OK && cts_media_stream_client_destroy(cs) == CTS_OK &&
          cts_media_stream_client_destroy(cf) == CTS_OK);
    return a;
}

}  // namespace

int main()
{
    // one thread: every feed agrees, clean and with exceptions
    uint32_t failed = 0, finished = 0;
    for (uint64_t seed = 1; seed <= 48; ++seed) {
        const cts_media_stream_stats a = run_stream(seed, seed % 3 == 0);
        failed += a.has_failure;
        finished += a.finished == 1;
    }
    CHECK(failed > 0 && finished > 0);

    // many clients at once: the process-wide counters are each client's statistics summed (x 3 feeds)
    cts_udp_status_details_reset();
    constexpr int kThreads = 6, kPer = 4;
    std::vector<cts_media_stream_stats> out(kThreads * kPer);
    std::vector<std::thread> th;
    for (int t = 0; t < kThreads; ++t)
        th.emplace_back([t, &out] {
            for (int k = 0; k < kPer; ++k) out[t * kPer + k] = run_stream(1000 + 31 * t + k, (t + k) % 2 == 0);
        });
    for (auto& x : th) x.join();
    cts_udp_status_details want{}, got{};
    for (const auto& a : out) {
        want.bits_received += 3 * a.bits_received;
        want.successful_frames += 3 * a.successful_frames;
        want.dropped_frames += 3 * a.dropped_frames;
        want.duplicate_frames += 3 * a.duplicate_frames;
        want.error_frames += 3 * a.error_frames;
    }
    CHECK(cts_udp_status_details_read(&got) == CTS_OK);
    CHECK(std::memcmp(&want, &got, sizeof want) == 0);

    char line[512];
    const cts_udp_status u{5000, 4000, 5000, got.bits_received, kThreads, got.successful_frames, got.dropped_frames,
                           got.duplicate_frames, got.error_frames};
    for (int fmt : {CTS_STATUS_CONSOLE, CTS_STATUS_CSV, CTS_STATUS_CLEAR_TEXT}) {
        CHECK(cts_status_udp_header(fmt, line, sizeof line) > 0);
        CHECK(cts_status_udp_legend(fmt, line, sizeof line) >= (fmt == CTS_STATUS_CSV ? 0 : 1));  // CSV: no legend
        CHECK(cts_status_udp_line(fmt, &u, line, sizeof line) > 0);
        CHECK(cts_status_udp_line(fmt, &u, line, 4) == -1);
    }
    CHECK(cts_status_udp_summary(kThreads * kPer, 0, failed, got.bits_received, got.successful_frames,
                                 got.dropped_frames, got.duplicate_frames, got.error_frames, line, sizeof line) > 0);
    std::printf("media_stream_client: ok\n");
    return 0;
}
