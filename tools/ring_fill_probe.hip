// ring_fill_probe.hip — why does the datagram fill write HBM at 3.5-3.9 TB/s when 64 KiB slabs write 5.2-5.9?
// 16 M MediaStream datagrams of 1472 B in a ring (datagram i at i * stride), filled four ways on the same arenas:
//   product  : cts::launch_media_stream_fill (one wave per datagram, descriptors + headers)
//   walk     : a flat walk of the ring's 16-byte chunks, each wave 64 consecutive chunks per round across
//              datagram boundaries (chunk k = datagram k / cps, chunk k % cps; headers read for chunks 0 and 1 only)
//   walk1536 : the same walk with a 1536-byte stride (whole 128-byte lines per datagram)
//   slab     : the pattern over the same bytes as one span (no datagram structure)
// nontemporal and plain stores. One JSON line per (case, round). Diagnostic only.
//   build: make tools/ring_fill_probe     run: tools/ring_fill_probe [datagrams] [rounds]
#define CTS_TUNING 1  // the round-3 wave-per-buffer fills too
#include "../ctstraffic_amd/csrc/cts_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace {

using namespace cts;

template <bool NTS>
__global__ void __launch_bounds__(256) ring_walk(u32x4* __restrict__ ring, uint32_t total_chunks, uint32_t cps,
                                                 const cts_datagram_header* __restrict__ headers)
{
    // each wave walks a contiguous run of the ring, 64 chunks per round
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * 4u, w = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t per = (total_chunks + waves - 1u) / waves;
    const uint32_t per64 = (per + 63u) & ~63u;
    const uint32_t k0 = w * per64;
    if (k0 >= total_chunks) return;
    const uint32_t k1 = k0 + per64 < total_chunks ? k0 + per64 : total_chunks;
    uint32_t k = k0 + lane;
    uint32_t i = k / cps, c = k - i * cps;
    for (; k < k1; k += 64u) {
        u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
        if (c < 2u) {
            const cts_datagram_header h = headers[i];
            const uint64_t seq = (uint64_t)h.sequence_number, qpc = (uint64_t)h.qpc, qpf = (uint64_t)h.qpf;
            if (c == 0u)
                e = u32x4{(uint32_t)(seq << 16), (uint32_t)(seq >> 16), (uint32_t)(seq >> 48) | (uint32_t)(qpc << 16),
                          (uint32_t)(qpc >> 16)};
            else
                e = u32x4{(uint32_t)(qpc >> 48) | (uint32_t)(qpf << 16), (uint32_t)(qpf >> 16),
                          (uint32_t)(qpf >> 48) | (e[2] & 0xFFFF0000u), e[3]};
        }
        if constexpr (NTS) __builtin_nontemporal_store(e, ring + k);
        else ring[k] = e;
        c += 64u;
        while (c >= cps) {
            c -= cps;
            ++i;
        }
    }
}

// the walk in the slab's order: round r writes chunks [r * G, (r + 1) * G) of the ring, G = grid * 256, lane t of
// workgroup b chunk r * G + 256 b + t (a 4 MiB front moving through the ring, as fill_span_kernel's)
template <bool NTS>
__global__ void __launch_bounds__(256) ring_walk_il(u32x4* __restrict__ ring, uint32_t total_chunks, uint32_t cps,
                                                    const cts_datagram_header* __restrict__ headers, uint32_t sdiv,
                                                    uint32_t smod)
{
    const uint32_t stride = gridDim.x * 256u;
    uint32_t k = blockIdx.x * 256u + threadIdx.x;
    uint32_t i = k / cps, c = k - i * cps;
    for (; k < total_chunks; k += stride) {
        u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
        if (c < 2u) {
            const cts_datagram_header h = headers[i];
            const uint64_t seq = (uint64_t)h.sequence_number, qpc = (uint64_t)h.qpc, qpf = (uint64_t)h.qpf;
            if (c == 0u)
                e = u32x4{(uint32_t)(seq << 16), (uint32_t)(seq >> 16), (uint32_t)(seq >> 48) | (uint32_t)(qpc << 16),
                          (uint32_t)(qpc >> 16)};
            else
                e = u32x4{(uint32_t)(qpc >> 48) | (uint32_t)(qpf << 16), (uint32_t)(qpf >> 16),
                          (uint32_t)(qpf >> 48) | (e[2] & 0xFFFF0000u), e[3]};
        }
        if constexpr (NTS) __builtin_nontemporal_store(e, ring + k);
        else ring[k] = e;
        i += sdiv;
        c += smod;
        if (c >= cps) {
            c -= cps;
            ++i;
        }
    }
}

// The walk with the headers as scalar loads: a wave's 64 chunks of one round hold at most two datagram starts (92
// chunks per datagram), so the wave loads headers[ib] and headers[ib + 1] (wave-uniform addresses: s_load, counted
// by lgkmcnt) and no store ever waits on a vector load. IL: waves interleaved (round r of wave w writes chunks
// (r * waves + w) * 64 ..), else each wave a contiguous run.
template <bool NTS, bool IL>
__global__ void __launch_bounds__(256) ring_walk_s(u32x4* __restrict__ ring, uint32_t total_chunks, uint32_t cps,
                                                   const cts_datagram_header* __restrict__ headers, uint32_t n)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * 4u;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    uint32_t kb, k1, step;
    if constexpr (IL) {
        kb = w * 64u;
        k1 = total_chunks;
        step = waves * 64u;
    } else {
        const uint32_t per = (total_chunks + waves - 1u) / waves;
        const uint32_t per64 = (per + 63u) & ~63u;
        kb = w * per64;
        k1 = kb + per64 < total_chunks ? kb + per64 : total_chunks;
        step = 64u;
    }
    if (kb >= k1) return;
    uint32_t ib = kb / cps, cb = kb - ib * cps;  // wave-uniform: the datagram and chunk of lane 0
    const uint32_t sdiv = step / cps, smod = step - sdiv * cps;
    for (; kb < k1; kb += step) {
        uint32_t c = cb + lane, i = ib;
        if (c >= cps) {
            c -= cps;
            i = ib + 1u;
        }
        u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
        const cts_datagram_header h0 = headers[ib];
        const cts_datagram_header h1 = headers[ib + 1u < n ? ib + 1u : ib];
        if (c < 2u) {
            const bool first = (i == ib);
            const uint64_t seq = (uint64_t)(first ? h0.sequence_number : h1.sequence_number);
            const uint64_t qpc = (uint64_t)(first ? h0.qpc : h1.qpc), qpf = (uint64_t)(first ? h0.qpf : h1.qpf);
            if (c == 0u)
                e = u32x4{(uint32_t)(seq << 16), (uint32_t)(seq >> 16), (uint32_t)(seq >> 48) | (uint32_t)(qpc << 16),
                          (uint32_t)(qpc >> 16)};
            else
                e = u32x4{(uint32_t)(qpc >> 48) | (uint32_t)(qpf << 16), (uint32_t)(qpf >> 16),
                          (uint32_t)(qpf >> 48) | (e[2] & 0xFFFF0000u), e[3]};
        }
        if (kb + lane < k1) {
            if constexpr (NTS) __builtin_nontemporal_store(e, ring + kb + lane);
            else ring[kb + lane] = e;
        }
        ib += sdiv;
        cb += smod;
        if (cb >= cps) {
            cb -= cps;
            ++ib;
        }
    }
}

// the product kernel before its descriptor/header prefetch (round 3's first aligned form)
template <bool NTS>
__global__ void __launch_bounds__(256) dgram_noprefetch(uint8_t* __restrict__ arena, const cts_buf_desc* __restrict__ descs,
                                                        const cts_datagram_header* __restrict__ headers, uint32_t n)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t i = blockIdx.x * 4u + wave; i < n; i += gridDim.x * 4u) {
        const cts_buf_desc d = descs[i];
        const cts_datagram_header h = headers[i];
        const uint64_t seq = (uint64_t)h.sequence_number, qpc = (uint64_t)h.qpc, qpf = (uint64_t)h.qpf;
        const uint32_t nchunks = (d.length + 15u) >> 4;
        u32x4* p = reinterpret_cast<u32x4*>(arena + d.byte_offset);
        for (uint32_t c = lane; c < nchunks; c += 64u) {
            u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
            if (c == 0u)
                e = u32x4{(uint32_t)(seq << 16), (uint32_t)(seq >> 16), (uint32_t)(seq >> 48) | (uint32_t)(qpc << 16),
                          (uint32_t)(qpc >> 16)};
            else if (c == 1u)
                e = u32x4{(uint32_t)(qpc >> 48) | (uint32_t)(qpf << 16), (uint32_t)(qpf >> 16),
                          (uint32_t)(qpf >> 48) | (e[2] & 0xFFFF0000u), e[3]};
            if constexpr (NTS) __builtin_nontemporal_store(e, p + c);
            else p[c] = e;
        }
    }
}

template <typename F>
double time_us(F f, int iters)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f(0);
    (void)hipEventRecord(a);
    for (int it = 0; it < iters; ++it) f(it + 1);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms * 1e3 / iters;
}

}  // namespace

int main(int argc, char** argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 16u * 1024u * 1024u;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 3;
    const uint32_t len = 1472;
    const uint64_t bytes1536 = (uint64_t)n * 1536u, bytes = (uint64_t)n * len;
    uint8_t* arena[2] = {nullptr, nullptr};
    for (auto& a : arena)
        if (hipMalloc(&a, bytes1536) != hipSuccess) return 1;
    std::vector<cts_buf_desc> d(n);
    std::vector<cts_datagram_header> h(n);
    for (uint32_t i = 0; i < n; ++i) {
        d[i] = cts_buf_desc{(uint64_t)i * len, len, 0, 0, 0};
        h[i] = cts_datagram_header{(int64_t)i + 1, 1000 + (int64_t)i, 10000000};
    }
    cts_buf_desc* dd = nullptr;
    cts_datagram_header* hd = nullptr;
    if (hipMalloc(&dd, sizeof(cts_buf_desc) * n) != hipSuccess || hipMalloc(&hd, sizeof(cts_datagram_header) * n) != hipSuccess)
        return 1;
    (void)hipMemcpy(dd, d.data(), sizeof(cts_buf_desc) * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(hd, h.data(), sizeof(cts_datagram_header) * n, hipMemcpyHostToDevice);
    cts_buf_desc* dp = nullptr;  // the payload fill's descriptors (26-byte header skipped, pattern offset 0)
    for (auto& x : d) x.skip_head = CTS_UDP_DATA_HEADER_LENGTH;
    if (hipMalloc(&dp, sizeof(cts_buf_desc) * n) != hipSuccess) return 1;
    (void)hipMemcpy(dp, d.data(), sizeof(cts_buf_desc) * n, hipMemcpyHostToDevice);
    cts::LaunchGeometry geo;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) == hipSuccess && cus > 0) geo.num_cus = cus;
    const uint32_t wgrid = (uint32_t)geo.num_cus * 8u;
    for (int r = 0; r < rounds; ++r) {
        for (int nt = 1; nt >= 0; --nt) {
            geo.fill_nt = nt;
            auto line = [&](const char* name, double us, uint64_t b) {
                std::printf("{\"round\": %d, \"case\": \"%s\", \"nt\": %d, \"us\": %.1f, \"GBps_written\": %.1f}\n", r, name,
                            nt, us, (double)b / us / 1e3);
                std::fflush(stdout);
            };
            for (int bpc : {4, 8}) {
                cts::LaunchGeometry g2 = geo;
                g2.ring_fill_blocks_per_cu = bpc;
                char name[64];
                std::snprintf(name, sizeof name, "product_batched_bpc%d", bpc);
                line(name, time_us([&](int it) {
                         (void)cts::launch_media_stream_fill(arena[it & 1], bytes, dd, hd, n, nullptr, g2);
                     }, 5), bytes);
                std::snprintf(name, sizeof name, "payload_wave_bpc%d", bpc);
                line(name, time_us([&](int it) {
                         (void)cts::launch_fill(arena[it & 1], bytes, dp, n, len, nullptr, g2);
                     }, 5), (uint64_t)n * (len - 26u));
            }
            for (uint32_t bpc : {4u, 8u, 16u}) {
                const uint32_t g = (uint32_t)geo.num_cus * bpc, stride = g * 256u;
                char name[64];
                std::snprintf(name, sizeof name, "walk_il_bpc%u", bpc);
                line(name, time_us([&](int it) {
                         u32x4* rp = reinterpret_cast<u32x4*>(arena[it & 1]);
                         if (nt) ring_walk_il<true><<<g, 256>>>(rp, n * 92u, 92u, hd, stride / 92u, stride % 92u);
                         else ring_walk_il<false><<<g, 256>>>(rp, n * 92u, 92u, hd, stride / 92u, stride % 92u);
                     }, 5), bytes);
            }
            for (uint32_t bpc : {8u, 64u}) {
                const uint32_t g = (uint32_t)geo.num_cus * bpc;
                char name[64];
                std::snprintf(name, sizeof name, "dgram_noprefetch_bpc%u", bpc);
                line(name, time_us([&](int it) {
                         if (nt) dgram_noprefetch<true><<<g, 256>>>(arena[it & 1], dd, hd, n);
                         else dgram_noprefetch<false><<<g, 256>>>(arena[it & 1], dd, hd, n);
                     }, 5), bytes);
            }
            {
                std::vector<uint32_t> lh(n, len);
                static uint32_t* ld = nullptr;
                if (ld == nullptr) {
                    (void)hipMalloc(&ld, sizeof(uint32_t) * n);
                    (void)hipMemcpy(ld, lh.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice);
                }
                for (int bpc : {2, 4, 8}) {
                    cts::LaunchGeometry g2 = geo;
                    g2.ring_fill_blocks_per_cu = bpc;
                    char name[64];
                    std::snprintf(name, sizeof name, "product_strided_bpc%d", bpc);
                    line(name, time_us([&](int it) {
                             (void)cts::launch_media_stream_fill_strided(arena[it & 1], bytes, len, ld, hd, n, nullptr, g2);
                         }, 5), bytes);
                }
            }
            for (uint32_t bpc : {4u, 8u}) {
                const uint32_t g = (uint32_t)geo.num_cus * bpc;
                char name[64];
                std::snprintf(name, sizeof name, "walk_s_bpc%u", bpc);
                line(name, time_us([&](int it) {
                         u32x4* rp = reinterpret_cast<u32x4*>(arena[it & 1]);
                         if (nt) ring_walk_s<true, false><<<g, 256>>>(rp, n * 92u, 92u, hd, n);
                         else ring_walk_s<false, false><<<g, 256>>>(rp, n * 92u, 92u, hd, n);
                     }, 5), bytes);
                std::snprintf(name, sizeof name, "walk_s_il_bpc%u", bpc);
                line(name, time_us([&](int it) {
                         u32x4* rp = reinterpret_cast<u32x4*>(arena[it & 1]);
                         if (nt) ring_walk_s<true, true><<<g, 256>>>(rp, n * 92u, 92u, hd, n);
                         else ring_walk_s<false, true><<<g, 256>>>(rp, n * 92u, 92u, hd, n);
                     }, 5), bytes);
            }
            line("walk", time_us([&](int it) {
                     if (nt) ring_walk<true><<<wgrid, 256>>>(reinterpret_cast<u32x4*>(arena[it & 1]), n * 92u, 92u, hd);
                     else ring_walk<false><<<wgrid, 256>>>(reinterpret_cast<u32x4*>(arena[it & 1]), n * 92u, 92u, hd);
                 }, 5), bytes);
            line("walk1536", time_us([&](int it) {
                     if (nt) ring_walk<true><<<wgrid, 256>>>(reinterpret_cast<u32x4*>(arena[it & 1]), n * 96u, 96u, hd);
                     else ring_walk<false><<<wgrid, 256>>>(reinterpret_cast<u32x4*>(arena[it & 1]), n * 96u, 96u, hd);
                 }, 5), bytes1536);
            line("slab", time_us([&](int it) {
                     cts::fill_span_kernel<<<(uint32_t)geo.num_cus * 4u, 256>>>(arena[it & 1], bytes, 0u);
                 }, 5), bytes);
        }
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return 0;
}
