// ring_order_probe.hip — the MediaStream ring fill (cts_media_stream_fill_strided) in piece order, beside the product
// kernel (cts_kernels.hip, included verbatim). Diagnostic only (profiles/r06/g/).
//
// The ring is cut into 8 KiB pieces of its 16-byte chunks, dealt round robin to the workgroups (as fill_pieces_kernel
// deals the pieces of 64 KiB buffers), so the grid's concurrent stores cover adjacent pieces. A batch of 16 pieces'
// datagram lengths and headers is staged in LDS (at most 10 datagrams touch a piece for strides >= 1024), the next
// batch loaded into registers before this batch's stores; each wave writes 2 rounds of 64 chunks of every piece.
// A second form (ring_wave_pieces_kernel, profiles/r06/q/) deals 2 KiB pieces to every wave, without LDS or barriers.
// Every datagram's bytes are compared with the product's output; 16 M x 1472 B with 1 % of the lengths random.
//   build: make tools/ring_order_probe     run: tools/ring_order_probe [datagrams] [reps]
#include "../ctstraffic_amd/csrc/cts_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

namespace {

using namespace cts;

constexpr uint32_t kPC = 512;  // chunks per piece (8 KiB)
constexpr int kB = 16;         // pieces per batch
constexpr int kS = 10;         // datagram slots per piece (stride >= 1024: at most 9 datagrams touch 8 KiB)

template <bool NTS>
__global__ void __launch_bounds__(256) ring_pieces_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                          uint32_t stride, const uint32_t* __restrict__ lengths,
                                                          const cts_datagram_header* __restrict__ headers, uint32_t n)
{
    __shared__ uint32_t ls[kB][kS];
    __shared__ RingHeader hs[kB][kS];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint32_t cps = stride >> 4;
    const uint32_t inv_cps = (uint32_t)(0xFFFFFFFFull / cps) + 1u;  // __umulhi(t, inv_cps) = t / cps for small t
    const uint64_t total = (uint64_t)n * cps;
    const uint64_t pieces = (total + kPC - 1) / kPC;
    const uint64_t G = gridDim.x;
    // thread t < kB * kS stages slot t % kS of piece t / kS
    const uint32_t sm = t / kS, ss = t % kS;
    auto fetch = [&](uint64_t v0, uint32_t& len, RingHeader& h) {
        len = 0xFFFFFFFFu;  // no datagram
        if (t >= (uint32_t)(kB * kS)) return;
        const uint64_t v = v0 + (uint64_t)sm * G;
        if (v >= pieces) return;
        const uint64_t j = v * kPC / cps + ss;
        if (j >= n || j * cps >= (v + 1) * kPC) return;
        len = lengths[j];
        const cts_datagram_header x = headers[j];
        h = RingHeader{(uint64_t)x.sequence_number, (uint64_t)x.qpc, (uint64_t)x.qpf};
    };
    uint32_t nlen;
    RingHeader nh{};
    fetch(blockIdx.x, nlen, nh);
    u32x4* const ring = reinterpret_cast<u32x4*>(arena);
    for (uint64_t v0 = blockIdx.x; v0 < pieces; v0 += (uint64_t)kB * G) {
        __syncthreads();  // the previous batch is written
        if (t < (uint32_t)(kB * kS)) {
            ls[sm][ss] = nlen;
            hs[sm][ss] = nh;
        }
        __syncthreads();
        fetch(v0 + (uint64_t)kB * G, nlen, nh);  // the next batch, in flight under this one's stores
#pragma unroll 1
        for (int m = 0; m < kB; ++m) {
            const uint64_t v = v0 + (uint64_t)m * G;
            if (v >= pieces) break;
            // per piece (wave-uniform): its first chunk, the first datagram touching it and that datagram's chunk
            const uint64_t kb = v * kPC;
            const uint64_t j0 = kb / cps;
            const uint32_t c0 = (uint32_t)(kb - j0 * cps);
            const uint64_t off0 = j0 * (uint64_t)stride;  // the first datagram's byte offset
#pragma unroll
            for (uint32_t r = 0; r < 2u; ++r) {
                const uint32_t kr = wave * 128u + r * 64u + lane;  // chunk within the piece
                if (kb + kr >= total) continue;
                // datagram slot s of the piece and chunk c within it: t = c0 + kr < 512 + cps, s = t / cps by a
                // 32-bit multiply-shift (exact for t < 2^16, cps >= 64)
                const uint32_t tt = c0 + kr;
                const uint32_t s = __umulhi(tt, inv_cps), c = tt - s * cps;
                const uint32_t len = ls[m][s];
                if (len < CTS_UDP_DATA_HEADER_LENGTH || len > stride || 16u * c >= len ||
                    off0 + (uint64_t)s * stride + len > arena_bytes)
                    continue;
                u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
                if (c < 2u) {
                    const RingHeader h = hs[m][s];
                    e = datagram_chunk(c, e, h.seq, h.qpc, h.qpf);
                }
                u32x4* const q = ring + (kb + kr);
                if (16u * c + 16u > len) {
                    store_chunk_bytes(reinterpret_cast<uint8_t*>(q), e, 0u, len - 16u * c);
                } else {
                    if constexpr (NTS) __builtin_nontemporal_store(e, q);
                    else *q = e;
                }
            }
        }
    }
}

// Round 6, second form: pieces of 128 chunks (2 KiB) per WAVE, dealt round robin over every wave of the grid, so
// at one workgroup per CU the grid's concurrent stores cover 2 MiB of adjacent ring (the config-2 fill's order). No
// LDS and no barrier: lane 4m + t of each wave loads the length and header of the t-th datagram touching piece m of
// the next batch (at most 3 for strides >= 1024) before this batch's stores, and each piece reads them by readlane
// (lengths always, a header only when its datagram starts in the piece). Invalid datagrams (length below the header,
// above the stride, past the arena) carry length 0: none of their chunks is written.
constexpr uint32_t kWPC = 128;  // chunks per wave piece

template <bool NTS, int B>
__global__ void __launch_bounds__(256) ring_wave_pieces_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                               uint32_t stride, const uint32_t* __restrict__ lengths,
                                                               const cts_datagram_header* __restrict__ headers,
                                                               uint32_t n)
{
    static_assert(B * 4 <= 64, "4 lanes per piece");
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t cps = stride >> 4;
    const uint32_t inv_cps = (uint32_t)(0xFFFFFFFFull / cps) + 1u;  // __umulhi(t, inv_cps) = t / cps, t < 2^16
    const uint64_t T = (uint64_t)n * cps;
    const uint64_t P = (T + kWPC - 1) / kWPC;
    const uint64_t W = (uint64_t)gridDim.x * 4u;
    const uint64_t gw = (uint64_t)blockIdx.x * 4u + wave;
    const uint32_t pm = lane >> 2, pt = lane & 3u;
    struct Pre {
        uint32_t len, c0, s_lo, s_hi, c_lo, c_hi, f_lo, f_hi;
    };
    auto fetch = [&](uint64_t v0) {
        Pre r{};
        const uint64_t v = v0 + (uint64_t)pm * W;
        if (pm >= (uint32_t)B || v >= P) return r;
        const uint64_t kb = v * kWPC;
        const uint64_t j0 = kb / cps;
        r.c0 = (uint32_t)(kb - j0 * cps);
        const uint64_t j = j0 + pt;
        if (pt > 2u || j >= n || j * cps >= kb + kWPC) return r;
        const uint32_t len = lengths[j];
        const cts_datagram_header h = headers[j];
        if (len >= CTS_UDP_DATA_HEADER_LENGTH && len <= stride && j * stride + len <= arena_bytes) r.len = len;
        r.s_lo = (uint32_t)(uint64_t)h.sequence_number;
        r.s_hi = (uint32_t)((uint64_t)h.sequence_number >> 32);
        r.c_lo = (uint32_t)(uint64_t)h.qpc;
        r.c_hi = (uint32_t)((uint64_t)h.qpc >> 32);
        r.f_lo = (uint32_t)(uint64_t)h.qpf;
        r.f_hi = (uint32_t)((uint64_t)h.qpf >> 32);
        return r;
    };
    auto rl = [](uint32_t x, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, (int)l); };
    u32x4* const ring = reinterpret_cast<u32x4*>(arena);
    Pre cur = fetch(gw);
    for (uint64_t v0 = gw; v0 < P; v0 += (uint64_t)B * W) {
        const Pre nxt = fetch(v0 + (uint64_t)B * W);
#pragma unroll 1
        for (uint32_t m = 0; m < (uint32_t)B; ++m) {
            const uint64_t v = v0 + (uint64_t)m * W;
            if (v >= P) break;
            const uint64_t kb = v * kWPC;
            const uint32_t c0 = rl(cur.c0, 4u * m);
            const uint32_t l0 = rl(cur.len, 4u * m), l1 = rl(cur.len, 4u * m + 1u), l2 = rl(cur.len, 4u * m + 2u);
            // header words of the datagrams starting in this piece (slot 0 only when the piece starts at its chunk 0
            // or 1; slots 1 and 2 when they exist)
            RingHeader h0{}, h1{}, h2{};
            auto hdr = [&](uint32_t t) {
                const uint32_t l = 4u * m + t;
                return RingHeader{((uint64_t)rl(cur.s_hi, l) << 32) | rl(cur.s_lo, l),
                                  ((uint64_t)rl(cur.c_hi, l) << 32) | rl(cur.c_lo, l),
                                  ((uint64_t)rl(cur.f_hi, l) << 32) | rl(cur.f_lo, l)};
            };
            if (c0 < 2u) h0 = hdr(0u);
            if (cps - c0 < kWPC) h1 = hdr(1u);
            if (2u * cps - c0 < kWPC) h2 = hdr(2u);
#pragma unroll
            for (uint32_t r = 0; r < kWPC / 64u; ++r) {
                const uint32_t kr = r * 64u + lane;
                if (kb + kr >= T) continue;
                const uint32_t tt = c0 + kr;
                const uint32_t sl = __umulhi(tt, inv_cps), c = tt - sl * cps;
                const uint32_t len = sl == 0u ? l0 : (sl == 1u ? l1 : l2);
                if (16u * c >= len) continue;
                u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
                if (c < 2u) {
                    const RingHeader& h = sl == 0u ? h0 : (sl == 1u ? h1 : h2);
                    e = datagram_chunk(c, e, h.seq, h.qpc, h.qpf);
                }
                u32x4* const q = ring + (kb + kr);
                if (16u * c + 16u > len) {
                    store_chunk_bytes(reinterpret_cast<uint8_t*>(q), e, 0u, len - 16u * c);
                } else {
                    if constexpr (NTS) __builtin_nontemporal_store(e, q);
                    else *q = e;
                }
            }
        }
        cur = nxt;
    }
}

__global__ void count_diff_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, uint64_t bytes,
                                  unsigned long long* bad)
{
    uint32_t c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < bytes; i += (uint64_t)gridDim.x * 256u)
        c += a[i] != b[i];
    if (c) atomicAdd(bad, (unsigned long long)c);
}

template <typename F>
double time_us(F f, int iters)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipEventRecord(a);
    for (int i = 0; i < iters; ++i) f();
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
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    const uint32_t stride = 1472;
    const uint64_t bytes = (uint64_t)n * stride;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess || cus <= 0) return 1;
    std::vector<uint32_t> hl(n, stride);
    std::vector<cts_datagram_header> hh(n);
    std::mt19937 rng(6);
    for (uint32_t i = 0; i < n; ++i) {
        hh[i] = cts_datagram_header{(int64_t)i + 1, (int64_t)rng(), (int64_t)rng()};
        if (rng() % 100u == 0u) hl[i] = rng() % (stride + 1u);
    }
    uint8_t *ra = nullptr, *rb = nullptr;
    uint32_t* dl = nullptr;
    cts_datagram_header* dh = nullptr;
    unsigned long long* bad = nullptr;
    if (hipMalloc((void**)&ra, bytes) != hipSuccess || hipMalloc((void**)&rb, bytes) != hipSuccess ||
        hipMalloc((void**)&dl, 4ull * n) != hipSuccess || hipMalloc((void**)&dh, sizeof(cts_datagram_header) * (uint64_t)n) != hipSuccess ||
        hipMalloc((void**)&bad, 8) != hipSuccess)
        return 1;
    (void)hipMemcpy(dl, hl.data(), 4ull * n, hipMemcpyHostToDevice);
    (void)hipMemcpy(dh, hh.data(), sizeof(cts_datagram_header) * (uint64_t)n, hipMemcpyHostToDevice);
    (void)hipMemset(ra, 0x5A, bytes);
    (void)hipMemset(rb, 0x5A, bytes);
    LaunchGeometry geo;
    geo.num_cus = cus;
    // correctness: the product into ra, the candidate into rb
    (void)launch_media_stream_fill_strided(ra, bytes, stride, dl, dh, n, nullptr, geo);
    auto check = [&](const char* name) {
        (void)hipMemset(bad, 0, 8);
        count_diff_kernel<<<2048, 256>>>(ra, rb, bytes, bad);
        unsigned long long nb = ~0ull;
        (void)hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        std::printf("{\"check\": \"%s vs product\", \"datagrams\": %u, \"bad_bytes\": %llu}\n", name, n, nb);
        std::fflush(stdout);
        (void)hipMemset(rb, 0x5A, bytes);
    };
    ring_pieces_kernel<true><<<cus, 256>>>(rb, bytes, stride, dl, dh, n);
    check("ring_pieces");
    ring_wave_pieces_kernel<false, 16><<<cus, 256>>>(rb, bytes, stride, dl, dh, n);
    check("ring_wave_pieces");
    ring_wave_pieces_kernel<true, 16><<<cus * 2, 256>>>(rb, bytes, stride, dl, dh, n);
    check("ring_wave_pieces_nt");
    for (int rep = 0; rep < reps; ++rep) {
        for (int bpc : {2, 4, 8}) {
            geo.ring_fill_blocks_per_cu = bpc;
            const double us = time_us([&] { (void)launch_media_stream_fill_strided(ra, bytes, stride, dl, dh, n, nullptr, geo); }, 5);
            std::printf("{\"case\": \"product_ring\", \"blocks_per_cu\": %d, \"rep\": %d, \"us\": %.1f, \"GBps\": %.1f}\n", bpc,
                        rep, us, bytes / (us * 1e3));
            std::fflush(stdout);
        }
        for (int bpc : {1, 2, 4}) {
            for (int nt = 0; nt < 2; ++nt) {
                const double us = time_us([&] {
                    if (nt) ring_wave_pieces_kernel<true, 16><<<cus * bpc, 256>>>(rb, bytes, stride, dl, dh, n);
                    else ring_wave_pieces_kernel<false, 16><<<cus * bpc, 256>>>(rb, bytes, stride, dl, dh, n);
                }, 5);
                std::printf("{\"case\": \"ring_wave_pieces\", \"nt\": %d, \"blocks_per_cu\": %d, \"rep\": %d, \"us\": %.1f, \"GBps\": %.1f}\n",
                            nt, bpc, rep, us, bytes / (us * 1e3));
                std::fflush(stdout);
            }
        }
        for (int bpc : {1, 2, 4}) {
            for (int nt = 0; nt < 2; ++nt) {
                const double us = time_us([&] {
                    if (nt) ring_pieces_kernel<true><<<cus * bpc, 256>>>(rb, bytes, stride, dl, dh, n);
                    else ring_pieces_kernel<false><<<cus * bpc, 256>>>(rb, bytes, stride, dl, dh, n);
                }, 5);
                std::printf("{\"case\": \"ring_pieces\", \"nt\": %d, \"blocks_per_cu\": %d, \"rep\": %d, \"us\": %.1f, \"GBps\": %.1f}\n",
                            nt, bpc, rep, us, bytes / (us * 1e3));
                std::fflush(stdout);
            }
        }
    }
    const hipError_t e = hipDeviceSynchronize();
    return e == hipSuccess ? 0 : 1;
}
