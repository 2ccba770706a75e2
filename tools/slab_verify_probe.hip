// slab_verify_probe.hip — can a one-buffer-per-workgroup verify reach the plain read's fastest shape?
//
// On every box the fastest plain streaming read of 256 MiB is one 64 KiB slab per workgroup over a 4 096-workgroup
// grid (tools/hbm_read_ceiling "slab": 39.4-39.9 us), where every workgroup is resident at once; the product verify
// grid-strides 4 buffers per workgroup over 1 024 workgroups (41.0 us) because round 4's one-buffer-per-workgroup
// form (46.4 us, profiles/r04/g/) paid a heavy per-workgroup start and could not be resident at once (58 VGPRs).
// This probe times, in one process over the same 8 rotated config-2 arenas:
//   product : cts::launch_verify (verify_wg_kernel, included verbatim);
//   slab    : the plain read, one slab per workgroup, U 16-B nontemporal loads per lane per round;
//   sv<U,C> : a slim verify of whole-line spans only, one buffer per workgroup: the descriptor (scalar loads), the
//             product's scan_rounds over the whole span, one __syncthreads_or verdict, lane 0 writes the clean
//             record (a failing buffer is only flagged: the product would re-scan it exactly); C = 1 adds the
//             counters (one atomic per counter per workgroup, shard blockIdx % 64).
// Every sv verdict is checked against the product's records. Diagnostic only (not the product).
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ictstraffic_amd/csrc
//          -mllvm -amdgpu-kernarg-preload-count=16 tools/slab_verify_probe.hip -o tools/slab_verify_probe
//   run:   tools/slab_verify_probe [passes] [launches]
#include "../ctstraffic_amd/csrc/cts_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

namespace {
using cts::u32x4;

__global__ void fill_arena(u32x4* a, const cts_buf_desc* d, uint32_t n)
{
    for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < (uint64_t)n * 4096; c += (uint64_t)gridDim.x * 256) {
        const uint32_t q = (d[c / 4096].expected_pattern_offset + 16u * (uint32_t)(c % 4096)) & 0xFFFFu;
        a[c] = cts::expected_chunk(q, q & 1u);
    }
}

template <int U>
__global__ void __launch_bounds__(256) slab_read(const u32x4* __restrict__ p, uint32_t* out)
{
    const u32x4* q = p + (uint64_t)blockIdx.x * 4096u;
    uint32_t acc = 0;
    for (uint32_t c = threadIdx.x; c < 4096u; c += 256u * U) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(q + c + u * 256u);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
    }
    acc = __syncthreads_or(acc == 0x12345678u) ? 1u : acc;
    if (acc == 0x12345678u) out[0] = acc;
}

// flags[i]: 1 = whole-line fast path, clean; 2 = fast path, mismatch (needs the exact re-scan); 3 = not fast-path shaped
template <int U, bool C>
__global__ void __launch_bounds__(256) slab_verify(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                   const cts_buf_desc* __restrict__ descs, cts_verify_result* results,
                                                   uint64_t* counters, uint32_t* flags)
{
    const uint32_t i = blockIdx.x;
    const cts_buf_desc d = descs[i];
    const cts::Span s = cts::make_span(arena, d);
    const bool fast = !cts::desc_bad(d, arena_bytes) && cts::span_whole_lines(s) && s.nchunks % (256u * U) == 0u;
    if (!fast) {
        if (threadIdx.x == 0) flags[i] = 3u;
        return;
    }
    const __amdgpu_buffer_rsrc_t r = cts::span_rsrc(s);
    const uint32_t acc = cts::scan_rounds<256, U, true, false>(s, r, threadIdx.x, 0u, s.nchunks);
    const bool bad = __syncthreads_or(acc != 0u);
    if (threadIdx.x == 0) {
        flags[i] = bad ? 2u : 1u;
        if (!bad) results[i] = cts_verify_result{s.len, 0u, 0u, 0u, 1u, 0u};
        if constexpr (C) {
            uint64_t* sh = counters + (size_t)(i % CTS_COUNTER_SHARDS) * cts::kCounterSlots;
            atomicAdd((unsigned long long*)&sh[cts::kBytesChecked], (unsigned long long)s.len);
            atomicAdd((unsigned long long*)&sh[cts::kBuffersChecked], 1ull);
            if (!bad) atomicAdd((unsigned long long*)&sh[cts::kBytesOk], (unsigned long long)s.len);
        }
    }
}

template <typename F>
double time_us(F launch, int reps, hipStream_t s)
{
    launch(0);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) launch(i);
    CHECK(hipEventRecord(b, s));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms * 1e3 / reps;
}

}  // namespace

int main(int argc, char** argv)
{
    const int passes = argc > 1 ? atoi(argv[1]) : 3;
    const int reps = argc > 2 ? atoi(argv[2]) : 64;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t n = 4096;
    const uint64_t bytes = (uint64_t)n << 16;
    constexpr int R = 8;
    std::vector<cts_buf_desc> hd(n);
    uint64_t x = 0xC75;
    auto rnd = [&] {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return x;
    };
    for (uint32_t i = 0; i < n; ++i) {
        const bool random_phase = rnd() % 4 == 0;
        hd[i] = cts_buf_desc{(uint64_t)i << 16, 65536u, random_phase ? (uint32_t)(rnd() & 0xFFFFu) : 0u, i, 0u};
    }
    cts_buf_desc* d = nullptr;
    CHECK(hipMalloc((void**)&d, n * sizeof(cts_buf_desc)));
    CHECK(hipMemcpy(d, hd.data(), n * sizeof(cts_buf_desc), hipMemcpyHostToDevice));
    std::vector<uint8_t*> arena(R);
    for (auto& a : arena) {
        CHECK(hipMalloc((void**)&a, bytes));
        fill_arena<<<4096, 256>>>(reinterpret_cast<u32x4*>(a), d, n);
        for (uint32_t b : {0u, 1024u, 2048u, 3072u}) {  // one corrupt byte per 1024 buffers
            const uint64_t off = ((uint64_t)b << 16) + 77u;
            uint8_t v = 0;
            CHECK(hipMemcpy(&v, a + off, 1, hipMemcpyDeviceToHost));
            v ^= 0x5A;
            CHECK(hipMemcpy(a + off, &v, 1, hipMemcpyHostToDevice));
        }
    }
    cts_verify_result* res = nullptr;
    cts_verify_result* res2 = nullptr;
    uint64_t* ctr = nullptr;
    uint32_t *cff = nullptr, *flags = nullptr, *out = nullptr;
    CHECK(hipMalloc((void**)&res, n * sizeof(cts_verify_result)));
    CHECK(hipMalloc((void**)&res2, n * sizeof(cts_verify_result)));
    CHECK(hipMalloc((void**)&ctr, CTS_COUNTER_SHARDS * 64));
    CHECK(hipMalloc((void**)&cff, n * 4));
    CHECK(hipMalloc((void**)&flags, n * 4));
    CHECK(hipMalloc((void**)&out, 64));
    CHECK(hipMemset(ctr, 0, CTS_COUNTER_SHARDS * 64));
    CHECK(hipMemset(cff, 0xFF, n * 4));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    cts::LaunchGeometry geo;
    geo.num_cus = cus;
    CHECK(hipDeviceSynchronize());

    // parity of the verdicts: sv<2,1> and sv<4,1> against the product's records on arena 0
    CHECK(cts::launch_verify(arena[0], bytes, d, n, 65536u, res, ctr, cff, n, s, geo));
    CHECK(hipStreamSynchronize(s));
    std::vector<cts_verify_result> hr(n);
    CHECK(hipMemcpy(hr.data(), res, n * sizeof(cts_verify_result), hipMemcpyDeviceToHost));
    int mismatched = 0, flagged = 0;
    for (int form = 0; form < 2; ++form) {
        CHECK(hipMemset(flags, 0, n * 4));
        if (form == 0) slab_verify<2, true><<<n, 256, 0, s>>>(arena[0], bytes, d, res2, ctr, flags);
        else slab_verify<4, true><<<n, 256, 0, s>>>(arena[0], bytes, d, res2, ctr, flags);
        CHECK(hipStreamSynchronize(s));
        std::vector<uint32_t> hf(n);
        CHECK(hipMemcpy(hf.data(), flags, n * 4, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t want = hr[i].pass ? 1u : 2u;
            if (hf[i] != want) ++mismatched;
            if (hf[i] == 2u) ++flagged;
        }
    }
    std::printf("{\"kind\":\"parity\",\"verdicts_differ\":%d,\"flagged_for_exact\":%d}\n", mismatched, flagged);
    std::fflush(stdout);
    if (mismatched != 0) return 2;

    auto a = [&](int i) { return arena[i % R]; };
    for (int pass = 0; pass < passes; ++pass) {
        const double prod = time_us([&](int i) { (void)cts::launch_verify(a(i), bytes, d, n, 65536u, res, ctr, cff, n, s, geo); },
                                    reps, s);
        const double sl4 = time_us([&](int i) {
            slab_read<4><<<n, 256, 0, s>>>(reinterpret_cast<const u32x4*>(a(i)), out);
        }, reps, s);
        const double sl2 = time_us([&](int i) {
            slab_read<2><<<n, 256, 0, s>>>(reinterpret_cast<const u32x4*>(a(i)), out);
        }, reps, s);
        const double v20 = time_us([&](int i) { slab_verify<2, false><<<n, 256, 0, s>>>(a(i), bytes, d, res2, ctr, flags); },
                                   reps, s);
        const double v21 = time_us([&](int i) { slab_verify<2, true><<<n, 256, 0, s>>>(a(i), bytes, d, res2, ctr, flags); },
                                   reps, s);
        const double v40 = time_us([&](int i) { slab_verify<4, false><<<n, 256, 0, s>>>(a(i), bytes, d, res2, ctr, flags); },
                                   reps, s);
        const double v41 = time_us([&](int i) { slab_verify<4, true><<<n, 256, 0, s>>>(a(i), bytes, d, res2, ctr, flags); },
                                   reps, s);
        std::printf("{\"kind\":\"time\",\"pass\":%d,\"launches\":%d,\"product_us\":%.2f,\"slab_read_u4_us\":%.2f,"
                    "\"slab_read_u2_us\":%.2f,\"sv_u2_us\":%.2f,\"sv_u2_counters_us\":%.2f,\"sv_u4_us\":%.2f,"
                    "\"sv_u4_counters_us\":%.2f}\n",
                    pass, reps, prod, sl4, sl2, v20, v21, v40, v41);
        std::fflush(stdout);
    }
    return 0;
}
