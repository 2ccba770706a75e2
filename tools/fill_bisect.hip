// fill_bisect.hip — the product fill kernel (cts_kernels.hip, included verbatim) launched directly, on
// one arena written over and over and on 4 arenas rotated per launch (1 GiB: more than the 256 MB MALL
// can keep). Rewriting one 256 MiB arena runs from the MALL and reads as 6.9 TB/s; rotated, the same
// kernel writes HBM at the rate cts_fill shows in bench.py. Diagnostic only.
#include "../ctstraffic_amd/csrc/cts_kernels.hip"

#include <cstdio>
#include <vector>

template <typename F>
static double time_us(F f, int iters = 20)
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
    return ms * 1e3 / iters;
}

int main()
{
    const uint32_t n = 4096;
    const uint64_t bytes = (uint64_t)n << 16;
    uint8_t* arena = nullptr;
    cts_buf_desc* d = nullptr;
    if (hipMalloc((void**)&arena, 4 * bytes) != hipSuccess || hipMalloc((void**)&d, n * sizeof(cts_buf_desc)) != hipSuccess)
        return 1;
    std::vector<cts_buf_desc> h(n);
    for (uint32_t i = 0; i < n; ++i) h[i] = cts_buf_desc{(uint64_t)i << 16, 65536u, 0u, i, 0u};
    (void)hipMemcpy(d, h.data(), n * sizeof(cts_buf_desc), hipMemcpyHostToDevice);
    for (int grid : {256, 1024}) {
        const double t_prod = time_us([&] { cts::fill_kernel<256, false><<<grid, 256>>>(arena, bytes, d, n); });
        const double t_nts = time_us([&] { cts::fill_kernel<256, true><<<grid, 256>>>(arena, bytes, d, n); });
        int k = 0;
        const double t_rot = time_us([&] { cts::fill_kernel<256, false><<<grid, 256>>>(arena + (uint64_t)(k++ % 4) * bytes, bytes, d, n); });
        std::printf("{\"grid\": %d, \"fill_kernel_plain_us\": %.2f, \"fill_kernel_nt_us\": %.2f, \"fill_kernel_plain_rotated_us\": %.2f}\n",
                    grid, t_prod, t_nts, t_rot);
        std::fflush(stdout);
    }
    return 0;
}
