// fill_abi_probe.cpp — cts_fill through the C ABI on hipMalloc'd arenas (no PyTorch), config-2 shape:
// 4096 x 64 KiB, phase 0, 4 arenas rotated; prints us per launch. Separates the kernel from the
// Python/torch environment the bench runs it in.   build: make tools/fill_abi_probe
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <vector>

#include "cts_engine.h"

int main()
{
    cts_engine* e = nullptr;
    if (cts_engine_create(0, &e) != CTS_OK) return 1;
    const uint32_t n = 4096;
    const uint64_t bytes = (uint64_t)n << 16;
    std::vector<void*> arenas(4);
    for (auto& a : arenas)
        if (hipMalloc(&a, bytes) != hipSuccess) return 1;
    std::vector<cts_buf_desc> h(n);
    for (uint32_t i = 0; i < n; ++i) h[i] = cts_buf_desc{(uint64_t)i << 16, 65536u, 0u, i, 0u};
    cts_buf_desc* d = nullptr;
    if (hipMalloc((void**)&d, n * sizeof(cts_buf_desc)) != hipSuccess) return 1;
    if (hipMemcpy(d, h.data(), n * sizeof(cts_buf_desc), hipMemcpyHostToDevice) != hipSuccess) return 1;
    for (int bpc : {1, 2, 4}) {
        cts_engine_set_attr(e, CTS_ATTR_FILL_BLOCKS_PER_CU, bpc);
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        cts_fill(e, arenas[0], bytes, d, n, 65536, nullptr);
        (void)hipEventRecord(a, nullptr);
        for (int i = 0; i < 40; ++i) cts_fill(e, arenas[i % 4], bytes, d, n, 65536, nullptr);
        (void)hipEventRecord(b, nullptr);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        std::printf("{\"probe\": \"cts_fill_abi\", \"fill_blocks_per_cu\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", bpc,
                    ms * 1e3 / 40, bytes / (ms * 1e3 / 40) / 1e3);
    }
    cts_engine_destroy(e);
    return 0;
}
