// write_shape_probe.hip — store shapes writing 256 MiB: widths (4/8/16 B per lane), interleaved vs
// per-workgroup 64 KiB slabs, data content (distinct words / the ctsTraffic pattern / zeros), and a
// copy of the fill's round structure. Caution, measured: every shape that rewrites ONE 256 MiB arena
// launch after launch runs largely from the 256 MB MALL (6.8-7.0 TB/s, zeros 8.1 TB/s); the "_rot"
// shapes rotate 8 arenas per launch and show the HBM write rate (tools/fill_bisect.hip: the product
// fill 39.6 us on one arena, 47.7 us rotated). One JSON line per (shape, grid).
#include <hip/hip_runtime.h>

#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int W, int U, bool NT>  // W = bytes per lane per store
__global__ void __launch_bounds__(256) write_kernel(uint8_t* __restrict__ p, uint64_t bytes, uint32_t seed)
{
    const uint64_t per_round = (uint64_t)gridDim.x * 256u * W * U;
    for (uint64_t base = (uint64_t)blockIdx.x * 256u * W * U; base < bytes; base += per_round) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t o = base + (uint64_t)u * 256u * W + (uint64_t)threadIdx.x * W;
            const uint32_t v = (uint32_t)o ^ seed;
            if constexpr (W == 4) {
                if (NT) __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(p + o));
                else *reinterpret_cast<uint32_t*>(p + o) = v;
            } else if constexpr (W == 8) {
                if (NT) __builtin_nontemporal_store(u32x2{v, v + 1}, reinterpret_cast<u32x2*>(p + o));
                else *reinterpret_cast<u32x2*>(p + o) = u32x2{v, v + 1};
            } else {
                if (NT) __builtin_nontemporal_store(u32x4{v, v + 1, v + 2, v + 3}, reinterpret_cast<u32x4*>(p + o));
                else *reinterpret_cast<u32x4*>(p + o) = u32x4{v, v + 1, v + 2, v + 3};
            }
        }
    }
}

// the fill kernel's shape: workgroup b writes whole 64 KiB slabs b, b + grid, ... (16-B stores, U per round).
// DATA 0: distinct words (offset ^ seed); 1: the ctsTraffic pattern (u16 ramp, identical in every 64 KiB
// slab); 2: zeros
template <int U, int DATA>
__global__ void __launch_bounds__(256) write_slab_kernel(uint8_t* __restrict__ p, uint64_t bytes, uint32_t seed)
{
    const uint64_t nslabs = bytes >> 16;
    for (uint64_t sl = blockIdx.x; sl < nslabs; sl += gridDim.x) {
        uint8_t* q = p + (sl << 16);
        for (uint32_t r = 0; r < 65536u / (256u * 16u * U); ++r) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t o = (r * U + u) * 4096u + threadIdx.x * 16u;
                u32x4 w;
                if constexpr (DATA == 0) {
                    const uint32_t v = (o + (uint32_t)sl * 65536u) ^ seed;
                    w = u32x4{v, v + 1, v + 2, v + 3};
                } else if constexpr (DATA == 1) {
                    const uint32_t k = o >> 1;  // u16 values k..k+7 (o < 65536: no wrap)
                    w = u32x4{k | ((k + 1) << 16), (k + 2) | ((k + 3) << 16), (k + 4) | ((k + 5) << 16),
                              (k + 6) | ((k + 7) << 16)};
                } else {
                    w = u32x4{0u, 0u, 0u, 0u};
                }
                *reinterpret_cast<u32x4*>(q + o) = w;
            }
        }
    }
}

// a copy of cts_kernels.hip's whole-span fill round (fill_whole_rounds, even phase): the expected words
// stepped from a packed u16-pair base with an opaque-register barrier, global stores for full rounds
template <int U, bool BARRIER>
__device__ __forceinline__ u32x4 fill_step(uint32_t B, int u)
{
    uint32_t bb = B;
    if constexpr (BARRIER) asm volatile("" : "+v"(bb));
    const uint32_t b = bb + (uint32_t)u * (uint32_t)(8 * 256) * 0x10001u;
    return u32x4{b & 0x7FFF7FFFu, (b + 0x20002u) & 0x7FFF7FFFu, (b + 0x40004u) & 0x7FFF7FFFu, (b + 0x60006u) & 0x7FFF7FFFu};
}

template <int U, bool BARRIER>
__global__ void __launch_bounds__(256) fillcopy_kernel(uint8_t* __restrict__ p, uint64_t bytes)
{
    typedef u32x4 __attribute__((address_space(1)))* gstore_ptr;
    const uint64_t nslabs = bytes >> 16;
    const uint32_t lane = threadIdx.x;
    for (uint64_t sl = blockIdx.x; sl < nslabs; sl += gridDim.x) {
        u32x4* q = reinterpret_cast<u32x4*>(p + (sl << 16));
        const uint32_t nchunks = 4096;
        for (uint32_t cb = 0; cb + 256u * U <= nchunks; cb += 256u * U) {
            const uint32_t k = ((16u * (cb + lane)) & 0xFFFFu) >> 1;
            const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
            const gstore_ptr g = (gstore_ptr)(q + cb + lane);
#pragma unroll
            for (int u = 0; u < U; ++u) g[u * 256] = fill_step<U, BARRIER>(B, u);
        }
    }
}

// fillcopy with the product's loop shape: runtime chunk count (not unrolled), the slab address from a
// descriptor array, optionally prefetched
struct PDesc {
    uint64_t off;
    uint32_t len, exp, conn, skip;
};
template <int U, int MODE>  // MODE 0: runtime loop, slab from blockIdx; 1: + descriptor load; 2: + prefetch
__global__ void __launch_bounds__(256) fillshape_kernel(uint8_t* __restrict__ p, const PDesc* __restrict__ d,
                                                        uint32_t n)
{
    typedef u32x4 __attribute__((address_space(1)))* gstore_ptr;
    const uint32_t lane = threadIdx.x;
    PDesc dn;
    if (MODE == 2 && blockIdx.x < n) dn = d[blockIdx.x];
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        uint64_t off;
        uint32_t len;
        if constexpr (MODE == 0) {
            off = (uint64_t)i << 16;
            len = 65536;
        } else if constexpr (MODE == 1) {
            const PDesc x = d[i];
            off = x.off;
            len = x.len;
        } else {
            const PDesc x = dn;
            if (i + gridDim.x < n) dn = d[i + gridDim.x];
            off = x.off;
            len = x.len;
        }
        u32x4* q = reinterpret_cast<u32x4*>(p + off);
        const uint32_t nchunks = len >> 4;
        for (uint32_t cb = 0; cb + 256u * U <= nchunks; cb += 256u * U) {
            const uint32_t k = ((16u * (cb + lane)) & 0xFFFFu) >> 1;
            const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
            const gstore_ptr g = (gstore_ptr)(q + cb + lane);
#pragma unroll
            for (int u = 0; u < U; ++u) g[u * 256] = fill_step<U, true>(B, u);
        }
    }
}

template <int U, int MODE>
static void run_fillshape(const char* name, uint8_t* p, const PDesc* d, uint32_t n, int grid)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    fillshape_kernel<U, MODE><<<grid, 256>>>(p, d, n);
    (void)hipEventRecord(a);
    const int iters = 20;
    for (int i = 0; i < iters; ++i) fillshape_kernel<U, MODE><<<grid, 256>>>(p, d, n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    std::printf("{\"shape\": \"%s\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", name, grid, us,
                (double)n * 65536.0 / (us * 1e3));
    std::fflush(stdout);
}

template <int U, bool BARRIER>
static void run_fillcopy(const char* name, uint8_t* p, uint64_t bytes, int grid)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    fillcopy_kernel<U, BARRIER><<<grid, 256>>>(p, bytes);
    (void)hipEventRecord(a);
    const int iters = 20;
    for (int i = 0; i < iters; ++i) fillcopy_kernel<U, BARRIER><<<grid, 256>>>(p, bytes);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    std::printf("{\"shape\": \"%s\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", name, grid, us, bytes / (us * 1e3));
    std::fflush(stdout);
}

template <int U, int DATA = 0>
static void run_slab(const char* name, uint8_t* p, uint64_t bytes, int grid)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    write_slab_kernel<U, DATA><<<grid, 256>>>(p, bytes, 1);
    (void)hipEventRecord(a);
    const int iters = 20;
    for (int i = 0; i < iters; ++i) write_slab_kernel<U, DATA><<<grid, 256>>>(p, bytes, (uint32_t)i);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    std::printf("{\"shape\": \"%s\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", name, grid, us, bytes / (us * 1e3));
    std::fflush(stdout);
}

template <int W, int U, bool NT>
static void run(const char* name, uint8_t* p, uint64_t bytes, int grid)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    write_kernel<W, U, NT><<<grid, 256>>>(p, bytes, 1);
    (void)hipEventRecord(a);
    const int iters = 20;
    for (int i = 0; i < iters; ++i) write_kernel<W, U, NT><<<grid, 256>>>(p, bytes, (uint32_t)i);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    std::printf("{\"shape\": \"%s\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n", name, grid, us, bytes / (us * 1e3));
    std::fflush(stdout);
}

int main()
{
    const uint64_t bytes = 256ull << 20;
    uint8_t* p = nullptr;
    if (hipMalloc((void**)&p, bytes) != hipSuccess) return 1;
    // arenas rotated as in bench.py (8 x 256 MiB: more than the 256 MB MALL holds), and a single arena
    uint8_t* big = nullptr;
    if (hipMalloc((void**)&big, 8 * bytes) == hipSuccess) {
        for (int grid : {256, 1024, 4096}) {  // a different arena for every launch
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            for (int shape = 0; shape < 2; ++shape) {
                (void)hipEventRecord(a);
                for (int i = 0; i < 24; ++i) {
                    uint8_t* q = big + (uint64_t)(i % 8) * bytes;
                    if (shape == 0) write_slab_kernel<4, 1><<<grid, 256>>>(q, bytes, (uint32_t)i);
                    else write_kernel<16, 4, false><<<grid, 256>>>(q, bytes, (uint32_t)i);
                }
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, a, b);
                const double us = ms * 1e3 / 24;
                std::printf("{\"shape\": \"%s\", \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
                            shape == 0 ? "slab_u4_pattern_rot" : "b16_u4_rot", grid, us, bytes / (us * 1e3));
                std::fflush(stdout);
            }
        }
        (void)hipFree(big);
    }
    {
        const uint32_t n = (uint32_t)(bytes >> 16);
        PDesc* hd = new PDesc[n];
        for (uint32_t i = 0; i < n; ++i) hd[i] = PDesc{(uint64_t)i << 16, 65536u, 0u, i, 0u};
        PDesc* dd = nullptr;
        if (hipMalloc((void**)&dd, n * sizeof(PDesc)) == hipSuccess &&
            hipMemcpy(dd, hd, n * sizeof(PDesc), hipMemcpyHostToDevice) == hipSuccess) {
            for (int grid : {256, 1024}) {
                run_fillshape<4, 0>("fillshape_runtime_loop", p, dd, n, grid);
                run_fillshape<4, 1>("fillshape_desc", p, dd, n, grid);
                run_fillshape<4, 2>("fillshape_desc_prefetch", p, dd, n, grid);
            }
        }
        delete[] hd;
    }
    for (int grid : {256, 1024}) {
        run_fillcopy<4, true>("fillcopy_u4_barrier", p, bytes, grid);
        run_fillcopy<4, false>("fillcopy_u4", p, bytes, grid);
    }
    for (int grid : {256, 1024, 4096}) {
        run_slab<4>("slab_u4", p, bytes, grid);
        run_slab<4, 1>("slab_u4_pattern", p, bytes, grid);
        run_slab<4, 2>("slab_u4_zeros", p, bytes, grid);
        run_slab<1>("slab_u1", p, bytes, grid);
    }
    for (int grid : {256, 512, 1024, 2048, 4096}) {
        run<16, 4, false>("b16_u4", p, bytes, grid);
        run<16, 1, false>("b16_u1", p, bytes, grid);
        run<8, 4, false>("b8_u4", p, bytes, grid);
        run<4, 4, false>("b4_u4", p, bytes, grid);
        run<4, 8, false>("b4_u8", p, bytes, grid);
        run<16, 4, true>("b16_u4_nt", p, bytes, grid);
        run<4, 4, true>("b4_u4_nt", p, bytes, grid);
    }
    return 0;
}
