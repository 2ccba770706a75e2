// rw_mix_probe.hip — what does a small write stream cost next to a streaming read? The
// MediaStream receive kernel writes 44 B of records + results per 1472-B datagram read (3 %), and
// those writes cost it 20-27 % of its time (tools/media_stream_probe.py). This probe streams a
// 2 GiB buffer with 16-B loads (4 per lane per round, grid-stride, like read_or in
// hbm_read_ceiling.hip) and writes ~3 % as many bytes as it reads, in different shapes:
//   none      no writes (the read ceiling)
//   dword     every round, lanes 0..29 of each wave store one dword each (120 B per 4 KiB read)
//   dword_nt  the same, nontemporal stores
//   line16    every round, lanes 0..7 store 16 B each (128 B, one line)
//   burst     every 8th round, lanes 0..59 store 16 B each (960 B per 32 KiB read)
//   wt        dword with write-through (sc1) stores
// Output positions follow the read position (output i belongs to the 4 KiB read as i), as the
// verify kernels' records follow their datagrams. (The 128 MiB output region is rewritten by every launch and
// may partly stay in the 256 MB MALL; the 2 GiB read stream cannot.) Prints one JSON line per shape.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256) rw_kernel(const u32x4* __restrict__ p, uint64_t nchunks, uint32_t* __restrict__ out)
{
    constexpr int U = 4;
    uint32_t acc = 0;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * 256u * U;
    uint64_t c = (uint64_t)blockIdx.x * 256u * U + threadIdx.x;
    for (uint64_t r = 0; c + 256u * (U - 1) < nchunks; c += stride, ++r) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(p + c + u * 256u);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
        // this wave's 4 KiB of the round: output slot = global round-wave index
        const uint64_t slot = ((c - threadIdx.x) / (256u * U)) * 4u + wave;
        const uint32_t v = acc | (uint32_t)r;
        if constexpr (MODE == 1) {
            if (lane < 30u) out[slot * 32u + lane] = v;
        } else if constexpr (MODE == 2) {
            if (lane < 30u) __builtin_nontemporal_store(v, out + slot * 32u + lane);
        } else if constexpr (MODE == 3) {
            if (lane < 8u) *reinterpret_cast<u32x4*>(out + slot * 32u + 4u * lane) = u32x4{v, v, v, v};
        } else if constexpr (MODE == 4) {
            if ((r & 7u) == 7u && lane < 60u)
                *reinterpret_cast<u32x4*>(out + (slot / 8u) * 256u + 4u * lane) = u32x4{v, v, v, v};
        } else if constexpr (MODE == 5) {
            if (lane < 30u) __hip_atomic_store(out + slot * 32u + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int MODE>
static void run(const char* name, const u32x4* p, uint64_t nchunks, uint32_t* out, int grid)
{
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    rw_kernel<MODE><<<grid, 256>>>(p, nchunks, out);
    (void)hipEventRecord(a);
    const int iters = 10;
    for (int i = 0; i < iters; ++i) rw_kernel<MODE><<<grid, 256>>>(p, nchunks, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / iters;
    std::printf("{\"shape\": \"%s\", \"grid\": %d, \"us\": %.1f, \"read_GBps\": %.1f}\n", name, grid, us,
                nchunks * 16.0 / (us * 1e3));
    std::fflush(stdout);
}

int main()
{
    const uint64_t bytes = 2ull << 30, nchunks = bytes / 16;
    u32x4* p = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc((void**)&p, bytes) != hipSuccess || hipMalloc((void**)&out, bytes / 16) != hipSuccess) return 1;
    (void)hipMemset(p, 1, bytes);
    (void)hipMemset(out, 0, bytes / 16);
    for (int grid : {2048, 4096}) {
        run<0>("none", p, nchunks, out, grid);
        run<1>("dword", p, nchunks, out, grid);
        run<2>("dword_nt", p, nchunks, out, grid);
        run<3>("line16", p, nchunks, out, grid);
        run<4>("burst", p, nchunks, out, grid);
        run<5>("wt_sc1", p, nchunks, out, grid);
    }
    return 0;
}
