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
//   *_deferred the round's outputs stored after the NEXT round's loads are issued (a store counts in
//             vmcnt, in issue order with the loads: stored before them, its ack joins their wait)
//   dword_everyK / dword_once_at_end: the dword shape on every K-th round only / once per wave at its end
//   frac_NB   (argv: any two arguments) dword stores of N bytes per 4 KiB read, N = 4 .. 120
//   phasedP_B the dword outputs of P rounds kept in LDS, then written by every workgroup at once: a
//             co-resident grid meets at a grid barrier (B = 1: before the write phase; B = 2: before and
//             after it), so the memory sees read phases and write phases instead of a mix
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
    // MODE 6/7: the previous round's output, stored after this round's loads, by every lane with no branch
    // (an exec-skip branch around the store makes the compiler's vmcnt at the join count it as if issued:
    // the loads' wait would then include it). Round 0 stores a placeholder to its own slot, overwritten later.
    uint32_t pend_v = 0;
    uint64_t pend_slot = ((c - threadIdx.x) / (256u * U)) * 4u + wave;
    for (uint64_t r = 0; c + 256u * (U - 1) < nchunks; c += stride, ++r) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(p + c + u * 256u);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (MODE == 6) {
            out[pend_slot * 32u + (lane < 30u ? lane : 29u)] = pend_v;
            __builtin_amdgcn_sched_barrier(0);
        } else if constexpr (MODE == 7) {
            *reinterpret_cast<u32x4*>(out + pend_slot * 32u + 4u * (lane & 7u)) = u32x4{pend_v, pend_v, pend_v, pend_v};
            __builtin_amdgcn_sched_barrier(0);
        }
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
        } else if constexpr (MODE == 9) {
            if ((r & 15u) == 15u && lane < 30u) out[slot * 32u + lane] = v;
        } else if constexpr (MODE == 10) {
            if ((r & 63u) == 63u && lane < 30u) out[slot * 32u + lane] = v;
        } else if constexpr (MODE == 6 || MODE == 7 || MODE == 8) {
            pend_v = v;
            pend_slot = slot;
        } else if constexpr (MODE > 100) {  // write fraction sweep: lanes 0..MODE-101 store one dword each
            if (lane < (uint32_t)(MODE - 100)) out[slot * 32u + lane] = v;
        }
    }
    if constexpr (MODE == 6 || MODE == 7 || MODE == 8)
        if (lane < 30u) out[pend_slot * 32u + lane] = pend_v;
    if (acc == 0x12345678u) out[0] = acc;
}

// Grid barrier for a co-resident grid: workgroup b adds to sub-counter b % nsub (its own 128-B line); the
// last arriver of a sub-counter adds to the top counter; everyone waits for the top to reach the generation.
// Counters only grow (generation gen counts from the launch's gen0), so launches need no reset. A barrier
// that waits past ~200 ms (a grid that is not co-resident) sets *err and lets the waves go.
template <int SLEEP>
__device__ __forceinline__ void grid_sync(uint32_t* bar, uint32_t nsub, uint32_t gen, uint32_t* err)
{
    // lines: 0 = top arrivals, 1..nsub = sub arrivals, 1+nsub..2*nsub = sub release words
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t s = blockIdx.x % nsub;
        const uint32_t per = gridDim.x / nsub + (s < gridDim.x % nsub ? 1u : 0u);
        const uint32_t old = __hip_atomic_fetch_add(bar + 32u * (1u + s), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1u == gen * per) {
            const uint32_t top = __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (top + 1u == gen * nsub)
                for (uint32_t i = 0; i < nsub; ++i)
                    __hip_atomic_store(bar + 32u * (1u + nsub + i), gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t t0 = wall_clock64();
        uint32_t* const rel = bar + 32u * (1u + nsub + s);
        while (__hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
            __builtin_amdgcn_s_sleep(SLEEP);
            if (wall_clock64() - t0 > 20000000ull) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

template <int P, int BARS, int SLEEP = 4>
__global__ void __launch_bounds__(256) phased_kernel(const u32x4* __restrict__ p, uint64_t nchunks, uint32_t* __restrict__ out,
                                                     uint32_t* bar, uint32_t nsub, uint32_t gen0, uint32_t* err)
{
    constexpr int U = 4;
    __shared__ uint32_t stage[P][4][32];
    uint32_t acc = 0, gen = gen0;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * 256u * U;
    uint64_t c = (uint64_t)blockIdx.x * 256u * U + threadIdx.x;
    uint64_t slot0 = 0;
    for (uint64_t r = 0; c + 256u * (U - 1) < nchunks; c += stride, ++r) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(p + c + u * 256u);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
        const uint32_t k = (uint32_t)(r % P);
        if (k == 0) slot0 = ((c - threadIdx.x) / (256u * U)) * 4u;
        if (lane < 30u) stage[k][wave][lane] = acc | (uint32_t)r;
        if (k == P - 1) {  // end of a read phase: meet, write the phase's outputs, (meet)
            grid_sync<SLEEP>(bar, nsub, ++gen, err);
            for (uint32_t i = threadIdx.x; i < P * 128u; i += 256u) {
                const uint32_t kk = i / 128u, w = (i / 32u) & 3u, l = i & 31u;
                if (l < 30u) out[(slot0 + (uint64_t)kk * (gridDim.x * 4u) + w) * 32u + l] = stage[kk][w][l];
            }
            if constexpr (BARS == 2) grid_sync<SLEEP>(bar, nsub, ++gen, err);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int P, int BARS, int SLEEP = 4>
static void run_phased(const char* name, const u32x4* p, uint64_t nchunks, uint32_t* out, uint32_t* bar, uint32_t* err)
{
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, phased_kernel<P, BARS, SLEEP>, 256, 0);
    int grid = cus * (per_cu < 8 ? per_cu : 8);
    // every workgroup must run the same number of rounds, a multiple of P (each meets every barrier)
    while (grid > 0 && (nchunks / (256u * 4u)) % ((uint64_t)grid * P) != 0) grid -= cus;
    if (grid <= 0) return;
    const uint32_t nsub = 32;
    const uint32_t phases = (uint32_t)(nchunks / (256u * 4u) / ((uint64_t)grid * P));
    const uint32_t per_launch = phases * BARS;
    (void)hipMemset(bar, 0, 65 * 128);
    (void)hipMemset(err, 0, 4);
    uint32_t gen0 = 0;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    phased_kernel<P, BARS, SLEEP><<<grid, 256>>>(p, nchunks, out, bar, nsub, gen0, err);
    gen0 += per_launch;
    (void)hipEventRecord(a);
    const int iters = 10;
    for (int i = 0; i < iters; ++i, gen0 += per_launch) phased_kernel<P, BARS, SLEEP><<<grid, 256>>>(p, nchunks, out, bar, nsub, gen0, err);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    uint32_t e = 0;
    (void)hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
    const double us = ms * 1e3 / iters;
    std::printf("{\"shape\": \"%s\", \"grid\": %d, \"phases\": %u, \"us\": %.1f, \"read_GBps\": %.1f, \"barrier_timeout\": %u}\n",
                name, grid, phases, us, nchunks * 16.0 / (us * 1e3), e);
    std::fflush(stdout);
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

int main(int argc, char**)
{
    const uint64_t bytes = 2ull << 30, nchunks = bytes / 16;
    u32x4* p = nullptr;
    uint32_t* out = nullptr;
    uint32_t *bar = nullptr, *err = nullptr;
    if (hipMalloc((void**)&p, bytes) != hipSuccess || hipMalloc((void**)&out, bytes / 16) != hipSuccess ||
        hipMalloc((void**)&bar, 65 * 128) != hipSuccess || hipMalloc((void**)&err, 4) != hipSuccess)
        return 1;
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
    if (argc > 2) {  // how the cost scales with the written fraction (dword shape, bytes per 4 KiB read)
        for (int pass = 0; pass < 2; ++pass) {
            run<0>("none", p, nchunks, out, 2048);
            run<101>("frac_4B", p, nchunks, out, 2048);
            run<102>("frac_8B", p, nchunks, out, 2048);
            run<104>("frac_16B", p, nchunks, out, 2048);
            run<108>("frac_32B", p, nchunks, out, 2048);
            run<115>("frac_60B", p, nchunks, out, 2048);
            run<130>("frac_120B", p, nchunks, out, 2048);
            run<1>("dword", p, nchunks, out, 2048);
            run<6>("dword_deferred", p, nchunks, out, 2048);
            run<3>("line16", p, nchunks, out, 2048);
            run<7>("line16_deferred", p, nchunks, out, 2048);
            run<9>("dword_every16", p, nchunks, out, 2048);
            run<10>("dword_every64", p, nchunks, out, 2048);
            run<8>("dword_once_at_end", p, nchunks, out, 2048);
        }
        return 0;
    }
    if (argc > 1) {
        run<0>("none", p, nchunks, out, 2048);
        run<1>("dword", p, nchunks, out, 2048);
        run_phased<8, 1, 1>("phased8_1_s1", p, nchunks, out, bar, err);
        run_phased<8, 1, 4>("phased8_1_s4", p, nchunks, out, bar, err);
        run_phased<8, 1, 16>("phased8_1_s16", p, nchunks, out, bar, err);
        run_phased<8, 2, 4>("phased8_2_s4", p, nchunks, out, bar, err);
        run_phased<16, 1, 4>("phased16_1_s4", p, nchunks, out, bar, err);
        run_phased<32, 1, 4>("phased32_1_s4", p, nchunks, out, bar, err);
        run_phased<32, 2, 4>("phased32_2_s4", p, nchunks, out, bar, err);
    }
    return 0;
}
