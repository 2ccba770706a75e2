// hbm_read_ceiling.hip — known-good reference for the verify roofline: how fast
// can a plain streaming READ kernel pull bytes from HBM on this MI355X?
// (methodology rule 10: a ceiling claim needs a reference measured on the same
// hardware). OR-reduces a large buffer with 16-byte loads, sweeping unroll,
// grid size and cache policy; prints one JSON line per configuration.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/hbm_read_ceiling.hip -o tools/hbm_read_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

// grid-stride over chunks; each lane issues U loads per round (straight line)
template <int U, bool NT>
__global__ void __launch_bounds__(256) read_or(const u32x4* __restrict__ p, uint64_t nchunks, uint32_t* out)
{
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256u * U;
    uint64_t c = (uint64_t)blockIdx.x * 256u * U + threadIdx.x;
    for (; c + 256u * (U - 1) < nchunks; c += stride) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = NT ? __builtin_nontemporal_load(p + c + u * 256u) : p[c + u * 256u];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

// contiguous per-block slabs: block b reads chunks [b*per, (b+1)*per) (like one buffer per block)
template <int U, bool NT>
__global__ void __launch_bounds__(256) read_or_slab(const u32x4* __restrict__ p, uint32_t per_block, uint32_t* out)
{
    uint32_t acc = 0;
    const u32x4* q = p + (uint64_t)blockIdx.x * per_block;
    for (uint32_t c = threadIdx.x; c + 256u * (U - 1) < per_block; c += 256u * U) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = NT ? __builtin_nontemporal_load(q + c + u * 256u) : q[c + u * 256u];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// verify's access shape: grid = G blocks, block b reads slabs b, b+G, ... (64 KiB each,
// U*4 KiB rounds); STAG rotates the round order by block so concurrently active blocks
// do not all start at the same 4 KiB offset of their slab (HBM channel/bank spread).
template <int U, bool NT, bool STAG>
__global__ void __launch_bounds__(256) read_or_slab_gs(const u32x4* __restrict__ p, uint32_t per_block,
                                                       uint32_t nslabs, uint32_t* out)
{
    uint32_t acc = 0;
    const uint32_t rounds = per_block / (256u * U);
    for (uint32_t sl = blockIdx.x; sl < nslabs; sl += gridDim.x) {
        const u32x4* q = p + (uint64_t)sl * per_block;
        const uint32_t r0 = STAG ? (sl / 8u) % rounds : 0u;  // blocks b..b+7 land on 8 XCDs
        for (uint32_t k = 0; k < rounds; ++k) {
            uint32_t r = r0 + k;
            r = r >= rounds ? r - rounds : r;
            const uint32_t c = r * 256u * U + threadIdx.x;
            u32x4 d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = NT ? __builtin_nontemporal_load(q + c + u * 256u) : q[c + u * 256u];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
        }
        acc = __syncthreads_or(acc == 0x12345678u) ? 1u : acc;  // verify's per-buffer barrier
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Timeline of the verify-shaped read (grid = BPC x CUs, block b reads 64-KiB slabs b, b + grid, ...):
// s_memrealtime (100 MHz) stamps per workgroup at start, after each slab, at the end, and the XCC id,
// to see where a 256 MiB launch's fixed cost goes (ramp-up, uneven finish).
template <int U>
__global__ void __launch_bounds__(256) read_slab_timeline(const u32x4* __restrict__ p, uint32_t per_block,
                                                          uint32_t nslabs, uint64_t* stamps, uint32_t* out)
{
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    const uint32_t rounds = per_block / (256u * U);
    uint32_t k = 0;
    for (uint32_t sl = blockIdx.x; sl < nslabs; sl += gridDim.x, ++k) {
        const u32x4* q = p + (uint64_t)sl * per_block;
        for (uint32_t r = 0; r < rounds; ++r) {
            const uint32_t c = r * 256u * U + threadIdx.x;
            u32x4 d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(q + c + u * 256u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
        }
        acc = __syncthreads_or(acc == 0x12345678u) ? 1u : acc;
        if (threadIdx.x == 0 && k < 6) stamps[(uint64_t)blockIdx.x * 8 + 1 + k] = __builtin_amdgcn_s_memrealtime();
    }
    if (threadIdx.x == 0) {
        stamps[(uint64_t)blockIdx.x * 8] = t0;
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        stamps[(uint64_t)blockIdx.x * 8 + 7] = (uint64_t)(xcc & 0xFu) | ((uint64_t)k << 8);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// LDS-DMA stream (global_load_lds_dwordx4): each wave reads its own contiguous region through a
// ring of D 1-KiB LDS slots, D DMAs in flight; lane l reads back the 16 bytes it requested
// (the DMA destination is lane-linear), so no barrier is needed, only counted vmcnt waits.
template <int D, int AUX>
__global__ void __launch_bounds__(256) read_ldsdma(const u32x4* __restrict__ p, uint32_t per_wave, uint32_t* out)
{
    __shared__ u32x4 ring[4][D][64];
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    const u32x4* base = p + ((uint64_t)blockIdx.x * 4u + w) * per_wave * 64u + l;
    typedef __attribute__((address_space(3))) void* lds_ptr;
#pragma unroll
    for (int d = 0; d < D; ++d)
        __builtin_amdgcn_global_load_lds(base + d * 64, (lds_ptr)&ring[w][d][0], 16, 0, AUX);
    uint32_t acc = 0;
    uint32_t k = 0;
    for (; k + D < per_wave; ++k) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D - 1) : "memory");
        const u32x4 v = ring[w][k % D][l];
        acc |= v[0] ^ v[1] ^ v[2] ^ v[3];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_global_load_lds(base + (uint64_t)(k + D) * 64, (lds_ptr)&ring[w][k % D][0], 16, 0, AUX);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; k < per_wave; ++k) {
        const u32x4 v = ring[w][k % D][l];
        acc |= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Static slabs, then a dynamically claimed tail: block b reads slabs b, b + G, ... below nstatic * G
// (the verify's shape), then the remaining slabs as ITEM-chunk work items drawn from 8 per-XCD pools
// (one head counter per pool, each on its own 128-B line; a block draws from its own XCD's pool and
// steals from the others once that is dry). The next item is claimed while the current one streams.
// Heads come in two sets: launch k uses set k & 1 and zeroes the other set for launch k + 1 (launches on
// one stream only). nread counts the chunks read (checked against the arena by the host).
template <int U, int ITEM, int STEAL>
__global__ void __launch_bounds__(256) read_dyntail(const u32x4* __restrict__ p, uint32_t nslabs, uint32_t nstatic,
                                                    uint32_t* heads, uint32_t set, uint32_t* nread, uint32_t* out)
{
    // STEAL 0: a block draws from its own XCD's pool only; 1: then from the others one returning atomic at a
    // time; 2: then wave 0 probes all 8 heads with one parallel load, claims from the first open pool
    // (rotated from its own) and leaves after one probe that finds every pool dry.
    constexpr uint32_t PER = 4096u;  // chunks per 64 KiB slab
    static_assert(ITEM % (256 * U) == 0 && PER % ITEM == 0, "item shape");
    if (blockIdx.x == 0 && threadIdx.x < 8)
        __hip_atomic_store(&heads[((set ^ 1u) * 8u + threadIdx.x) * 32u], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t* h = heads + set * 8u * 32u;
    uint32_t acc = 0, cnt = 0;
    const uint32_t G = gridDim.x;
    const uint32_t dyn0 = nstatic * G < nslabs ? nstatic * G : nslabs;
    for (uint32_t sl = blockIdx.x; sl < dyn0; sl += G) {
        const u32x4* q = p + (uint64_t)sl * PER;
        for (uint32_t c = threadIdx.x; c < PER; c += 256u * U) {
            u32x4 d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(q + c + u * 256u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
            cnt += U;
        }
        acc = __syncthreads_or(acc == 0x12345678u) ? 1u : acc;
    }
    const uint32_t items = (nslabs - dyn0) * (PER / ITEM);
    const uint32_t pool = (items + 7u) / 8u;
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7u;
    __shared__ uint32_t slot[2];
    uint32_t dry = 0;  // pools seen empty (wave 0, wave-uniform)
    const uint32_t lane = threadIdx.x;
    auto hi_of = [&](uint32_t x) { return x * pool + pool < items ? x * pool + pool : items; };
    // wave 0 only (all its lanes)
    auto other = [&]() -> uint32_t {
        if constexpr (STEAL == 0) {
            return ~0u;
        } else if constexpr (STEAL == 1) {
            uint32_t r = ~0u;
            if (lane == 0) {
                for (uint32_t t = 0; t < 8u; ++t) {
                    const uint32_t x = (xcc + t) & 7u;
                    if (dry & (1u << x)) continue;
                    if (x * pool < hi_of(x)) {
                        const uint32_t v = __hip_atomic_fetch_add(&h[x * 32u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (x * pool + v < hi_of(x)) { r = x * pool + v; break; }
                    }
                    dry |= 1u << x;
                }
            }
            return __shfl(r, 0);
        } else {
            for (;;) {
                bool open = false;
                if (lane < 8u && !(dry & (1u << lane)) && lane * pool < hi_of(lane)) {
                    const uint32_t v = __hip_atomic_load(&h[lane * 32u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    open = lane * pool + v < hi_of(lane);
                }
                const uint32_t m = (uint32_t)__ballot(open) & 0xFFu;
                dry |= ~m & 0xFFu;
                if (!m) return ~0u;
                const uint32_t rot = ((m >> xcc) | (m << (8u - xcc))) & 0xFFu;
                const uint32_t x = (xcc + (uint32_t)__builtin_ctz(rot)) & 7u;
                uint32_t r = ~0u;
                if (lane == 0) {
                    const uint32_t v = __hip_atomic_fetch_add(&h[x * 32u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (x * pool + v < hi_of(x)) r = x * pool + v;
                }
                r = __shfl(r, 0);
                if (r != ~0u) return r;
                dry |= 1u << x;
            }
        }
    };
    if (lane < 64u) {
        uint32_t r = ~0u;
        if (items && lane == 0) {
            const uint32_t v = __hip_atomic_fetch_add(&h[xcc * 32u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (xcc * pool + v < hi_of(xcc)) r = xcc * pool + v;
        }
        r = __shfl(r, 0);
        if (items && r == ~0u) { dry |= 1u << xcc; r = other(); }
        if (lane == 0) slot[0] = r;
    }
    __syncthreads();
    uint32_t cur = slot[0], par = 1;
    while (cur != ~0u) {
        uint32_t v = 0;
        const bool own = !(dry & (1u << xcc));
        if (lane == 0 && own) v = __hip_atomic_fetch_add(&h[xcc * 32u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t sl = dyn0 + cur / (PER / ITEM), part = cur % (PER / ITEM);
        const u32x4* q = p + (uint64_t)sl * PER + part * ITEM;
        for (uint32_t c = threadIdx.x; c < ITEM; c += 256u * U) {
            u32x4 d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = __builtin_nontemporal_load(q + c + u * 256u);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
            cnt += U;
        }
        if (lane < 64u) {
            uint32_t r = ~0u;
            if (lane == 0 && own && xcc * pool + v < hi_of(xcc)) r = xcc * pool + v;
            r = __shfl(r, 0);
            if (r == ~0u) {
                dry |= 1u << xcc;
                r = other();
            }
            if (lane == 0) slot[par] = r;
        }
        __syncthreads();
        cur = slot[par];
        par ^= 1u;
    }
    if (nread && threadIdx.x == 0) atomicAdd(nread, cnt * 256u);  // every lane reads the same chunk count
    if (acc == 0x12345678u) out[0] = acc;
}

// write reference for the fill kernel: the same slab shape, 16-byte stores (POL 0 = nontemporal,
// 1 = plain, 2 = write-through sc1 via an agent-scope relaxed atomic store of each dword)
template <int U, int POL = 0>
__global__ void __launch_bounds__(256) write_slab_gs(u32x4* __restrict__ p, uint32_t per_block, uint32_t nslabs)
{
    for (uint32_t sl = blockIdx.x; sl < nslabs; sl += gridDim.x) {
        u32x4* q = p + (uint64_t)sl * per_block;
        for (uint32_t c = threadIdx.x; c < per_block; c += 256u * U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t v = sl + c + (uint32_t)u;
                const u32x4 x = u32x4{v, v + 1u, v + 2u, v + 3u};
                if constexpr (POL == 0) __builtin_nontemporal_store(x, q + c + u * 256u);
                else q[c + u * 256u] = x;
            }
        }
    }
}

// ctsTraffic's byte pattern (u16 ramp mod 32768, 64 KiB period) instead of a constant:
// the verify stream reads bytes that toggle; a memset arena does not
__global__ void fill_ramp(uint32_t* p, uint64_t nwords)
{
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t k = (uint32_t)((2 * w) & 0x7FFFu);
        p[w] = k | ((k + 1u) << 16);
    }
}

template <typename F>
static float time_ms(F launch, int reps, hipStream_t s)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch(0);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) launch(i);
    CHECK(hipEventRecord(b, s));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char** argv)
{
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    // argv: [reps] [arena MiB (256 = one config-2 batch)] [quick: 1 = two configs only] [ramp] [writes: 1 = store sweep]
    //       [dma: 1 = LDS-DMA sweep] [timeline: 1 = per-workgroup s_memrealtime stamps]
    const size_t arena = (size_t)(argc > 2 ? atoi(argv[2]) : 256) << 20;
    const bool quick = argc > 3 && atoi(argv[3]) != 0;
    const bool ramp = argc > 4 && atoi(argv[4]) != 0;  // arena holds the ctsTraffic pattern
    const int R = 8;                     // rotate: 2 GiB total, defeats the 256 MiB MALL
    std::vector<u32x4*> bufs(R);
    for (int r = 0; r < R; ++r) {
        CHECK(hipMalloc(&bufs[r], arena));
        if (ramp) fill_ramp<<<2048, 256>>>(reinterpret_cast<uint32_t*>(bufs[r]), arena / 4);
        else CHECK(hipMemset(bufs[r], r + 1, arena));
    }
    uint32_t* out;
    CHECK(hipMalloc(&out, 64));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    const uint64_t nchunks = arena / 16;
    const int reps = argc > 1 ? atoi(argv[1]) : 64;

#define RUN_GS(U, NT, BPC)                                                                                           \
    do {                                                                                                             \
        const uint32_t grid = (uint32_t)cus * (BPC);                                                                 \
        float ms = time_ms([&](int i) { read_or<U, NT><<<grid, 256, 0, s>>>(bufs[i % R], nchunks, out); }, reps, s); \
        printf("{\"kind\":\"gridstride\",\"U\":%d,\"nt\":%d,\"blocks_per_cu\":%d,\"us\":%.2f,\"GBps\":%.1f}\n", U,     \
               (int)NT, BPC, ms * 1e3, arena / (ms * 1e-3) / 1e9);                                                    \
    } while (0)
#define RUN_SLAB(U, NT, SLAB)                                                                                       \
    do {                                                                                                            \
        const uint32_t per = (SLAB) / 16;                                                                           \
        const uint32_t grid = (uint32_t)(arena / (SLAB));                                                          \
        float ms = time_ms([&](int i) { read_or_slab<U, NT><<<grid, 256, 0, s>>>(bufs[i % R], per, out); }, reps, s); \
        printf("{\"kind\":\"slab\",\"U\":%d,\"nt\":%d,\"slab\":%d,\"us\":%.2f,\"GBps\":%.1f}\n", U, (int)NT, SLAB,    \
               ms * 1e3, arena / (ms * 1e-3) / 1e9);                                                                 \
    } while (0)

#define RUN_SLABGS(U, NT, STAG, BPC)                                                                             \
    do {                                                                                                         \
        const uint32_t per = 65536 / 16;                                                                         \
        const uint32_t nsl = (uint32_t)(arena / 65536);                                                          \
        const uint32_t grid = (uint32_t)cus * (BPC);                                                             \
        float ms = time_ms(                                                                                      \
            [&](int i) { read_or_slab_gs<U, NT, STAG><<<grid, 256, 0, s>>>(bufs[i % R], per, nsl, out); }, reps, \
            s);                                                                                                  \
        printf("{\"kind\":\"slab_gs\",\"U\":%d,\"nt\":%d,\"stagger\":%d,\"blocks_per_cu\":%d,\"us\":%.2f,"        \
               "\"GBps\":%.1f}\n",                                                                               \
               U, (int)NT, (int)STAG, BPC, ms * 1e3, arena / (ms * 1e-3) / 1e9);                                 \
    } while (0)

#define RUN_WRP(U, BPC, POL)                                                                                  \
    do {                                                                                                      \
        const uint32_t nsl = (uint32_t)(arena / 65536);                                                       \
        const uint32_t grid = (uint32_t)cus * (BPC);                                                          \
        float ms = time_ms([&](int i) { write_slab_gs<U, POL><<<grid, 256, 0, s>>>(bufs[i % R], 4096u, nsl); }, reps, \
                           s);                                                                                \
        printf("{\"kind\":\"write_slab_gs\",\"U\":%d,\"nt\":%d,\"blocks_per_cu\":%d,\"us\":%.2f,\"GBps\":%.1f}\n", U, \
               POL == 0 ? 1 : 0, BPC, ms * 1e3, arena / (ms * 1e-3) / 1e9);                                 \
    } while (0)
#define RUN_WR(U, BPC) RUN_WRP(U, BPC, 0)

#define RUN_DMA(D, AUX, BPC)                                                                                   \
    do {                                                                                                       \
        const uint32_t grid = (uint32_t)cus * (BPC);                                                           \
        const uint32_t per_wave = (uint32_t)(nchunks / 64 / (grid * 4u));                                      \
        const double bytes = (double)per_wave * 64 * 16 * grid * 4;                                            \
        float ms = time_ms([&](int i) { read_ldsdma<D, AUX><<<grid, 256, 0, s>>>(bufs[i % R], per_wave, out); }, \
                           reps, s);                                                                           \
        printf("{\"kind\":\"ldsdma\",\"D\":%d,\"aux\":%d,\"blocks_per_cu\":%d,\"us\":%.2f,\"GBps\":%.1f}\n", D, AUX, \
               BPC, ms * 1e3, bytes / (ms * 1e-3) / 1e9);                                                       \
    } while (0)

#define RUN_DYN(U, ITEM, NSTATIC, BPC, ST)                                                                            \
    do {                                                                                                          \
        const uint32_t nsl = (uint32_t)(arena / 65536);                                                           \
        const uint32_t grid = (uint32_t)cus * (BPC);                                                              \
        CHECK(hipMemsetAsync(heads, 0, 2 * 8 * 32 * 4, s));                                                       \
        CHECK(hipMemsetAsync(nread, 0, 4, s));                                                                    \
        read_dyntail<U, ITEM, ST><<<grid, 256, 0, s>>>(bufs[0], nsl, NSTATIC, heads, 0u, nread, out);                 \
        uint32_t got = 0;                                                                                         \
        CHECK(hipMemcpy(&got, nread, 4, hipMemcpyDeviceToHost));                                                  \
        CHECK(hipMemsetAsync(heads, 0, 2 * 8 * 32 * 4, s));                                                       \
        CHECK(hipStreamSynchronize(s));                                                                           \
        uint32_t k = 0;                                                                                           \
        float ms = time_ms(                                                                                       \
            [&](int i) {                                                                                          \
                read_dyntail<U, ITEM, ST><<<grid, 256, 0, s>>>(bufs[i % R], nsl, NSTATIC, heads, k & 1u, nullptr, out); \
                ++k;                                                                                              \
            },                                                                                                    \
            reps, s);                                                                                             \
        printf("{\"kind\":\"dyntail\",\"steal\":%d,\"U\":%d,\"item_KiB\":%d,\"nstatic\":%d,\"blocks_per_cu\":%d,\"chunks_ok\":%d,"  \
               "\"us\":%.2f,\"GBps\":%.1f}\n",                                                                     \
               ST, U, (ITEM) / 64, NSTATIC, BPC, (int)(got == nchunks), ms * 1e3, arena / (ms * 1e-3) / 1e9);          \
    } while (0)

    const bool dyn = argc > 8 && atoi(argv[8]) != 0;
    if (dyn) {
        uint32_t *heads, *nread;
        CHECK(hipMalloc(&heads, 2 * 8 * 32 * 4));
        CHECK(hipMalloc(&nread, 4));
        for (int pass = 0; pass < 3; ++pass) {
            RUN_SLABGS(2, true, false, 4);
            RUN_DYN(2, 2048, 3, 4, 0);
            RUN_DYN(2, 2048, 3, 4, 1);
            RUN_DYN(2, 2048, 3, 4, 2);
            RUN_DYN(2, 1024, 3, 4, 0);
            RUN_DYN(2, 1024, 3, 4, 2);
            RUN_DYN(2, 4096, 2, 4, 0);
            RUN_DYN(2, 4096, 2, 4, 2);
            RUN_DYN(2, 2048, 2, 4, 2);
            RUN_DYN(2, 4096, 0, 4, 0);
            RUN_DYN(2, 4096, 0, 4, 2);
        }
        return 0;
    }
    const bool timeline = argc > 7 && atoi(argv[7]) != 0;
    if (timeline) {
        // one timeline per (U, blocks per CU): 3 launches each, the last one's stamps printed as percentiles
        uint64_t* st;
        const int maxgrid = cus * 16;
        CHECK(hipMalloc(&st, (size_t)maxgrid * 8 * sizeof(uint64_t)));
        const int cfg[][2] = {{4, 4}, {2, 4}};
        for (auto& c : cfg) {
            const uint32_t grid = (uint32_t)cus * c[1];
            const uint32_t nsl = (uint32_t)(arena / 65536);
            for (int rep = 0; rep < 3; ++rep) {
                CHECK(hipMemsetAsync(st, 0, (size_t)grid * 8 * sizeof(uint64_t), s));
                if (c[0] == 4) read_slab_timeline<4><<<grid, 256, 0, s>>>(bufs[rep % R], 4096u, nsl, st, out);
                else read_slab_timeline<2><<<grid, 256, 0, s>>>(bufs[rep % R], 4096u, nsl, st, out);
                CHECK(hipStreamSynchronize(s));
            }
            std::vector<uint64_t> h((size_t)grid * 8);
            CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            uint64_t t_min = ~0ull;
            for (uint32_t b = 0; b < grid; ++b) t_min = h[b * 8] < t_min ? h[b * 8] : t_min;
            std::vector<double> starts, ends, firsts;
            for (uint32_t b = 0; b < grid; ++b) {
                const uint32_t k = (uint32_t)(h[b * 8 + 7] >> 8);
                starts.push_back((h[b * 8] - t_min) * 0.01);
                ends.push_back((h[b * 8 + (k < 6 ? k : 6)] - t_min) * 0.01);
                firsts.push_back((h[b * 8 + 1] - h[b * 8]) * 0.01);
            }
            auto pct = [](std::vector<double> v, double q) {
                std::sort(v.begin(), v.end());
                return v[(size_t)(q * (v.size() - 1))];
            };
            printf("{\"kind\":\"timeline\",\"U\":%d,\"blocks_per_cu\":%d,\"start_us\":[%.2f,%.2f,%.2f],"
                   "\"first_slab_us\":[%.2f,%.2f,%.2f],\"end_us\":[%.2f,%.2f,%.2f,%.2f,%.2f],\"end_by_xcc\":[",
                   c[0], c[1], pct(starts, 0), pct(starts, 0.5), pct(starts, 1.0), pct(firsts, 0), pct(firsts, 0.5),
                   pct(firsts, 1.0), pct(ends, 0), pct(ends, 0.1), pct(ends, 0.5), pct(ends, 0.9), pct(ends, 1.0));
            for (uint32_t x = 0; x < 8; ++x) {  // per XCC: min / median / max end
                std::vector<double> ex;
                for (uint32_t b = 0; b < grid; ++b)
                    if ((h[b * 8 + 7] & 0xFu) == x) ex.push_back(ends[b]);
                if (ex.empty()) continue;
                printf("%s[%u,%.2f,%.2f,%.2f]", x ? "," : "", x, pct(ex, 0), pct(ex, 0.5), pct(ex, 1.0));
            }
            printf("]}\n");
        }
        return 0;
    }
    const bool dma = argc > 6 && atoi(argv[6]) != 0;
    if (dma) {
        for (int pass = 0; pass < 2; ++pass) {
            RUN_GS(4, true, 8);
            RUN_SLAB(4, true, 65536);
            RUN_DMA(4, 2, 2);
            RUN_DMA(8, 2, 2);
            RUN_DMA(8, 2, 1);
            RUN_DMA(16, 2, 1);
            RUN_DMA(8, 0, 2);
            RUN_DMA(4, 2, 4);
            RUN_DMA(16, 2, 2);
        }
        return 0;
    }
    const bool writes = argc > 5 && atoi(argv[5]) != 0;
    if (writes) {
        for (int pass = 0; pass < 2; ++pass) {
            RUN_WRP(4, 2, 1);
            RUN_WRP(4, 4, 1);
            RUN_WRP(2, 8, 1);
            RUN_WRP(4, 2, 0);
            RUN_WR(1, 4);
            RUN_WR(2, 4);
            RUN_WR(4, 4);
            RUN_WR(4, 8);
            RUN_WR(2, 8);
            RUN_WR(1, 8);
            RUN_WR(4, 2);
            RUN_WR(4, 16);
        }
        return 0;
    }
    if (quick) {
        for (int pass = 0; pass < 2; ++pass) {
            RUN_GS(8, true, 8);
            RUN_GS(4, true, 8);
            RUN_SLAB(8, true, 65536);
            RUN_SLAB(4, true, 65536);
            RUN_SLABGS(4, true, false, 8);
            RUN_SLABGS(4, true, true, 8);
            RUN_SLABGS(8, true, false, 8);
            RUN_SLABGS(8, true, true, 8);
            RUN_SLABGS(4, true, false, 4);
            RUN_SLABGS(4, true, true, 4);
        }
        return 0;
    }
    for (int pass = 0; pass < 2; ++pass) {
        RUN_GS(4, true, 4);
        RUN_GS(4, true, 8);
        RUN_GS(4, true, 16);
        RUN_GS(8, true, 4);
        RUN_GS(8, true, 8);
        RUN_GS(2, true, 8);
        RUN_GS(2, true, 16);
        RUN_GS(1, true, 32);
        RUN_GS(4, false, 8);
        RUN_GS(8, false, 4);
        RUN_SLAB(8, true, 65536);
        RUN_SLAB(4, true, 65536);
        RUN_SLAB(16, true, 65536);
        RUN_SLAB(4, true, 32768);
        RUN_SLAB(8, true, 131072);
        RUN_SLAB(8, false, 65536);
    }
    return 0;
}
