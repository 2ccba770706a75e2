// verify_ablation.hip — where do the microseconds between a plain streaming read
// (tools/hbm_read_ceiling.hip) and cts::verify_wg_kernel go? One 256-lane
// workgroup per 64 KiB slab, U x 16-byte nontemporal buffer loads per lane per
// round, and the verify kernel's extra work switched on one piece at a time:
//   desc  : the slab address comes from a 24-byte descriptor loaded first
//   alu   : the expected pattern is regenerated and XORed (verify's ALU)
//   sync  : __syncthreads_or after every slab
//   grid  : grid-stride over slabs (blocks_per_cu x CUs workgroups) vs one slab each
// Diagnostic only (not part of the product). Prints one JSON line per config.
//
// build: hipcc --offload-arch=gfx950 -O3 tools/verify_ablation.hip -o tools/verify_ablation
#include <hip/hip_runtime.h>

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

struct Desc {
    uint64_t off;
    uint32_t len, exp, conn, skip;
};

__device__ __forceinline__ u32x4 expected(uint32_t B, int u)
{
    uint32_t bb = B;
    asm volatile("" : "+v"(bb));
    const uint32_t b = bb + (uint32_t)u * 2048u * 0x10001u;
    return u32x4{b & 0x7FFF7FFFu, (b + 0x20002u) & 0x7FFF7FFFu, (b + 0x40004u) & 0x7FFF7FFFu,
                 (b + 0x60006u) & 0x7FFF7FFFu};
}

// EDGE: like cts::scan_buffer — lanes 0..8 load chunk 0 / the last chunk / head chunks first,
//       the interior [8, 4095) streams in a full round + a masked tail round (voffset form)
// REC : lane 0 writes a 12-byte per-buffer record and adds 5 u64 counters in LDS, flushed at the end
template <int U, bool DESC, bool ALU, bool SYNC, bool EDGE = false, bool REC = false>
__global__ void __launch_bounds__(256, 8)
    slab(const uint8_t* __restrict__ arena, const Desc* __restrict__ descs, uint32_t n, uint32_t* out)
{
    __shared__ uint64_t ctr[5];
    if (threadIdx.x < 5) ctr[threadIdx.x] = 0;
    __syncthreads();
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        uint64_t off = (uint64_t)i * 65536u;
        if constexpr (DESC) off = descs[i].off;
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(arena + off), (short)0, 65536, 0x00020000);
        const uint32_t voff = threadIdx.x * 16u;
        uint32_t a = 0;
        u32x4 edge = {0, 0, 0, 0};
        if constexpr (EDGE) {
            const uint32_t lane = threadIdx.x;
            const uint32_t ce = lane == 1u ? 4095u : (lane >= 2u && lane <= 8u ? lane - 1u : 0u);
            edge = __builtin_amdgcn_raw_buffer_load_b128(r, lane <= 8u ? ce * 16u : 0x7FFFFFF0u, 0u, 2);
            uint32_t cb = 8;
            for (; cb + 256u * U <= 4095u; cb += 256u * U) {
                u32x4 d[U];
#pragma unroll
                for (int u = 0; u < U; ++u) d[u] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, (cb + u * 256u) * 16u, 2);
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t k = (((cb + threadIdx.x) * 16u) & 0xFFFFu) >> 1;
                const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    u32x4 x = d[u];
                    if constexpr (ALU) x ^= expected(B, u);
                    a |= x[0] | x[1] | x[2] | x[3];
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (cb < 4095u) {
                u32x4 d[U];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    d[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (cb + u * 256u + threadIdx.x) * 16u, 0u, 2);
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t k = (((cb + threadIdx.x) * 16u) & 0xFFFFu) >> 1;
                const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    u32x4 x = d[u];
                    if constexpr (ALU) x ^= expected(B, u);
                    const uint32_t any = x[0] | x[1] | x[2] | x[3];
                    a |= (cb + u * 256u + threadIdx.x < 4095u) ? any : 0u;
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            a |= lane <= 8u ? (edge[0] | edge[1] | edge[2] | edge[3]) : 0u;
        } else {
            for (uint32_t cb = 0; cb < 4096u; cb += 256u * U) {
                u32x4 d[U];
#pragma unroll
                for (int u = 0; u < U; ++u) d[u] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, (cb + u * 256u) * 16u, 2);
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t k = (((cb + threadIdx.x) * 16u) & 0xFFFFu) >> 1;
                const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    u32x4 x = d[u];
                    if constexpr (ALU) x ^= expected(B, u);
                    a |= x[0] | x[1] | x[2] | x[3];
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        bool bad;
        if constexpr (SYNC) {
            bad = __syncthreads_or(a == 0x12345678u);
        } else {
            bad = a == 0x12345678u;
            acc |= a;
        }
        if constexpr (REC) {
            if (threadIdx.x == 0) {
                uint32_t rec[3] = {65536u, 0u, bad ? 0u : 0x00010000u};
                uint32_t* dst = out + 16 + 3 * (size_t)i;
                dst[0] = rec[0];
                dst[1] = rec[1];
                dst[2] = rec[2];
                ctr[0] += 65536;
                ctr[2] += 1;
                ctr[1] += bad ? 0 : 65536;
            }
        } else if (bad) {
            acc ^= 1;
        }
    }
    if constexpr (REC) {
        __syncthreads();
        if (threadIdx.x < 5 && ctr[threadIdx.x]) atomicAdd((unsigned long long*)(out + 2 * threadIdx.x), ctr[threadIdx.x]);
    }
    if (acc == 0x12345678u) out[0] = acc;
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
    return ms / reps;
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? atoi(argv[1]) : 100;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t n = 4096;
    const size_t arena = (size_t)n * 65536;
    const int R = 8;
    std::vector<uint8_t*> bufs(R);
    for (int r = 0; r < R; ++r) {
        CHECK(hipMalloc(&bufs[r], arena));
        CHECK(hipMemset(bufs[r], 0, arena));
    }
    std::vector<Desc> hd(n);
    for (uint32_t i = 0; i < n; ++i) hd[i] = Desc{(uint64_t)i * 65536u, 65536u, 0u, i, 0u};
    Desc* dd;
    CHECK(hipMalloc(&dd, n * sizeof(Desc)));
    CHECK(hipMemcpy(dd, hd.data(), n * sizeof(Desc), hipMemcpyHostToDevice));
    uint32_t* out;
    CHECK(hipMalloc(&out, 64 + 16 * (size_t)n));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));

#define RUN(U, DESC, ALU, SYNC, EDGE, REC, BPC)                                                                \
    do {                                                                                                      \
        const uint32_t grid = (BPC) == 0 ? n : (uint32_t)cus * (BPC);                                         \
        float ms = time_ms(                                                                                   \
            [&](int i) { slab<U, DESC, ALU, SYNC, EDGE, REC><<<grid, 256, 0, s>>>(bufs[i % R], dd, n, out); }, reps, s); \
        printf("{\"U\":%d,\"desc\":%d,\"alu\":%d,\"sync\":%d,\"edge\":%d,\"rec\":%d,\"blocks_per_cu\":%d,"     \
               "\"us\":%.2f,\"GBps\":%.1f}\n", U, (int)DESC, (int)ALU, (int)SYNC, (int)EDGE, (int)REC, BPC, ms * 1e3,  \
               arena / (ms * 1e-3) / 1e9);                                                                     \
    } while (0)

    const bool isolate = argc > 2 && atoi(argv[2]) != 0;
    if (isolate) {  // one piece at a time over the plain read (U4 = verify's default round)
        for (int pass = 0; pass < 2; ++pass) {
            RUN(4, false, false, false, false, false, 8);
            RUN(4, true, false, false, false, false, 8);
            RUN(4, false, true, false, false, false, 8);
            RUN(4, false, false, true, false, false, 8);
            RUN(4, true, true, false, false, false, 8);
            RUN(4, true, true, true, false, false, 8);
            RUN(8, false, true, false, false, false, 8);
            RUN(8, false, false, true, false, false, 8);
        }
        return 0;
    }
    for (int pass = 0; pass < 2; ++pass) {
        RUN(8, false, false, false, false, false, 8);
        RUN(8, true, true, true, false, false, 8);
        RUN(8, true, true, true, true, false, 8);
        RUN(8, true, true, true, false, true, 8);
        RUN(8, true, true, true, true, true, 8);
        RUN(8, true, true, false, true, true, 8);
        RUN(4, true, true, true, true, true, 8);
        RUN(8, true, true, true, true, true, 0);
    }
    return 0;
}
