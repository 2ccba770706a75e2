// verify_timeline.hip — where does a config-2 verify launch spend the time a plain streaming read of the same
// bytes does not? (DESIGN.md §3 "Where a 256 MiB launch's last few percent go"; VERDICT r03 "Next round" 3.)
//
// The product kernel (cts_kernels.hip, included verbatim) against the plain read of the same shape, in one process on
// one box, 8 rotated 256 MiB arenas (4096 x 64 KiB buffers each; 75 % phase-0 / 25 % random expected offsets, one
// corrupt byte per 1024 buffers, as bench.py's config 2):
//   time    : HIP events around R launches, per launch: the product verify_wg_kernel ("product_verify_us"), a
//             replica of its whole-line path built from the same device helpers with the stamps compiled out (must
//             equal the product), a depth-2 pipelined form (pipe2), and the plain read (grid = 4 x CUs, workgroup b
//             reads 64-KiB slabs b, b + grid, ..., U = 2, the verify's per-buffer barrier);
//   timeline: per-workgroup s_memrealtime stamps (100 MHz) of the stamped replica and of the plain read:
//             entry, first data issue (after the first descriptor arrived), the end of every buffer, the end
//             after the counter flush; printed as percentiles over the 1024 workgroups and by XCC.
// Built twice by the Makefile: tools/verify_timeline and tools/verify_timeline_kp (kernel arguments preloaded into
// SGPRs: -mllvm -amdgpu-kernarg-preload-count=16), so one call compares both prologues. Diagnostic only.
// CTS_KERNELS_FILE: another revision of the product kernels for an A/B on one box (CTS_TL_COUNTERS: its counter
// count per shard row, 5 before round 6)
#ifdef CTS_KERNELS_FILE
#include CTS_KERNELS_FILE
#else
#include "../ctstraffic_amd/csrc/cts_kernels.hip"
#endif
#ifndef CTS_TL_COUNTERS
#define CTS_TL_COUNTERS cts::kCounterCount
#endif

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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
constexpr int kSt = 16;  // stamp slots per workgroup

__device__ __forceinline__ uint64_t stamp() { return __builtin_amdgcn_s_memrealtime(); }
// a stamp taken once `dep` is available (the asm's input makes the compiler wait for it first)
__device__ __forceinline__ uint64_t stamp_after(uint32_t dep)
{
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "s"(dep));
    return t;
}
__device__ __forceinline__ uint32_t xcc_id()
{
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 0xFu;
}

// the test arena: buffer i = the pattern from its expected offset, written 16 bytes at a time
__global__ void fill_arena(u32x4* a, const cts_buf_desc* d, uint32_t n)
{
    for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < (uint64_t)n * 4096; c += (uint64_t)gridDim.x * 256) {
        const uint32_t q = (d[c / 4096].expected_pattern_offset + 16u * (uint32_t)(c % 4096)) & 0xFFFFu;
        a[c] = cts::expected_chunk(q, q & 1u);
    }
}

// A whole-line span streamed one chunk per lane per step with the next two steps' loads in flight (a pipeline of depth
// 2 at U = 1): at most 2 KiB in flight per wave, as the product's U = 2 rounds, but never none while the wave compares.
template <bool EVEN>
__device__ __forceinline__ void scan_pipe2(const cts::Span& s, uint32_t lane, uint32_t& first, uint32_t& count)
{
    const __amdgpu_buffer_rsrc_t r = cts::span_rsrc(s);
    const uint32_t steps = s.nchunks / 256u;
    const uint32_t voff = lane * 16u;
    u32x4 a = cts::buf_load<true>(r, voff, 0u);
    u32x4 b = cts::buf_load<true>(r, voff, 256u * 16u);  // past the span: reads 0, no request
    for (uint32_t j = 0; j < steps; ++j) {
        const u32x4 nxt = cts::buf_load<true>(r, voff, (j + 2u) * 256u * 16u);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t B = cts::chunk_base(s, j * 256u + lane);
        const u32x4 x = a ^ cts::expected_step<256, 1, EVEN>(B, 0, s.sh);
        if (cts::or4(x) != 0u) cts::take_diff(s, j * 256u + lane, x, first, count);
        a = b;
        b = nxt;
    }
}

template <bool STAMP>
__global__ void __launch_bounds__(256, 8)
    verify_pipe(const uint8_t* __restrict__ arena, uint64_t arena_bytes, const cts_buf_desc* __restrict__ descs,
                uint32_t n, cts_verify_result* __restrict__ results, uint64_t* __restrict__ counters,
                uint32_t* __restrict__ conn_first_fail, uint32_t n_conns)
{
    __shared__ uint64_t ctr[1][CTS_TL_COUNTERS];
    const uint32_t lane = threadIdx.x;
    uint32_t i = blockIdx.x;
    const uint32_t step = gridDim.x;
    cts_buf_desc dn;
    if (i < n) dn = descs[i];
    cts::zero_counters<1>(ctr);
    for (; i < n; i = i + step < n ? i + step : n) {
        const cts_buf_desc d = dn;
        if (i + step < n) dn = descs[i + step];
        if (cts::desc_bad(d, arena_bytes)) continue;
        const cts::Span s = cts::make_span(arena, d);
        uint32_t first = cts::kNone, count = 0;
        if (__builtin_amdgcn_readfirstlane((cts::span_whole_lines(s) && s.nchunks % 256u == 0u) ? 1u : 0u)) {
            if (__builtin_amdgcn_readfirstlane(s.sh) == 0u) scan_pipe2<true>(s, lane, first, count);
            else scan_pipe2<false>(s, lane, first, count);
        } else {
            cts::scan_whole_exact<256, 2, true, true>(s, lane, first, count);
        }
        const bool dirty = __builtin_amdgcn_readfirstlane(__syncthreads_or(first != cts::kNone)) != 0;
        if (dirty) cts::block_reduce_mismatch(first, count);
        if (lane == 0) cts::finish_buffer(s, d, i, first, count, results, ctr[0], conn_first_fail, n_conns);
    }
    cts::flush_counters<1>(counters, ctr);
}

// verify_wg_kernel<true> on the whole-line path every config-2 buffer takes, built from the same helpers; STAMP adds the
// timeline stores (lane 0, one 8-byte store per event).
template <bool STAMP>
__global__ void __launch_bounds__(256, 4)
    verify_replica(const uint8_t* __restrict__ arena, uint64_t arena_bytes, const cts_buf_desc* __restrict__ descs,
                   uint32_t n, cts_verify_result* __restrict__ results, uint64_t* __restrict__ counters,
                   uint32_t* __restrict__ conn_first_fail, uint32_t n_conns, uint64_t* __restrict__ st)
{
    const uint64_t t_entry = STAMP ? stamp() : 0;
    __shared__ uint64_t ctr[1][CTS_TL_COUNTERS];
    const uint32_t lane = threadIdx.x;
    uint32_t i = blockIdx.x, k = 0;
    const uint32_t step = gridDim.x;
    cts_buf_desc dn;
    if (i < n) dn = descs[i];
    cts::zero_counters<1>(ctr);
    uint64_t* my = st + (uint64_t)blockIdx.x * kSt;
    for (; i < n; i = i + step < n ? i + step : n, ++k) {
        const cts_buf_desc d = dn;
        if (i + step < n) dn = descs[i + step];
        if (cts::desc_bad(d, arena_bytes)) continue;
        const cts::Span s = cts::make_span(arena, d);
        if (STAMP && k == 0 && lane == 0) my[1] = stamp_after((uint32_t)d.byte_offset);
        uint32_t first = cts::kNone, count = 0;
        cts::scan_whole_exact<256, 2, true, true>(s, lane, first, count);
        const bool dirty = __builtin_amdgcn_readfirstlane(__syncthreads_or(first != cts::kNone)) != 0;
        if (dirty) cts::block_reduce_mismatch(first, count);
        if (lane == 0) cts::finish_buffer(s, d, i, first, count, results, ctr[0], conn_first_fail, n_conns);
        if (STAMP && lane == 0 && k < 8) my[2 + k] = stamp();
    }
    cts::flush_counters<1>(counters, ctr);
    if (STAMP && lane == 0) {
        my[0] = t_entry;
        my[10] = stamp();
        my[11] = (uint64_t)xcc_id() | ((uint64_t)k << 8);
    }
}

// the plain read of the same shape (hbm_read_ceiling.hip read_slab_timeline): no descriptor, no compare, no output.
// MAP (the "map" mode): which slab workgroup b reads in its k-th step: 0 = b + k G (the verify's walk), 1 = (b ^ 1) + k G
// (each XCC reads the other parity of 64 KiB slots), 2 = ((b + k) mod G) + k G (each XCC's slots alternate in parity)
template <bool STAMP, int MAP = 0>
__global__ void __launch_bounds__(256) plain_read(const u32x4* __restrict__ p, uint32_t nslabs, uint64_t* st,
                                                  uint32_t* out)
{
    const uint64_t t_entry = STAMP ? stamp() : 0;
    uint32_t acc = 0, k = 0;
    uint64_t* my = st + (uint64_t)blockIdx.x * kSt;
    for (uint32_t sl0 = blockIdx.x; sl0 < nslabs; sl0 += gridDim.x, ++k) {
        uint32_t sl = sl0;
        if constexpr (MAP == 1) sl = sl0 ^ 1u;
        if constexpr (MAP == 2) sl = sl0 - blockIdx.x + (blockIdx.x + k) % gridDim.x;
        const u32x4* q = p + (uint64_t)sl * 4096u;
        if (STAMP && k == 0 && threadIdx.x == 0) my[1] = stamp();
        for (uint32_t r = 0; r < 8; ++r) {
            const uint32_t c = r * 512u + threadIdx.x;
            u32x4 d[2];
            d[0] = __builtin_nontemporal_load(q + c);
            d[1] = __builtin_nontemporal_load(q + c + 256u);
            __builtin_amdgcn_sched_barrier(0);
            acc |= d[0][0] ^ d[0][1] ^ d[0][2] ^ d[0][3] ^ d[1][0] ^ d[1][1] ^ d[1][2] ^ d[1][3];
        }
        acc = __syncthreads_or(acc == 0x12345678u) ? 1u : acc;
        if (STAMP && threadIdx.x == 0 && k < 8) my[2 + k] = stamp();
    }
    if (acc == 0x12345678u) out[0] = acc;
    if (STAMP && threadIdx.x == 0) {
        my[0] = t_entry;
        my[10] = stamp();
        my[11] = (uint64_t)xcc_id() | ((uint64_t)k << 8);
    }
}

#define PRODUCT cts::verify_wg_kernel<true>

// XCD-skewed plain read ("skew" mode): the grid has S = gridDim.x / 8 slots per XCD (workgroup b runs on XCD b mod 8,
// the dispatcher's round robin); on the odd XCDs only S - 2 dd of them work, dd = S * SKEW / (64 + SKEW), so the even
// XCDs read (S) / (S - 2 dd) times as many slabs. The active workgroups are ranked even XCDs first and walk slabs
// rank, rank + A, ... (A = active count): every slab is read once whatever the placement.
template <bool STAMP, int SKEW>
__global__ void __launch_bounds__(256) plain_read_skew(const u32x4* __restrict__ p, uint32_t nslabs, uint64_t* st,
                                                       uint32_t* out)
{
    const uint64_t t_entry = STAMP ? stamp() : 0;
    // SKEW < 0: the even XCDs get the fewer workgroups instead
    constexpr uint32_t AS = (uint32_t)(SKEW < 0 ? -SKEW : SKEW);
    const uint32_t S = gridDim.x / 8u, dd = S * AS / (64u + AS), So = S - 2u * dd;
    const uint32_t x = blockIdx.x & 7u, q = blockIdx.x >> 3;
    const uint32_t few = (x & 1u) ^ (SKEW < 0 ? 1u : 0u);  // this XCD runs So workgroups
    if (few && q >= So) return;
    const uint32_t rank = few ? 4u * S + (x >> 1) * So + q : (x >> 1) * S + q;
    const uint32_t A = 4u * S + 4u * So;
    uint32_t acc = 0, k = 0;
    uint64_t* my = st + (uint64_t)rank * kSt;
    for (uint32_t sl = rank; sl < nslabs; sl += A, ++k) {
        const u32x4* qq = p + (uint64_t)sl * 4096u;
        if (STAMP && k == 0 && threadIdx.x == 0) my[1] = stamp();
        for (uint32_t r = 0; r < 8; ++r) {
            const uint32_t c = r * 512u + threadIdx.x;
            u32x4 d[2];
            d[0] = __builtin_nontemporal_load(qq + c);
            d[1] = __builtin_nontemporal_load(qq + c + 256u);
            __builtin_amdgcn_sched_barrier(0);
            acc |= d[0][0] ^ d[0][1] ^ d[0][2] ^ d[0][3] ^ d[1][0] ^ d[1][1] ^ d[1][2] ^ d[1][3];
        }
        acc = __syncthreads_or(acc == 0x12345678u) ? 1u : acc;
        if (STAMP && threadIdx.x == 0 && k < 8) my[2 + k] = stamp();
    }
    if (acc == 0x12345678u) out[0] = acc;
    if (STAMP && threadIdx.x == 0) {
        my[0] = t_entry;
        my[10] = stamp();
        my[11] = (uint64_t)xcc_id() | ((uint64_t)k << 8);
    }
}

// the grid plain_read_skew<SKEW> needs for about `active` working workgroups
inline uint32_t skew_grid(uint32_t active, int skew)
{
    const uint32_t P = active / 8u, a = (uint32_t)(skew < 0 ? -skew : skew);
    return 8u * (P + (P * a + 63u) / 64u);
}

// The plain read with UO loads per lane per round on the odd XCDs (by HW_REG_XCC_ID) and 2 on the even ones ("xu"
// mode): do the late XCDs want more bytes in flight?
template <int UO>
__global__ void __launch_bounds__(256) plain_read_xu(const u32x4* __restrict__ p, uint32_t nslabs, uint32_t* out)
{
    uint32_t acc = 0;
    const bool odd = (xcc_id() & 1u) != 0u;
    for (uint32_t sl = blockIdx.x; sl < nslabs; sl += gridDim.x) {
        const u32x4* q = p + (uint64_t)sl * 4096u;
        if (odd) {
            for (uint32_t r = 0; r < 16u / UO; ++r) {
                u32x4 d[UO];
#pragma unroll
                for (int u = 0; u < UO; ++u) d[u] = __builtin_nontemporal_load(q + r * 256u * UO + u * 256u + threadIdx.x);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < UO; ++u) acc |= d[u][0] ^ d[u][1] ^ d[u][2] ^ d[u][3];
            }
        } else {
            for (uint32_t r = 0; r < 8; ++r) {
                const uint32_t c = r * 512u + threadIdx.x;
                u32x4 d[2];
                d[0] = __builtin_nontemporal_load(q + c);
                d[1] = __builtin_nontemporal_load(q + c + 256u);
                __builtin_amdgcn_sched_barrier(0);
                acc |= d[0][0] ^ d[0][1] ^ d[0][2] ^ d[0][3] ^ d[1][0] ^ d[1][1] ^ d[1][2] ^ d[1][3];
            }
        }
        acc = __syncthreads_or(acc == 0x12345678u) ? 1u : acc;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// ---- "tail" mode (VERDICT r04 "Next round" 6): the last round's buffers cut into PARTS sub-buffers, one per extra
// workgroup. The first main_grid workgroups run the product's grid-stride walk over the first full_rounds rounds; the
// PARTS x (n - full_rounds x main_grid) tail workgroups come after them in the grid, so the dispatcher hands them out
// as main workgroups retire and the faster CUs take more of the tail. The parts of a buffer merge their verdicts
// through a per-buffer global slot {~first (atomicMax), count (atomicAdd), arrivals}; the last to arrive writes the
// record and counts the buffer, and resets the slot (the slots start zeroed and stay so between launches).
struct TailSlot {
    uint32_t first, count, arrive, pad;
};

__device__ __forceinline__ void verify_one_product(const cts::Span& s, uint32_t lane, uint32_t& first, uint32_t& count)
{
    if (cts::span_giant(s)) {
        cts::scan_giant_exact<256, true>(s, lane, first, count);
    } else if (__builtin_amdgcn_readfirstlane(cts::span_whole_lines(s) ? 1u : 0u)) {
        cts::scan_whole_exact<256, 2, true, true>(s, lane, first, count);
        return;
    } else {
        const uint32_t acc = cts::scan_buffer<256, 2, true, true>(s, lane);
        if (__builtin_amdgcn_readfirstlane(__syncthreads_or(acc != 0u)) != 0 && acc != 0u)
            cts::scan_exact_owned<256, 2, true>(s, lane, first, count);
    }
}

template <int PARTS>
__global__ void __launch_bounds__(256, 4)
    verify_tail(const uint8_t* __restrict__ arena, uint64_t arena_bytes, const cts_buf_desc* __restrict__ descs, uint32_t n,
                cts_verify_result* __restrict__ results, uint64_t* __restrict__ counters,
                uint32_t* __restrict__ conn_first_fail, uint32_t n_conns, uint32_t main_grid, uint32_t full_rounds,
                TailSlot* __restrict__ slots)
{
    __shared__ uint64_t ctr[1][CTS_TL_COUNTERS];
    const uint32_t lane = threadIdx.x;
    cts::zero_counters<1>(ctr);
    if (blockIdx.x < main_grid) {
        const uint32_t end = full_rounds * main_grid < n ? full_rounds * main_grid : n;
        uint32_t i = blockIdx.x;
        cts_buf_desc dn;
        if (i < end) dn = descs[i];
        for (; i < end; i += main_grid) {
            const cts_buf_desc d = dn;
            if (i + main_grid < end) dn = descs[i + main_grid];
            if (cts::desc_bad(d, arena_bytes)) {
                if (lane == 0) cts::write_bad(results, i);
                continue;
            }
            const cts::Span s = cts::make_span(arena, d);
            uint32_t first = cts::kNone, count = 0;
            verify_one_product(s, lane, first, count);
            if (__builtin_amdgcn_readfirstlane(__syncthreads_or(first != cts::kNone)) != 0)
                cts::block_reduce_mismatch(first, count);
            if (lane == 0) cts::finish_buffer(s, d, i, first, count, results, ctr[0], conn_first_fail, n_conns);
        }
    } else {
        const uint32_t t = blockIdx.x - main_grid;
        const uint32_t i = full_rounds * main_grid + t / PARTS, part = t % PARTS;
        if (i < n) {
            const cts_buf_desc d = descs[i];
            if (cts::desc_bad(d, arena_bytes)) {
                if (lane == 0 && part == 0) cts::write_bad(results, i);
            } else {
                const cts::Span s = cts::make_span(arena, d);
                uint32_t first = cts::kNone, count = 0;
                const uint32_t per = s.nchunks / PARTS;
                if (__builtin_amdgcn_readfirstlane((cts::span_whole_lines(s) && !cts::span_giant(s) &&
                                                    s.nchunks % (PARTS * 512u) == 0u) ? 1u : 0u)) {
                    // this part's whole-line sub-span [part x per, (part + 1) x per) chunks
                    cts::Span q = s;
                    const uint32_t c0 = part * per;
                    q.p = s.p + c0;
                    q.sp = s.sp + 16u * c0;
                    q.nchunks = per;
                    q.len = 16u * per;
                    q.q0 = (s.q0 + 16u * c0) & 0xFFFFu;
                    q.expected = q.q0;
                    cts::scan_whole_exact<256, 2, true, true>(q, lane, first, count);
                    if (first != cts::kNone) first += 16u * c0;
                } else if (part == 0) {
                    verify_one_product(s, lane, first, count);  // any other span: part 0 takes it whole
                }
                if (__builtin_amdgcn_readfirstlane(__syncthreads_or(first != cts::kNone)) != 0)
                    cts::block_reduce_mismatch(first, count);
                if (lane == 0) {
                    TailSlot* sl = slots + i;
                    // device-scope atomics only, no fences: an agent-scope fence on gfx950 writes back / invalidates
                    // the XCD's L2 (~70-100 ns each, serialised: the first form of this tool ran 139-1095 us)
                    if (first != cts::kNone) {  // stored as ~first (0 = none: the slots start zeroed)
                        atomicMax(&sl->first, ~first);
                        atomicAdd(&sl->count, count);
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // both done before the arrival
                    }
                    if (atomicAdd(&sl->arrive, 1u) == (uint32_t)PARTS - 1u) {  // the last part finishes the buffer
                        const uint32_t f = atomicAdd(&sl->first, 0u), c = atomicAdd(&sl->count, 0u);
                        cts::finish_buffer(s, d, i, f == 0u ? cts::kNone : ~f, c, results, ctr[0], conn_first_fail,
                                           n_conns);
                        atomicExch(&sl->first, 0u);
                        atomicExch(&sl->count, 0u);
                        atomicExch(&sl->arrive, 0u);
                    }
                }
            }
        }
    }
    cts::flush_counters<1>(counters, ctr);
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

double pct(std::vector<double> v, double q)
{
    if (v.empty()) return -1;
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (double)(v.size() - 1))];
}

void print_timeline(const char* kind, const std::vector<uint64_t>& h, uint32_t grid, bool kp)
{
    uint64_t t0 = ~0ull;
    for (uint32_t b = 0; b < grid; ++b) t0 = std::min(t0, h[(size_t)b * kSt]);
    std::vector<double> entry, first_issue, first_buf, per_buf, last_buf, tail, end;
    for (uint32_t b = 0; b < grid; ++b) {
        const uint64_t* m = &h[(size_t)b * kSt];
        const uint32_t k = (uint32_t)(m[11] >> 8);
        if (k == 0) continue;
        const uint32_t kk = std::min<uint32_t>(k, 8);
        entry.push_back((m[0] - t0) * 0.01);
        first_issue.push_back((m[1] - m[0]) * 0.01);
        first_buf.push_back((m[2] - m[1]) * 0.01);
        for (uint32_t j = 1; j < kk; ++j) per_buf.push_back((m[2 + j] - m[1 + j]) * 0.01);
        last_buf.push_back((m[1 + kk] - t0) * 0.01);
        tail.push_back((m[10] - m[1 + kk]) * 0.01);
        end.push_back((m[10] - t0) * 0.01);
    }
    auto p3 = [&](const std::vector<double>& v) {
        static char buf[8][96];
        static int slot = 0;
        char* o = buf[slot++ & 7];
        std::snprintf(o, 96, "[%.2f,%.2f,%.2f,%.2f,%.2f]", pct(v, 0), pct(v, 0.1), pct(v, 0.5), pct(v, 0.9), pct(v, 1));
        return o;
    };
    std::printf("{\"kind\":\"timeline\",\"kernel\":\"%s\",\"kernarg_preload\":%d,\"workgroups\":%u,"
                "\"pcts\":\"p0,p10,p50,p90,p100 in us\",\"entry_us\":%s,\"entry_to_first_issue_us\":%s,"
                "\"first_buffer_us\":%s,\"later_buffer_us\":%s,\"last_buffer_end_us\":%s,\"flush_after_last_us\":%s,"
                "\"end_us\":%s,\"end_by_xcc\":[",
                kind, kp ? 1 : 0, grid, p3(entry), p3(first_issue), p3(first_buf), p3(per_buf), p3(last_buf), p3(tail),
                p3(end));
    for (uint32_t x = 0, first = 1; x < 8; ++x) {
        std::vector<double> ex;
        for (uint32_t b = 0; b < grid; ++b) {
            const uint64_t* m = &h[(size_t)b * kSt];
            if ((m[11] >> 8) != 0 && (m[11] & 0xFu) == x) ex.push_back((m[10] - t0) * 0.01);
        }
        if (ex.empty()) continue;
        std::printf("%s[%u,%.2f,%.2f,%.2f]", first ? "" : ",", x, pct(ex, 0), pct(ex, 0.5), pct(ex, 1));
        first = 0;
    }
    // per XCC: medians of entry, entry to first issue, first buffer, later buffers
    std::printf("],\"phases_by_xcc\":[");
    for (uint32_t x = 0, first = 1; x < 8; ++x) {
        std::vector<double> en, fi, fb, lb;
        for (uint32_t b = 0; b < grid; ++b) {
            const uint64_t* m = &h[(size_t)b * kSt];
            const uint32_t k = (uint32_t)(m[11] >> 8);
            if (k == 0 || (m[11] & 0xFu) != x) continue;
            const uint32_t kk = std::min<uint32_t>(k, 8);
            en.push_back((m[0] - t0) * 0.01);
            fi.push_back((m[1] - m[0]) * 0.01);
            fb.push_back((m[2] - m[1]) * 0.01);
            for (uint32_t j = 1; j < kk; ++j) lb.push_back((m[2 + j] - m[1 + j]) * 0.01);
        }
        if (en.empty()) continue;
        std::printf("%s[%u,%.2f,%.2f,%.2f,%.2f]", first ? "" : ",", x, pct(en, 0.5), pct(fi, 0.5), pct(fb, 0.5),
                    pct(lb, 0.5));
        first = 0;
    }
    std::printf("]}\n");
    std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv)
{
#ifdef CTS_TOOL_KERNARG_PRELOAD
    const bool kp = true;
#else
    const bool kp = false;
#endif
    const int passes = argc > 1 ? atoi(argv[1]) : 3;
    const bool map_mode = argc > 3 && std::string(argv[3]) == "map";
    const bool skew_mode = argc > 3 && std::string(argv[3]) == "skew";
    const bool xu_mode = argc > 3 && std::string(argv[3]) == "xu";
    const bool tail_mode = argc > 3 && std::string(argv[3]) == "tail";
    const int reps = argc > 2 ? atoi(argv[2]) : 64;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t n = 4096, grid = (uint32_t)cus * 4u;  // the engine's grid for 4096 x 64 KiB: 4 buffers per workgroup
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
        // one corrupt byte per 1024 buffers (in the second round), and two in a first round (the SPEC round)
        for (uint32_t b : {0u, 1024u, 2048u, 3072u, 5u, 1029u}) {
            const uint64_t off = ((uint64_t)b << 16) + (b % 1024u ? 77u : 12345u);
            uint8_t v = 0;
            CHECK(hipMemcpy(&v, a + off, 1, hipMemcpyDeviceToHost));
            v ^= 0x5A;
            CHECK(hipMemcpy(a + off, &v, 1, hipMemcpyHostToDevice));
        }
    }
    cts_verify_result* res = nullptr;
    uint64_t* ctr = nullptr;
    uint32_t *cff = nullptr, *out = nullptr;
    uint64_t* st = nullptr;
    CHECK(hipMalloc((void**)&res, n * sizeof(cts_verify_result)));
    CHECK(hipMalloc((void**)&ctr, CTS_COUNTER_SHARDS * 64));
    CHECK(hipMalloc((void**)&cff, n * 4));
    CHECK(hipMalloc((void**)&out, 64));
    CHECK(hipMalloc((void**)&st, (size_t)grid * kSt * 8));
    CHECK(hipMemset(ctr, 0, CTS_COUNTER_SHARDS * 64));
    CHECK(hipMemset(cff, 0xFF, n * 4));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    CHECK(hipDeviceSynchronize());

    if (xu_mode) {
        // more bytes in flight on the late XCDs (U 4 / 8 on the odd ones), or more workgroups there (skew -4 / -8)
        for (int pass = 0; pass < passes; ++pass) {
            auto a = [&](int i) { return reinterpret_cast<const u32x4*>(arena[i % R]); };
            const double t2 = time_us([&](int i) { plain_read_xu<2><<<grid, 256, 0, s>>>(a(i), n, out); }, reps, s);
            const double t4 = time_us([&](int i) { plain_read_xu<4><<<grid, 256, 0, s>>>(a(i), n, out); }, reps, s);
            const double t8 = time_us([&](int i) { plain_read_xu<8><<<grid, 256, 0, s>>>(a(i), n, out); }, reps, s);
            const double m4 = time_us([&](int i) {
                plain_read_skew<false, -4><<<skew_grid(grid, -4), 256, 0, s>>>(a(i), n, st, out);
            }, reps, s);
            const double m8 = time_us([&](int i) {
                plain_read_skew<false, -8><<<skew_grid(grid, -8), 256, 0, s>>>(a(i), n, st, out);
            }, reps, s);
            const double p0 = time_us([&](int i) { plain_read<false><<<grid, 256, 0, s>>>(a(i), n, st, out); }, reps, s);
            std::printf("{\"kind\":\"xu_time\",\"pass\":%d,\"launches\":%d,\"plain_us\":%.2f,\"odd_u2_us\":%.2f,"
                        "\"odd_u4_us\":%.2f,\"odd_u8_us\":%.2f,\"more_wg_on_odd_skew4_us\":%.2f,"
                        "\"more_wg_on_odd_skew8_us\":%.2f}\n", pass, reps, p0, t2, t4, t8, m4, m8);
            std::fflush(stdout);
        }
        return 0;
    }
    if (skew_mode) {
        // does reading fewer slabs on the late (odd) XCDs shorten the launch? active workgroups stay ~1024
        std::vector<uint64_t> h((size_t)grid * 2 * kSt);
        uint64_t* st2 = nullptr;
        CHECK(hipMalloc((void**)&st2, h.size() * 8));
        for (int pass = 0; pass < passes; ++pass) {
            double t[5];
            const int sk[5] = {0, 2, 4, 6, 8};
            for (int v = 0; v < 5; ++v) {
                const uint32_t g = skew_grid(grid, sk[v]);
                t[v] = time_us([&](int i) {
                    const u32x4* a = reinterpret_cast<const u32x4*>(arena[i % R]);
                    switch (sk[v]) {
                    case 0: plain_read_skew<false, 0><<<g, 256, 0, s>>>(a, n, st2, out); break;
                    case 2: plain_read_skew<false, 2><<<g, 256, 0, s>>>(a, n, st2, out); break;
                    case 4: plain_read_skew<false, 4><<<g, 256, 0, s>>>(a, n, st2, out); break;
                    case 6: plain_read_skew<false, 6><<<g, 256, 0, s>>>(a, n, st2, out); break;
                    default: plain_read_skew<false, 8><<<g, 256, 0, s>>>(a, n, st2, out); break;
                    }
                }, reps, s);
            }
            const double t_plain = time_us([&](int i) {
                plain_read<false><<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(arena[i % R]), n, st, out);
            }, reps, s);
            std::printf("{\"kind\":\"skew_time\",\"pass\":%d,\"launches\":%d,\"plain_us\":%.2f,\"skew0_us\":%.2f,"
                        "\"skew2_us\":%.2f,\"skew4_us\":%.2f,\"skew6_us\":%.2f,\"skew8_us\":%.2f}\n",
                        pass, reps, t_plain, t[0], t[1], t[2], t[3], t[4]);
            std::fflush(stdout);
            for (int v : {0, 4}) {
                const uint32_t g = skew_grid(grid, v);
                for (int rep = 0; rep < 3; ++rep) {
                    CHECK(hipMemsetAsync(st2, 0, h.size() * 8, s));
                    const u32x4* a = reinterpret_cast<const u32x4*>(arena[rep % R]);
                    if (v == 0) plain_read_skew<true, 0><<<g, 256, 0, s>>>(a, n, st2, out);
                    else plain_read_skew<true, 4><<<g, 256, 0, s>>>(a, n, st2, out);
                    CHECK(hipStreamSynchronize(s));
                }
                CHECK(hipMemcpy(h.data(), st2, h.size() * 8, hipMemcpyDeviceToHost));
                print_timeline(v == 0 ? "plain_skew0" : "plain_skew4", h, grid, kp);  // ranks 0..1023 (A = 1024 at 0 and 4)
            }
        }
        return 0;
    }
    if (tail_mode) {
        // the last round(s) split into sub-buffers handed out by the dispatcher, against the product
        TailSlot* slots = nullptr;
        CHECK(hipMalloc((void**)&slots, n * sizeof(TailSlot)));
        CHECK(hipMemset(slots, 0, n * sizeof(TailSlot)));
        auto read_ctr = [&] {
            std::vector<uint64_t> h(CTS_COUNTER_SHARDS * 8);
            CHECK(hipMemcpy(h.data(), ctr, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<uint64_t> v(5, 0);
            for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh)
                for (int k = 0; k < 5; ++k) v[k] += h[sh * 8 + k];
            return v;
        };
        auto run = [&](int form, int i, uint32_t fr) {
            const uint32_t tail = n - fr * grid;
            switch (form) {
            case 0: PRODUCT<<<grid, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n); break;
            case 1: verify_tail<1><<<grid + tail, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n, grid, fr, slots); break;
            case 2: verify_tail<2><<<grid + 2 * tail, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n, grid, fr, slots); break;
            case 4: verify_tail<4><<<grid + 4 * tail, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n, grid, fr, slots); break;
            default: verify_tail<8><<<grid + 8 * tail, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n, grid, fr, slots); break;
            }
        };
        // parity on arena 0: records, first-failure slots and counters against the product's
        std::vector<cts_verify_result> a(n), b(n);
        std::vector<uint32_t> ca(n), cb(n);
        CHECK(hipMemset(ctr, 0, CTS_COUNTER_SHARDS * 64));
        CHECK(hipMemset(cff, 0xFF, n * 4));
        run(0, 0, 3);
        CHECK(hipMemcpy(a.data(), res, n * sizeof(cts_verify_result), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(ca.data(), cff, n * 4, hipMemcpyDeviceToHost));
        const std::vector<uint64_t> c0 = read_ctr();
        int ok = 1;
        for (int form : {1, 2, 4, 8})
            for (uint32_t fr : {3u, 2u}) {
                CHECK(hipMemset(res, 0, n * sizeof(cts_verify_result)));
                CHECK(hipMemset(ctr, 0, CTS_COUNTER_SHARDS * 64));
                CHECK(hipMemset(cff, 0xFF, n * 4));
                run(form, 0, fr);
                CHECK(hipMemcpy(b.data(), res, n * sizeof(cts_verify_result), hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(cb.data(), cff, n * 4, hipMemcpyDeviceToHost));
                const bool same = std::memcmp(a.data(), b.data(), n * sizeof(cts_verify_result)) == 0 && ca == cb &&
                                  read_ctr() == c0;
                std::printf("{\"kind\":\"tail_parity\",\"parts\":%d,\"full_rounds\":%u,\"equals_product\":%d}\n", form,
                            fr, same ? 1 : 0);
                ok &= same ? 1 : 0;
            }
        std::fflush(stdout);
        if (!ok) return 3;
        for (int pass = 0; pass < passes; ++pass) {
            double t[9];
            int k = 0;
            t[k++] = time_us([&](int i) { run(0, i, 3); }, reps, s);
            for (int form : {1, 2, 4, 8})
                for (uint32_t fr : {3u, 2u}) t[k++] = time_us([&](int i) { run(form, i, fr); }, reps, s);
            const double tp = time_us([&](int i) {
                plain_read<false><<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(arena[i % R]), n, st, out);
            }, reps, s);
            std::printf("{\"kind\":\"tail_time\",\"pass\":%d,\"launches\":%d,\"product_us\":%.2f,\"p1_r3_us\":%.2f,"
                        "\"p1_r2_us\":%.2f,\"p2_r3_us\":%.2f,\"p2_r2_us\":%.2f,\"p4_r3_us\":%.2f,\"p4_r2_us\":%.2f,"
                        "\"p8_r3_us\":%.2f,\"p8_r2_us\":%.2f,\"plain_read_us\":%.2f}\n", pass, reps, t[0], t[1], t[2], t[3],
                        t[4], t[5], t[6], t[7], t[8], tp);
            std::fflush(stdout);
        }
        return 0;
    }
    if (map_mode) {
        // does a late XCC follow the XCC or the addresses it reads? the plain read under three slab maps, and the
        // product verify with its descriptors permuted the way map 2 permutes the slabs (workgroup b's k-th buffer at
        // slot ((b + k) mod G) + k G)
        std::vector<cts_buf_desc> pd(n);
        for (uint32_t j = 0; j < n; ++j) {
            const uint32_t b = j % grid, k = j / grid;
            pd[j] = hd[k * grid + (b + k) % grid];
        }
        cts_buf_desc* dp = nullptr;
        CHECK(hipMalloc((void**)&dp, n * sizeof(cts_buf_desc)));
        CHECK(hipMemcpy(dp, pd.data(), n * sizeof(cts_buf_desc), hipMemcpyHostToDevice));
        std::vector<uint64_t> h((size_t)grid * kSt);
        for (int pass = 0; pass < passes; ++pass) {
            const double t0 = time_us([&](int i) {
                plain_read<false, 0><<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(arena[i % R]), n, st, out);
            }, reps, s);
            const double t1 = time_us([&](int i) {
                plain_read<false, 1><<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(arena[i % R]), n, st, out);
            }, reps, s);
            const double t2 = time_us([&](int i) {
                plain_read<false, 2><<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(arena[i % R]), n, st, out);
            }, reps, s);
            const double v0 = time_us([&](int i) {
                PRODUCT<<<grid, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n);
            }, reps, s);
            const double v2 = time_us([&](int i) {
                PRODUCT<<<grid, 256, 0, s>>>(arena[i % R], bytes, dp, n, res, ctr, cff, n);
            }, reps, s);
            std::printf("{\"kind\":\"map_time\",\"pass\":%d,\"launches\":%d,\"plain_map0_us\":%.2f,\"plain_map1_us\":%.2f,"
                        "\"plain_map2_us\":%.2f,\"verify_descs_in_order_us\":%.2f,\"verify_descs_map2_us\":%.2f}\n",
                        pass, reps, t0, t1, t2, v0, v2);
            std::fflush(stdout);
            for (int m = 0; m < 3; ++m) {
                for (int rep = 0; rep < 3; ++rep) {
                    CHECK(hipMemsetAsync(st, 0, (size_t)grid * kSt * 8, s));
                    const u32x4* a = reinterpret_cast<const u32x4*>(arena[rep % R]);
                    if (m == 0) plain_read<true, 0><<<grid, 256, 0, s>>>(a, n, st, out);
                    if (m == 1) plain_read<true, 1><<<grid, 256, 0, s>>>(a, n, st, out);
                    if (m == 2) plain_read<true, 2><<<grid, 256, 0, s>>>(a, n, st, out);
                    CHECK(hipStreamSynchronize(s));
                }
                CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
                print_timeline(m == 0 ? "plain_map0" : m == 1 ? "plain_map1" : "plain_map2", h, grid, kp);
            }
        }
        return 0;
    }
    // parity of the replica and the pipelined form against the product on arena 0
    {
        std::vector<cts_verify_result> a(n), b(n);
        PRODUCT<<<grid, 256, 0, s>>>(arena[0], bytes, d, n, res, ctr, cff, n);
        CHECK(hipMemcpy(a.data(), res, n * sizeof(cts_verify_result), hipMemcpyDeviceToHost));
        CHECK(hipMemset(res, 0, n * sizeof(cts_verify_result)));
        verify_replica<true><<<grid, 256, 0, s>>>(arena[0], bytes, d, n, res, ctr, cff, n, st);
        CHECK(hipMemcpy(b.data(), res, n * sizeof(cts_verify_result), hipMemcpyDeviceToHost));
        uint32_t failed = 0;
        for (uint32_t i = 0; i < n; ++i) failed += a[i].pass ? 0u : 1u;
        auto eq = [](const std::vector<cts_verify_result>& x, const std::vector<cts_verify_result>& y) {
            return std::equal(x.begin(), x.end(), y.begin(), [](const cts_verify_result& p, const cts_verify_result& q) {
                return p.first_mismatch == q.first_mismatch && p.mismatch_bytes == q.mismatch_bytes && p.pass == q.pass &&
                       p.expected == q.expected && p.actual == q.actual;
            });
        };
        const bool same = eq(a, b);
        CHECK(hipMemset(res, 0, n * sizeof(cts_verify_result)));
        verify_pipe<false><<<grid, 256, 0, s>>>(arena[0], bytes, d, n, res, ctr, cff, n);
        CHECK(hipMemcpy(b.data(), res, n * sizeof(cts_verify_result), hipMemcpyDeviceToHost));
        std::printf("{\"kind\":\"parity\",\"kernarg_preload\":%d,\"replica_equals_product\":%d,"
                    "\"pipe2_equals_product\":%d,\"failed_buffers\":%u}\n",
                    kp ? 1 : 0, same ? 1 : 0, eq(a, b) ? 1 : 0, failed);
    }

    for (int pass = 0; pass < passes; ++pass) {
        const double t_prod = time_us([&](int i) {
            PRODUCT<<<grid, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n);
        }, reps, s);
        const double t_rep = time_us([&](int i) {
            verify_replica<false><<<grid, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n, st);
        }, reps, s);
        const double t_plain = time_us([&](int i) {
            plain_read<false><<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(arena[i % R]), n, st, out);
        }, reps, s);
        const double t_pipe = time_us([&](int i) {
            verify_pipe<false><<<grid, 256, 0, s>>>(arena[i % R], bytes, d, n, res, ctr, cff, n);
        }, reps, s);
        std::printf("{\"kind\":\"time\",\"kernarg_preload\":%d,\"pass\":%d,\"launches\":%d,\"product_verify_us\":%.2f,"
                    "\"replica_verify_us\":%.2f,\"pipe2_us\":%.2f,\"plain_read_us\":%.2f,\"product_GBps\":%.1f,"
                    "\"plain_GBps\":%.1f,\"product_over_plain\":%.4f}\n",
                    kp ? 1 : 0, pass, reps, t_prod, t_rep, t_pipe, t_plain, bytes / t_prod / 1e3, bytes / t_plain / 1e3,
                    t_prod / t_plain);
        std::fflush(stdout);
    }
    // timelines: the last of 3 launches of each (rotating arenas), alternating
    std::vector<uint64_t> h((size_t)grid * kSt);
    for (int pass = 0; pass < passes; ++pass) {
        for (int which = 0; which < 2; ++which) {
            for (int rep = 0; rep < 3; ++rep) {
                CHECK(hipMemsetAsync(st, 0, (size_t)grid * kSt * 8, s));
                if (which == 0)
                    verify_replica<true><<<grid, 256, 0, s>>>(arena[rep % R], bytes, d, n, res, ctr, cff, n, st);
                else
                    plain_read<true><<<grid, 256, 0, s>>>(reinterpret_cast<const u32x4*>(arena[rep % R]), n, st, out);
                CHECK(hipStreamSynchronize(s));
            }
            CHECK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
            print_timeline(which == 0 ? "verify_replica" : "plain_read", h, grid, kp);
        }
    }
    return 0;
}
