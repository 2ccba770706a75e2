// cts_kernels.hip — CDNA4 (gfx950) fill and verify kernels for ctsTraffic's
// data-integrity path.
//
// Reference semantics (microsoft/ctsTraffic):
//   pattern  ctsTraffic/ctsIOPattern.cpp:35-36,55-80 — byte at stream position j
//            (mod 65536) is P(j) = (j & 1) ? j >> 9 : (j >> 1) & 0xFF, i.e. the
//            little-endian u16 ramp 0..32767 repeated every 64 KiB.
//   verify   ctsTraffic/ctsIOPattern.cpp:745-775 — RtlCompareMemory(S + expected,
//            buf + bufferOffset, n): matching-prefix length; pass iff == n.
//
// Design: a pure HBM-read stream, no MFMA. A buffer's
// verified span is cut into 16-byte chunks aligned in memory (1 KiB per
// wave-instruction). Chunk 0 and the last chunk may be partial ("edges") and are
// checked with byte masks by two lanes; the interior chunks are streamed by a
// branch-free fast pass that only ORs (received ^ expected). The expected chunk
// is regenerated in registers from the stream position (no pattern table is
// read): one v_mad_u32_u24 + add/and per u16 pair, one v_alignbyte per dword for
// the byte phase. Only when a team's OR is nonzero (rare) does an exact re-scan
// compute the first differing byte and the differing-byte count.
//
// Paths:
//   verify_wg_kernel    one 256-lane workgroup per buffer (64 KiB TCP buffers)
//   verify_wg_lds_kernel the same, chunks land in LDS by LDS-DMA (global_load_lds)
//   verify_wave_kernel  one wave per buffer, G buffers in flight per wave
//                       (1472-byte MediaStream datagrams)
#include <hip/hip_runtime.h>

#include "cts_internal.hpp"

namespace cts {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t pattern_byte_dev(uint32_t pos)
{
    pos &= 0xFFFFu;
    return (pos & 1u) ? (pos >> 9) : ((pos >> 1) & 0xFFu);
}

// Expected 16 bytes for a chunk whose first byte sits at pattern position q
// (0 <= q < 65536); sh = q & 1. The chunk is bytes sh..sh+15 of the u16 values
// k..k+8 (k = q >> 1, mod 32768). Packed: dword j = (k+2j) | (k+2j+1) << 16 =
// base + j*0x20002 with base = k*0x10001 + 0x10000; & 0x7FFF7FFF wraps
// 32768 -> 0 in each half (the low half never exceeds 32775: no carry crosses).
// v_alignbyte with a register shift handles both phases without a branch.
__device__ __forceinline__ u32x4 expected_chunk(uint32_t q, uint32_t sh)
{
    const uint32_t k = q >> 1;
    const uint32_t base = __umul24(k, 0x10001u) + 0x10000u;
    const uint32_t w0 = base & 0x7FFF7FFFu;
    const uint32_t w1 = (base + 0x20002u) & 0x7FFF7FFFu;
    const uint32_t w2 = (base + 0x40004u) & 0x7FFF7FFFu;
    const uint32_t w3 = (base + 0x60006u) & 0x7FFF7FFFu;
    const uint32_t w4 = (base + 0x80008u) & 0x7FFF7FFFu;
    return u32x4{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                 __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
}

// 0x80 in every byte of x that is nonzero.
__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t x)
{
    return (((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

__device__ __forceinline__ uint32_t low_bytes_mask(int nb)  // nb in [0,4]
{
    return (uint32_t)((1ull << (8 * nb)) - 1ull);
}

// Mask keeping bytes [lo, hi) of a 16-byte chunk (0 <= lo <= hi <= 16).
__device__ __forceinline__ u32x4 range_mask(uint32_t lo, uint32_t hi)
{
    u32x4 m;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        int a = (int)lo - 4 * w;
        int b = (int)hi - 4 * w;
        a = a < 0 ? 0 : (a > 4 ? 4 : a);
        b = b < 0 ? 0 : (b > 4 ? 4 : b);
        m[w] = (b > a) ? (low_bytes_mask(b) & ~low_bytes_mask(a)) : 0u;
    }
    return m;
}

template <bool NT>
__device__ __forceinline__ u32x4 load_chunk(const u32x4* p)
{
    if constexpr (NT) {
        return __builtin_nontemporal_load(p);
    } else {
        return *p;
    }
}

__device__ __forceinline__ uint32_t or4(u32x4 x) { return x[0] | x[1] | x[2] | x[3]; }

// A buffer's verified span [sp, sp + len) as 16-byte chunks of p = sp - lo.
struct Span {
    const u32x4* p;
    const uint8_t* sp;
    uint32_t len;
    uint32_t nchunks;  // chunks covering [lo, lo + len)
    uint32_t q0;       // pattern position of the byte at p (mod 65536)
    uint32_t sh;       // q0 & 1 (byte phase), uniform over the span
    uint32_t lo;       // bytes of chunk 0 before the span
    uint32_t hi_last;  // bytes of the last chunk inside the span (1..16)
    uint32_t expected; // ctsTask::m_expectedPatternOffset
};

__device__ __forceinline__ bool desc_bad(const cts_buf_desc& d, uint64_t arena_bytes)
{
    // FAIL_FAST conditions of the reference (offset >= c_bufferPatternSize,
    // ctsIOPattern.cpp:723-725) and buffers outside the arena are flagged, not read.
    return d.expected_pattern_offset >= 65536u || d.length < d.skip_head || d.byte_offset > arena_bytes ||
           arena_bytes - d.byte_offset < (uint64_t)d.length;
}

__device__ __forceinline__ Span make_span(const uint8_t* __restrict__ arena, const cts_buf_desc& d)
{
    Span s;
    s.len = d.length - d.skip_head;
    // pointer arithmetic from the kernel argument keeps the global address
    // space (global_load_dwordx4, not flat_load: flat loads also count in
    // lgkmcnt and force full drains)
    s.sp = arena + d.byte_offset + d.skip_head;
    s.lo = (uint32_t)((uintptr_t)s.sp & 15u);
    s.nchunks = s.len == 0 ? 0u : (uint32_t)(((uint64_t)s.lo + s.len + 15u) >> 4);
    s.hi_last = s.len == 0 ? 0u : (uint32_t)((uint64_t)s.lo + s.len - 16ull * (s.nchunks - 1u));
    s.q0 = (d.expected_pattern_offset - s.lo) & 0xFFFFu;
    s.sh = s.q0 & 1u;
    s.p = reinterpret_cast<const u32x4*>(s.sp - s.lo);
    s.expected = d.expected_pattern_offset;
    return s;
}

__device__ __forceinline__ u32x4 chunk_xor(const Span& s, uint32_t c, u32x4 data)
{
    return data ^ expected_chunk((s.q0 + 16u * c) & 0xFFFFu, s.sh);
}

// XOR of one (possibly partial) chunk with its expected bytes, bytes outside
// the span masked to zero.
__device__ __forceinline__ u32x4 chunk_diff_masked(const Span& s, uint32_t c)
{
    u32x4 x = chunk_xor(s, c, s.p[c]);
    if (c == 0u || c == s.nchunks - 1u) x &= range_mask(c == 0u ? s.lo : 0u, c == s.nchunks - 1u ? s.hi_last : 16u);
    return x;
}

// Edge chunks (first and last, possibly partial) by lanes 0 and 1.
__device__ __forceinline__ uint32_t scan_edges(const Span& s, uint32_t lane)
{
    uint32_t acc = 0;
    if (lane < 2u && s.nchunks > 0u && (lane == 0u || s.nchunks > 1u)) {
        acc = or4(chunk_diff_masked(s, lane == 0u ? 0u : s.nchunks - 1u));
    }
    return acc;
}

// Fast pass over interior chunks [c_begin, c_end) (all 16 bytes valid): OR of
// (received ^ expected) over this lane's chunks. Straight-line rounds of U
// loads per lane, all issued before the first compare (sched_barrier stops the
// scheduler from interleaving them with the compares); no load under a branch
// (a load under an exec branch makes hipcc drain vmcnt(0) at every join). The
// tail round clamps its chunk index and discards the excess.
template <int TEAM, int U, bool NT>
__device__ __forceinline__ uint32_t scan_interior(const Span& s, uint32_t c_begin, uint32_t c_end, uint32_t lane)
{
    uint32_t acc = 0;
    if (c_end <= c_begin) return 0;
    uint32_t cb = c_begin;
    for (; cb + (uint32_t)(TEAM * U) <= c_end; cb += (uint32_t)(TEAM * U)) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = load_chunk<NT>(s.p + cb + (uint32_t)(u * TEAM) + lane);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc |= or4(chunk_xor(s, cb + (uint32_t)(u * TEAM) + lane, d[u]));
    }
    if (cb < c_end) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = cb + (uint32_t)(u * TEAM) + lane;
            d[u] = load_chunk<NT>(s.p + (c < c_end ? c : c_end - 1u));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = cb + (uint32_t)(u * TEAM) + lane;
            const uint32_t any = or4(chunk_xor(s, c < c_end ? c : c_end - 1u, d[u]));
            acc |= (c < c_end) ? any : 0u;
        }
    }
    return acc;
}

// Exact scan of a whole span (rare path: a span the fast pass flagged): first
// differing byte position (relative to the span start) and # differing bytes
// over this lane's chunks.
template <int TEAM>
__device__ __forceinline__ void scan_exact(const Span& s, uint32_t lane, uint32_t& first, uint32_t& count)
{
    for (uint32_t c = lane; c < s.nchunks; c += TEAM) {
        const u32x4 x = chunk_diff_masked(s, c);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t nz = nonzero_bytes(x[w]);
            if (nz) {
                const uint32_t idx = 4u * (uint32_t)w + ((uint32_t)__builtin_ctz(nz) >> 3);
                const uint32_t pos = 16u * c + idx - s.lo;
                first = pos < first ? pos : first;
                count += (uint32_t)__builtin_popcount(nz);
            }
        }
    }
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
    return v;
}

struct TeamCounters {
    uint64_t v[5];
};

__device__ __forceinline__ void write_bad(cts_verify_result* results, uint32_t i)
{
    if (results != nullptr) {
        cts_verify_result r;
        r.first_mismatch = 0;
        r.mismatch_bytes = 0;
        r.expected = 0;
        r.actual = 0;
        r.pass = 0;
        r.flags = CTS_RESULT_FLAG_BAD_DESC;
        results[i] = r;
    }
}

// Record one verified buffer (called by the team leader).
__device__ __forceinline__ void finish_buffer(const Span& s, const cts_buf_desc& d, uint32_t i, uint32_t first,
                                              uint32_t count, cts_verify_result* results, TeamCounters& tc,
                                              uint32_t* conn_first_fail, uint32_t n_conns)
{
    const bool pass = (first == kNone);
    if (results != nullptr) {
        cts_verify_result r;
        r.first_mismatch = pass ? s.len : first;
        r.mismatch_bytes = pass ? 0u : count;
        r.expected = pass ? 0 : (uint8_t)pattern_byte_dev(s.expected + first);
        r.actual = pass ? 0 : s.sp[first];
        r.pass = pass ? 1 : 0;
        r.flags = 0;
        results[i] = r;
    }
    tc.v[kBytesChecked] += s.len;
    tc.v[kBuffersChecked] += 1;
    if (pass) {
        tc.v[kBytesOk] += s.len;
    } else {
        tc.v[kBuffersFailed] += 1;
        tc.v[kMismatchedBytes] += count;
        if (conn_first_fail != nullptr && d.conn_index < n_conns) atomicMin(&conn_first_fail[d.conn_index], i);
    }
}

// Fold the per-team counters of a workgroup and add them to the counter shard
// of this workgroup (one 64-byte line per shard, CTS_COUNTER_SHARDS shards).
template <int TEAMS>
__device__ __forceinline__ void flush_counters(uint64_t* counters, const TeamCounters& tc, uint32_t team, bool leader)
{
    __shared__ uint64_t red_ctr[TEAMS][5];
    if (counters == nullptr) return;
    if (leader) {
#pragma unroll
        for (int k = 0; k < 5; ++k) red_ctr[team][k] = tc.v[k];
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        uint64_t sum = 0;
#pragma unroll
        for (int t = 0; t < TEAMS; ++t) sum += red_ctr[t][threadIdx.x];
        if (sum)
            atomicAdd((unsigned long long*)&counters[(blockIdx.x % CTS_COUNTER_SHARDS) * kCounterSlots + threadIdx.x],
                      (unsigned long long)sum);
    }
}

// Workgroup-wide reduction of (first, count) when some lane saw a mismatch.
__device__ __forceinline__ void block_reduce_mismatch(uint32_t& first, uint32_t& count)
{
    __shared__ uint32_t red_first[kBlock / 64];
    __shared__ uint32_t red_count[kBlock / 64];
    const uint32_t wave = threadIdx.x / 64;
    first = wave_min(first);
    count = wave_sum(count);
    if ((threadIdx.x & 63) == 0) {
        red_first[wave] = first;
        red_count[wave] = count;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) {
            first = red_first[w] < first ? red_first[w] : first;
            count += red_count[w];
        }
    }
    __syncthreads();  // red_* reused by the next buffer
}

// ---------------------------------------------------------------------------------------------
// One 256-lane workgroup per buffer (grid-strides over buffers).
template <int U, bool NT>
__global__ void __launch_bounds__(kBlock) verify_wg_kernel(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                           const cts_buf_desc* __restrict__ descs, uint32_t n,
                                                           cts_verify_result* __restrict__ results,
                                                           uint64_t* __restrict__ counters,
                                                           uint32_t* __restrict__ conn_first_fail, uint32_t n_conns)
{
    const uint32_t lane = threadIdx.x;
    TeamCounters tc = {{0, 0, 0, 0, 0}};
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const cts_buf_desc d = descs[i];
        if (desc_bad(d, arena_bytes)) {
            if (lane == 0) write_bad(results, i);
            continue;
        }
        const Span s = make_span(arena, d);
        uint32_t acc = s.nchunks >= 3u ? scan_interior<kBlock, U, NT>(s, 1u, s.nchunks - 1u, lane) : 0u;
        acc |= scan_edges(s, lane);
        uint32_t first = kNone, count = 0;
        if (__syncthreads_or(acc != 0u)) {  // rare: exact re-scan + reduction
            scan_exact<kBlock>(s, lane, first, count);
            block_reduce_mismatch(first, count);
        }
        if (lane == 0) finish_buffer(s, d, i, first, count, results, tc, conn_first_fail, n_conns);
    }
    flush_counters<1>(counters, tc, 0, threadIdx.x == 0);
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA variant: each wave streams its chunks with global_load_lds_dwordx4
// (1 KiB per wave-instruction lands in the wave's private LDS slot, lane i at
// +16 i) and reads them back with ds_read_b128 behind a counted vmcnt. The
// in-flight bytes live in LDS, not VGPRs. No cross-wave LDS sharing: no barrier.
template <int N>
__device__ __forceinline__ void wait_vmcnt()
{
    static_assert(N >= 0 && N < 64, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int U, bool NT>
__device__ __forceinline__ uint32_t scan_interior_lds(const Span& s, uint32_t c_begin, uint32_t c_end, uint32_t lane,
                                                      u32x4 (*slot)[64])
{
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(1))) const void gbl_void;
    uint32_t acc = 0;
    if (c_end <= c_begin) return 0;
    for (uint32_t cb = c_begin; cb < c_end; cb += (uint32_t)(kBlock * U)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = cb + (uint32_t)(u * kBlock) + lane;
            const u32x4* src = s.p + (c < c_end ? c : c_end - 1u);
            __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)&slot[u][0], 16, 0, NT ? 2 : 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            // wait until the u-th piece has landed (the U-1-u younger ones may still fly)
            if constexpr (U == 8) {
                switch (u) {
                case 0: wait_vmcnt<7>(); break;
                case 1: wait_vmcnt<6>(); break;
                case 2: wait_vmcnt<5>(); break;
                case 3: wait_vmcnt<4>(); break;
                case 4: wait_vmcnt<3>(); break;
                case 5: wait_vmcnt<2>(); break;
                case 6: wait_vmcnt<1>(); break;
                default: wait_vmcnt<0>(); break;
                }
            } else {
                wait_vmcnt<0>();
            }
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t c = cb + (uint32_t)(u * kBlock) + lane;
            const u32x4 data = slot[u][lane];
            const uint32_t any = or4(chunk_xor(s, c < c_end ? c : c_end - 1u, data));
            acc |= (c < c_end) ? any : 0u;
        }
        // every lane has read its slot entries before the next round overwrites them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

template <int U, bool NT>
__global__ void __launch_bounds__(kBlock) verify_wg_lds_kernel(const uint8_t* __restrict__ arena,
                                                               uint64_t arena_bytes,
                                                               const cts_buf_desc* __restrict__ descs, uint32_t n,
                                                               cts_verify_result* __restrict__ results,
                                                               uint64_t* __restrict__ counters,
                                                               uint32_t* __restrict__ conn_first_fail, uint32_t n_conns)
{
    __shared__ __attribute__((aligned(16))) u32x4 ring[kBlock / 64][U][64];
    const uint32_t lane = threadIdx.x;
    const uint32_t wave = threadIdx.x / 64;
    TeamCounters tc = {{0, 0, 0, 0, 0}};
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const cts_buf_desc d = descs[i];
        if (desc_bad(d, arena_bytes)) {
            if (lane == 0) write_bad(results, i);
            continue;
        }
        const Span s = make_span(arena, d);
        uint32_t acc = s.nchunks >= 3u ? scan_interior_lds<U, NT>(s, 1u, s.nchunks - 1u, lane, ring[wave]) : 0u;
        acc |= scan_edges(s, lane);
        uint32_t first = kNone, count = 0;
        if (__syncthreads_or(acc != 0u)) {
            scan_exact<kBlock>(s, lane, first, count);
            block_reduce_mismatch(first, count);
        }
        if (lane == 0) finish_buffer(s, d, i, first, count, results, tc, conn_first_fail, n_conns);
    }
    flush_counters<1>(counters, tc, 0, threadIdx.x == 0);
}

// ---------------------------------------------------------------------------------------------
// One wave per buffer, G buffers in flight per wave (datagram-sized buffers).
// A group of G descriptors whose interiors fit U chunks per lane takes the
// grouped fast path (G*U loads per lane issued together); any other group is
// processed buffer by buffer.
template <int G, int U, bool NT>
__global__ void __launch_bounds__(kBlock) verify_wave_kernel(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                             const cts_buf_desc* __restrict__ descs, uint32_t n,
                                                             cts_verify_result* __restrict__ results,
                                                             uint64_t* __restrict__ counters,
                                                             uint32_t* __restrict__ conn_first_fail, uint32_t n_conns)
{
    constexpr int WAVES = kBlock / 64;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t gw = blockIdx.x * WAVES + wave;
    const uint32_t nw = gridDim.x * WAVES;
    TeamCounters tc = {{0, 0, 0, 0, 0}};

    for (uint32_t base = gw * G; base < n; base += nw * G) {
        cts_buf_desc d[G];
        Span s[G];
        bool ok[G];
        bool simple = true;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t i = base + (uint32_t)g;
            ok[g] = false;
            s[g].nchunks = 0;
            if (i < n) {
                d[g] = descs[i];
                ok[g] = !desc_bad(d[g], arena_bytes);
                if (ok[g]) s[g] = make_span(arena, d[g]);
            }
            simple = simple && ok[g] && s[g].nchunks >= 3u && s[g].nchunks - 2u <= (uint32_t)(64 * U);
        }
        uint32_t acc[G];
        if (simple) {
            u32x4 x[G][U];
#pragma unroll
            for (int g = 0; g < G; ++g) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t c = 1u + (uint32_t)(u * 64) + lane;
                    const uint32_t cl = s[g].nchunks - 2u;  // last interior chunk
                    x[g][u] = load_chunk<NT>(s[g].p + (c < cl ? c : cl));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int g = 0; g < G; ++g) {
                acc[g] = 0;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t c = 1u + (uint32_t)(u * 64) + lane;
                    const uint32_t cl = s[g].nchunks - 2u;
                    const uint32_t any = or4(chunk_xor(s[g], c < cl ? c : cl, x[g][u]));
                    acc[g] |= (c <= cl) ? any : 0u;
                }
                acc[g] |= scan_edges(s[g], lane);
            }
        } else {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                acc[g] = 0;
                if (ok[g]) {
                    if (s[g].nchunks >= 3u) acc[g] = scan_interior<64, U, NT>(s[g], 1u, s[g].nchunks - 1u, lane);
                    acc[g] |= scan_edges(s[g], lane);
                }
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint32_t i = base + (uint32_t)g;
            if (i >= n) break;
            if (!ok[g]) {
                if (lane == 0) write_bad(results, i);
                continue;
            }
            uint32_t first = kNone, count = 0;
            if (__any(acc[g] != 0u)) {
                scan_exact<64>(s[g], lane, first, count);
                first = wave_min(first);
                count = wave_sum(count);
            }
            if (lane == 0) finish_buffer(s[g], d[g], i, first, count, results, tc, conn_first_fail, n_conns);
        }
    }
    flush_counters<WAVES>(counters, tc, wave, lane == 0);
}

// ---------------------------------------------------------------------------------------------
// fill: the write-bound twin. Interior chunks are 16-byte stores; the (at most
// two) edge chunks of a span are written bytewise so neighbouring buffers
// sharing a 16-byte line are never touched.
__device__ __forceinline__ void fill_chunk(u32x4* a0, uint32_t c, uint32_t nchunks, uint32_t q0, uint32_t lo,
                                           uint32_t hi_last)
{
    const u32x4 e = expected_chunk((q0 + 16u * c) & 0xFFFFu, q0 & 1u);
    const bool first_c = (c == 0u);
    const bool last_c = (c == nchunks - 1u);
    const uint32_t b0 = first_c ? lo : 0u;
    const uint32_t b1 = last_c ? hi_last : 16u;
    if (b0 == 0u && b1 == 16u) {
        __builtin_nontemporal_store(e, a0 + c);
    } else {
        uint8_t* dst = reinterpret_cast<uint8_t*>(a0 + c);
        for (uint32_t b = b0; b < b1; ++b) dst[b] = (uint8_t)(e[b >> 2] >> (8 * (b & 3)));
    }
}

template <int TEAM>
__global__ void __launch_bounds__(kBlock) fill_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                      const cts_buf_desc* __restrict__ descs, uint32_t n)
{
    constexpr int TEAMS = kBlock / TEAM;
    const uint32_t lane = threadIdx.x % TEAM;
    const uint32_t team = (TEAM == kBlock) ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / TEAM);
    for (uint32_t i = blockIdx.x * TEAMS + team; i < n; i += gridDim.x * TEAMS) {
        const cts_buf_desc d = descs[i];
        if (desc_bad(d, arena_bytes)) continue;
        const uint32_t len = d.length - d.skip_head;
        if (len == 0) continue;
        uint8_t* sp = arena + d.byte_offset + d.skip_head;
        const uint32_t lo = (uint32_t)((uintptr_t)sp & 15u);
        const uint32_t nchunks = (uint32_t)(((uint64_t)lo + len + 15u) >> 4);
        const uint32_t hi_last = (uint32_t)((uint64_t)lo + len - 16ull * (nchunks - 1u));
        const uint32_t q0 = (d.expected_pattern_offset - lo) & 0xFFFFu;
        u32x4* p = reinterpret_cast<u32x4*>(sp - lo);
        for (uint32_t c = lane; c < nchunks; c += TEAM) fill_chunk(p, c, nchunks, q0, lo, hi_last);
    }
}

// One long span, all workgroups cooperating (sender buffer materialisation).
__global__ void __launch_bounds__(kBlock) fill_span_kernel(uint8_t* __restrict__ dst, uint64_t bytes, uint32_t e)
{
    const uint32_t lo = (uint32_t)((uintptr_t)dst & 15u);
    const uint32_t nchunks = (uint32_t)((lo + bytes + 15u) >> 4);
    const uint32_t hi_last = (uint32_t)(lo + bytes - 16ull * (nchunks - 1u));
    const uint32_t q0 = (e - lo) & 0xFFFFu;
    u32x4* p = reinterpret_cast<u32x4*>(dst - lo);
    for (uint32_t c = blockIdx.x * kBlock + threadIdx.x; c < nchunks; c += gridDim.x * kBlock)
        fill_chunk(p, c, nchunks, q0, lo, hi_last);
}

// ---------------------------------------------------------------------------------------------
static inline uint32_t grid_for(uint32_t n, int teams_per_block, const LaunchGeometry& geo)
{
    const uint64_t want = ((uint64_t)n + teams_per_block - 1) / teams_per_block;
    const uint64_t cap = (uint64_t)geo.num_cus * (uint64_t)(geo.blocks_per_cu > 0 ? geo.blocks_per_cu : 16);
    const uint64_t g = want < cap ? want : cap;
    return (uint32_t)(g == 0 ? 1 : g);
}

#define CTS_VERIFY_ARGS arena, arena_bytes, descs, n, results, counters, conn_first_fail, n_conns

template <bool NT>
static void launch_verify_nt(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                             bool small, cts_verify_result* results, uint64_t* counters, uint32_t* conn_first_fail,
                             uint32_t n_conns, hipStream_t stream, const LaunchGeometry& geo)
{
    if (small) {
        // variant (small path): 0 = G4 U2, 1 = G2 U2, 2 = G8 U2, 3 = G1 U2
        constexpr int U = 2;
        int G = 4;
        switch (geo.verify_variant) {
        case 1: G = 2; break;
        case 2: G = 8; break;
        case 3: G = 1; break;
        default: G = 4; break;
        }
        const uint32_t grid = grid_for((n + G - 1) / G, kBlock / 64, geo);
        switch (G) {
        case 1: verify_wave_kernel<1, U, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        case 2: verify_wave_kernel<2, U, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        case 8: verify_wave_kernel<8, U, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        default: verify_wave_kernel<4, U, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        }
    } else {
        // variant (workgroup path): 0 = U8, 1 = U16, 2 = U4, 3 = LDS-DMA U8
        const uint32_t grid = grid_for(n, 1, geo);
        switch (geo.verify_variant) {
        case 1: verify_wg_kernel<16, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        case 2: verify_wg_kernel<4, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        case 3: verify_wg_lds_kernel<8, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        default: verify_wg_kernel<8, NT><<<grid, kBlock, 0, stream>>>(CTS_VERIFY_ARGS); break;
        }
    }
}

hipError_t launch_verify(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                         uint32_t max_length_hint, cts_verify_result* results, uint64_t* counters,
                         uint32_t* conn_first_fail, uint32_t n_conns, hipStream_t stream,
                         const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    const bool small = max_length_hint != 0 && max_length_hint <= (uint32_t)geo.small_threshold;
    if (geo.nontemporal) {
        launch_verify_nt<true>(arena, arena_bytes, descs, n, small, results, counters, conn_first_fail, n_conns,
                               stream, geo);
    } else {
        launch_verify_nt<false>(arena, arena_bytes, descs, n, small, results, counters, conn_first_fail, n_conns,
                                stream, geo);
    }
    return hipGetLastError();
}

hipError_t launch_fill(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                       uint32_t max_length_hint, hipStream_t stream, const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    const bool small = max_length_hint != 0 && max_length_hint <= (uint32_t)geo.small_threshold;
    if (small) {
        fill_kernel<64><<<grid_for(n, kBlock / 64, geo), kBlock, 0, stream>>>(arena, arena_bytes, descs, n);
    } else {
        fill_kernel<kBlock><<<grid_for(n, 1, geo), kBlock, 0, stream>>>(arena, arena_bytes, descs, n);
    }
    return hipGetLastError();
}

hipError_t launch_fill_span(uint8_t* dst, uint64_t bytes, uint32_t pattern_offset, hipStream_t stream,
                            const LaunchGeometry& geo)
{
    if (bytes == 0) return hipSuccess;
    const uint64_t chunks = (bytes + 30) / 16 + 1;
    const uint32_t grid = grid_for((uint32_t)((chunks + kBlock - 1) / kBlock), 1, geo);
    fill_span_kernel<<<grid, kBlock, 0, stream>>>(dst, bytes, pattern_offset & 0xFFFFu);
    return hipGetLastError();
}

}  // namespace cts
