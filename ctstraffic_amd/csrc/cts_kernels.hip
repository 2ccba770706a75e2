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
// Design: a pure HBM-read stream, no MFMA. Each team (a
// 256-lane workgroup for 64 KiB TCP buffers, one 64-lane wave for datagrams)
// owns one buffer at a time and walks it in 16-byte chunks (global_load_dwordx4,
// 1 KiB per wave-instruction, all U loads of a round issued before any compare).
// The expected chunk is regenerated in registers from the stream position: one
// v_mad_u32_u24 + adds/ands for four u16 pairs, and for an odd byte phase one
// v_alignbyte per dword. The byte phase is uniform per buffer (chunks are
// 16-aligned in memory, so the parity of the pattern position of every chunk
// equals that of expected - (start mod 16)), so the odd/even choice is a
// wave-uniform branch outside the loop. Mismatch analysis (first differing byte,
// popcount of differing bytes) only runs in the rare branch where a chunk's
// XOR is nonzero. Per buffer the team reduces (min first, sum count) only when
// some lane saw a mismatch (wave __any / workgroup __syncthreads_or).
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
// (0 <= q < 65536). For even q the chunk holds the u16 values k..k+7
// (k = q >> 1, mod 32768); for odd q it is bytes 1..16 of values k..k+8.
// Packed: dword j = (k+2j) | (k+2j+1) << 16 = base + j*0x20002 with
// base = k*0x10001 + 0x10000; the & 0x7FFF7FFF wraps 32768 -> 0 in each half
// (low half never exceeds 32775, so no carry crosses into the high half).
template <bool ODD>
__device__ __forceinline__ u32x4 expected_chunk(uint32_t q)
{
    const uint32_t k = q >> 1;
    const uint32_t base = __umul24(k, 0x10001u) + 0x10000u;
    const uint32_t w0 = base & 0x7FFF7FFFu;
    const uint32_t w1 = (base + 0x20002u) & 0x7FFF7FFFu;
    const uint32_t w2 = (base + 0x40004u) & 0x7FFF7FFFu;
    const uint32_t w3 = (base + 0x60006u) & 0x7FFF7FFFu;
    if constexpr (!ODD) {
        return u32x4{w0, w1, w2, w3};
    } else {
        const uint32_t w4 = (base + 0x80008u) & 0x7FFF7FFFu;
        return u32x4{__builtin_amdgcn_alignbyte(w1, w0, 1), __builtin_amdgcn_alignbyte(w2, w1, 1),
                     __builtin_amdgcn_alignbyte(w3, w2, 1), __builtin_amdgcn_alignbyte(w4, w3, 1)};
    }
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
        const uint32_t mw = (b > a) ? (low_bytes_mask(b) & ~low_bytes_mask(a)) : 0u;
        m[w] = mw;
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

// Fast pass over the INTERIOR chunks [1, nchunks-1) of a span (all 16 bytes
// valid): returns the OR of (received ^ expected) over the lane's chunks.
// Straight-line code — every load of a round is issued before the first
// compare and no load sits under a branch (a load under an exec branch makes
// hipcc drain vmcnt(0) at every join, serialising the stream). The tail round
// clamps its chunk index to the last interior chunk and discards the excess.
template <int TEAM, int U, bool ODD, bool NT>
__device__ __forceinline__ uint32_t scan_interior(const u32x4* __restrict__ a0, uint32_t nchunks, uint32_t q0,
                                                  uint32_t lane)
{
    uint32_t acc = 0;
    if (nchunks < 3u) return 0;
    const uint32_t c_end = nchunks - 1u;
    uint32_t cb = 1u;
    for (; cb + (uint32_t)(TEAM * U) <= c_end; cb += (uint32_t)(TEAM * U)) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = load_chunk<NT>(a0 + cb + (uint32_t)(u * TEAM) + lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = cb + (uint32_t)(u * TEAM) + lane;
            const u32x4 x = d[u] ^ expected_chunk<ODD>((q0 + 16u * c) & 0xFFFFu);
            acc |= x[0] | x[1] | x[2] | x[3];
        }
    }
    if (cb < c_end) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = cb + (uint32_t)(u * TEAM) + lane;
            d[u] = load_chunk<NT>(a0 + (c < c_end ? c : c_end - 1u));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = cb + (uint32_t)(u * TEAM) + lane;
            const uint32_t cc = c < c_end ? c : c_end - 1u;
            const u32x4 x = d[u] ^ expected_chunk<ODD>((q0 + 16u * cc) & 0xFFFFu);
            const uint32_t any = x[0] | x[1] | x[2] | x[3];
            acc |= (c < c_end) ? any : 0u;
        }
    }
    return acc;
}

// XOR of one (possibly partial) chunk with its expected bytes, bytes outside
// the span [lo, 16*(nchunks-1)+hi_last) masked to zero.
template <bool ODD>
__device__ __forceinline__ u32x4 chunk_diff(const u32x4* __restrict__ a0, uint32_t c, uint32_t nchunks, uint32_t q0,
                                            uint32_t lo, uint32_t hi_last)
{
    u32x4 x = a0[c] ^ expected_chunk<ODD>((q0 + 16u * c) & 0xFFFFu);
    if (c == 0u || c == nchunks - 1u) x &= range_mask(c == 0u ? lo : 0u, c == nchunks - 1u ? hi_last : 16u);
    return x;
}

// Exact scan of a whole span (rare path: only for a span the fast pass
// flagged, or for its two edge chunks): first differing byte position
// (relative to the span start) and # of differing bytes over the lane's chunks.
template <int TEAM, bool ODD>
__device__ __noinline__ void scan_exact(const u32x4* __restrict__ a0, uint32_t c_begin, uint32_t c_end,
                                        uint32_t nchunks, uint32_t q0, uint32_t lo, uint32_t hi_last, uint32_t lane,
                                        uint32_t& first, uint32_t& count)
{
    for (uint32_t c = c_begin + lane; c < c_end; c += TEAM) {
        const u32x4 x = chunk_diff<ODD>(a0, c, nchunks, q0, lo, hi_last);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t nz = nonzero_bytes(x[w]);
            if (nz) {
                const uint32_t idx = 4u * (uint32_t)w + ((uint32_t)__builtin_ctz(nz) >> 3);
                const uint32_t pos = 16u * c + idx - lo;
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

// One verify pass over n descriptors. TEAM = 256 (one workgroup per buffer) or
// 64 (one wave per buffer, 4 buffers per workgroup). Grid-strides over buffers.
template <int TEAM, int U, bool NT>
__global__ void __launch_bounds__(kBlock) verify_kernel(const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                        const cts_buf_desc* __restrict__ descs, uint32_t n,
                                                        cts_verify_result* __restrict__ results,
                                                        uint64_t* __restrict__ counters,
                                                        uint32_t* __restrict__ conn_first_fail, uint32_t n_conns)
{
    constexpr int TEAMS = kBlock / TEAM;
    __shared__ uint32_t red_first[kBlock / 64];
    __shared__ uint32_t red_count[kBlock / 64];
    __shared__ uint64_t red_ctr[TEAMS][5];

    const uint32_t lane = threadIdx.x % TEAM;
    const uint32_t team = (TEAM == kBlock) ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / TEAM);
    const uint32_t wave = threadIdx.x / 64;

    TeamCounters tc = {{0, 0, 0, 0, 0}};

    for (uint32_t i = blockIdx.x * TEAMS + team; i < n; i += gridDim.x * TEAMS) {
        const cts_buf_desc d = descs[i];
        const bool bad = d.expected_pattern_offset >= 65536u || d.length < d.skip_head ||
                         d.byte_offset > arena_bytes || arena_bytes - d.byte_offset < (uint64_t)d.length;
        if (bad) {
            if (results != nullptr && lane == 0) {
                cts_verify_result r;
                r.first_mismatch = 0;
                r.mismatch_bytes = 0;
                r.expected = 0;
                r.actual = 0;
                r.pass = 0;
                r.flags = CTS_RESULT_FLAG_BAD_DESC;
                results[i] = r;
            }
            continue;
        }
        const uint32_t len = d.length - d.skip_head;
        // pointer arithmetic from the kernel argument keeps the global address
        // space (global_load_dwordx4, not flat_load: flat loads also count in
        // lgkmcnt and force full drains)
        const uint8_t* sp = arena + d.byte_offset + d.skip_head;  // span start
        const uint32_t lo = (uint32_t)((uintptr_t)sp & 15u);
        const uint32_t nchunks = len == 0 ? 0u : (uint32_t)(((uint64_t)lo + len + 15u) >> 4);
        const uint32_t hi_last = len == 0 ? 0u : (uint32_t)((uint64_t)lo + len - 16ull * (nchunks - 1u));
        const uint32_t q0 = (d.expected_pattern_offset - lo) & 0xFFFFu;

        uint32_t first = kNone, count = 0;
        const u32x4* p = reinterpret_cast<const u32x4*>(sp - lo);
        const bool odd = (q0 & 1u) != 0u;
        // fast pass: interior chunks, branch-free streaming compare
        uint32_t acc = odd ? scan_interior<TEAM, U, true, NT>(p, nchunks, q0, lane)
                           : scan_interior<TEAM, U, false, NT>(p, nchunks, q0, lane);
        // edge chunks (first and last; possibly partial) by lanes 0 and 1
        if (lane < 2u && nchunks > 0u && (lane == 0u || nchunks > 1u)) {
            const uint32_t c = lane == 0u ? 0u : nchunks - 1u;
            const u32x4 x = odd ? chunk_diff<true>(p, c, nchunks, q0, lo, hi_last)
                                : chunk_diff<false>(p, c, nchunks, q0, lo, hi_last);
            acc |= x[0] | x[1] | x[2] | x[3];
        }
        // rare path: some lane of the team saw a difference -> exact re-scan
        bool team_bad;
        if constexpr (TEAM == 64) {
            team_bad = __any(acc != 0u);
        } else {
            team_bad = __syncthreads_or(acc != 0u) != 0;
        }
        if (team_bad) {
            if (odd) {
                scan_exact<TEAM, true>(p, 0u, nchunks, nchunks, q0, lo, hi_last, lane, first, count);
            } else {
                scan_exact<TEAM, false>(p, 0u, nchunks, nchunks, q0, lo, hi_last, lane, first, count);
            }
        }

        // team reduction, only if some lane saw a mismatch
        if constexpr (TEAM == 64) {
            if (team_bad) {
                first = wave_min(first);
                count = wave_sum(count);
            }
        } else {
            if (team_bad) {
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
        }

        if (lane == 0) {
            const bool pass = (first == kNone);
            cts_verify_result r;
            r.first_mismatch = pass ? len : first;
            r.mismatch_bytes = pass ? 0u : count;
            r.expected = pass ? 0 : (uint8_t)pattern_byte_dev(d.expected_pattern_offset + first);
            r.actual = pass ? 0 : sp[first];
            r.pass = pass ? 1 : 0;
            r.flags = 0;
            if (results != nullptr) results[i] = r;
            tc.v[kBytesChecked] += len;
            tc.v[kBuffersChecked] += 1;
            if (pass) {
                tc.v[kBytesOk] += len;
            } else {
                tc.v[kBuffersFailed] += 1;
                tc.v[kMismatchedBytes] += count;
                if (conn_first_fail != nullptr && d.conn_index < n_conns) atomicMin(&conn_first_fail[d.conn_index], i);
            }
        }
    }

    if (counters == nullptr) return;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) red_ctr[team][k] = tc.v[k];
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        uint64_t sum = 0;
#pragma unroll
        for (int t = 0; t < TEAMS; ++t) sum += red_ctr[t][threadIdx.x];
        if (sum) atomicAdd((unsigned long long*)&counters[(blockIdx.x % CTS_COUNTER_SHARDS) * kCounterSlots + threadIdx.x],
                           (unsigned long long)sum);
    }
}

// ---------------------------------------------------------------------------------------------
// fill: the write-bound twin. Interior chunks are 16-byte stores; the (at most
// two) edge chunks of a span are written bytewise so neighbouring buffers
// sharing a 16-byte line are never touched.
template <bool ODD>
__device__ __forceinline__ void fill_chunk(u32x4* a0, uint32_t c, uint32_t nchunks, uint32_t q0, uint32_t lo,
                                           uint32_t hi_last)
{
    const u32x4 e = expected_chunk<ODD>((q0 + 16u * c) & 0xFFFFu);
    const bool first_c = (c == 0u);
    const bool last_c = (c == nchunks - 1u);
    if (!first_c && !last_c) {
        __builtin_nontemporal_store(e, a0 + c);
    } else {
        const uint32_t b0 = first_c ? lo : 0u;
        const uint32_t b1 = last_c ? hi_last : 16u;
        if (b0 == 0u && b1 == 16u) {
            __builtin_nontemporal_store(e, a0 + c);
        } else {
            uint8_t* dst = reinterpret_cast<uint8_t*>(a0 + c);
            for (uint32_t b = b0; b < b1; ++b) dst[b] = (uint8_t)(e[b >> 2] >> (8 * (b & 3)));
        }
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
        const bool bad = d.expected_pattern_offset >= 65536u || d.length < d.skip_head ||
                         d.byte_offset > arena_bytes || arena_bytes - d.byte_offset < (uint64_t)d.length;
        if (bad) continue;
        const uint32_t len = d.length - d.skip_head;
        if (len == 0) continue;
        uint8_t* sp = arena + d.byte_offset + d.skip_head;
        const uint32_t lo = (uint32_t)((uintptr_t)sp & 15u);
        const uint32_t nchunks = (uint32_t)(((uint64_t)lo + len + 15u) >> 4);
        const uint32_t hi_last = (uint32_t)((uint64_t)lo + len - 16ull * (nchunks - 1u));
        const uint32_t q0 = (d.expected_pattern_offset - lo) & 0xFFFFu;
        u32x4* p = reinterpret_cast<u32x4*>(sp - lo);
        if (q0 & 1u) {
            for (uint32_t c = lane; c < nchunks; c += TEAM) fill_chunk<true>(p, c, nchunks, q0, lo, hi_last);
        } else {
            for (uint32_t c = lane; c < nchunks; c += TEAM) fill_chunk<false>(p, c, nchunks, q0, lo, hi_last);
        }
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
    for (uint32_t c = blockIdx.x * kBlock + threadIdx.x; c < nchunks; c += gridDim.x * kBlock) {
        if (q0 & 1u) {
            fill_chunk<true>(p, c, nchunks, q0, lo, hi_last);
        } else {
            fill_chunk<false>(p, c, nchunks, q0, lo, hi_last);
        }
    }
}

// ---------------------------------------------------------------------------------------------
static inline uint32_t grid_for(uint32_t n, int teams_per_block, const LaunchGeometry& geo)
{
    const uint64_t want = ((uint64_t)n + teams_per_block - 1) / teams_per_block;
    const uint64_t cap = (uint64_t)geo.num_cus * (uint64_t)(geo.blocks_per_cu > 0 ? geo.blocks_per_cu : 8);
    const uint64_t g = want < cap ? want : cap;
    return (uint32_t)(g == 0 ? 1 : g);
}

hipError_t launch_verify(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                         uint32_t max_length_hint, cts_verify_result* results, uint64_t* counters,
                         uint32_t* conn_first_fail, uint32_t n_conns, hipStream_t stream,
                         const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    const bool small = max_length_hint != 0 && max_length_hint <= (uint32_t)geo.small_threshold;
    if (small) {
        const uint32_t grid = grid_for(n, kBlock / 64, geo);
        if (geo.nontemporal) {
            verify_kernel<64, 2, true><<<grid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n, results, counters,
                                                                     conn_first_fail, n_conns);
        } else {
            verify_kernel<64, 2, false><<<grid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n, results, counters,
                                                                      conn_first_fail, n_conns);
        }
    } else {
        const uint32_t grid = grid_for(n, 1, geo);
        if (geo.nontemporal) {
            verify_kernel<kBlock, 8, true><<<grid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n, results,
                                                                         counters, conn_first_fail, n_conns);
        } else {
            verify_kernel<kBlock, 8, false><<<grid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n, results,
                                                                          counters, conn_first_fail, n_conns);
        }
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
