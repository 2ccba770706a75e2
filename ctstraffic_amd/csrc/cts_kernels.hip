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
// Paths (one kernel per path; nontemporal and plain-load forms of each):
//   verify_wg_kernel                  one 256-lane workgroup per buffer (64 KiB TCP buffers)
//   verify_quad_kernel                four buffers per wave (datagram-sized buffers; descriptors or a strided ring)
//   media_stream_verify_quad_kernel   MediaStream receive: header + payload, four datagrams per wave
//   fill_kernel / fill_span_kernel / fill_batched_kernel / media_stream_fill_ring_kernel   the sender side
//   mailbox_kernel                    SYNC-mode VerifyBuffer without a launch per call (resident grid)
// Every alternative measured on the way to these (other unroll depths, barrier-free and wave-per-buffer
// workgroups, windowed and rotated walks, staged records, speculative first loads, LDS-DMA, line policies,
// two-pass MediaStream receives) was removed from the source once it lost; DESIGN.md §10 lists them with
// their numbers, and git history (up to round 4, commit fe0efda) holds their code.
#include <hip/hip_runtime.h>

#include <type_traits>

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

// load_chunk through an explicitly global (address space 1) pointer: a pointer that
// went through a select or a phi can lose its address space and become a flat load,
// which also counts in lgkmcnt and forces full drains
typedef const u32x4 __attribute__((address_space(1)))* gchunk_ptr;
template <bool NT>
__device__ __forceinline__ u32x4 load_chunk_g(const u32x4* p)
{
    const gchunk_ptr g = (gchunk_ptr)p;
    if constexpr (NT) {
        return __builtin_nontemporal_load(g);
    } else {
        return *g;
    }
}

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
    uint32_t cb0;      // first interior chunk on a 128-byte line boundary (1..8)
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
    // Interior rounds start on a 128-byte line: a wave's 1 KiB load then covers 8
    // lines instead of straddling 9 (chunks [1, cb0) are head chunks, see scan_buffer).
    const uint32_t a = (uint32_t)(((uintptr_t)s.p >> 4) & 7u);  // chunk 0's slot in its line
    s.cb0 = 8u - a;                                             // (a + cb0) % 8 == 0, cb0 in [1, 8]
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

// Buffer resource over the span's chunks [0, nchunks): 16-byte buffer loads
// address it with ONE lane offset VGPR (+ an SGPR offset per unrolled load)
// instead of a 64-bit address per load, and the hardware range check returns 0
// for any byte past num_records instead of faulting.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const Span& s)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4*>(s.p), (short)0, (int)(s.nchunks * 16u), 0x00020000);
}

template <bool NT>
__device__ __forceinline__ u32x4 buf_load(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, NT ? 2 : 0);  // aux 2 = nt
}

// Expected chunk u of a round: k advances by TEAM*8 per unrolled step (16*TEAM
// bytes / 2), added to the packed base before the per-half wrap mask. The low
// half stays below 65536 (k <= 32767 + 8*TEAM*(U-1) + 8), so no carry crosses.
template <int TEAM, int U, bool EVEN = false>
__device__ __forceinline__ u32x4 expected_step(uint32_t B, int u, uint32_t sh)
{
    static_assert(32767 + 8 * TEAM * (U - 1) + 8 < 65536, "packed k must not carry");
    // B is made opaque so each word is v_add(literal) + v_and: left visible,
    // hipcc folds the adds into v_mad_u32_u24 whose 32-bit addends (VOP3 takes
    // no literal on gfx950) it then parks in ~40 VGPRs, halving occupancy.
    uint32_t bb = B;
    asm volatile("" : "+v"(bb));
    const uint32_t b = bb + (uint32_t)u * (uint32_t)(8 * TEAM) * 0x10001u;
    const uint32_t w0 = b & 0x7FFF7FFFu;
    const uint32_t w1 = (b + 0x20002u) & 0x7FFF7FFFu;
    const uint32_t w2 = (b + 0x40004u) & 0x7FFF7FFFu;
    const uint32_t w3 = (b + 0x60006u) & 0x7FFF7FFFu;
    if constexpr (EVEN) {
        // byte phase 0 (every 16-aligned expected offset, 75 % of config 2): the chunk IS
        // the four packed pairs, no funnel shift and no fifth word
        return u32x4{w0, w1, w2, w3};
    } else {
        const uint32_t w4 = (b + 0x80008u) & 0x7FFF7FFFu;
        return u32x4{__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                     __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
    }
}

// packed base (k*0x10001 + 0x10000) of the chunk at index c
__device__ __forceinline__ uint32_t chunk_base(const Span& s, uint32_t c)
{
    const uint32_t k = ((s.q0 + 16u * c) & 0xFFFFu) >> 1;
    return __umul24(k, 0x10001u) + 0x10000u;
}

// Fast pass over the interior chunks [1, nchunks-1) (all 16 bytes valid): OR
// of (received ^ expected) over this lane's chunks. Straight-line rounds of U
// buffer loads per lane, all issued before the first compare (sched_barrier
// keeps the scheduler from interleaving them with the compares); no load under
// a branch (a load under an exec branch makes hipcc drain vmcnt(0) at every
// join). Full rounds use SGPR offsets; the tail round puts the whole offset in
// the VGPR so the range check (which covers voffset + imm) zero-fills the
// excess lanes, which are then masked out.
template <int TEAM, int U, bool NT, bool EVEN>
__device__ __forceinline__ uint32_t scan_rounds(const Span& s, __amdgpu_buffer_rsrc_t r, uint32_t lane, uint32_t cb,
                                                uint32_t c_end)
{
    uint32_t acc = 0;
    const uint32_t voff = lane * 16u;
    for (; cb + (uint32_t)(TEAM * U) <= c_end; cb += (uint32_t)(TEAM * U)) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = buf_load<NT>(r, voff, (cb + (uint32_t)(u * TEAM)) * 16u);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t B = chunk_base(s, cb + lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc |= or4(d[u] ^ expected_step<TEAM, U, EVEN>(B, u, s.sh));
            // one chunk's expected words live at a time (else hipcc hoists all
            // U*5 of them ahead of the compares: +40 VGPRs, half the occupancy)
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (cb < c_end) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = buf_load<NT>(r, (cb + (uint32_t)(u * TEAM) + lane) * 16u, 0u);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t B = chunk_base(s, cb + lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t any = or4(d[u] ^ expected_step<TEAM, U, EVEN>(B, u, s.sh));
            acc |= (cb + (uint32_t)(u * TEAM) + lane < c_end) ? any : 0u;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    return acc;
}

// interior = [cb0, nchunks-1); [1, cb0) are head chunks
template <int TEAM, int U, bool NT, bool EVEN>
__device__ __forceinline__ uint32_t scan_interior_impl(const Span& s, __amdgpu_buffer_rsrc_t r, uint32_t lane)
{
    if (s.nchunks < 3u) return 0;
    return scan_rounds<TEAM, U, NT, EVEN>(s, r, lane, s.cb0, s.nchunks - 1u);
}

// SPLIT: a span-uniform (scalar) branch on the byte phase selects the
// funnel-shift-free even-phase stream.
template <int TEAM, int U, bool NT, bool SPLIT>
__device__ __forceinline__ uint32_t scan_interior(const Span& s, __amdgpu_buffer_rsrc_t r, uint32_t lane)
{
    if constexpr (SPLIT) {
        if (__builtin_amdgcn_readfirstlane(s.sh) == 0u) return scan_interior_impl<TEAM, U, NT, true>(s, r, lane);
    }
    return scan_interior_impl<TEAM, U, NT, false>(s, r, lane);
}

// A span of whole chunks starting on a 128-byte line (lo == 0, hi_last == 16,
// chunk 0 line-aligned: every buffer of a 64 KiB-strided arena or recv ring
// whose completion is a multiple of 16 bytes) has no partial chunk to mask: all
// of [0, nchunks) streams in rounds, with no edge/head load and, for 64 KiB, no
// tail round (4096 chunks = 8 full rounds of 256 lanes x U2; scan_whole_exact).
__device__ __forceinline__ bool span_whole_lines(const Span& s)
{
    return s.lo == 0u && s.hi_last == 16u && s.cb0 == 8u;
}

// Fast pass over a whole span: OR of (received ^ expected) over this lane's
// share. The two edge chunks (first and last, possibly partial) are loaded
// FIRST by every lane (lane 1 the last chunk, the others chunk 0: the same
// lines, no extra traffic), so their latency hides under the interior stream
// instead of adding a dependent round trip per buffer; their byte-masked
// compare runs at the end, branch-free, on registers. For an empty span the
// edge offset is out of the resource's range and reads 0.
// Edge/head chunk of a lane: lane 0 = chunk 0, lane 1 = the last chunk, lanes
// 2..8 = head chunks 1..7 (those below cb0 and the last chunk); other lanes
// re-load chunk 0 (same line, no extra traffic) and discard it.
__device__ __forceinline__ uint32_t edge_chunk_of(const Span& s, uint32_t lane)
{
    return lane == 1u ? s.nchunks - 1u : ((lane >= 2u && lane <= 8u) ? lane - 1u : 0u);
}
__device__ __forceinline__ bool edge_chunk_used(const Span& s, uint32_t lane)
{
    if (s.nchunks == 0u) return false;
    if (lane == 0u) return true;
    if (lane == 1u) return s.nchunks > 1u;
    const uint32_t h = s.nchunks - 1u < s.cb0 ? s.nchunks - 1u : s.cb0;  // head = [1, min(cb0, nchunks-1))
    return lane >= 2u && lane <= 8u && lane - 1u < h;
}

template <int TEAM, int U, bool NT, bool SPLIT = false>
__device__ __forceinline__ uint32_t scan_buffer(const Span& s, uint32_t lane)
{
    const __amdgpu_buffer_rsrc_t r = span_rsrc(s);
    const uint32_t ce = edge_chunk_of(s, lane);
    // lanes without an edge/head chunk address past the resource: the range check
    // returns 0 without a memory request (waves 1..3 of a workgroup fetch nothing)
    const u32x4 edge = buf_load<NT>(r, edge_chunk_used(s, lane) ? ce * 16u : 0x7FFFFFF0u, 0u);
    uint32_t acc = scan_interior<TEAM, U, NT, SPLIT>(s, r, lane);
    const u32x4 x = chunk_xor(s, ce, edge) & range_mask(ce == 0u ? s.lo : 0u, ce == s.nchunks - 1u ? s.hi_last : 16u);
    acc |= edge_chunk_used(s, lane) ? or4(x) : 0u;
    return acc;
}

// Exact diff of one chunk's XOR: first differing byte (span-relative) and count.
__device__ __forceinline__ void take_diff(const Span& s, uint32_t c, u32x4 x, uint32_t& first, uint32_t& count)
{
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

// Exact re-scan of exactly the chunks this lane owns in scan_buffer (interior
// chunk c in [cb0, nchunks-1) -> lane (c-cb0) % TEAM; edge/head chunks -> lanes
// 0..8, edge_chunk_of). Only lanes whose fast pass saw a difference call it, so
// a corrupt buffer costs one lane's re-read, not the team's; the loads go out U
// at a time like the fast pass, so the re-read is a few round trips, not one per
// chunk. Yields the lane's first differing byte and differing-byte count.
template <int TEAM, int U, bool NT>
__device__ __forceinline__ void scan_exact_owned(const Span& s, uint32_t lane, uint32_t& first, uint32_t& count)
{
    if (s.nchunks == 0) return;
    const __amdgpu_buffer_rsrc_t r = span_rsrc(s);
    if (s.nchunks >= 3u) {
        const uint32_t c_end = s.nchunks - 1u;
        for (uint32_t cb = s.cb0; cb < c_end; cb += (uint32_t)(TEAM * U)) {
            u32x4 d[U];
#pragma unroll
            for (int u = 0; u < U; ++u) d[u] = buf_load<NT>(r, (cb + (uint32_t)(u * TEAM) + lane) * 16u, 0u);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = cb + (uint32_t)(u * TEAM) + lane;
                if (c < c_end) take_diff(s, c, chunk_xor(s, c, d[u]), first, count);
            }
        }
    }
    if (edge_chunk_used(s, lane)) {
        const uint32_t c = edge_chunk_of(s, lane);
        const u32x4 x = chunk_xor(s, c, buf_load<NT>(r, c * 16u, 0u)) &
                        range_mask(c == 0u ? s.lo : 0u, c == s.nchunks - 1u ? s.hi_last : 16u);
        take_diff(s, c, x, first, count);
    }
}

// The whole-span stream with the exact diff done in registers: a lane whose round
// saw a difference computes its first differing byte and differing-byte count from
// the XORs it still holds, so a corrupt buffer costs no re-read. (A re-read is 8
// dependent rounds for a 64 KiB buffer: several microseconds during which the
// workgroup's next buffer waits, and with one corrupt buffer in a thousand that
// workgroup is the launch's last to finish.) The clean-path cost is one compare and
// branch per round.
// One whole round: XOR the U loaded chunks with the expected words, then the exact diff of a round that differs.
template <int TEAM, int U, bool EVEN>
__device__ __forceinline__ void whole_exact_round(const Span& s, u32x4 (&d)[U], uint32_t cb, uint32_t lane,
                                                  uint32_t& first, uint32_t& count)
{
    const uint32_t B = chunk_base(s, cb + lane);
    uint32_t any = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        d[u] ^= expected_step<TEAM, U, EVEN>(B, u, s.sh);
        any |= or4(d[u]);
        __builtin_amdgcn_sched_barrier(0);
    }
    if (any != 0u) {
#pragma unroll
        for (int u = 0; u < U; ++u) take_diff(s, cb + (uint32_t)(u * TEAM) + lane, d[u], first, count);
    }
}

template <int TEAM, int U, bool NT, bool EVEN>
__device__ __forceinline__ void scan_whole_exact_impl(const Span& s, __amdgpu_buffer_rsrc_t r, uint32_t lane,
                                                      uint32_t& first, uint32_t& count)
{
    const uint32_t voff = lane * 16u;
    uint32_t cb = 0;
    const uint32_t c_end = s.nchunks;
    for (; cb + (uint32_t)(TEAM * U) <= c_end; cb += (uint32_t)(TEAM * U)) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = buf_load<NT>(r, voff, (cb + (uint32_t)(u * TEAM)) * 16u);
        __builtin_amdgcn_sched_barrier(0);
        whole_exact_round<TEAM, U, EVEN>(s, d, cb, lane, first, count);
    }
    if (cb < c_end) {
        u32x4 d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = buf_load<NT>(r, (cb + (uint32_t)(u * TEAM) + lane) * 16u, 0u);
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t B = chunk_base(s, cb + lane);
        uint32_t any = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = cb + (uint32_t)(u * TEAM) + lane < c_end;
            d[u] = in ? (d[u] ^ expected_step<TEAM, U, EVEN>(B, u, s.sh)) : u32x4{0u, 0u, 0u, 0u};
            any |= or4(d[u]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (any != 0u) {
#pragma unroll
            for (int u = 0; u < U; ++u) take_diff(s, cb + (uint32_t)(u * TEAM) + lane, d[u], first, count);
        }
    }
}

// SPLIT: a span-uniform branch on the byte phase selects the funnel-shift-free even-phase stream
template <int TEAM, int U, bool NT, bool SPLIT>
__device__ __forceinline__ void scan_whole_exact(const Span& s, uint32_t lane, uint32_t& first, uint32_t& count)
{
    const __amdgpu_buffer_rsrc_t r = span_rsrc(s);
    if constexpr (SPLIT) {
        if (__builtin_amdgcn_readfirstlane(s.sh) == 0u) {
            scan_whole_exact_impl<TEAM, U, NT, true>(s, r, lane, first, count);
            return;
        }
    }
    scan_whole_exact_impl<TEAM, U, NT, false>(s, r, lane, first, count);
}

// Spans of 2 GiB or more (a u32 ctsTask length allows 4 GiB - 1). The buffer-resource streams above
// address a span with 32-bit byte offsets and a 32-bit num_records (and use 0x7FFFFFF0 as an
// out-of-range offset), so such spans take this plain pass instead: 64-bit pointers, exact from the
// start (first differing byte and count, RtlCompareMemory semantics), TEAM lanes striding the chunks
// G loads at a time (2: the pass must not raise the hot kernels' register count). Positions are span-relative u32 (16c + idx - lo < 2^32 even when 16c wraps).
constexpr uint32_t kGiantChunks = 1u << 27;

__device__ __forceinline__ bool span_giant(const Span& s)
{
    return __builtin_amdgcn_readfirstlane(s.nchunks >= kGiantChunks ? 1u : 0u) != 0u;
}

template <int TEAM, bool NT, uint32_t G = 2>
__device__ __forceinline__ void scan_giant_exact(const Span& s, uint32_t lane, uint32_t& first, uint32_t& count)
{
    for (uint32_t cb = 0; cb < s.nchunks; cb += G * TEAM) {
        u32x4 d[G];
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t c = cb + g * TEAM + lane;
            d[g] = load_chunk_g<NT>(s.p + (c < s.nchunks ? c : 0u));
        }
#pragma unroll
        for (uint32_t g = 0; g < G; ++g) {
            const uint32_t c = cb + g * TEAM + lane;
            if (c < s.nchunks) {
                u32x4 x = chunk_xor(s, c, d[g]);
                if (c == 0u || c == s.nchunks - 1u)
                    x &= range_mask(c == 0u ? s.lo : 0u, c == s.nchunks - 1u ? s.hi_last : 16u);
                take_diff(s, c, x, first, count);
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
// rslot != nullptr: the record goes there (an LDS staging slot) instead of to results[i].
__device__ __forceinline__ void finish_buffer(const Span& s, const cts_buf_desc& d, uint32_t i, uint32_t first,
                                              uint32_t count, cts_verify_result* results, uint64_t* tc,
                                              uint32_t* conn_first_fail, uint32_t n_conns,
                                              cts_verify_result* rslot = nullptr)
{
    const bool pass = (first == kNone);
    if (rslot != nullptr) {
        cts_verify_result r;
        r.first_mismatch = pass ? s.len : first;
        r.mismatch_bytes = pass ? 0u : count;
        r.expected = pass ? 0 : (uint8_t)pattern_byte_dev(s.expected + first);
        r.actual = pass ? 0 : s.sp[first];
        r.pass = pass ? 1 : 0;
        r.flags = 0;
        *rslot = r;
    } else if (results != nullptr) {
        cts_verify_result r;
        r.first_mismatch = pass ? s.len : first;
        r.mismatch_bytes = pass ? 0u : count;
        r.expected = pass ? 0 : (uint8_t)pattern_byte_dev(s.expected + first);
        r.actual = pass ? 0 : s.sp[first];
        r.pass = pass ? 1 : 0;
        r.flags = 0;
        results[i] = r;
    }
    // the team's running counters live in LDS (tc[kCounterCount]), not in 12 VGPRs across the stream loop
    tc[kBytesChecked] += s.len;
    tc[kBuffersChecked] += 1;
    if (pass) {
        tc[kBytesOk] += s.len;
    } else {
        tc[kBuffersFailed] += 1;
        tc[kMismatchedBytes] += count;
        if (conn_first_fail != nullptr && d.conn_index < n_conns &&
            atomicMin(&conn_first_fail[d.conn_index], i) == 0xFFFFFFFFu)
            tc[kConnectionsFailed] += 1;
    }
}

// Per-team running counters in LDS: ctr[team][kCounterCount], zeroed at kernel start.
template <int TEAMS>
__device__ __forceinline__ void zero_counters(uint64_t (*ctr)[kCounterCount])
{
    if (threadIdx.x < (unsigned)(TEAMS * kCounterCount)) ctr[threadIdx.x / kCounterCount][threadIdx.x % kCounterCount] = 0;
    __syncthreads();
}

// Fold the per-team counters of a workgroup and add them to the counter shard
// of this workgroup (one 64-byte line per shard, CTS_COUNTER_SHARDS shards).
template <int TEAMS>
__device__ __forceinline__ void flush_counters(uint64_t* counters, uint64_t (*ctr)[kCounterCount])
{
    __syncthreads();
    if (counters == nullptr) return;
    if (threadIdx.x < (unsigned)kCounterCount) {
        uint64_t sum = 0;
#pragma unroll
        for (int t = 0; t < TEAMS; ++t) sum += ctr[t][threadIdx.x];
        if (sum)
            atomicAdd((unsigned long long*)&counters[(blockIdx.x % CTS_COUNTER_SHARDS) * kCounterSlots + threadIdx.x],
                      (unsigned long long)sum);
    }
}

// Workgroup-wide reduction of (first, count) when some lane saw a mismatch.
// red = 2 * (kBlock/64) u32 of LDS scratch.
__device__ __forceinline__ void block_reduce_mismatch_with(uint32_t& first, uint32_t& count, uint32_t* red)
{
    const uint32_t wave = threadIdx.x / 64;
    first = wave_min(first);
    count = wave_sum(count);
    if ((threadIdx.x & 63) == 0) {
        red[wave] = first;
        red[kBlock / 64 + wave] = count;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) {
            first = red[w] < first ? red[w] : first;
            count += red[kBlock / 64 + w];
        }
    }
    __syncthreads();  // red reused by the next buffer
}

__device__ __forceinline__ void block_reduce_mismatch(uint32_t& first, uint32_t& count)
{
    __shared__ uint32_t red[2 * (kBlock / 64)];
    block_reduce_mismatch_with(first, count, red);
}

// ---------------------------------------------------------------------------------------------
// One 256-lane workgroup per buffer (64 KiB TCP buffers; grid-strides over the descriptors). The next
// buffer's descriptor is fetched while the current one streams. A whole-line span (every buffer of a
// 64 KiB-strided arena whose completion is a multiple of 16 bytes) streams in rounds of kWgLoads 16-byte
// buffer loads per lane with the exact diff in registers (scan_whole_exact); any other span takes the
// edge-first fast pass (scan_buffer) and, when it differs, an exact re-read by the lanes that saw it. The
// per-buffer verdict is workgroup-uniform (__syncthreads_or); only a corrupt buffer reduces (first, count)
// over the workgroup. Registers are allocated for 4 waves per SIMD, the 4 workgroups per CU the launch runs
// at (LaunchGeometry::blocks_per_cu): no SGPR spills in the per-buffer set-up (41.18-41.27 against 41.42-41.45
// us per config-2 launch for the 8-wave allocation, profiles/r04/h/wpe.jsonl).
constexpr int kWgLoads = 2;  // loads per lane per round: 4 workgroups x 4 waves x 2 = 32 KiB in flight per CU

template <bool NT>
__global__ void __launch_bounds__(kBlock, 4)
    verify_wg_kernel(const uint8_t* __restrict__ arena, uint64_t arena_bytes, const cts_buf_desc* __restrict__ descs,
                     uint32_t n, cts_verify_result* __restrict__ results, uint64_t* __restrict__ counters,
                     uint32_t* __restrict__ conn_first_fail, uint32_t n_conns)
{
    __shared__ uint64_t ctr[1][kCounterCount];
    const uint32_t lane = threadIdx.x;
    zero_counters<1>(ctr);
    const uint32_t step = gridDim.x;
    uint32_t i = blockIdx.x;
    cts_buf_desc dn;
    if (i < n) dn = descs[i];
    for (; i < n; i = (uint64_t)i + step < n ? i + step : n) {
        const cts_buf_desc d = dn;
        if ((uint64_t)i + step < n) dn = descs[i + step];
        if (desc_bad(d, arena_bytes)) {
            if (lane == 0) write_bad(results, i);
            continue;
        }
        const Span s = make_span(arena, d);
        uint32_t first = kNone, count = 0;
        bool dirty;
        if (span_giant(s)) {  // >= 2 GiB: 64-bit exact pass
            scan_giant_exact<kBlock, NT>(s, lane, first, count);
            dirty = __builtin_amdgcn_readfirstlane(__syncthreads_or(first != kNone)) != 0;
            if (dirty) block_reduce_mismatch(first, count);
        } else if (__builtin_amdgcn_readfirstlane(span_whole_lines(s) ? 1u : 0u)) {
            // whole-line span, exact diff in registers: only the reduction is left
            scan_whole_exact<kBlock, kWgLoads, NT, true>(s, lane, first, count);
            dirty = __builtin_amdgcn_readfirstlane(__syncthreads_or(first != kNone)) != 0;
            if (dirty) block_reduce_mismatch(first, count);
        } else {
            const uint32_t acc = scan_buffer<kBlock, kWgLoads, NT, true>(s, lane);
            dirty = __builtin_amdgcn_readfirstlane(__syncthreads_or(acc != 0u)) != 0;
            if (dirty) {  // rare: exact re-scan by the dirty lanes + reduction
                if (acc != 0u) scan_exact_owned<kBlock, 2, NT>(s, lane, first, count);
                block_reduce_mismatch(first, count);
            }
        }
        if (lane == 0) finish_buffer(s, d, i, first, count, results, ctr[0], conn_first_fail, n_conns);
    }
    flush_counters<1>(counters, ctr);
}

// ---------------------------------------------------------------------------------------------
// Four buffers per wave: 16-lane teams, one buffer each (datagram-sized spans).
// A whole wave per 1472-byte datagram issues its per-buffer scalar work (descriptor,
// span set-up, edge lanes, record, counters) once per datagram, and a third of its
// lanes' loads fall past the span (4.71 against 5.95 TB/s of payload for this form on
// config 3, tools/rounds/r04/media_stream_probe.py). Here a wave's instructions serve four datagrams at once: the span fields live in VGPRs (one
// descriptor per team), each load instruction fetches four 256-byte runs, and
// U loads per lane cover 16*U chunks per round (U = 6: 1536 B, one round for a
// 1446-byte payload at any alignment). Loads are global (per-lane 64-bit
// addresses: a buffer resource must be wave-uniform); addresses of chunks outside
// a span are clamped into it (same lines, no extra traffic) and their compare is
// discarded. The rounds start on the 128-byte line of chunk 0 (the line-aligned
// interior of scan_buffer), so a team's run covers 2 lines, not 3.
// A team whose OR is nonzero (rare; the verdict is a wave ballot) re-reads its own
// chunks exactly and reduces (first, count) over its 16 lanes.
__device__ __forceinline__ void take_diff_at(uint32_t c, uint32_t lo, u32x4 x, uint32_t& first, uint32_t& count)
{
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t nz = nonzero_bytes(x[w]);
        if (nz) {
            const uint32_t pos = 16u * c + 4u * (uint32_t)w + ((uint32_t)__builtin_ctz(nz) >> 3) - lo;
            first = pos < first ? pos : first;
            count += (uint32_t)__builtin_popcount(nz);
        }
    }
}

constexpr int kQuadTeam = 16;  // lanes per buffer in the four-buffers-per-wave kernels

// A team's span, all fields per lane (VGPRs): the four teams of a wave hold four buffers.
struct QSpan {
    const u32x4* p;     // chunk 0 (16-byte aligned)
    const uint8_t* sp;  // first verified byte
    uint32_t len, nch, hi_last, lo, q0, sh;
    int last;  // address clamp: the last chunk (0 for an empty span)
    int cs;    // first chunk of round 0: the first chunk of chunk 0's 128-byte line (-7..0)
    int c_hi;  // last interior chunk (nch - 2)
};

// Span of [sp, sp + len) at pattern offset `expected`; an empty span (len 0: an idle
// team, a bad descriptor, a non-DATA datagram) points at `dummy`, 16-byte-aligned
// memory the clamped loads may read (every compare of an empty span is discarded).
__device__ __forceinline__ QSpan quad_span(const uint8_t* sp, uint32_t len, uint32_t expected, const void* dummy)
{
    QSpan q;
    q.sp = len ? sp : reinterpret_cast<const uint8_t*>(dummy);
    q.len = len;
    q.lo = (uint32_t)((uintptr_t)q.sp & 15u);
    q.nch = len == 0u ? 0u : (uint32_t)(((uint64_t)q.lo + len + 15u) >> 4);
    q.hi_last = len == 0u ? 0u : (uint32_t)((uint64_t)q.lo + len - 16ull * (q.nch - 1u));
    q.q0 = (expected - q.lo) & 0xFFFFu;
    q.sh = q.q0 & 1u;
    q.p = reinterpret_cast<const u32x4*>(q.sp - q.lo);
    q.last = q.nch == 0u ? 0 : (int)q.nch - 1;
    q.cs = -(int)(((uintptr_t)q.p >> 4) & 7u);
    q.c_hi = (int)q.nch - 2;
    return q;
}

// Edge chunk of a team lane: lane 0 chunk 0, lane 1 the last chunk (others: none).
__device__ __forceinline__ bool quad_edge_used(const QSpan& q, uint32_t lane)
{
    return (lane == 0u && q.nch >= 1u) || (lane == 1u && q.nch >= 2u);
}
__device__ __forceinline__ uint32_t quad_edge_chunk(const QSpan& q, uint32_t lane) { return lane == 1u ? (uint32_t)q.last : 0u; }
__device__ __forceinline__ u32x4 quad_edge_xor(const QSpan& q, uint32_t ce, u32x4 data)
{
    return (data ^ expected_chunk((q.q0 + 16u * ce) & 0xFFFFu, q.sh)) &
           range_mask(ce == 0u ? q.lo : 0u, ce == (uint32_t)q.last ? q.hi_last : 16u);
}

// Interior [1, nch-1) in rounds of U loads per lane starting at chunk cs (the wave loops
// while any of its teams has chunks left); returns the OR of this lane's differences.
// Chunks outside the span are clamped to its first / last chunk.
template <int U, bool NT>
__device__ __forceinline__ uint32_t quad_scan_interior(const QSpan& q, uint32_t lane)
{
    constexpr int ROUND = kQuadTeam * U;
    uint32_t acc = 0;
    for (int r = 0; __any(q.cs + r * ROUND <= q.c_hi); ++r) {
        const int cb = q.cs + r * ROUND + (int)lane;
        u32x4 dd[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int c = cb + u * kQuadTeam;
            c = c < 0 ? 0 : (c > q.last ? q.last : c);
            dd[u] = load_chunk_g<NT>(q.p + c);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t k = ((q.q0 + 16u * (uint32_t)cb) & 0xFFFFu) >> 1;
        const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = cb + u * kQuadTeam;
            const uint32_t any = or4(dd[u] ^ expected_step<kQuadTeam, U>(B, u, q.sh));
            acc |= (c >= 1 && c <= q.c_hi) ? any : 0u;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    return acc;
}

// Exact re-read of exactly the chunks this lane owns (interior chunks = cs + lane mod 16,
// plus its edge chunk): first differing byte (span-relative) and differing-byte count.
template <bool NT>
__device__ __forceinline__ void quad_scan_exact(const QSpan& q, uint32_t lane, uint32_t& first, uint32_t& count)
{
    for (int c = q.cs + (int)lane; c <= q.c_hi; c += kQuadTeam) {
        if (c >= 1)
            take_diff_at((uint32_t)c, q.lo,
                         load_chunk_g<NT>(q.p + c) ^ expected_chunk((q.q0 + 16u * (uint32_t)c) & 0xFFFFu, q.sh), first,
                         count);
    }
    if (quad_edge_used(q, lane)) {
        const uint32_t ce = quad_edge_chunk(q, lane);
        take_diff_at(ce, q.lo, quad_edge_xor(q, ce, load_chunk_g<NT>(q.p + ce)), first, count);
    }
}

// min / sum over the 16 lanes of each team (all lanes of the wave take part)
__device__ __forceinline__ void quad_team_reduce(uint32_t& first, uint32_t& count)
{
#pragma unroll
    for (int off = kQuadTeam / 2; off > 0; off >>= 1) {
        const uint32_t of = (uint32_t)__shfl_xor((int)first, off, kQuadTeam);
        first = of < first ? of : first;
        count += (uint32_t)__shfl_xor((int)count, off, kQuadTeam);
    }
}

// Team-leader running counters (registers), written to LDS once at the end.
struct QCounters {
    uint64_t bytes = 0, ok = 0, mism = 0;
    uint32_t bufs = 0, fail = 0, conns = 0;
    __device__ __forceinline__ void add(uint32_t len, bool pass, uint32_t count)
    {
        bytes += len;
        bufs += 1u;
        if (pass) {
            ok += len;
        } else {
            fail += 1u;
            mism += count;
        }
    }
    template <int TEAMS>
    __device__ __forceinline__ void flush(uint64_t (*ctr)[kCounterCount], uint32_t team, uint32_t lane,
                                          uint64_t* counters) const
    {
        if (lane == 0u) {
            ctr[team][kBytesChecked] = bytes;
            ctr[team][kBytesOk] = ok;
            ctr[team][kBuffersChecked] = bufs;
            ctr[team][kBuffersFailed] = fail;
            ctr[team][kMismatchedBytes] = mism;
            ctr[team][kConnectionsFailed] = conns;
        }
        flush_counters<TEAMS>(counters, ctr);
    }
};

// Per-wave output staging for the four-buffers-per-wave kernels. Each team leader puts its
// 12-byte result (and, for MediaStream, its 32-byte record) in LDS as whole dwords; the wave
// then writes the four teams' outputs from consecutive lanes: one coalesced dword store covers
// 4 x 12 = 48 contiguous result bytes, one covers 4 x 32 = 128 record bytes. Written directly,
// each leader's struct became 4-lane sub-dword and unaligned stores (global_store_short/byte,
// dword at +7): on 4 M datagrams the records alone added 265 us to a 920 us launch
// (tools/rounds/r04/media_stream_probe.py). Nontemporal stores here measured 2-4 % slower; write-through
// (sc1) stores helped the records and hurt the results, and deferring the stores until the next
// buffer's loads were in flight changed nothing (+-0.5 %).
struct QuadOut {
    uint32_t res[4][3];
    uint32_t rec[4][8];
};

__device__ __forceinline__ uint32_t result_dw2(uint32_t expected, uint32_t actual, uint32_t pass, uint32_t flags)
{
    return (expected & 0xFFu) | ((actual & 0xFFu) << 8) | (pass << 16) | (flags << 24);  // bytes 8..11
}

template <typename O>
__device__ __forceinline__ void quad_stage_result(O& o, uint32_t t, uint32_t first_mismatch,
                                                  uint32_t mismatch_bytes, uint32_t dw2)
{
    o.res[t][0] = first_mismatch;
    o.res[t][1] = mismatch_bytes;
    o.res[t][2] = dw2;
}

// All 64 lanes of the wave call this after the leaders staged their results; i = this lane's buffer index
// (the wave's four teams hold i0 .. i0 + 3, i0 = lane 0's), n = buffers in the launch.
__device__ __forceinline__ void quad_flush_results(const QuadOut& o, uint32_t i, uint32_t n, cts_verify_result* results)
{
    __builtin_amdgcn_wave_barrier();
    // (64-bit: i0 + t may pass 2^32 on the wave's last round when n is close to it)
    const uint64_t i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)i);
    const uint32_t l = threadIdx.x & 63u;
    if (results != nullptr && l < 12u) {
        const uint32_t t = l / 3u;
        const uint32_t v = o.res[t][l - 3u * t];
        if (i0 + t < n) reinterpret_cast<uint32_t*>(results)[3ull * i0 + l] = v;
    }
    __builtin_amdgcn_wave_barrier();
}

// The MediaStream receive writes its records + results every kMsRing rounds from the per-wave ring: for config 3
// (1 024 datagrams per workgroup, 64 rounds per wave) once, at the workgroup's end. 4.25 vs 4.30 ms per 16 M
// datagrams written every round (two boxes, profiles/r02/ms_records_ring/); 45 KB of LDS per workgroup.
constexpr int kMsRing = 64;

// Per-wave output ring: the staged outputs of K rounds (QuadOut slots) and each round's first buffer
// index, written by the wave every K rounds instead of every round. A read stream slows down with the
// FREQUENCY of the writes mixed into it, not with their bytes (tools/rw_mix_probe.hip: one dword per wave
// per 4 KiB round costs the read 18 %, the same store on every 16th round 5 %, on every 64th round
// nothing measurable; 4 to 120 bytes per store cost the same).
// A ring slot of the compact receive: four cts_datagram_status entries (4 dwords each), no result records.
struct QuadStatusOut {
    uint32_t rec[4][4];
};

template <int K, typename SlotT = QuadOut>
struct QuadRing {
    SlotT slot[K];
    uint32_t i0[K];
};

// All 64 lanes: write rounds [0, m) of the ring (round j's four buffers start at i0[j]); n = buffers in
// the launch. Records go as agent-scope relaxed atomic dwords, RECDW x 4 per round, results as plain dwords,
// 12 per round.
// RECDW = dwords per record: 8 (cts_datagram_record) or 4 (cts_datagram_status, staged in rec[t][0..3]).
template <int K, int RECDW = 8, typename SlotT = QuadOut>
__device__ __forceinline__ void quad_ring_flush(const QuadRing<K, SlotT>& g, uint32_t m, uint32_t n,
                                                cts_verify_result* results, void* records)
{
    __builtin_amdgcn_wave_barrier();
    const uint32_t l = threadIdx.x & 63u;
    if (records != nullptr) {
#pragma unroll 1  // (unrolled, the LDS reads are hoisted into ~80 VGPRs: occupancy 4 -> 2 waves/SIMD)
        for (uint32_t k = 0; k < (K * 4u * RECDW + 63u) / 64u; ++k) {
            const uint32_t e = k * 64u + l, j = e / (4u * RECDW), d = e % (4u * RECDW);
            if (j < m) {
                const uint64_t i0 = g.i0[j];
                if (i0 + d / RECDW < n)
                    __hip_atomic_store(reinterpret_cast<uint32_t*>(records) + (uint64_t)RECDW * i0 + d,
                                       g.slot[j].rec[d / RECDW][d % RECDW], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if constexpr (!std::is_same<SlotT, QuadStatusOut>::value)
    if (results != nullptr) {
#pragma unroll 1
        for (uint32_t k = 0; k < (K * 12u + 63u) / 64u; ++k) {
            const uint32_t e = k * 64u + l, j = e / 12u, d = e - 12u * j;
            if (j < m) {
                const uint64_t i0 = g.i0[j];
                const uint32_t t = d / 3u;
                if (i0 + t < n) reinterpret_cast<uint32_t*>(results)[3ull * i0 + d] = g.slot[j].res[t][d - 3u * t];
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// Which buffers a team visits: the buffers are cut into chunks of `per` consecutive buffers (a multiple of
// TEAMS); block b walks chunks b, b + grid, ... TEAMS buffers at a time, so the rounds of a wave write adjacent
// outputs and a 128-byte line of 12-byte results fills up in ONE CU's L2 (a grid-stride walk spreads a line over
// workgroups on different XCDs: partial-line writes, 0-5 % slower, tools/rounds/r04/media_stream_probe.py). One chunk per
// block (contig_grid's default) is a fully block-contiguous walk.
template <int TEAMS>
struct QuadWalk {
    uint32_t i, end;
    uint64_t cbase;  // first buffer of the current chunk
    uint32_t per, team;
    __device__ __forceinline__ QuadWalk(uint32_t n, uint32_t per_, uint32_t team_) : end(n), per(per_), team(team_)
    {
        cbase = (uint64_t)blockIdx.x * per;
        i = cbase + team < (uint64_t)n ? (uint32_t)(cbase + team) : n;
    }
    // the buffer after i (end when none); moves to the block's next chunk at a chunk's end
    __device__ __forceinline__ uint32_t next()
    {
        uint64_t nx = (uint64_t)i + TEAMS;
        if (nx - cbase >= per) {
            cbase += (uint64_t)gridDim.x * per;
            nx = cbase + team;
        }
        return nx < (uint64_t)end ? (uint32_t)nx : end;
    }
};

// Where the buffers of a quad-team walk come from: a descriptor array, or (STRIDED) a uniformly strided
// receive ring -- buffer i at i * stride, completed length lens[i], one skip / expected offset /
// connection for the whole ring (a UDP socket's datagrams: skip 26, expected 0), read as 4 bytes of
// metadata per buffer instead of a 24-byte descriptor.
struct VSource {
    const cts_buf_desc* descs;  // !STRIDED
    const uint32_t* lens;       // STRIDED
    uint32_t stride, skip_head, expected, conn_index;
};

template <bool STRIDED>
__device__ __forceinline__ cts_buf_desc vs_desc(const VSource& src, uint32_t i)
{
    if constexpr (STRIDED) {
        const uint32_t len = src.lens[i];
        // a completion longer than its slot would overlap the next one: flagged (an out-of-range
        // expected offset makes desc_bad reject it) rather than read
        return cts_buf_desc{(uint64_t)i * src.stride, len, len <= src.stride ? src.expected : 65536u, src.conn_index,
                            src.skip_head};
    } else {
        return src.descs[i];
    }
}

// U = 6 loads per lane per round: 1536 B per team, one round for a 1446-byte payload at any alignment.
// The two edge chunks are loaded first with the default (L2-allocating) policy, so the lines they bring into L2
// stay there for the round loads that request them again (nontemporal, they sat at L2's LRU position and were
// often gone: config 3, 4 M datagrams, 8 M extra L2 requests and FETCH_SIZE 1.7 % over the arena,
// profiles/r03/dg_probe/).
constexpr int kQuadLoads = 6;

template <bool NT, bool STRIDED>
__global__ void __launch_bounds__(kBlock)
    verify_quad_kernel(const uint8_t* __restrict__ arena, uint64_t arena_bytes, VSource src, uint32_t n,
                       cts_verify_result* __restrict__ results, uint64_t* __restrict__ counters,
                       uint32_t* __restrict__ conn_first_fail, uint32_t n_conns, uint32_t per)
{
    constexpr int TEAMS = kBlock / kQuadTeam;
    __shared__ uint64_t ctr[TEAMS][kCounterCount];
    __shared__ QuadOut qout[kBlock / 64];
    const uint32_t lane = threadIdx.x & (kQuadTeam - 1);
    const uint32_t team = threadIdx.x / kQuadTeam;
    // the dummy target of an empty span's clamped loads: the descriptor array (>= 24 bytes) or, for a
    // strided ring, the arena (>= 16 bytes, 16-aligned), rounded up to 16 bytes
    const void* dummy = STRIDED ? static_cast<const void*>(arena)
                                : reinterpret_cast<const void*>(((uintptr_t)src.descs + 15u) & ~(uintptr_t)15u);
    QCounters qc;
    QuadWalk<TEAMS> w(n, per, team);
    cts_buf_desc dn = vs_desc<STRIDED>(src, w.i < n ? w.i : n - 1u);  // n >= 1 (launch_verify returns early on 0)
    while (__any(w.i < w.end)) {
        const uint32_t i = w.i;
        const cts_buf_desc d = dn;
        const uint32_t inext = w.next();
        dn = vs_desc<STRIDED>(src, inext < n ? inext : n - 1u);  // clamped: no load under a branch
        const bool live = i < w.end;
        const bool ok = live && !desc_bad(d, arena_bytes);
        const QSpan q = quad_span(arena + d.byte_offset + d.skip_head, ok ? d.length - d.skip_head : 0u,
                                  d.expected_pattern_offset, dummy);
        // edge chunks first (their latency hides under the interior rounds)
        const uint32_t ce = quad_edge_chunk(q, lane);
        const u32x4 edge = load_chunk_g<false>(q.p + ce);
        uint32_t acc = quad_scan_interior<kQuadLoads, NT>(q, lane);
        acc |= quad_edge_used(q, lane) ? or4(quad_edge_xor(q, ce, edge)) : 0u;
        uint32_t first = kNone, count = 0;
        if (__any(acc != 0u)) {  // rare: exact re-read of the dirty lanes' own chunks
            if (acc != 0u) quad_scan_exact<NT>(q, lane, first, count);
            quad_team_reduce(first, count);
        }
        if (lane == 0u && live) {
            QuadOut& o = qout[team >> 2];
            if (!ok) {
                quad_stage_result(o, team & 3u, 0u, 0u, result_dw2(0u, 0u, 0u, CTS_RESULT_FLAG_BAD_DESC));
            } else {
                const bool pass = first == kNone;
                if (results != nullptr)
                    quad_stage_result(o, team & 3u, pass ? q.len : first, pass ? 0u : count,
                                      pass ? result_dw2(0u, 0u, 1u, 0u)
                                           : result_dw2(pattern_byte_dev(d.expected_pattern_offset + first),
                                                        q.sp[first], 0u, 0u));
                qc.add(q.len, pass, count);
                if (!pass && conn_first_fail != nullptr && d.conn_index < n_conns &&
                    atomicMin(&conn_first_fail[d.conn_index], i) == 0xFFFFFFFFu)
                    qc.conns += 1u;  // this connection's first recorded failure (kConnectionsFailed)
            }
        }
        quad_flush_results(qout[team >> 2], i, w.end, results);
        w.i = inext;
    }
    qc.flush<TEAMS>(ctr, team, lane, counters);
}

// ---------------------------------------------------------------------------------------------
// fill: the write-bound twin. Interior chunks are 16-byte stores; the (at most
// two) edge chunks of a span write only their own bytes, so neighbouring buffers
// sharing a 16-byte line are never touched.

// Bytes [b0, b1) of the 16-byte chunk e at dst: whole dwords as dword stores, a partial dword as one
// aligned short and/or one byte store (at most 6 stores; a byte loop took up to 15).
__device__ __forceinline__ void store_chunk_bytes(uint8_t* dst, const u32x4& e, uint32_t b0, uint32_t b1)
{
#pragma unroll
    for (uint32_t w = 0; w < 4u; ++w) {
        const uint32_t lo = b0 > 4u * w ? b0 - 4u * w : 0u, hi = b1 < 4u * w + 4u ? (b1 > 4u * w ? b1 - 4u * w : 0u) : 4u;
        if (lo >= hi) continue;
        uint8_t* q = dst + 4u * w;
        const uint32_t v = e[w];
        if (lo == 0u && hi == 4u) {
            *reinterpret_cast<uint32_t*>(q) = v;
            continue;
        }
        uint32_t b = lo;
        if ((b & 1u) && b < hi) {  // odd start: one byte
            q[b] = (uint8_t)(v >> (8u * b));
            ++b;
        }
        if (b + 2u <= hi) {  // an aligned pair
            *reinterpret_cast<uint16_t*>(q + b) = (uint16_t)(v >> (8u * b));
            b += 2u;
        }
        if (b < hi) q[b] = (uint8_t)(v >> (8u * b));  // one byte left
    }
}

template <bool NTS = false>
__device__ __forceinline__ void fill_chunk(u32x4* a0, uint32_t c, uint32_t nchunks, uint32_t q0, uint32_t lo,
                                           uint32_t hi_last)
{
    const u32x4 e = expected_chunk((q0 + 16u * c) & 0xFFFFu, q0 & 1u);
    const bool first_c = (c == 0u);
    const bool last_c = (c == nchunks - 1u);
    const uint32_t b0 = first_c ? lo : 0u;
    const uint32_t b1 = last_c ? hi_last : 16u;
    if (b0 == 0u && b1 == 16u) {
        if constexpr (NTS) __builtin_nontemporal_store(e, a0 + c);
        else a0[c] = e;
    } else {
        store_chunk_bytes(reinterpret_cast<uint8_t*>(a0 + c), e, b0, b1);
    }
}

// A span of whole 16-byte chunks (lo == 0, last chunk full): straight-line rounds of
// U 16-byte buffer stores per lane, the expected words stepped like the verify
// stream; the tail round needs no mask (stores past num_records are dropped).
template <int TEAM, int U, bool EVEN, bool NTS>
__device__ __forceinline__ void fill_whole_rounds(u32x4* p, uint32_t nchunks, uint32_t q0, uint32_t lane)
{
    const uint32_t sh = q0 & 1u;
    typedef u32x4 __attribute__((address_space(1)))* gstore_ptr;
    uint32_t cb = 0;
    for (; cb + (uint32_t)(TEAM * U) <= nchunks; cb += (uint32_t)(TEAM * U)) {  // full rounds: global stores
        const uint32_t k = ((q0 + 16u * (cb + lane)) & 0xFFFFu) >> 1;
        const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
        const gstore_ptr g = (gstore_ptr)(p + cb + lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32x4 e = expected_step<TEAM, U, EVEN>(B, u, sh);
            if constexpr (NTS) __builtin_nontemporal_store(e, g + u * TEAM);
            else g[u * TEAM] = e;
        }
    }
    if (cb < nchunks) {  // tail round: buffer stores past num_records are dropped
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)(nchunks * 16u), 0x00020000);
        const uint32_t k = ((q0 + 16u * (cb + lane)) & 0xFFFFu) >> 1;
        const uint32_t B = __umul24(k, 0x10001u) + 0x10000u;
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(expected_step<TEAM, U, EVEN>(B, u, sh), r,
                                                   (cb + (uint32_t)(u * TEAM) + lane) * 16u, 0u, NTS ? 2 : 0);
    }
}

// NTS: nontemporal stores. Plain stores measured faster for whole 64 KiB buffers (tools/hbm_read_ceiling
// writes: 5.51-5.60 TB/s plain vs 4.98-5.35 nt on the same slab shape), nontemporal for datagrams.
// One buffer's payload (descriptor d: bytes [skip_head, length) at pattern offset expected_pattern_offset) by a team of
// TEAM lanes, FU stores per lane per whole-span round.
template <int TEAM, int FU, bool NTS>
__device__ __forceinline__ void fill_one(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc& d, uint32_t lane)
{
    if (desc_bad(d, arena_bytes)) return;
    const uint32_t len = d.length - d.skip_head;
    if (len == 0) return;
    uint8_t* sp = arena + d.byte_offset + d.skip_head;
    const uint32_t lo = (uint32_t)((uintptr_t)sp & 15u);
    const uint32_t nchunks = (uint32_t)(((uint64_t)lo + len + 15u) >> 4);
    const uint32_t hi_last = (uint32_t)((uint64_t)lo + len - 16ull * (nchunks - 1u));
    const uint32_t q0 = (d.expected_pattern_offset - lo) & 0xFFFFu;
    u32x4* p = reinterpret_cast<u32x4*>(sp - lo);
    // (whole-chunk spans stream buffer stores: 32-bit offsets, so spans >= 2 GiB take the pointer loop)
    if (__builtin_amdgcn_readfirstlane((lo == 0u && hi_last == 16u && nchunks < kGiantChunks) ? 1u : 0u)) {
        if (__builtin_amdgcn_readfirstlane(q0 & 1u) == 0u) fill_whole_rounds<TEAM, FU, true, NTS>(p, nchunks, q0, lane);
        else fill_whole_rounds<TEAM, FU, false, NTS>(p, nchunks, q0, lane);
        return;
    }
    for (uint32_t c = lane; c < nchunks; c += TEAM) fill_chunk<NTS>(p, c, nchunks, q0, lo, hi_last);
}

template <int TEAM, bool NTS = false>
__global__ void __launch_bounds__(kBlock) fill_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                      const cts_buf_desc* __restrict__ descs, uint32_t n)
{
    constexpr int TEAMS = kBlock / TEAM;
    constexpr int FU = TEAM == kBlock ? 4 : 2;  // stores per lane per whole-span round
    const uint32_t lane = threadIdx.x % TEAM;
    const uint32_t team = (TEAM == kBlock) ? 0u : (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x / TEAM);
    const uint32_t step = gridDim.x * TEAMS;
    uint32_t i = blockIdx.x * TEAMS + team;
    // the next buffer's descriptor is loaded while this one's stores go out: with one workgroup per CU
    // nothing else hides a dependent descriptor load per buffer (49.4 -> see DESIGN §3 fill)
    cts_buf_desc dn;
    if (i < n) dn = descs[i];
    for (; i < n; i = (uint64_t)i + step < n ? i + step : n) {
        const cts_buf_desc d = dn;
        if ((uint64_t)i + step < n) dn = descs[i + step];
        fill_one<TEAM, FU, NTS>(arena, arena_bytes, d, lane);
    }
}

// The workgroup path's fill in piece order. Every buffer is cut into ppb pieces of kFillPiece bytes (the last
// piece of a buffer also takes whatever lies past ppb pieces, so any length is filled whatever the hint said);
// pieces are numbered buffer-major and dealt to the workgroups round robin, so at any moment the grid's stores
// cover adjacent pieces -- adjacent buffers of an arena that holds them in order -- rather than one 64 KiB slab per
// workgroup spread over the arena. Rotated over 4 GiB of arenas at one workgroup per CU, plain 16-B stores of the
// pattern write 6.4-6.5 TB/s in this order against 5.5-5.6 in the slab order (tools/write_ceiling_rot.hip,
// profiles/r06/). One workgroup per CU leaves nothing to hide a wave's scalar work between its stores, so the
// pieces of a batch are decoded together: lane m of every wave loads piece m's descriptor and works out its span
// (checks, alignment, chunk range, pattern phase) in vector registers, the next batch's load is issued before this
// batch's stores, and each piece then costs a few readlanes and its stores. (Decoded piece by piece on the scalar
// unit, the same order wrote 3.9 TB/s at one workgroup per CU.)
constexpr uint32_t kFillPiece = 8192;
constexpr int kPieceBatch = 16;

struct PieceJob {   // one piece, decoded by its lane of the batch
    uint64_t base;  // 16-B-aligned address of the span's chunk 0
    uint32_t q0;    // pattern position of chunk 0's first byte
    uint32_t cb, ce;  // chunk range of the piece
    uint32_t nchunks, lo, hi_last;
    uint32_t kind;  // 0 nothing to write, 1 whole 16-B chunks, 2 edge chunks in the range
};

template <uint32_t PIECE>
__device__ __forceinline__ PieceJob decode_piece(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs,
                                                 uint64_t v, uint64_t total, uint32_t ppb, bool mine)
{
    constexpr uint32_t kChunks = PIECE / 16;
    PieceJob j{};
    if (!mine || v >= total) return j;
    const uint32_t i = (uint32_t)(v / ppb), pc = (uint32_t)(v - (uint64_t)i * ppb);
    const cts_buf_desc d = descs[i];
    if (desc_bad(d, arena_bytes) || d.length == d.skip_head) return j;
    const uint32_t len = d.length - d.skip_head;
    const uint64_t sp = (uint64_t)(uintptr_t)arena + d.byte_offset + d.skip_head;
    j.lo = (uint32_t)(sp & 15u);
    j.nchunks = (uint32_t)(((uint64_t)j.lo + len + 15u) >> 4);
    j.hi_last = (uint32_t)((uint64_t)j.lo + len - 16ull * (j.nchunks - 1u));
    j.q0 = (d.expected_pattern_offset - j.lo) & 0xFFFFu;
    j.base = sp - j.lo;
    const uint64_t cb = (uint64_t)pc * kChunks;
    if (cb >= j.nchunks) return j;
    j.cb = (uint32_t)cb;
    j.ce = pc + 1u == ppb ? j.nchunks : (uint32_t)(cb + kChunks < j.nchunks ? cb + kChunks : j.nchunks);
    j.kind = (j.lo == 0u && j.hi_last == 16u) ? 1u : 2u;
    return j;
}

__device__ __forceinline__ uint32_t lane_u32(uint32_t x, int m) { return (uint32_t)__builtin_amdgcn_readlane((int)x, m); }

// (PIECE and BATCH other than the defaults: tools/write_ceiling_rot.hip's sweep only)
template <bool NTS, uint32_t PIECE = kFillPiece, int BATCH = kPieceBatch>
__global__ void __launch_bounds__(kBlock) fill_pieces_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                             const cts_buf_desc* __restrict__ descs, uint32_t n,
                                                             uint32_t ppb)
{
    typedef u32x4 __attribute__((address_space(1)))* gstore_ptr;
    constexpr uint32_t kChunks = PIECE / 16;
    static_assert(PIECE % (16 * kBlock) == 0 && BATCH <= 64, "whole rounds per piece; one lane per piece");
    const uint64_t total = (uint64_t)n * ppb;
    const uint32_t lane = threadIdx.x;
    const uint32_t m_own = lane & 63u;  // every wave decodes the batch for itself (readlane reads the own wave)
    const uint64_t G = gridDim.x;
    PieceJob cur = decode_piece<PIECE>(arena, arena_bytes, descs, blockIdx.x + (uint64_t)m_own * G, total, ppb,
                                       m_own < (uint32_t)BATCH);
    for (uint64_t v0 = blockIdx.x; v0 < total; v0 += (uint64_t)BATCH * G) {
        // the next batch, decoded before this batch's stores. Its load is waited for at once, which also waits for
        // the previous batch's stores (vector loads and stores share one in-order counter): once per batch, the wave
        // cadence that keeps the grid's stores adjacent (no wait 5.6 TB/s, a wait every 1-4 pieces 5.1-6.2, the
        // decode after the stores 5.7, against 6.2 here: profiles/r06/j, l)
        const PieceJob nxt = decode_piece<PIECE>(arena, arena_bytes, descs, v0 + (uint64_t)(BATCH + m_own) * G, total,
                                                 ppb, m_own < (uint32_t)BATCH);
#pragma unroll 1
        for (int m = 0; m < BATCH; ++m) {
            const uint32_t kind = lane_u32(cur.kind, m);
            if (kind == 0u) continue;
            const uint64_t base = ((uint64_t)lane_u32((uint32_t)(cur.base >> 32), m) << 32) | lane_u32((uint32_t)cur.base, m);
            const uint32_t q0 = lane_u32(cur.q0, m), cb = lane_u32(cur.cb, m), ce = lane_u32(cur.ce, m);
            if (kind == 1u) {  // whole 16-byte chunks: straight stores
                const gstore_ptr g = (gstore_ptr)base;
                const uint32_t sh = q0 & 1u;
                if (ce <= cb + kChunks) {  // one piece: kChunks / kBlock stores per lane, unrolled
#pragma unroll
                    for (uint32_t u = 0; u < kChunks / kBlock; ++u) {
                        const uint32_t c = cb + u * kBlock + lane;
                        if (c < ce) {
                            const u32x4 e = expected_chunk((q0 + 16u * c) & 0xFFFFu, sh);
                            if constexpr (NTS) __builtin_nontemporal_store(e, g + c);
                            else g[c] = e;
                        }
                    }
                } else {  // the last piece of a buffer longer than the hint said
                    for (uint32_t c = cb + lane; c < ce; c += kBlock) {
                        const u32x4 e = expected_chunk((q0 + 16u * c) & 0xFFFFu, sh);
                        if constexpr (NTS) __builtin_nontemporal_store(e, g + c);
                        else g[c] = e;
                    }
                }
            } else {  // the edge chunks write only their own bytes
                const uint32_t nchunks = lane_u32(cur.nchunks, m), lo = lane_u32(cur.lo, m),
                               hi_last = lane_u32(cur.hi_last, m);
                u32x4* p = reinterpret_cast<u32x4*>((uintptr_t)base);
                for (uint32_t c = cb + lane; c < ce; c += kBlock) fill_chunk<NTS>(p, c, nchunks, q0, lo, hi_last);
            }
        }
        cur = nxt;
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
// MediaStream (UDP) datagrams, four per wave (16-lane teams; see verify_quad_kernel).
// Receive: parse + validate the header (ctsMediaStreamProtocol.hpp:284-329), then verify the payload of
// DATA datagrams at pattern offset 0 after the 26-byte header (ctsIOPatternMediaStream.cpp:185-192).
// Team lanes 0..2 load the 16-byte chunks holding the header alongside the speculative DATA payload
// stream; the header dwords reach the team leader through DPP row shifts, with no dependent memory round
// trip (header bytes by byte loads and lane shuffles, and one wave per datagram, measured slower:
// tools/rounds/r04/media_stream_probe.py).

// Team lane 0 receives dword c of lane `from`'s u32x4 (from = 1, 2) within its 16-lane DPP
// row (row_shl:from; a VALU move, no LDS round trip).
template <int FROM>
__device__ __forceinline__ uint32_t row_shl(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 | FROM, 0xF, 0xF, true);
}

// Header dwords: team lanes 0..2 each hold one 16-byte chunk of
// the 48-byte window starting at the datagram's 16-byte-aligned base; header byte b sits at
// window byte ho + b. Returns dwords H[0..5] = header bytes 0..23 on team lane 0.
__device__ __forceinline__ void header_dwords_hdr16(u32x4 own, uint32_t ho, uint32_t (&H)[6])
{
    uint32_t W[12];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        W[c] = own[c];
        W[4 + c] = row_shl<1>(own[c]);
        W[8 + c] = row_shl<2>(own[c]);
    }
    // the 7 dwords starting at ho / 4 (a 4-way select each), then a byte funnel by ho % 4
    const uint32_t j0 = ho >> 2, s = ho & 3u;
    uint32_t V[7];
#pragma unroll
    for (int m = 0; m < 7; ++m)
        V[m] = j0 == 0u ? W[m] : (j0 == 1u ? W[m + 1] : (j0 == 2u ? W[m + 2] : W[m + 3]));
#pragma unroll
    for (int k = 0; k < 6; ++k) H[k] = __builtin_amdgcn_alignbyte(V[k + 1], V[k], s);
}

// Where a received datagram sits: a descriptor (cts_media_stream_verify), or slot i of a uniformly
// strided receive ring with its completed length in lens[i] (STRIDED: cts_media_stream_verify_strided,
// 4 B of metadata per datagram instead of a 24-B descriptor).
struct MsSource {
    const cts_buf_desc* descs;  // !STRIDED
    const uint32_t* lens;       // STRIDED
    uint32_t stride;
};

template <bool STRIDED>
__device__ __forceinline__ void ms_datagram(const MsSource& src, uint32_t i, uint64_t& off, uint32_t& len)
{
    if constexpr (STRIDED) {
        off = (uint64_t)i * src.stride;
        len = src.lens[i];
    } else {
        const cts_buf_desc d = src.descs[i];
        off = d.byte_offset;
        len = d.length;
    }
}

// The team leader's staging of its datagram's outputs into slot o (a QuadOut, or a ring slot).
#define CTS_MS_STAGE(o)                                                                                           \
    do {                                                                                                          \
            const uint32_t t = team & 3u;                                                                         \
            if constexpr (STATUS) {                                                                               \
                if (records != nullptr) {                                                                         \
                    /* cts_datagram_status as dwords: seq, completed bytes, flag | kind | pass */ \
                    o.rec[t][0] = data ? (H[0] >> 16) | (H[1] << 16) : 0u;                                        \
                    o.rec[t][1] = data ? (H[1] >> 16) | (H[2] << 16) : 0u;                                        \
                    o.rec[t][2] = completed;                                                                      \
                    o.rec[t][3] = (flag & 0xFFFFu) | (kind << 16) | ((data && first == kNone) ? 1u << 24 : 0u);   \
                }                                                                                                 \
            } else if (records != nullptr) {                                                                      \
                /* cts_datagram_record as dwords: seq = header bytes 2..9 (GetSequenceNumberFromTask); */ \
                /* ctsIOPatternMediaStream.cpp:218-219 read the sender qpc / qpf at bytes 8 and 16 */ \
                o.rec[t][0] = data ? (H[0] >> 16) | (H[1] << 16) : 0u;                                            \
                o.rec[t][1] = data ? (H[1] >> 16) | (H[2] << 16) : 0u;                                            \
                o.rec[t][2] = data ? H[2] : 0u;                                                                   \
                o.rec[t][3] = data ? H[3] : 0u;                                                                   \
                o.rec[t][4] = data ? H[4] : 0u;                                                                   \
                o.rec[t][5] = data ? H[5] : 0u;                                                                   \
                o.rec[t][6] = (flag & 0xFFFFu) | (kind << 16);  /* flag, kind, reserved = 0 */ \
                o.rec[t][7] = completed;                                                                          \
            }                                                                                                     \
            if (!data) {                                                                                          \
                if constexpr (!STATUS)                                                                            \
                quad_stage_result(o, t, 0u, 0u,                                                                   \
                                  result_dw2(0u, 0u, 0u, kind == CTS_DGRAM_BAD_DESC ? CTS_RESULT_FLAG_BAD_DESC    \
                                                                                   : CTS_RESULT_FLAG_NOT_DATA));  \
            } else {                                                                                              \
                const bool pass = first == kNone;                                                                 \
                if constexpr (!STATUS)                                                                            \
                if (results != nullptr)                                                                           \
                    quad_stage_result(o, t, pass ? q.len : first, pass ? 0u : count,                              \
                                      pass ? result_dw2(0u, 0u, 1u, 0u)                                           \
                                           : result_dw2(pattern_byte_dev(first), q.sp[first], 0u, 0u));           \
                qc.add(q.len, pass, count);                                                                       \
            }                                                                                                     \
    } while (0)

// RING: outputs staged in a per-wave ring of RING rounds and written every RING rounds (QuadRing); 0 only with
// FRAMES, which writes no per-datagram outputs.
// STATUS: records points at 16-byte cts_datagram_status entries (results unused).
// FRAMES (cts_media_stream_verify_frames): the client's accounting of the batch, summed on the GPU. The jitter window
// does not move between two render ticks, so CompleteTaskBackToPattern (ctsIOPatternMediaStream.cpp:150-272) over a
// batch is a sum over its clean DATA datagrams: bits received, the bytes of each frame in the window, an error frame
// for each one outside it. Every other datagram is an exception (its lowest index is kept): the client replays such a
// batch datagram by datagram.
constexpr uint32_t kFramesLds = 512;  // window slots summed in LDS per workgroup (larger windows: global atomics)
struct MsFrames {
    int64_t head;         // the window's first sequence number (the jitter queue's head)
    int64_t final_frame;  // m_finalFrame
    uint32_t frames;      // the window's size
    uint32_t finished;    // the stream finished: a zero-byte datagram is no exception
    uint64_t* totals;     // CTS_FRAME_TOTAL_SHARDS x {bits, error frames, datagrams, ~first exception | count << 32}
    uint64_t* frame_bytes;  // [frames]
};

// The header chunks and the payload's edge chunks are loaded ahead of the rounds with the default (L2-allocating)
// policy, as verify_quad_kernel's edges (nontemporal, their lines were often gone from L2 when the rounds asked again).
template <bool NT, bool STRIDED, int RING, bool STATUS = false, bool FRAMES = false>
__global__ void __launch_bounds__(kBlock)
    media_stream_verify_quad_kernel(const uint8_t* __restrict__ arena, uint64_t arena_bytes, MsSource src, uint32_t n,
                                    void* __restrict__ records, cts_verify_result* __restrict__ results,
                                    uint64_t* __restrict__ counters, uint32_t per, MsFrames fr = MsFrames{})
{
    static_assert(RING > 0 || FRAMES, "per-datagram outputs go through the per-wave ring");
    constexpr int U = kQuadLoads;
    constexpr int TEAMS = kBlock / kQuadTeam;
    __shared__ uint64_t s_fbytes[FRAMES ? kFramesLds : 1];  // FRAMES: this workgroup's bytes per window slot
    __shared__ uint64_t s_ftot[4];                          // FRAMES: bits, error frames, datagrams, exceptions
    uint64_t f_bits = 0;
    uint32_t f_err = 0, f_data = 0, f_exc = 0, f_inv_first = 0;
    const bool f_lds = FRAMES && fr.frames <= kFramesLds;
    if constexpr (FRAMES) {
        for (uint32_t k = threadIdx.x; k < kFramesLds; k += kBlock) s_fbytes[k] = 0;
        if (threadIdx.x < 4) s_ftot[threadIdx.x] = 0;
        __syncthreads();
    }
    __shared__ uint64_t ctr[TEAMS][kCounterCount];
    using RingSlot = typename std::conditional<STATUS, QuadStatusOut, QuadOut>::type;
    __shared__ QuadRing<RING ? RING : 1, RingSlot> qring[RING ? kBlock / 64 : 1];
    uint32_t rs = 0;  // RING: this wave's next ring slot (wave-uniform)
    const uint32_t lane = threadIdx.x & (kQuadTeam - 1);
    const uint32_t team = threadIdx.x / kQuadTeam;
    // dummy target of an empty span's clamped loads: 16-byte-aligned bytes the launch owns
    const void* dummy = STRIDED ? reinterpret_cast<const void*>(arena)
                                : reinterpret_cast<const void*>(((uintptr_t)src.descs + 15u) & ~(uintptr_t)15u);
    QCounters qc;
    QuadWalk<TEAMS> w(n, per, team);
    uint64_t noff;
    uint32_t nlen;
    ms_datagram<STRIDED>(src, w.i < n ? w.i : n - 1u, noff, nlen);
    while (__any(w.i < w.end)) {
        const uint32_t i = w.i;
        const uint64_t doff = noff;
        const uint32_t completed = nlen;
        const uint32_t inext = w.next();
        ms_datagram<STRIDED>(src, inext < n ? inext : n - 1u, noff, nlen);  // clamped: no load under a branch
        const bool live = i < w.end;
        const bool bad = doff > arena_bytes || arena_bytes - doff < (uint64_t)completed ||
                         (STRIDED && completed > src.stride);
        const bool in = live && !bad;
        const uint8_t* dg = arena + (in ? doff : 0u);
        u32x4 hch = u32x4{0u, 0u, 0u, 0u};
        const uint32_t ho = (uint32_t)((uintptr_t)dg & 15u);
        // header chunks: the 16-byte-aligned chunks holding bytes [0, min(completed, 26)); a
        // chunk is loaded only if it holds one of those bytes (never past the datagram's page)
        const uint32_t hbytes = completed < CTS_UDP_DATA_HEADER_LENGTH ? completed : CTS_UDP_DATA_HEADER_LENGTH;
        if (in && 16u * lane < ho + hbytes) hch = load_chunk_g<false>(reinterpret_cast<const u32x4*>(dg - ho) + lane);
        // speculative DATA payload: [26, completed) at pattern offset 0
        const bool maybe_data = in && completed >= CTS_UDP_DATA_HEADER_LENGTH;
        const QSpan q = quad_span(dg + CTS_UDP_DATA_HEADER_LENGTH, maybe_data ? completed - CTS_UDP_DATA_HEADER_LENGTH : 0u,
                                  0u, dummy);
        const uint32_t ce = quad_edge_chunk(q, lane);
        const u32x4 edge = load_chunk_g<false>(q.p + ce);
        uint32_t acc = quad_scan_interior<U, NT>(q, lane);
        acc |= quad_edge_used(q, lane) ? or4(quad_edge_xor(q, ce, edge)) : 0u;
        // header dwords, valid on team lane 0; bytes past the completed length are never read (the flag needs
        // completed >= 2, the DATA fields completed >= 26)
        uint32_t H[6];
        header_dwords_hdr16(hch, ho, H);
        // header: ctsMediaStreamMessage::ValidateBufferLengthFromTask (ctsMediaStreamProtocol.hpp:284-329)
        uint32_t flag = 0, kind;
        if (bad) {
            kind = CTS_DGRAM_BAD_DESC;
        } else if (completed == 0u) {
            kind = CTS_DGRAM_ZERO;
        } else if (completed < CTS_UDP_FLAG_LENGTH) {
            kind = CTS_DGRAM_SHORT;
        } else {
            flag = H[0] & 0xFFFFu;
            if (flag == CTS_UDP_FLAG_DATA)
                kind = completed < CTS_UDP_DATA_HEADER_LENGTH ? CTS_DGRAM_SHORT : CTS_DGRAM_DATA;
            else if (flag == CTS_UDP_FLAG_ID)
                kind = completed < CTS_UDP_CONNECTION_ID_HEADER_LENGTH ? CTS_DGRAM_SHORT : CTS_DGRAM_ID;
            else
                kind = CTS_DGRAM_UNKNOWN;
        }
        kind = (uint32_t)__shfl((int)kind, 0, kQuadTeam);  // lane 0's verdict, for every lane
        const bool data = kind == CTS_DGRAM_DATA;
        uint32_t first = kNone, count = 0;
        if (__any(acc != 0u && data)) {  // rare: exact re-read (non-DATA teams' differences are discarded)
            if (acc != 0u && data) quad_scan_exact<NT>(q, lane, first, count);
            quad_team_reduce(first, count);
        }
        if constexpr (FRAMES) {
            if (lane == 0u && live) {
                if (data && first == kNone) {
                    // GetSequenceNumberFromTask: header bytes 2..9; found in the window -> bytes to its frame
                    // (ctsIOPatternMediaStream.cpp:195-265)
                    const int64_t seq = (int64_t)((uint64_t)((H[0] >> 16) | (H[1] << 16)) |
                                                  ((uint64_t)((H[1] >> 16) | (H[2] << 16)) << 32));
                    const uint64_t k = (uint64_t)seq - (uint64_t)fr.head;
                    f_bits += (uint64_t)completed * 8u;
                    ++f_data;
                    if (seq > fr.final_frame || seq < fr.head || k >= fr.frames) {
                        ++f_err;
                    } else if (f_lds) {
                        __hip_atomic_fetch_add(&s_fbytes[k], (uint64_t)completed, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        atomicAdd((unsigned long long*)&fr.frame_bytes[k], (unsigned long long)completed);
                    }
                    qc.add(q.len, true, 0u);
                } else {
                    if (data) qc.add(q.len, false, count);  // a corrupt payload: CorruptedBytes
                    if (!(kind == CTS_DGRAM_ZERO && fr.finished)) {
                        ++f_exc;
                        f_inv_first = f_inv_first > ~i ? f_inv_first : ~i;  // the lowest index: the largest ~i
                    }
                }
            }
            w.i = inext;
            continue;
        }
        if constexpr (RING > 0) {
            if (lane == 0u && live) {
                auto& o_ = qring[team >> 2].slot[rs];
                CTS_MS_STAGE(o_);
            }
            auto& g = qring[team >> 2];
            const uint32_t i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)i);
            if ((threadIdx.x & 63u) == 0u) g.i0[rs] = i0;
            if (++rs == (uint32_t)RING) {
                quad_ring_flush<RING, STATUS ? 4 : 8, RingSlot>(g, RING, w.end, STATUS ? nullptr : results, records);
                rs = 0;
            }
        }
        w.i = inext;
    }
    if constexpr (RING > 0)
        if (rs)
            quad_ring_flush<RING, STATUS ? 4 : 8, RingSlot>(qring[team >> 2], rs, w.end, STATUS ? nullptr : results,
                                                           records);
    if constexpr (FRAMES) {
        // the team leaders' sums -> the workgroup's (LDS) -> one shard of the launch's totals
        uint64_t* const sh = fr.totals + (size_t)(blockIdx.x % CTS_FRAME_TOTAL_SHARDS) * 4u;
        if (lane == 0u) {
            if (f_bits) __hip_atomic_fetch_add(&s_ftot[0], f_bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (f_err) __hip_atomic_fetch_add(&s_ftot[1], (uint64_t)f_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (f_data) __hip_atomic_fetch_add(&s_ftot[2], (uint64_t)f_data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (f_exc) {  // rare: straight to the shard (u32 ~first exception, then u32 count)
                uint32_t* const w3 = reinterpret_cast<uint32_t*>(&sh[3]);
                atomicMax(&w3[0], f_inv_first);
                atomicAdd(&w3[1], f_exc);
            }
        }
        __syncthreads();
        if (f_lds)
            for (uint32_t k = threadIdx.x; k < fr.frames; k += kBlock)
                if (s_fbytes[k]) atomicAdd((unsigned long long*)&fr.frame_bytes[k], (unsigned long long)s_fbytes[k]);
        if (threadIdx.x < 3 && s_ftot[threadIdx.x])
            atomicAdd((unsigned long long*)&sh[threadIdx.x], (unsigned long long)s_ftot[threadIdx.x]);
    }
    qc.flush<TEAMS>(ctr, team, lane, counters);
}

// Send: header {u16 0, i64 seq, i64 qpc, i64 qpf} + P[0 .. length-26) per datagram
// (ctsMediaStreamSendRequests' WSABUF array, ctsMediaStreamProtocol.hpp:230-243).
// A datagram starting on a 16-byte boundary (every slot of a receive-ring-shaped arena, 1472 = 92 x 16) is written
// as whole 16-byte chunks: chunk c holds datagram bytes [16c, 16c + 16), i.e. pattern positions 16c - 26 on, with
// the header's 26 bytes assembled in registers into chunks 0 and 1. Only a partial last chunk writes bytes. (The
// header written bytewise by 26 lanes beside nontemporal payload chunks and 6 byte stores for payload bytes 26..31
// left the first line of every datagram written in pieces: 8.4 -> 7.0 ms for 16 M x 1472 B, tools/rounds/r04/media_stream_probe.py.)
// What still bounds this kernel is latency, not bytes: each datagram's descriptor and header are loaded before its
// stores, one datagram per wave at a time (a one-datagram prefetch was slower: 9.3 ms, tools/ring_fill_probe.hip).
// A ring of datagrams goes through media_stream_fill_ring_kernel instead (cts_media_stream_fill_strided: 4.3 ms).
// One whole datagram (header {0, seq, qpc, qpf} + payload) of descriptor d by one wave.
template <bool NTS>
__device__ __forceinline__ void ms_fill_one(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc& d, uint64_t seq,
                                            uint64_t qpc, uint64_t qpf, uint32_t lane)
{
    if (d.length < CTS_UDP_DATA_HEADER_LENGTH || d.byte_offset > arena_bytes ||
        arena_bytes - d.byte_offset < (uint64_t)d.length)
        return;
    uint8_t* dg = arena + d.byte_offset;
    if (__builtin_amdgcn_readfirstlane(((uintptr_t)dg & 15u) == 0u ? 1u : 0u)) {
        const uint32_t nchunks = (d.length + 15u) >> 4;
        const uint32_t hi_last = d.length - 16u * (nchunks - 1u);
        u32x4* p = reinterpret_cast<u32x4*>(dg);
        for (uint32_t c = lane; c < nchunks; c += 64u) {
            u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
            if (c == 0u)  // flag 0 | seq | qpc bytes 0..5
                e = u32x4{(uint32_t)(seq << 16), (uint32_t)(seq >> 16), (uint32_t)(seq >> 48) | (uint32_t)(qpc << 16),
                          (uint32_t)(qpc >> 16)};
            else if (c == 1u)  // qpc bytes 6..7 | qpf | payload bytes 0..5
                e = u32x4{(uint32_t)(qpc >> 48) | (uint32_t)(qpf << 16), (uint32_t)(qpf >> 16),
                          (uint32_t)(qpf >> 48) | (e[2] & 0xFFFF0000u), e[3]};
            if (c == nchunks - 1u && hi_last != 16u) {
                store_chunk_bytes(reinterpret_cast<uint8_t*>(p + c), e, 0u, hi_last);
            } else {
                if constexpr (NTS) __builtin_nontemporal_store(e, p + c);
                else p[c] = e;
            }
        }
        return;
    }
    if (lane < CTS_UDP_DATA_HEADER_LENGTH) {
        uint8_t b = 0;
        if (lane >= 2u && lane < 10u) b = (uint8_t)(seq >> (8 * (lane - 2u)));
        else if (lane >= 10u && lane < 18u) b = (uint8_t)(qpc >> (8 * (lane - 10u)));
        else if (lane >= 18u) b = (uint8_t)(qpf >> (8 * (lane - 18u)));
        dg[lane] = b;  // flag bytes 0..1 = c_udpDatagramProtocolHeaderFlagData = 0
    }
    const uint32_t len = d.length - CTS_UDP_DATA_HEADER_LENGTH;
    if (len == 0) return;
    uint8_t* sp = dg + CTS_UDP_DATA_HEADER_LENGTH;
    const uint32_t lo = (uint32_t)((uintptr_t)sp & 15u);
    const uint32_t nchunks = (uint32_t)(((uint64_t)lo + len + 15u) >> 4);
    const uint32_t hi_last = (uint32_t)((uint64_t)lo + len - 16ull * (nchunks - 1u));
    const uint32_t q0 = (0u - lo) & 0xFFFFu;
    u32x4* p = reinterpret_cast<u32x4*>(sp - lo);
    for (uint32_t c = lane; c < nchunks; c += 64u) fill_chunk<NTS>(p, c, nchunks, q0, lo, hi_last);
}

// Whole MediaStream datagrams through descriptors (cts_media_stream_fill), batched: each workgroup walks one
// contiguous range of descriptors in batches of kFillBatch, staged in LDS with their headers, and each wave fills a
// contiguous quarter of the batch, one datagram at a time. Nothing is loaded inside the per-datagram loop: the
// wave-per-datagram form waits for a descriptor (a scalar load of a far-away line: ~1 us) before every datagram's
// stores, which bounded it at 3.4-3.9 TB/s on 16 M x 1472 B (6.8-7.0 ms, tools/rounds/r04/media_stream_probe.py). (The same
// batching measured slower for cts_fill's payload-only small buffers, whose first chunk is a partial write either
// way: 6.9 against 6.1-6.8 ms per 16 M x 1446 B, tools/ring_fill_probe.hip.)
constexpr uint32_t kFillBatch = kBlock;

template <bool NTS>
__global__ void __launch_bounds__(kBlock)
    fill_batched_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes, const cts_buf_desc* __restrict__ descs,
                        const cts_datagram_header* __restrict__ headers, uint32_t n)
{
    constexpr uint32_t WAVES = kBlock / 64;
    __shared__ cts_buf_desc ds[kFillBatch];
    __shared__ cts_datagram_header hs[kFillBatch];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t per_wg = (uint32_t)(((uint64_t)n + gridDim.x - 1u) / gridDim.x);
    const uint64_t g0 = (uint64_t)blockIdx.x * per_wg;
    const uint64_t g1 = g0 + per_wg < n ? g0 + per_wg : n;
    for (uint64_t d0 = g0; d0 < g1; d0 += kFillBatch) {
        const uint32_t nb = (uint32_t)(g1 - d0 < kFillBatch ? g1 - d0 : kFillBatch);
        __syncthreads();  // every wave is done with the previous batch
        if (threadIdx.x < nb) {
            ds[threadIdx.x] = descs[d0 + threadIdx.x];
            hs[threadIdx.x] = headers[d0 + threadIdx.x];
        }
        __syncthreads();
        const uint32_t q = (nb + WAVES - 1u) / WAVES;
        const uint32_t t1 = (wave + 1u) * q < nb ? (wave + 1u) * q : nb;
        for (uint32_t t = wave * q; t < t1; ++t) {
            const cts_datagram_header h = hs[t];
            ms_fill_one<NTS>(arena, arena_bytes, ds[t], (uint64_t)h.sequence_number, (uint64_t)h.qpc, (uint64_t)h.qpf,
                             lane);
        }
    }
}


// MediaStream sender over a ring (cts_media_stream_fill_strided): datagram i occupies [i * stride, i * stride +
// lengths[i]) of a 16-byte aligned arena, stride a multiple of 16, so the ring is a flat array of 16-byte chunks and
// chunk k is chunk c = k mod (stride / 16) of datagram k / (stride / 16). A datagram with a length below the header,
// above the stride or past the arena is not written; nor are the bytes between a datagram's end and the next slot.
//
// Each workgroup walks one contiguous range of datagrams in batches of kRingBatch: the batch's headers and lengths
// are loaded into LDS (one vector load per thread, then one wait), and its chunks are cut into four contiguous runs,
// one per wave, written 64 consecutive chunks (1 KiB) per round across datagram boundaries. In the loop nothing is
// loaded from memory: a store never waits on a load (vmcnt counts loads and stores in issue order, so a vector load
// in the loop would wait for every store before it; scalar header loads wait for K$ misses at ~1 us each, and every
// SMEM wait is lgkmcnt(0), so they cannot be prefetched). A round of whole datagrams (the common case) writes its
// header chunks through two lane selects and checks nothing per lane. Measured on 16 M x 1472 B
// (tools/ring_fill_probe.hip, profiles/r03/fill_ring/): 4.6-4.9 ms (5.1-5.4 TB/s) at 4 workgroups per CU; scalar
// per-round header loads 4.4-5.8 ms by form; the descriptor fill 5.1-5.4 ms batched, 6.8-9.0 ms wave per datagram; the
// bare pattern as one span 4.0-4.3 ms.
constexpr uint32_t kRingBatch = 512;

struct RingHeader {
    uint64_t seq, qpc, qpf;
};

__device__ __forceinline__ u32x4 datagram_chunk(uint32_t c, const u32x4& pattern, uint64_t seq, uint64_t qpc,
                                                uint64_t qpf)
{
    if (c == 0u)  // flag 0 | seq | qpc bytes 0..5
        return u32x4{(uint32_t)(seq << 16), (uint32_t)(seq >> 16), (uint32_t)(seq >> 48) | (uint32_t)(qpc << 16),
                     (uint32_t)(qpc >> 16)};
    if (c == 1u)  // qpc bytes 6..7 | qpf | payload bytes 0..5
        return u32x4{(uint32_t)(qpc >> 48) | (uint32_t)(qpf << 16), (uint32_t)(qpf >> 16),
                     (uint32_t)(qpf >> 48) | (pattern[2] & 0xFFFF0000u), pattern[3]};
    return pattern;
}

// e with header h in lanes l0 (chunk 0) and l0 + 1 (chunk 1, whose bytes 10..15 are payload: the pattern e already
// holds there). l0 is wave-uniform and may be outside [0, 64) (wrapped), then no lane matches.
__device__ __forceinline__ u32x4 header_lanes(u32x4 e, uint32_t lane, uint32_t l0, const RingHeader& h)
{
    if (lane == l0) {
        e = u32x4{(uint32_t)(h.seq << 16), (uint32_t)(h.seq >> 16), (uint32_t)(h.seq >> 48) | (uint32_t)(h.qpc << 16),
                  (uint32_t)(h.qpc >> 16)};
    } else if (lane == l0 + 1u) {
        e[0] = (uint32_t)(h.qpc >> 48) | (uint32_t)(h.qpf << 16);
        e[1] = (uint32_t)(h.qpf >> 16);
        e[2] = (uint32_t)(h.qpf >> 48) | (e[2] & 0xFFFF0000u);
    }
    return e;
}

// One chunk with every check: chunk c of datagram j (batch slot t) at ring chunk k.
template <bool NTS>
__device__ __forceinline__ void ring_chunk_checked(u32x4* ring, uint64_t k, uint64_t j, uint32_t c, uint32_t len,
                                                   const RingHeader& h, uint32_t stride, uint64_t arena_bytes)
{
    if (len < CTS_UDP_DATA_HEADER_LENGTH || len > stride || 16u * c >= len || j * stride + len > arena_bytes) return;
    const u32x4 e = datagram_chunk(c, expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u), h.seq,
                                   h.qpc, h.qpf);
    if (16u * c + 16u > len) {
        store_chunk_bytes(reinterpret_cast<uint8_t*>(ring + k), e, 0u, len - 16u * c);
    } else {
        if constexpr (NTS) __builtin_nontemporal_store(e, ring + k);
        else ring[k] = e;
    }
}

// SCALAR: stride >= 1024, so a round holds at most two datagram starts and the wave tracks its datagram and chunk as
// wave-uniform values; otherwise each lane finds its own. full_slots: slots wholly inside the arena (clamped to 2^32-1).
template <bool NTS, bool SCALAR>
__global__ void __launch_bounds__(kBlock)
    media_stream_fill_ring_kernel(uint8_t* __restrict__ arena, uint64_t arena_bytes, uint32_t stride,
                                  const uint32_t* __restrict__ lengths, const cts_datagram_header* __restrict__ headers,
                                  uint32_t n, uint32_t full_slots)
{
    constexpr uint32_t WAVES = kBlock / 64;
    __shared__ RingHeader hs[kRingBatch];
    __shared__ uint32_t ls[kRingBatch];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t cps = stride >> 4;  // chunks per slot
    const uint32_t per_wg = (uint32_t)(((uint64_t)n + gridDim.x - 1u) / gridDim.x);
    const uint64_t g0 = (uint64_t)blockIdx.x * per_wg;
    const uint64_t g1 = g0 + per_wg < n ? g0 + per_wg : n;
    u32x4* const ring = reinterpret_cast<u32x4*>(arena);
    for (uint64_t d0 = g0; d0 < g1; d0 += kRingBatch) {
        const uint32_t nb = (uint32_t)(g1 - d0 < kRingBatch ? g1 - d0 : kRingBatch);
        __syncthreads();  // every wave is done with the previous batch's LDS
        for (uint32_t t = threadIdx.x; t < nb; t += kBlock) {
            const cts_datagram_header h = headers[d0 + t];
            hs[t] = RingHeader{(uint64_t)h.sequence_number, (uint64_t)h.qpc, (uint64_t)h.qpf};
            ls[t] = lengths[d0 + t];
        }
        __syncthreads();
        // this wave's run of the batch's chunks, whole 64-chunk rounds (the last run may end inside one)
        const uint32_t nk = nb * cps;
        const uint32_t per_w = ((nk + WAVES - 1u) / WAVES + 63u) & ~63u;
        uint32_t kl = wave * per_w;
        const uint32_t kl1 = kl + per_w < nk ? kl + per_w : nk;
        const uint64_t kbase = d0 * cps;  // the batch's first ring chunk
        if constexpr (SCALAR) {
            if (kl >= kl1) continue;
            uint32_t ib = kl / cps, cb = kl - ib * cps;  // lane 0's datagram (in the batch) and chunk
            for (; kl < kl1; kl += 64u) {
                const bool crosses = cb + 63u >= cps;
                const uint32_t i1 = ib + 1u < nb ? ib + 1u : ib;
                const uint32_t l0 = ls[ib], l1 = ls[i1];
                const bool whole = kl + 64u <= kl1 && l0 == stride && d0 + ib < full_slots &&
                                   (!crosses || (ib + 1u < nb && l1 == stride && d0 + ib + 1u < full_slots));
                uint32_t c = cb + lane;
                const bool second = c >= cps;
                if (second) c -= cps;
                if (__builtin_amdgcn_readfirstlane(whole ? 1 : 0)) {
                    u32x4 e = expected_chunk((16u * c - CTS_UDP_DATA_HEADER_LENGTH) & 0xFFFFu, 0u);
                    if (cb < 2u) e = header_lanes(e, lane, 0u - cb, hs[ib]);
                    if (crosses) e = header_lanes(e, lane, cps - cb, hs[i1]);
                    if constexpr (NTS) __builtin_nontemporal_store(e, ring + kbase + kl + lane);
                    else ring[kbase + kl + lane] = e;
                } else if (kl + lane < kl1) {
                    const uint32_t t = second ? i1 : ib;
                    ring_chunk_checked<NTS>(ring, kbase + kl + lane, d0 + t, c, ls[t], hs[t], stride, arena_bytes);
                }
                cb += 64u;
                if (cb >= cps) {
                    cb -= cps;
                    ++ib;
                }
            }
        } else {  // stride < 1024: several datagrams per round, each lane finds its own
            for (uint32_t k = kl + lane; k < kl1; k += 64u) {
                const uint32_t t = k / cps, c = k - t * cps;
                ring_chunk_checked<NTS>(ring, kbase + k, d0 + t, c, ls[t], hs[t], stride, arena_bytes);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
static inline uint32_t grid_for(uint32_t n, int teams_per_block, const LaunchGeometry& geo, int bpc_cap = 0)
{
    const uint64_t want = ((uint64_t)n + teams_per_block - 1) / teams_per_block;
    const int bpc = bpc_cap > 0 ? bpc_cap : (teams_per_block > 1 ? geo.small_blocks_per_cu : geo.blocks_per_cu);
    const uint64_t cap = (uint64_t)geo.num_cus * (uint64_t)(bpc > 0 ? bpc : 8);
    // grid-stride with the same number of teams' worth of work per workgroup: past the cap
    // the grid shrinks to ceil(want / per) so no workgroup runs one buffer more than the
    // rest (an uneven split, e.g. 4096 buffers over 1280 workgroups, leaves a tail of
    // workgroups with an extra buffer that alone sets the launch's end)
    const uint64_t per = want <= cap ? 1 : (want + cap - 1) / cap;
    const uint64_t g = (want + per - 1) / per;
    return (uint32_t)(g == 0 ? 1 : g);
}



// Chunked launch of a four-buffers-per-wave kernel (QuadWalk): chunk = geo.small_chunk
// buffers (rounded up to the block's 16 teams); 0 = one block-contiguous range per block, every
// block but the last with the same count.
struct ContigGrid {
    uint32_t grid, per;
};
static inline ContigGrid contig_grid(uint32_t n, const LaunchGeometry& geo)
{
    const uint32_t teams = kBlock / kQuadTeam;
    const uint32_t g = grid_for(n, teams, geo);
    if (geo.small_chunk > 0) {
        const uint64_t per = ((uint64_t)geo.small_chunk + teams - 1) / teams * teams;
        const uint64_t chunks = ((uint64_t)n + per - 1) / per;
        return ContigGrid{(uint32_t)(chunks < g ? chunks : g), (uint32_t)per};
    }
    const uint64_t groups = ((uint64_t)n + teams - 1) / teams;
    const uint64_t per = (groups + g - 1) / g * teams;
    return ContigGrid{(uint32_t)(((uint64_t)n + per - 1) / per), (uint32_t)per};
}

template <bool NT>
static void launch_verify_nt(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                             bool small, cts_verify_result* results, uint64_t* counters, uint32_t* conn_first_fail,
                             uint32_t n_conns, hipStream_t stream, const LaunchGeometry& geo)
{
    if (small) {
        const ContigGrid cg = contig_grid(n, geo);
        verify_quad_kernel<NT, false><<<cg.grid, kBlock, 0, stream>>>(
            arena, arena_bytes, VSource{descs, nullptr, 0u, 0u, 0u, 0u}, n, results, counters, conn_first_fail, n_conns,
            cg.per);
    } else {
        verify_wg_kernel<NT><<<grid_for(n, 1, geo), kBlock, 0, stream>>>(arena, arena_bytes, descs, n, results,
                                                                         counters, conn_first_fail, n_conns);
    }
}

// ---- SYNC mailbox: VerifyBuffer (ctsIOPattern.cpp:745-775) per completion without a launch per call ----
// A resident grid of G groups x kMailGroup workgroups; group g serves its own ring of S job slots.
// Every workgroup of the group sees each job itself (no inter-workgroup hand-off on the critical
// path), splits the job's buffer into 4 KiB pieces (one 16-B system-scope load per lane: the host
// rewrites a reused recv slot between jobs, so nothing may come from a cache), compares them with the
// pattern regenerated in registers, and posts one tagged part record to host memory; the caller folds
// the parts.
//
// Each workgroup is four data waves and one polling wave. Lane 0 of the poller reads the next job's
// slot (one 16-B system-scope load in flight) while the data waves still verify the current one, and
// publishes the job to them through LDS (job, then tag); the data waves fold their results with LDS
// atomics and the last one posts the part record. Pollers never join a barrier, and a publication
// slot is reused (two, by job parity) only after its job was folded. More pollers per workgroup, their
// phases spread over the PCIe round trip, were slower: 2 or 4 polling waves (each on its own copy of
// the slot) gave 9.5 us per 64 KiB verify against 6.3 with one, on the same box (tools/sync_probe) --
// the poll reads compete with the data reads. After kMailHotTicks without a job the poller slows
// down, which keeps idle groups' PCIe reads low (a caller's job goes to the least busy group).
constexpr int kMailAux = 1 | 16;                 // sc0 sc1: system scope
constexpr uint32_t kMailThreads = kBlock + 64;   // four data waves + the polling wave
constexpr uint64_t kMailHotTicks = 5000;         // 50 us (s_memrealtime, 100 MHz)

#if defined(CTS_MAILBOX_TRACE)
// diagnostic builds only (tools/mailbox_bisect.hip): per (job mod 1024, workgroup) the s_memrealtime
// stamps of the publication, the data compared (wave 0), the part record stored, the poll's start, and
// each data wave's compare (4 + wave)
__device__ uint64_t* cts_mail_trace;
#define CTS_MAIL_STAMP(which)                                                                      \
    do {                                                                                           \
        if (cts_mail_trace != nullptr)                                                             \
            cts_mail_trace[((j % 1024u) * kMailGroup + gi) * 8u + (which)] = wall_clock64();       \
    } while (0)
#else
#define CTS_MAIL_STAMP(which) \
    do {                      \
    } while (0)
#endif

// The poller keeps one read of the job slot in flight (two reads half a PCIe round trip apart measured 6.72-6.79 us
// per 64 KiB at one caller against 6.32-6.51 with one, and no gain at 8 / 16 callers: profiles/r03/mailbox_polls_ab/).
__global__ __launch_bounds__(kMailThreads) void mailbox_kernel(const MailSlot* slots, MailPart* parts, uint32_t per_group,
                                                               MailStarts starts, uint64_t idle_ticks,
                                                               uint64_t delay_ticks)
{
    __shared__ uint64_t s_job[2][2];              // published job by parity: ptr_exp, len_seq
    __shared__ uint32_t s_tag[2];                 // its tag, written after the job
    __shared__ uint32_t s_first[2], s_count[2], s_arrive[2];
    __shared__ uint32_t s_done;                   // jobs folded
    const uint32_t g = blockIdx.x / kMailGroup, gi = blockIdx.x % kMailGroup;
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    const uint64_t j0 = starts.j[g];
    const MailSlot* const ring = slots + (size_t)g * per_group;
    if (tid == 0) {
        s_tag[0] = s_tag[1] = (uint32_t)j0;  // j0's tag is j0 + 1: neither parity starts published
        s_first[0] = s_first[1] = kNone;
        s_count[0] = s_count[1] = s_arrive[0] = s_arrive[1] = 0;
        s_done = 0;
    }
    __syncthreads();  // the kernel's only barrier
    // LDS words shared with waves that never meet at a barrier: relaxed workgroup-scope atomics (ds_read /
    // ds_write), ordered by lds_order() -- one wave's LDS operations execute in issue order, so only the
    // compiler has to be kept from reordering them (no fence: a fence would wait for outstanding loads)
#define LDS_LD(x) __hip_atomic_load(&(x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define LDS_ST(x, v) __hip_atomic_store(&(x), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
    const auto lds_order = [] { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };

    if (wave == kBlock / 64) {  // ---- the poller ----
        if (lane != 0) return;
        if (delay_ticks != 0 && g == 0 && gi == kMailGroup - 1) {  // test hook (CTS_MAILBOX_DELAY_MS): a late poller
            const uint64_t t0 = wall_clock64();
            while (wall_clock64() - t0 < delay_ticks) __builtin_amdgcn_s_sleep(127);
        }
        for (uint32_t i = 0;; ++i) {
            const uint64_t j = j0 + i;
            const uint32_t tag = (uint32_t)(j + 1), par = i & 1u;
            while (LDS_LD(s_done) + 1u < i) __builtin_amdgcn_s_sleep(1);  // job i-2 folded: its parity is free
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<MailSlot*>(ring + (uint32_t)(j % per_group)), (short)0, 16, 0x00020000);
            const uint64_t start = wall_clock64();
            CTS_MAIL_STAMP(3);
            u32x4 v;
            // this slot's job arrived (or a later one holds it); idle: no job within idle_ticks
            const auto seen = [&](const u32x4& x) { return x[3] == tag || (int32_t)(x[3] - tag) > 0; };
            const auto idle = [&](bool& leave) {
                const uint64_t waited = wall_clock64() - start;
                leave = waited > idle_ticks;
                if (waited > kMailHotTicks) __builtin_amdgcn_s_sleep(40);
            };
            bool leave = false;
            for (;;) {
                v = __builtin_amdgcn_raw_buffer_load_b128(r, 0u, 0u, kMailAux);
                if (seen(v)) break;
                idle(leave);
                if (leave) break;
                __builtin_amdgcn_s_sleep(2);
            }
            if (leave) {
                v = u32x4{0u, 0u, 0u, ~tag};  // no job within idle_ticks: publish one whose tag word is not the tag
            } else if (v[3] != tag) {
                // a later job already holds this slot: the host reuses a slot only once every part record of its
                // job was folded (or at once for a no-op), so job j needed nothing from this workgroup; take it as a
                // no-op and catch up (a workgroup that fell per_group jobs behind would otherwise wait for a tag
                // that never comes back)
                v = u32x4{0u, 0u, kMailSkip, tag};
            }
            LDS_ST(s_job[par][0], (uint64_t)v[0] | ((uint64_t)v[1] << 32));
            LDS_ST(s_job[par][1], (uint64_t)v[2] | ((uint64_t)v[3] << 32));
            lds_order();
            LDS_ST(s_tag[par], tag);
            CTS_MAIL_STAMP(0);
            if (v[3] != tag || v[2] == 0u) return;  // idle leave or stop
        }
    }

    // ---- data waves ----
    for (uint32_t i = 0;; ++i) {
        const uint64_t j = j0 + i;
        const uint32_t tag = (uint32_t)(j + 1), par = i & 1u;
        while (LDS_LD(s_tag[par]) != tag) __builtin_amdgcn_s_sleep(1);
        lds_order();
        const uint64_t ptr_exp = LDS_LD(s_job[par][0]), len_seq = LDS_LD(s_job[par][1]);
        if ((uint32_t)(len_seq >> 32) != tag) return;  // idle leave
        const uint64_t ptr = ptr_exp & 0xFFFFFFFFFFFFull;
        const uint32_t expected = (uint32_t)(ptr_exp >> 48), len = (uint32_t)len_seq;
        const bool mine = len != kMailSkip && gi < mail_parts(ptr, len);
        const uint32_t d = (uint32_t)ptr & 15u;
        const uint8_t* const base = reinterpret_cast<const uint8_t*>(ptr - d);
        uint32_t first = kNone, count = 0;
        if (mine && len != 0) {
            const uint64_t nchunks = ((uint64_t)d + len + 15u) >> 4;
            const uint32_t pieces = (uint32_t)((nchunks * 16u + kMailPieceBytes - 1) / kMailPieceBytes);
            const uint32_t q_base = (expected + 65536u - d) & 0xFFFFu;  // pattern position of base[0]
            const uint32_t hi_last = ((d + len - 1u) & 15u) + 1u;
            for (uint32_t u0 = gi; u0 < pieces; u0 += 4 * kMailGroup) {
                u32x4 v[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {  // four pieces' loads in flight before any compare
                    const uint32_t u = u0 + jj * kMailGroup;
                    const uint64_t off = (uint64_t)u * kMailPieceBytes;
                    const uint64_t rem = u < pieces ? nchunks * 16u - off : 0u;
                    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                        const_cast<uint8_t*>(base + (u < pieces ? off : 0u)), (short)0,
                        (int)(rem < kMailPieceBytes ? rem : kMailPieceBytes), 0x00020000);
                    v[jj] = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0u, kMailAux);
                }
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const uint64_t c = (uint64_t)(u0 + jj * kMailGroup) * (kMailPieceBytes / 16u) + tid;
                    if (u0 + jj * kMailGroup >= pieces || c >= nchunks) continue;
                    const uint32_t q = (uint32_t)((q_base + c * 16u) & 0xFFFFu);
                    u32x4 x = v[jj] ^ expected_chunk(q, q & 1u);
                    if (c == 0 || c == nchunks - 1) x &= range_mask(c == 0 ? d : 0u, c == nchunks - 1 ? hi_last : 16u);
                    if (or4(x) == 0u) continue;
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const uint32_t nz = nonzero_bytes(x[w]);
                        if (nz == 0u) continue;
                        const uint32_t pos = (uint32_t)(c * 16u - d) + 4u * w + ((uint32_t)__builtin_ctz(nz) >> 3);
                        first = pos < first ? pos : first;
                        count += (uint32_t)__builtin_popcount(nz);
                    }
                }
            }
        }
        first = wave_min(first);
        count = wave_sum(count);
        if (tid == 0) CTS_MAIL_STAMP(1);
        if (lane == 0) CTS_MAIL_STAMP(4 + wave);
        if (lane == 0) {
            __hip_atomic_fetch_min(&s_first[par], first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(&s_count[par], count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            lds_order();
            if (__hip_atomic_fetch_add(&s_arrive[par], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ==
                kBlock / 64 - 1) {  // the last data wave: post the part record, free the parity
                lds_order();
                const uint32_t f = LDS_LD(s_first[par]);
                const uint32_t n = LDS_LD(s_count[par]);
                if (mine) {
                    MailPart* const out = parts + ((size_t)g * per_group + (uint32_t)(j % per_group)) * kMailGroup + gi;
                    uint64_t g0 = 0xFFFFFFFFull | ((uint64_t)tag << 32), g1 = (uint64_t)(tag & 0xFFFFFFu) << 40;
                    if (len != 0) {
                        uint32_t actual = 0;
                        if (f != kNone) {  // the received byte there (ctsIOPattern.cpp:761-772 prints it)
                            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                                const_cast<uint8_t*>(base + d + f), (short)0, 1, 0x00020000);
                            actual = (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, 0u, 0u, kMailAux);
                        }
                        g0 = (uint64_t)f | ((uint64_t)tag << 32);
                        g1 |= (uint64_t)n | ((uint64_t)actual << 32);
                    }
                    __hip_atomic_store(&out->g0, g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(&out->g1, g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    CTS_MAIL_STAMP(2);
                }
                LDS_ST(s_first[par], kNone);
                LDS_ST(s_count[par], 0u);
                LDS_ST(s_arrive[par], 0u);
                lds_order();
                LDS_ST(s_done, i + 1u);
            }
        }
        if (len == 0) return;  // stop: acknowledged above
    }
#undef LDS_LD
#undef LDS_ST
}

hipError_t launch_mailbox(const MailSlot* slots, MailPart* parts, uint32_t per_group, const MailStarts& starts,
                          uint32_t groups, uint64_t idle_ticks, hipStream_t stream, uint64_t delay_ticks)
{
    if (slots == nullptr || parts == nullptr || per_group == 0 || groups == 0 || groups > kMailMaxGroups)
        return hipErrorInvalidValue;
    mailbox_kernel<<<groups * kMailGroup, kMailThreads, 0, stream>>>(slots, parts, per_group, starts, idle_ticks,
                                                                     delay_ticks);
    return hipGetLastError();
}

// ---- counter fold (cts_counters_allreduce): one lane per shard, the kCounterCount sums by lanes 0.. ----
static_assert(CTS_COUNTER_SHARDS == 64, "one lane per counter shard");
__global__ void __launch_bounds__(64) counters_fold_kernel(const uint64_t* __restrict__ block, uint64_t* __restrict__ out,
                                                           int accumulate)
{
    __shared__ uint64_t part[CTS_COUNTER_SHARDS][kCounterCount];
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (int k = 0; k < kCounterCount; ++k) part[t][k] = block[t * kCounterSlots + k];
    __syncthreads();
    if (t < (uint32_t)kCounterCount) {
        uint64_t s = accumulate ? out[t] : 0u;
        for (uint32_t sh = 0; sh < CTS_COUNTER_SHARDS; ++sh) s += part[sh][t];
        out[t] = s;
    }
}

hipError_t launch_counters_fold(const void* block, uint64_t* out, bool accumulate, hipStream_t stream)
{
    if (block == nullptr || out == nullptr) return hipErrorInvalidValue;
    counters_fold_kernel<<<1, 64, 0, stream>>>(static_cast<const uint64_t*>(block), out, accumulate ? 1 : 0);
    return hipGetLastError();
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

// cts_verify_strided: the small-buffer walk (verify_quad_kernel) over a uniformly strided ring
hipError_t launch_verify_strided(const uint8_t* arena, uint64_t arena_bytes, uint32_t stride, const uint32_t* lens,
                                 uint32_t n, uint32_t skip_head, uint32_t expected, uint32_t conn_index,
                                 cts_verify_result* results, uint64_t* counters, uint32_t* conn_first_fail,
                                 uint32_t n_conns, hipStream_t stream, const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    const VSource src{nullptr, lens, stride, skip_head, expected, conn_index};
    const ContigGrid cg = contig_grid(n, geo);
    if (geo.nontemporal)
        verify_quad_kernel<true, true><<<cg.grid, kBlock, 0, stream>>>(arena, arena_bytes, src, n, results, counters,
                                                                       conn_first_fail, n_conns, cg.per);
    else
        verify_quad_kernel<false, true><<<cg.grid, kBlock, 0, stream>>>(arena, arena_bytes, src, n, results, counters,
                                                                        conn_first_fail, n_conns, cg.per);
    return hipGetLastError();
}

// grid of the batched datagram fills: whole batches per workgroup, at most ring_fill_blocks_per_cu per CU
static inline uint32_t batched_fill_grid(uint32_t n, const LaunchGeometry& geo)
{
    const uint64_t cap = (uint64_t)geo.num_cus * (uint64_t)(geo.ring_fill_blocks_per_cu > 0 ? geo.ring_fill_blocks_per_cu : 4);
    const uint64_t want = ((uint64_t)n + kFillBatch - 1) / kFillBatch;
    return (uint32_t)(want < cap ? want : cap);
}

hipError_t launch_fill(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                       uint32_t max_length_hint, hipStream_t stream, const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    const bool small = max_length_hint != 0 && max_length_hint <= (uint32_t)geo.small_threshold;
    // store policy: fill_nt 0 = plain, 1 = nontemporal, 2 = by path (plain for the workgroup path:
    // config 2 48.7 vs 51.1 us; nontemporal for datagrams: 1.46 vs 1.68 ms per 4 M; tools/rounds/r04/tune_verify.py --op fill)
    const bool nts = geo.fill_nt == 2 ? small : geo.fill_nt != 0;
    const uint32_t sgrid = grid_for(n, kBlock / 64, geo), lgrid = grid_for(n, 1, geo, geo.fill_blocks_per_cu);
    if (!small && max_length_hint != 0) {  // the workgroup path in piece order (fill_pieces_kernel)
        const uint32_t ppb = (uint32_t)(((uint64_t)max_length_hint + kFillPiece - 1) / kFillPiece);
        const uint64_t total = (uint64_t)n * ppb;
        const uint64_t cap = (uint64_t)geo.num_cus * (uint64_t)(geo.fill_blocks_per_cu > 0 ? geo.fill_blocks_per_cu : 1);
        const uint32_t pgrid = (uint32_t)(total < cap ? total : cap);
        if (nts) fill_pieces_kernel<true><<<pgrid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n, ppb);
        else fill_pieces_kernel<false><<<pgrid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n, ppb);
        return hipGetLastError();
    }
    if (nts) {
        if (small) fill_kernel<64, true><<<sgrid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n);
        else fill_kernel<kBlock, true><<<lgrid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n);
    } else {
        if (small) fill_kernel<64><<<sgrid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n);
        else fill_kernel<kBlock><<<lgrid, kBlock, 0, stream>>>(arena, arena_bytes, descs, n);
    }
    return hipGetLastError();
}

// The MediaStream receive: four datagrams per wave walking block-contiguous ranges (contig_grid), records + results
// staged in a per-wave LDS ring and written every kMsRing rounds (for config 3 once, at the workgroup's end).
hipError_t launch_media_stream_verify(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                                     cts_datagram_record* records, cts_verify_result* results, uint64_t* counters,
                                     hipStream_t stream, const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    const ContigGrid cg = contig_grid(n, geo);
    const MsSource src{descs, nullptr, 0u};
    if (geo.nontemporal)
        media_stream_verify_quad_kernel<true, false, kMsRing><<<cg.grid, kBlock, 0, stream>>>(
            arena, arena_bytes, src, n, records, results, counters, cg.per);
    else
        media_stream_verify_quad_kernel<false, false, kMsRing><<<cg.grid, kBlock, 0, stream>>>(
            arena, arena_bytes, src, n, records, results, counters, cg.per);
    return hipGetLastError();
}

hipError_t launch_media_stream_verify_strided(const uint8_t* arena, uint64_t arena_bytes, uint32_t stride,
                                             const uint32_t* lengths, uint32_t n, cts_datagram_record* records,
                                             cts_verify_result* results, uint64_t* counters, hipStream_t stream,
                                             const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    // the same walk over the ring's slots
    const ContigGrid cg = contig_grid(n, geo);
    const MsSource src{nullptr, lengths, stride};
    if (geo.nontemporal)
        media_stream_verify_quad_kernel<true, true, kMsRing><<<cg.grid, kBlock, 0, stream>>>(
            arena, arena_bytes, src, n, records, results, counters, cg.per);
    else
        media_stream_verify_quad_kernel<false, true, kMsRing><<<cg.grid, kBlock, 0, stream>>>(
            arena, arena_bytes, src, n, records, results, counters, cg.per);
    return hipGetLastError();
}

hipError_t launch_media_stream_status(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs,
                                     const uint32_t* lengths, uint32_t stride, uint32_t n, cts_datagram_status* status,
                                     uint64_t* counters, hipStream_t stream, const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    // one pass over descriptors, or (descs == nullptr) the strided ring: the receive walk, each wave staging its
    // datagrams' 16-byte statuses in an LDS ring and writing 64 rounds of them at a time -- for config 3 (1024
    // datagrams per workgroup) once, at the workgroup's end. Per 16 M datagrams 4.30-4.31 ms against 4.44 with 32
    // rounds and 4.54 written every round, one box (profiles/r02/ms_status/); a two-pass form (headers -> statuses,
    // then the payload clearing pass on failures) measured 4.25 against 4.08 ms (the header gather's scattered
    // 16-byte reads cost more than the writes it takes out of the payload pass)
    const ContigGrid cg = contig_grid(n, geo);
    const MsSource src{descs, lengths, stride};
#define CTS_MS_STATUS(NT, STR)                                                                                \
    media_stream_verify_quad_kernel<NT, STR, 64, true><<<cg.grid, kBlock, 0, stream>>>(arena, arena_bytes, src, n, \
                                                                                       status, nullptr, counters, \
                                                                                       cg.per)
    if (descs == nullptr) {
        if (geo.nontemporal) CTS_MS_STATUS(true, true);
        else CTS_MS_STATUS(false, true);
    } else {
        if (geo.nontemporal) CTS_MS_STATUS(true, false);
        else CTS_MS_STATUS(false, false);
    }
#undef CTS_MS_STATUS
    return hipGetLastError();
}

hipError_t launch_media_stream_frames(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs,
                                     const uint32_t* lengths, uint32_t stride, uint32_t n, const cts_frame_window& win,
                                     uint64_t* totals, uint64_t* frame_bytes, uint64_t* counters, hipStream_t stream,
                                     const LaunchGeometry& geo)
{
    // the sums start from zero on the launch's stream (a batch's totals, not a running sum); frame bytes placed right
    // after the totals (the pattern's layout) are cleared with them in one call
    const size_t tb = (size_t)CTS_FRAME_TOTAL_SHARDS * 4u * sizeof(uint64_t);
    const bool adjacent = frame_bytes == totals + CTS_FRAME_TOTAL_SHARDS * 4u;
    hipError_t err = hipMemsetAsync(totals, 0, tb + (adjacent ? (size_t)win.frames * 8u : 0u), stream);
    if (err == hipSuccess && win.frames != 0 && !adjacent)
        err = hipMemsetAsync(frame_bytes, 0, (size_t)win.frames * 8u, stream);
    if (err != hipSuccess || n == 0) return err;
    // descs == nullptr: the strided-ring form; the variant-3 walk without per-datagram outputs
    const ContigGrid cg = contig_grid(n, geo);
    const MsSource src{descs, lengths, stride};
    const MsFrames fr{win.head_sequence_number, win.final_frame, win.frames, win.finished, totals, frame_bytes};
#define CTS_MS_FRAMES(NT, STR)                                                                        \
    media_stream_verify_quad_kernel<NT, STR, 0, false, true><<<cg.grid, kBlock, 0, stream>>>(           \
        arena, arena_bytes, src, n, nullptr, nullptr, counters, cg.per, fr)
    if (descs == nullptr) {
        if (geo.nontemporal) CTS_MS_FRAMES(true, true);
        else CTS_MS_FRAMES(false, true);
    } else {
        if (geo.nontemporal) CTS_MS_FRAMES(true, false);
        else CTS_MS_FRAMES(false, false);
    }
#undef CTS_MS_FRAMES
    return hipGetLastError();
}

hipError_t launch_media_stream_fill(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs,
                                   const cts_datagram_header* headers, uint32_t n, hipStream_t stream,
                                   const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    // store policy: fill_nt 0 or 2 (by path) = plain, 1 = nontemporal (batched: 5.08 ms plain vs 5.37 nt per 16 M x
    // 1472 B, tools/ring_fill_probe.hip)
    const bool nts = geo.fill_nt == 1;
    const uint32_t grid = batched_fill_grid(n, geo);
    if (nts) fill_batched_kernel<true><<<grid, kBlock, 0, stream>>>(arena, arena_bytes, descs, headers, n);
    else fill_batched_kernel<false><<<grid, kBlock, 0, stream>>>(arena, arena_bytes, descs, headers, n);
    return hipGetLastError();
}

hipError_t launch_media_stream_fill_strided(uint8_t* arena, uint64_t arena_bytes, uint32_t stride, const uint32_t* lengths,
                                           const cts_datagram_header* headers, uint32_t n, hipStream_t stream,
                                           const LaunchGeometry& geo)
{
    if (n == 0) return hipSuccess;
    // (stride <= 1 MiB keeps a batch's chunk count, 512 x stride / 16, in 32 bits; a UDP datagram is < 64 KiB)
    if ((stride & 15u) != 0u || stride < 32u || stride > (1u << 20) || ((uintptr_t)arena & 15u) != 0u)
        return hipErrorInvalidValue;
    const uint64_t cap = (uint64_t)geo.num_cus * (uint64_t)(geo.ring_fill_blocks_per_cu > 0 ? geo.ring_fill_blocks_per_cu : 4);
    // every workgroup gets at least a batch's worth of datagrams, or the whole ring
    const uint64_t want = ((uint64_t)n + kRingBatch - 1) / kRingBatch;
    const uint32_t grid = (uint32_t)(want < cap ? want : cap);
    const uint64_t slots = arena_bytes / stride;
    const uint32_t full_slots = (uint32_t)(slots < 0xFFFFFFFFull ? slots : 0xFFFFFFFFull);
    const bool nts = geo.fill_nt != 0;
#define CTS_RING_FILL(NT_, SC_)                                                                                   \
    media_stream_fill_ring_kernel<NT_, SC_><<<grid, kBlock, 0, stream>>>(arena, arena_bytes, stride, lengths, headers, n, \
                                                                         full_slots)
    if (stride >= 1024u) {
        if (nts) CTS_RING_FILL(true, true);
        else CTS_RING_FILL(false, true);
    } else {
        if (nts) CTS_RING_FILL(true, false);
        else CTS_RING_FILL(false, false);
    }
#undef CTS_RING_FILL
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
