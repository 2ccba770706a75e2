// cts_internal.hpp — launchers shared between the kernel TU and the C-ABI TU.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include "cts_engine.h"
#include "cts_media_stream.h"

namespace cts {

// Device counter block: CTS_COUNTER_SHARDS rows of 8 u64 (64 B each); a
// workgroup adds its totals to row (blockIdx.x % CTS_COUNTER_SHARDS) so the
// adds of a 2048-block grid spread over 64 lines instead of one.
constexpr int kCounterSlots = 8;  // kCounterCount used, padded to one 64-byte line
enum CounterSlot {
    kBytesChecked = 0,
    kBytesOk = 1,
    kBuffersChecked = 2,
    kBuffersFailed = 3,
    kMismatchedBytes = 4,
    // conn_first_fail slots a launch moved off 0xFFFFFFFF: the atomicMin that returned the empty value is the
    // connection's first recorded failure, so each failed connection counts once however many of its buffers fail
    // and however many launches share the slot array (ctsSocketState.cpp:221-228, m_protocolErrorCount)
    kConnectionsFailed = 5
};
constexpr int kCounterCount = 6;
static_assert(kCounterCount <= kCounterSlots, "counters fit a shard line");

// The folded sums v[kCounterCount] as the ABI's structs.
inline cts_counters_ex counters_ex_of(const uint64_t* v)
{
    return cts_counters_ex{v[kBytesChecked],  v[kBytesOk],         v[kBuffersChecked],
                           v[kBuffersFailed], v[kMismatchedBytes], v[kConnectionsFailed]};
}
inline cts_counters counters_of(const cts_counters_ex& x)
{
    return cts_counters{x.bytes_checked, x.bytes_ok, x.buffers_checked, x.buffers_failed, x.mismatched_bytes};
}

// One kernel per path. CTS_ATTR_VERIFY_VARIANT / SMALL_VARIANT / MS_VARIANT report which one, by the number it
// had among the alternatives measured in rounds 1-4; setting any other value is CTS_E_INVALID.
constexpr int kVerifyKernelId = 25;       // verify_wg_kernel: U2 whole-line exact stream, 4 waves per SIMD (round 4)
constexpr int kSmallKernelId = 15;        // verify_quad_kernel: block-contiguous, edge loads L2-allocating (round 3)
constexpr int kMediaStreamKernelId = 3;   // media_stream_verify_quad_kernel: DPP header, per-wave output ring

struct LaunchGeometry {
    int num_cus = 256;        // hipDeviceAttributeMultiprocessorCount
    int blocks_per_cu = 4;        // workgroup-per-buffer grid cap = num_cus * this (grid-stride beyond);
                                  // 4 x 4 waves x U2 = 32 KiB of loads in flight per CU measured best
                                  // (config 2: 41.0-41.2 us vs 42.6-43.9 at 8; tools/rounds/r04/tune_verify.py)
    int small_blocks_per_cu = 64; // small-buffer (quad) path grid cap
    int nontemporal = 1;      // nt loads for the once-read verify stream
    int small_threshold = 8192;  // max_length_hint <= this -> small-buffer path
    int small_chunk = 0;         // chunked walk of the quad kernels: buffers per chunk (0 = one contiguous range per
                                 // workgroup)
    int fill_nt = 2;             // fill store policy: 0 plain, 1 nontemporal, 2 by path (plain for the workgroup
                                 // path, nontemporal for datagrams; tools/rounds/r04/tune_verify.py --op fill)
    int fill_blocks_per_cu = 1;  // fill grid cap (write-bound; plain stores: 1 measured best, 48.7 vs 49.1-49.4 us)
    int ring_fill_blocks_per_cu = 4;  // MediaStream ring fill grid cap (16 M x 1472 B: 4.3 ms at 4, 5.0 at 8;
                                      // CTS_RING_FILL_BLOCKS_PER_CU; tools/ring_fill_probe.hip)
};

// ---- SYNC mailbox (cts_verify_mapped): a resident verify grid fed through pinned host memory ----
// Host-coherent pinned memory (hipHostMallocCoherent) holds G rings of S 64-B job slots, one ring per
// group, and one 16-B part record per (slot, piece). Group g's j-th job (j counts per group) uses
// slot g * S + j mod S and carries the tag j + 1. The caller writes the job's first 8 bytes, then the 8
// bytes carrying the sequence tag, so the grid's single 16-B read of a slot never sees a new tag
// with an old job. Every workgroup that verified a piece answers with one 16-B part record whose two
// 8-byte halves each carry the ticket's tag (each half is one naturally aligned 8-B store, so a
// half is never torn); the caller folds the parts: min of first differing bytes, sum of counts.
struct alignas(64) MailSlot {
    uint64_t ptr_exp;  // device address (bits 0-47) | expected pattern offset << 48
    uint64_t len_seq;  // length (bits 0-31; 0 = stop: the grid exits) | (j + 1) << 32
    uint64_t pad[6];
};
static_assert(sizeof(MailSlot) == 64, "one cache line per slot");
// Host side: the job half, then the tagged half (x86 keeps the two stores in order), so the grid's one
// 16-B read of a slot never sees a new tag with an old job.
inline void mail_write(MailSlot* s, uint64_t ptr_exp, uint64_t len_seq)
{
    __atomic_store_n(&s->ptr_exp, ptr_exp, __ATOMIC_RELAXED);
    __atomic_store_n(&s->len_seq, len_seq, __ATOMIC_RELEASE);
}
struct alignas(16) MailPart {
    uint64_t g0;  // first differing byte of the piece(s), 0xFFFFFFFF = none | (j + 1) << 32
    uint64_t g1;  // differing bytes | received byte at g0's first << 32 | ((j + 1) & 0xFFFFFF) << 40
};
constexpr uint32_t kMailPieceBytes = 4096;  // one 16-B load per lane of a 256-lane workgroup
// The grid is G groups of kMailGroup workgroups; a group's workgroups alone poll its ring and verify
// its jobs' pieces (piece u by workgroup u mod kMailGroup of the group, up to four pieces per workgroup
// per round, their loads in flight together). The caller gives each job to the group with the fewest jobs
// outstanding, so one caller keeps one group busy and the others idle. Four workgroups cover a 64 KiB
// buffer in one PCIe round trip. Every workgroup polls its group's slot, and the pollers' PCIe reads
// compete with the data reads: 16 workgroups per group answered a 64 KiB verify in 6.1-6.7 / 26.2-26.3 /
// 42.3-42.5 us at 1 / 8 / 16 callers, 8 in 5.8-6.7 / 12.8-19.0 / 32.6-36.9, 4 in 5.5 / 11.5-11.8 / 28.1-29.1
// (tools/sync_probe, tools/mailbox_group_ab.sh, profiles/r02/mailbox_group_ab.jsonl).
#ifndef CTS_MAIL_GROUP
#define CTS_MAIL_GROUP 4  // (a -D override builds the A/B libraries of tools/mailbox_group_ab.sh)
#endif
constexpr uint32_t kMailGroup = CTS_MAIL_GROUP;
// Part records a job is answered with (a stop job: one per workgroup of its group).
#if defined(__HIP__)
__host__ __device__
#endif
inline uint32_t mail_parts(uint64_t ptr, uint32_t len)
{
    if (len == 0) return kMailGroup;
    const uint64_t pieces = (((ptr & 15u) + (uint64_t)len + 15u) / 16u * 16u + kMailPieceBytes - 1) / kMailPieceBytes;
    return pieces < kMailGroup ? (uint32_t)pieces : kMailGroup;
}
constexpr uint32_t kMailMaxGroups = 64;
// Job length of a no-op: the host's keepalive for an idle group (its pollers' idle exit restarts), and what a
// poller publishes for a job whose slot a later job already holds. No workgroup answers it.
constexpr uint32_t kMailSkip = 0xFFFFFFFFu;
struct MailStarts {
    uint64_t j[kMailMaxGroups];  // each group's first job number (passed by value)
};
// Each group polls its jobs from starts.j[g] on until a stop job, or until it has waited idle_ticks
// (s_memrealtime, 100 MHz) for one job: every wave reaches one of the two exits. per_group = S.
// groups * kMailGroup workgroups of kMailThreads threads.
// delay_ticks (test hook, 0 in production): group 0's last workgroup starts polling that much later.
hipError_t launch_mailbox(const MailSlot* slots, MailPart* parts, uint32_t per_group, const MailStarts& starts,
                          uint32_t groups, uint64_t idle_ticks, hipStream_t stream, uint64_t delay_ticks = 0);

// out[0..kCounterCount) = (accumulate ? out : 0) + the counters of a device counter block, summed over its
// CTS_COUNTER_SHARDS shards (one 64-thread workgroup; cts_counters_allreduce folds on the device with it).
hipError_t launch_counters_fold(const void* block, uint64_t* out, bool accumulate, hipStream_t stream);

hipError_t launch_verify(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                         uint32_t max_length_hint, cts_verify_result* results, uint64_t* counters,
                         uint32_t* conn_first_fail, uint32_t n_conns, hipStream_t stream,
                         const LaunchGeometry& geo);

hipError_t launch_verify_strided(const uint8_t* arena, uint64_t arena_bytes, uint32_t stride, const uint32_t* lens,
                                 uint32_t n, uint32_t skip_head, uint32_t expected, uint32_t conn_index,
                                 cts_verify_result* results, uint64_t* counters, uint32_t* conn_first_fail,
                                 uint32_t n_conns, hipStream_t stream, const LaunchGeometry& geo);

hipError_t launch_fill(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                       uint32_t max_length_hint, hipStream_t stream, const LaunchGeometry& geo);

// dst[i] = P((pattern_offset + i) mod 65536) for i < bytes; many blocks per span.
hipError_t launch_fill_span(uint8_t* dst, uint64_t bytes, uint32_t pattern_offset, hipStream_t stream,
                            const LaunchGeometry& geo);

hipError_t launch_media_stream_verify(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs, uint32_t n,
                                     cts_datagram_record* records, cts_verify_result* results, uint64_t* counters,
                                     hipStream_t stream, const LaunchGeometry& geo);

// Receive ring: datagram i at arena + i * stride, lengths[i] completed bytes (the windowed kernel).
hipError_t launch_media_stream_verify_strided(const uint8_t* arena, uint64_t arena_bytes, uint32_t stride,
                                             const uint32_t* lengths, uint32_t n, cts_datagram_record* records,
                                             cts_verify_result* results, uint64_t* counters, hipStream_t stream,
                                             const LaunchGeometry& geo);

// The receive pass writing 16-byte statuses (cts_media_stream_verify_status); descs == nullptr: the strided ring.
hipError_t launch_media_stream_status(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs,
                                     const uint32_t* lengths, uint32_t stride, uint32_t n, cts_datagram_status* status,
                                     uint64_t* counters, hipStream_t stream, const LaunchGeometry& geo);

// The receive pass summing the client's frame accounting (cts_media_stream_verify_frames); descs == nullptr: the
// strided ring. Zeroes totals (cts_frame_totals_device_bytes()) and frame_bytes[win.frames] first.
hipError_t launch_media_stream_frames(const uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs,
                                     const uint32_t* lengths, uint32_t stride, uint32_t n, const cts_frame_window& win,
                                     uint64_t* totals, uint64_t* frame_bytes, uint64_t* counters, hipStream_t stream,
                                     const LaunchGeometry& geo);

hipError_t launch_media_stream_fill(uint8_t* arena, uint64_t arena_bytes, const cts_buf_desc* descs,
                                   const cts_datagram_header* headers, uint32_t n, hipStream_t stream,
                                   const LaunchGeometry& geo);
hipError_t launch_media_stream_fill_strided(uint8_t* arena, uint64_t arena_bytes, uint32_t stride, const uint32_t* lengths,
                                           const cts_datagram_header* headers, uint32_t n, hipStream_t stream,
                                           const LaunchGeometry& geo);

}  // namespace cts
