/*
 * cts_engine.h — C ABI of the MI355X-native ctsTraffic data-integrity engine.
 *
 * The engine replaces the two hot-path pieces of ctsTraffic's ctsIoPattern
 * (reference: /root/reference, microsoft/ctsTraffic):
 *
 *   fill   = InitOnceIoPatternCallback            ctsTraffic/ctsIOPattern.cpp:52-90
 *            (+ per-buffer materialisation of the sender stream)
 *   verify = ctsIoPattern::VerifyBuffer            ctsTraffic/ctsIOPattern.cpp:745-775
 *            (decl. ctsTraffic/ctsIOPattern.h:329), RtlCompareMemory semantics
 *
 * Both are reached in the reference only through ctsIoPattern::CompleteIo
 * (ctsIOPattern.cpp:364-534) and the ctsIoPattern constructor, so the IO
 * functors (ctsSendRecvIocp.cpp, ctsRioIocp.cpp, ctsMediaStreamClient.cpp)
 * stay unchanged; the host-side ctsIoPattern mirror lives in cts_pattern.h.
 *
 * Conventions (ctsIOPattern.h:143-144 are noexcept; FAIL_FAST on internal
 * inconsistency): every entry point is noexcept and returns an int status,
 * 0 = CTS_OK, negative = error (see cts_status). No entry point throws.
 * Device pointers are plain pointers obtained from hipMalloc (or any
 * allocator of the same process/runtime); `stream` is a hipStream_t passed
 * as void* (NULL = the legacy null stream). No torch types cross this ABI.
 *
 * Thread safety: an engine may be used concurrently from many threads as
 * long as each thread passes its own stream (the reference serialises per
 * connection under the ctsSocket lock, ctsSocket.h:189, and runs many
 * connections concurrently on the NT threadpool).
 */
#ifndef CTS_ENGINE_H
#define CTS_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* c_bufferPatternSize = 0xffff + 1 (ctsIOPattern.cpp:35). The byte stream
 * repeats every 65536 bytes: u16 little-endian values 0..32767
 * (ctsIOPattern.cpp:55-58 build 0..65535, but only the first 65536 bytes are
 * ever copied into the sender buffer, ctsIOPattern.cpp:72-80). */
#define CTS_PATTERN_PERIOD 65536u
/* c_udpDatagramDataHeaderLength = 2 + 8 + 8 + 8 (ctsMediaStreamProtocol.hpp:43-52) */
#define CTS_UDP_DATA_HEADER_LENGTH 26u
/* c_statusErrorDataDidNotMatchBitPattern = MAXINT - 3 (ctsIOPattern.h:49) */
#define CTS_STATUS_ERROR_DATA_DID_NOT_MATCH_BIT_PATTERN 2147483644u
/* Number of 64-byte counter shards in a device counter block. */
#define CTS_COUNTER_SHARDS 64u

typedef enum cts_status {
    CTS_OK = 0,
    CTS_E_INVALID = -1,   /* bad argument (null, misaligned, out of range) */
    CTS_E_HIP = -2,       /* a HIP runtime call or kernel launch failed */
    CTS_E_NOMEM = -3,     /* allocation failed */
    CTS_E_NO_DEVICE = -4, /* no HIP device / device index out of range */
    CTS_E_UNAVAILABLE = -5, /* an optional runtime library (RCCL) could not be loaded */
    CTS_E_TIMEOUT = -6      /* a bounded wait ran out; nothing was freed, the call may be repeated
                             * (cts_io_pattern_destroy while a kernel still reads the pattern's buffers) */
} cts_status;

/* One received (verify) or outgoing (fill) buffer inside a device arena.
 * Mirrors the fields of ctsTask (ctsIOTask.hpp:37-60) that the hot path
 * reads: m_buffer (as an arena offset), the transferred length, the
 * m_bufferOffset where payload starts, and m_expectedPatternOffset. */
typedef struct cts_buf_desc {
    uint64_t byte_offset;             /* buffer start = arena + byte_offset */
    uint32_t length;                  /* bytes transferred incl. skip_head (currentTransfer) */
    uint32_t expected_pattern_offset; /* ctsTask::m_expectedPatternOffset, < 65536 */
    uint32_t conn_index;              /* connection slot (DataError accounting) */
    uint32_t skip_head;               /* ctsTask::m_bufferOffset: 0 TCP, 26 MediaStream payload */
} cts_buf_desc;                       /* 24 bytes */

#define CTS_RESULT_FLAG_BAD_DESC 0x1u /* descriptor out of arena / offset >= 65536 / length < skip_head */

/* Per-buffer verify record. first_mismatch is RtlCompareMemory's return
 * value (matching-prefix length) over the verified region
 * [byte_offset+skip_head, byte_offset+length) — ctsIOPattern.cpp:757-760;
 * pass iff first_mismatch == length - skip_head (ctsIOPattern.cpp:774).
 * expected/actual are the two bytes ctsIOPattern.cpp:761-772 prints. */
typedef struct cts_verify_result {
    uint32_t first_mismatch;
    uint32_t mismatch_bytes;  /* extension: # of differing bytes (not in the reference) */
    uint8_t expected;         /* pattern byte at first_mismatch (0 when clean) */
    uint8_t actual;           /* received byte at first_mismatch (0 when clean) */
    uint8_t pass;             /* 1 = buffer matched the bit pattern */
    uint8_t flags;            /* CTS_RESULT_FLAG_* */
} cts_verify_result;          /* 12 bytes */

/* Aggregate counters (the aggregation target is ctsStatistics.hpp:87-373).
 * bytes_checked  : sum of verified bytes (length - skip_head)
 * bytes_ok       : sum of verified bytes of buffers that passed
 * buffers_checked: # buffers verified (bad descriptors excluded)
 * buffers_failed : # buffers that did not match
 * mismatched_bytes: extension, sum of cts_verify_result.mismatch_bytes */
typedef struct cts_counters {
    uint64_t bytes_checked;
    uint64_t bytes_ok;
    uint64_t buffers_checked;
    uint64_t buffers_failed;
    uint64_t mismatched_bytes;
} cts_counters;

/* cts_counters plus the DataError count, read by the *_ex entry points (cts_counters keeps its size and meaning).
 * connections_failed: # connections with a failing buffer, i.e. the ConnectionStatusDetails.m_protocolErrorCount
 * increments of ctsSocketState.cpp:221-228 (one per connection whose verify failed, however many of its buffers
 * did). Counted on the device when a verify's atomicMin on dev_conn_first_fail[c] finds the slot still
 * 0xFFFFFFFF, so it counts only in launches given a dev_conn_first_fail array, once per slot over the life of
 * that array (re-initialise the slots when the counter block is reset). */
typedef struct cts_counters_ex {
    uint64_t bytes_checked;
    uint64_t bytes_ok;
    uint64_t buffers_checked;
    uint64_t buffers_failed;
    uint64_t mismatched_bytes;
    uint64_t connections_failed;
} cts_counters_ex;

typedef struct cts_engine cts_engine;

/* ---- library / pattern helpers ------------------------------------------ */
const char* cts_version(void);
const char* cts_status_string(int status);
/* P(stream_offset mod 65536): the byte g_senderSharedBuffer holds at that
 * offset (ctsIOPattern.cpp:55-80). Pure arithmetic, no device needed. */
uint8_t cts_pattern_byte(uint64_t stream_offset);
/* g_maximumBufferSize = c_bufferPatternSize + GetMaxBufferSize() (ctsIOPattern.cpp:60) */
uint64_t cts_sender_buffer_size(uint32_t max_buffer_size);

/* Which of n_shards GPUs owns a connection: fmix32(conn_index) mod n_shards (the murmur3
 * finaliser). Every buffer of a connection goes to one GPU, so its first failing buffer and its
 * DataError decision (ctsSocketState.cpp:221-232) stay GPU-local. */
uint32_t cts_shard_of(uint32_t conn_index, uint32_t n_shards);

/* ---- engine lifetime ------------------------------------------------------ */
int cts_engine_create(int device, cts_engine** out);
int cts_engine_destroy(cts_engine* engine);
int cts_engine_device(const cts_engine* engine);
/* The host NUMA node the engine's GPU hangs off (its PCI device's numa_node), or -1 if unknown. In
 * tools/sync_probe, threads posting SYNC verifies (cts_verify_mapped / cts_verify_host) answered faster
 * pinned there: 6.0-7.5 / 9.9-12.7 / 14.5-15.0 us per 64 KiB at 1 / 8 / 16 callers, against 6.1-9.6 /
 * 16.1-17.3 / 15.5-24.8 unpinned. Whole loopback runs pinned there were not faster. */
int cts_engine_numa_node(const cts_engine* engine);

/* Launch-geometry attributes (defaults tuned for MI355X; env overrides
 * CTS_BLOCKS_PER_CU / CTS_NT_LOADS / CTS_SMALL_THRESHOLD / CTS_SMALL_BLOCKS_PER_CU /
 * CTS_FILL_BLOCKS_PER_CU / CTS_SMALL_CHUNK / CTS_FILL_NT / CTS_RING_FILL_BLOCKS_PER_CU
 * are read at create time). */
typedef enum cts_engine_attr {
    CTS_ATTR_BLOCKS_PER_CU = 1,   /* grid cap = CUs x this (grid-strides beyond) */
    CTS_ATTR_NT_LOADS = 2,        /* 1 = nontemporal loads on the verify stream */
    CTS_ATTR_SMALL_THRESHOLD = 3, /* max_length_hint <= this -> one wave per buffer */
    CTS_ATTR_VERIFY_VARIANT = 4,  /* read-only id of the workgroup-per-buffer kernel (25); set: that id only */
    CTS_ATTR_SMALL_BLOCKS_PER_CU = 5, /* grid cap of the small-buffer path */
    CTS_ATTR_SMALL_VARIANT = 6,       /* read-only id of the small-buffer (datagram) kernel (15) */
    CTS_ATTR_FILL_BLOCKS_PER_CU = 7,  /* grid cap of the fill kernels */
    CTS_ATTR_MS_VARIANT = 8,          /* read-only id of the MediaStream receive kernel (3) */
    CTS_ATTR_SMALL_CHUNK = 9,         /* chunked small-buffer walk: buffers per chunk (0 = contiguous) */
    CTS_ATTR_FILL_NT = 10,            /* cts_fill stores: 0 plain, 1 nontemporal, 2 by path (default) */
    CTS_ATTR_SYNC_MAILBOX = 11        /* 1 (default) = SYNC-mode pattern verifies of pinned recv buffers and
                                       * cts_verify_host go through cts_verify_mapped (the resident mailbox
                                       * grid); 0 = one sliced launch + synchronize per call */
} cts_engine_attr;
int cts_engine_set_attr(cts_engine* engine, int attr, int value);
/* A non-blocking HIP stream on the engine's device, whatever device the calling
 * thread has current (one per connection: the reference serialises IO per
 * connection under the ctsSocket lock, ctsSocket.h:189). */
int cts_engine_stream_create(cts_engine* engine, void** stream);
int cts_engine_stream_destroy(cts_engine* engine, void* stream);
int cts_engine_get_attr(const cts_engine* engine, int attr, int* value);

/* ---- fill (write-bound) --------------------------------------------------- */
/* Materialise g_senderSharedBuffer on the device: dst[i] = P(i) for
 * i < 65536 + max_buffer_size (InitOnceIoPatternCallback, ctsIOPattern.cpp:52-90).
 * dst must be 16-byte aligned. */
int cts_sender_buffer_fill(cts_engine* engine, void* dev_dst, uint32_t max_buffer_size, void* stream);

/* For every descriptor d: arena[d.byte_offset + d.skip_head + b] =
 * P(d.expected_pattern_offset + b) for b < d.length - d.skip_head, i.e. what a
 * sender at stream offset d.expected_pattern_offset puts on the wire
 * (ctsTask{m_buffer = S, m_bufferOffset = m_sendPatternOffset}, ctsIOPattern.cpp:676-697).
 * Header bytes [0, skip_head) are left untouched. max_length_hint selects the
 * launch geometry (0 = unknown). dev_arena must be 16-byte aligned, dev_descs
 * 8-byte aligned (CTS_E_INVALID otherwise). */
int cts_fill(cts_engine* engine, void* dev_arena, uint64_t arena_bytes,
             const cts_buf_desc* dev_descs, uint32_t n, uint32_t max_length_hint, void* stream);

/* ---- verify (read-bound, the headline path) -------------------------------- */
/* Verify n device-resident buffers against the pattern. Any of the three
 * outputs may be NULL:
 *   dev_results[i]        : per-buffer record (cts_verify_result)
 *   dev_counters          : device counter block (cts_counters_device_bytes()),
 *                           ACCUMULATED into (like ctsStatsTracking::Add)
 *   dev_conn_first_fail   : n_conns u32 slots; for every failing buffer i of
 *                           connection c (< n_conns): atomicMin(slot[c], i).
 *                           Initialise to 0xFFFFFFFF. The DataError count
 *                           (ctsSocketState.cpp:221-232) is the number of slots
 *                           != 0xFFFFFFFF when descriptors of one connection are
 *                           in stream order; with dev_counters given it is also
 *                           accumulated on the device (connections_failed,
 *                           cts_counters_read_ex).
 * dev_arena must be 16-byte aligned and its allocation must extend to a
 * multiple of 16 bytes (every hipMalloc allocation does); dev_descs must be
 * 8-byte aligned, dev_results and dev_conn_first_fail 4-byte aligned and
 * dev_counters 8-byte aligned (CTS_E_INVALID otherwise; the same holds for the
 * outputs of every verify entry point). */
int cts_verify(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes,
               const cts_buf_desc* dev_descs, uint32_t n, uint32_t max_length_hint,
               cts_verify_result* dev_results, void* dev_counters,
               uint32_t* dev_conn_first_fail, uint32_t n_conns, void* stream);

/* ---- counters --------------------------------------------------------------- */
size_t cts_counters_device_bytes(void);
int cts_counters_reset(cts_engine* engine, void* dev_counters, void* stream);
/* Folds the shards into *out. Synchronises `stream`. */
int cts_counters_read(cts_engine* engine, const void* dev_counters, cts_counters* out, void* stream);
/* The process-wide counters of a node: one process drives one engine per GPU (the reference is one
 * process per host), and ctsStatsTracking (ctsStatistics.hpp:87-198) is the sum of every engine's
 * device block, folded on the host. dev_counters[i] belongs to engines[i]; streams may be NULL
 * (each engine's legacy stream) or hold one stream per engine (each is synchronised). */
int cts_counters_read_multi(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                            uint32_t n, cts_counters* out);
/* The same node-wide counters reduced on the GPUs over RCCL (ncclAllReduce, sum,
 * ncclUint64, over xGMI; count 6 since round 6: the five below and the DataError count of cts_counters_ex), for
 * ctsTraffic's one-process host: each engine's block is folded on its own
 * device (engines sharing a device fold into one slot), then one ncclAllReduce per device runs inside
 * ncclGroupStart/End on that device's stream (the stream of its first engine in the list; streams may be NULL =
 * each engine's legacy stream; another engine's stream on the same device is synchronised first). Every device's
 * result is read back and must agree. The communicators (ncclCommInitAll over the distinct devices, in list
 * order) are created by cts_counters_allreduce_prepare, or else on the first call for a device set, and reused. RCCL is loaded on first use (librccl.so.1,
 * or the path in $CTS_RCCL_LIBRARY): CTS_E_UNAVAILABLE when it cannot be; CTS_E_HIP when an RCCL or HIP call
 * fails or the devices' results disagree. Thread-safe (calls are serialised). Replaces the reads behind
 * ctsConfig::TcpStatusDetails / ctsStatsTracking (ctsConfig.h:415-417, ctsStatistics.hpp:87-198). */
int cts_counters_allreduce(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                           uint32_t n, cts_counters* out);
/* Destroys the communicators and device slots cts_counters_allreduce keeps (call before the engines' devices go
 * away, e.g. at shutdown); the next all-reduce creates them again. */
int cts_counters_allreduce_release(void);

/* The same three reads with the DataError count (cts_counters_ex.connections_failed): the all-reduce is one
 * ncclAllReduce of count 6. cts_counters_read / _read_multi / _allreduce return the first five fields of these. */
int cts_counters_read_ex(cts_engine* engine, const void* dev_counters, cts_counters_ex* out, void* stream);
int cts_counters_read_multi_ex(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                               uint32_t n, cts_counters_ex* out);
int cts_counters_allreduce_ex(cts_engine* const* engines, const void* const* dev_counters, void* const* streams,
                              uint32_t n, cts_counters_ex* out);

/* Everything the first cts_counters_allreduce of a device set would set up, done now: RCCL loaded, the device
 * slots allocated, ncclCommInitAll over the engines' distinct devices (in list order, as the all-reduce groups
 * them) and one dry run of a counter read per device (a zeroed block folded, all-reduced and copied back), so
 * RCCL's first-collective set-up and the fold's first launch are paid here too. Call it next
 * to cts_engine_create, before the status timer's first tick (ctsTraffic.cpp:107-113 prints at t = 0); later
 * all-reduces over the same device set reuse the clique. Idempotent. Errors as cts_counters_allreduce. */
int cts_counters_allreduce_prepare(cts_engine* const* engines, uint32_t n);

/* Where the set-up time of the newest clique went (ms, host wall clock); all zero before one was built. */
typedef struct cts_allreduce_setup {
    double rccl_load_ms;       /* dlopen of librccl + dlsym (0 when RCCL was already loaded by an earlier clique) */
    double slots_ms;           /* the per-device result slots: hipMallocAsync + synchronize */
    double comm_init_ms;       /* ncclCommInitAll */
    double first_allreduce_ms; /* the dry run: fold of a zeroed block, the first grouped ncclAllReduce, copy back */
    uint32_t devices;          /* ranks in that clique */
    uint32_t prepared;         /* 1 = built by cts_counters_allreduce_prepare, 0 = by a first all-reduce */
    /* the newest completed cts_counters_allreduce(_ex) call, in us: the folds launched (and other streams'
     * synchronised), the grouped all-reduce enqueued, the copies back and their synchronisation; and the whole call
     * from entry to return (argument checks, the device grouping, the lock and the clique lookup included) */
    double last_fold_us;
    double last_allreduce_us;
    double last_readback_us;
    double last_total_us;
} cts_allreduce_setup;
int cts_counters_allreduce_setup_times(cts_allreduce_setup* out);

/* cts_verify over a uniformly strided receive ring (a UDP socket's datagrams): buffer i occupies
 * [i * stride, i * stride + dev_lengths[i]) of the arena, its first skip_head bytes are skipped and the rest
 * is checked against the pattern from expected_offset (MediaStream payloads: skip 26, expected 0,
 * ctsIOPatternMediaStream.cpp:185-192); every buffer belongs to connection conn_index. The kernel reads 4
 * bytes of metadata per buffer instead of a 24-byte descriptor. A length above the stride (or one that
 * leaves the arena) is flagged CTS_RESULT_FLAG_BAD_DESC. Outputs and counters as cts_verify. dev_lengths must
 * be 4-byte aligned, dev_arena 16-byte aligned with arena_bytes >= 16, stride > 0. */
int cts_verify_strided(cts_engine* engine, const void* dev_arena, uint64_t arena_bytes, uint32_t stride,
                       const uint32_t* dev_lengths, uint32_t n, uint32_t skip_head, uint32_t expected_offset,
                       uint32_t conn_index, cts_verify_result* dev_results, void* dev_counters,
                       uint32_t* dev_conn_first_fail, uint32_t n_conns, void* stream);

/* ---- host-buffer drop-in for ctsIoPattern::VerifyBuffer ---------------------- */
/* Verifies `len` bytes at host_buf against the pattern starting at
 * expected_offset and waits. Returns the record in *out (RtlCompareMemory
 * semantics, ctsIOPattern.cpp:753-774). Thread-safe. With CTS_ATTR_SYNC_MAILBOX
 * (the default) the bytes are copied into a pinned staging buffer of the
 * call's own and posted to the resident mailbox grid (cts_verify_mapped), so
 * concurrent callers run side by side; with it off, they are staged into one
 * shared buffer and verified by a launch + synchronize on the engine's stream. */
int cts_verify_host(cts_engine* engine, const void* host_buf, uint32_t len,
                    uint32_t expected_offset, cts_verify_result* out);

/* The same one-buffer VerifyBuffer (ctsIOPattern.cpp:745-775) for a buffer the
 * GPU can already address (a cts_host_alloc dev_view, or HBM), verified in
 * place and waited for, without a kernel launch per call: a resident grid on
 * the engine's device (groups of workgroups, each group polling its own ring
 * of host-coherent pinned job slots) verifies each posted buffer as 4 KiB
 * pieces spread over a group's workgroups, which answer with part records
 * the caller spins on and folds. Thread-safe: concurrent connections'
 * CompleteIo (each serialised per connection by its ctsSocket lock,
 * ctsSocket.h:189) post independent jobs, each to the least busy group, and
 * those run side by side. The grid starts on the first call and stops after
 * CTS_MAILBOX_IDLE_MS (default 50) ms without calls (env CTS_MAILBOX_GROUPS,
 * CTS_MAILBOX_SLOTS size it); cts_engine_destroy stops it. Each group also
 * leaves by itself after CTS_MAILBOX_EXIT_MS (default 1000) ms without a job;
 * while posts come, the watchdog gives idle groups no-op jobs to keep them
 * inside that bound, and a post relaunches a grid that left. A job unanswered
 * after CTS_MAILBOX_TIMEOUT_MS (default 2000) does not fail the call: it and
 * later calls verify with one sliced launch + synchronize until the grid has
 * drained, then the mailbox starts over. While the grid is resident a device-
 * wide wait (hipDeviceSynchronize, torch.cuda.synchronize) waits for it too,
 * i.e. until CTS_MAILBOX_IDLE_MS after the last call; cts_host_free stops the
 * grids of every engine on its device first (with that device current), so a
 * free does not wait on other threads' posts. */
int cts_verify_mapped(cts_engine* engine, const void* dev_buf, uint32_t len,
                      uint32_t expected_offset, cts_verify_result* out);
/* How many times the mailbox grid was launched (0 = never used): each launch serves every
 * cts_verify_mapped call until the grid goes idle. */
uint64_t cts_mailbox_launches(const cts_engine* engine);

/* Pinned host arenas (the recv-buffer container of a GPU-verified
 * ctsIoPattern, ctsIOPattern.cpp:156-175): page-locked and mapped into the
 * device address space, so cts_verify can read them in place over PCIe
 * (zero-copy) or hipMemcpyAsync can DMA them. *dev_view receives the device
 * address to pass as dev_arena. */
int cts_host_alloc(cts_engine* engine, uint64_t bytes, void** host_ptr, void** dev_view);
/* Frees cts_host_alloc memory. hipHostFree synchronizes the current device, so the
 * engine's device is made current and every engine's resident mailbox grid on it is
 * stopped first (they relaunch on their next cts_verify_mapped). */
int cts_host_free(cts_engine* engine, void* host_ptr);
/* Device address of pinned+mapped host memory (hipHostGetDevicePointer);
 * CTS_E_INVALID if host_ptr is not device-accessible pinned memory. */
int cts_host_device_pointer(void* host_ptr, void** dev_view);

/* Batched host path (PCIe-inclusive): verifies n host buffers
 * (bufs[i] + skip_heads[i], lens[i] - skip_heads[i] bytes, expected offsets
 * expected[i]) in one kernel launch: the buffers are copied into the engine's
 * pinned, device-mapped staging arena (kept and grown across calls) and the
 * kernel reads them in place over PCIe (zero copy). skip_heads may be NULL
 * (all 0). results[n] host memory; counters (host) accumulated into if
 * non-NULL. Thread-safe (serialised per engine); synchronous. */
int cts_verify_host_batch(cts_engine* engine, const void* const* bufs, const uint32_t* lens,
                          const uint32_t* expected, const uint32_t* skip_heads, uint32_t n,
                          cts_verify_result* results, cts_counters* counters);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* CTS_ENGINE_H */
