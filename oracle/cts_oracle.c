/*
 * cts_oracle.c — CPU restatement of ctsTraffic's pattern fill + verify.
 * TEST INFRASTRUCTURE ONLY (see cts_oracle.h). Plain C11 + pthreads.
 */
#include "cts_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ctsIOPattern.cpp:55-58: for fillSlot in [0, c_bufferPatternSize):
 *   *(unsigned short*)&g_bufferPattern[fillSlot * 2] = (unsigned short)fillSlot;
 * (x86/x64 Windows is little-endian, so the u16 is stored low byte first.) */
void ora_build_pattern_table(uint8_t* out)
{
    for (uint32_t fillSlot = 0; fillSlot < ORA_PATTERN_SIZE; ++fillSlot) {
        const uint16_t v = (uint16_t)fillSlot;
        out[fillSlot * 2 + 0] = (uint8_t)(v & 0xFFu);
        out[fillSlot * 2 + 1] = (uint8_t)(v >> 8);
    }
}

/* ctsIOPattern.cpp:60: g_maximumBufferSize = c_bufferPatternSize + GetMaxBufferSize() */
uint64_t ora_sender_buffer_size(uint32_t max_buffer_size)
{
    return (uint64_t)ORA_PATTERN_SIZE + max_buffer_size;
}

/* ctsIOPattern.cpp:72-80: copy at most c_bufferPatternSize bytes of
 * g_bufferPattern per iteration until g_maximumBufferSize bytes are written.
 * Only the first 65536 bytes of the 131072-byte table are ever used. */
static uint8_t g_table[ORA_PATTERN_SIZE * 2]; /* g_bufferPattern, built once (callers may run on many threads) */
static pthread_once_t g_table_once = PTHREAD_ONCE_INIT;
static void build_table(void) { ora_build_pattern_table(g_table); }

void ora_build_sender_buffer(uint8_t* dst, uint32_t max_buffer_size)
{
    pthread_once(&g_table_once, build_table);
    const uint8_t* const table = g_table;
    uint8_t* protectedDestination = dst;
    uint64_t writeSizeRemaining = ora_sender_buffer_size(max_buffer_size);
    while (writeSizeRemaining > 0) {
        const uint64_t bytesToWrite =
            writeSizeRemaining > ORA_PATTERN_SIZE ? ORA_PATTERN_SIZE : writeSizeRemaining;
        memcpy(protectedDestination, table, (size_t)bytesToWrite);
        protectedDestination += bytesToWrite;
        writeSizeRemaining -= bytesToWrite;
    }
}

/* RtlCompareMemory (ntdll): "returns the number of bytes in the two blocks
 * that match", counting from the start — i.e. the offset of the first
 * mismatch, or n. Vectorised block memcmp, byte scan inside the first
 * differing block. */
size_t ora_compare_memory(const void* a, const void* b, size_t n)
{
    const uint8_t* pa = (const uint8_t*)a;
    const uint8_t* pb = (const uint8_t*)b;
    size_t i = 0;
    const size_t block = 4096;
    while (i < n) {
        const size_t len = (n - i) < block ? (n - i) : block;
        if (memcmp(pa + i, pb + i, len) != 0) {
            for (size_t j = 0; j < len; ++j) {
                if (pa[i + j] != pb[i + j]) return i + j;
            }
        }
        i += len;
    }
    return n;
}

/* ctsIOPattern.cpp:745-775 (VerifyBuffer):
 *   patternBuffer = g_senderSharedBuffer + m_expectedPatternOffset
 *   lengthMatched = RtlCompareMemory(patternBuffer, m_buffer + m_bufferOffset, transferred)
 *   on mismatch prints lengthMatched, patternBuffer[lengthMatched], buf[lengthMatched]
 *   return lengthMatched == transferred
 * mismatch_bytes is an extension (not computed by the reference). */
int ora_verify_buffer(const uint8_t* sender, const uint8_t* buf, uint32_t buffer_offset,
                      uint32_t expected, uint32_t transferred, ora_result* out)
{
    const uint8_t* patternBuffer = sender + expected;
    const uint8_t* received = buf + buffer_offset;
    const size_t lengthMatched = ora_compare_memory(patternBuffer, received, transferred);
    ora_result r;
    memset(&r, 0, sizeof(r));
    r.first_mismatch = (uint32_t)lengthMatched;
    r.pass = (uint8_t)(lengthMatched == transferred);
    if (!r.pass) {
        r.expected = patternBuffer[lengthMatched];
        r.actual = received[lengthMatched];
        uint32_t cnt = 0;
        for (size_t j = lengthMatched; j < transferred; ++j) cnt += (patternBuffer[j] != received[j]);
        r.mismatch_bytes = cnt;
    }
    if (out) *out = r;
    return r.pass;
}

/* ctsIOPattern.cpp:491-492 and :695-697:
 *   m_PatternOffset += bytes; m_PatternOffset %= c_bufferPatternSize; */
uint32_t ora_advance_offset(uint32_t offset, uint64_t bytes)
{
    return (uint32_t)(((uint64_t)offset + bytes) % ORA_PATTERN_SIZE);
}

static uint8_t g_sender[ORA_PATTERN_SIZE]; /* one period of S */
static pthread_once_t g_sender_once = PTHREAD_ONCE_INIT;
static void build_sender_period(void) { ora_build_sender_buffer(g_sender, 0); }

uint8_t ora_pattern_byte(uint64_t stream_offset)
{
    pthread_once(&g_sender_once, build_sender_period);
    return g_sender[stream_offset % ORA_PATTERN_SIZE];
}

static int desc_bad(const ora_desc* d, uint64_t arena_bytes)
{
    if (d->expected_pattern_offset >= ORA_PATTERN_SIZE) return 1; /* FAIL_FAST ctsIOPattern.cpp:723-725 */
    if (d->length < d->skip_head) return 1;                        /* ValidateBufferLengthFromTask */
    if (d->byte_offset > arena_bytes || arena_bytes - d->byte_offset < d->length) return 1;
    return 0;
}

static uint32_t max_verified_len(const ora_desc* descs, uint32_t n)
{
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t v = descs[i].length >= descs[i].skip_head ? descs[i].length - descs[i].skip_head : 0;
        if (v > m) m = v;
    }
    return m;
}

/* Sender-side materialisation: the bytes a send task
 * {m_buffer = S, m_bufferOffset = m_sendPatternOffset, len} puts on the wire
 * (ctsIOPattern.cpp:676-681) land in the receiver's buffer. */
void ora_fill(uint8_t* arena, uint64_t arena_bytes, const ora_desc* descs, uint32_t n)
{
    const uint32_t maxlen = max_verified_len(descs, n);
    uint8_t* S = (uint8_t*)malloc((size_t)ora_sender_buffer_size(maxlen));
    if (!S) return;
    ora_build_sender_buffer(S, maxlen);
    for (uint32_t i = 0; i < n; ++i) {
        const ora_desc* d = &descs[i];
        if (desc_bad(d, arena_bytes)) continue;
        memcpy(arena + d->byte_offset + d->skip_head, S + d->expected_pattern_offset,
               d->length - d->skip_head);
    }
    free(S);
}

typedef struct verify_job {
    const uint8_t* arena;
    uint64_t arena_bytes;
    const ora_desc* descs;
    uint32_t begin, end;
    ora_result* results;
    ora_counters counters;
    uint32_t* conn_first_fail;
    uint32_t n_conns;
    const uint8_t* S;
} verify_job;

static void* verify_worker(void* arg)
{
    verify_job* j = (verify_job*)arg;
    memset(&j->counters, 0, sizeof(j->counters));
    for (uint32_t i = j->begin; i < j->end; ++i) {
        const ora_desc* d = &j->descs[i];
        ora_result r;
        if (desc_bad(d, j->arena_bytes)) {
            memset(&r, 0, sizeof(r));
            r.flags = 1;
        } else {
            const uint32_t transferred = d->length - d->skip_head;
            ora_verify_buffer(j->S, j->arena + d->byte_offset, d->skip_head,
                              d->expected_pattern_offset, transferred, &r);
            j->counters.bytes_checked += transferred;
            j->counters.buffers_checked += 1;
            if (r.pass) {
                j->counters.bytes_ok += transferred;
            } else {
                j->counters.buffers_failed += 1;
                j->counters.mismatched_bytes += r.mismatch_bytes;
                if (j->conn_first_fail && d->conn_index < j->n_conns) {
                    uint32_t* slot = &j->conn_first_fail[d->conn_index];
                    uint32_t cur = __atomic_load_n(slot, __ATOMIC_RELAXED);
                    while (i < cur && !__atomic_compare_exchange_n(slot, &cur, i, 0, __ATOMIC_RELAXED,
                                                                   __ATOMIC_RELAXED)) {
                    }
                }
            }
        }
        if (j->results) j->results[i] = r;
    }
    return NULL;
}

int ora_verify_batch(const uint8_t* arena, uint64_t arena_bytes, const ora_desc* descs,
                     uint32_t n, ora_result* results, ora_counters* counters,
                     uint32_t* conn_first_fail, uint32_t n_conns, int nthreads)
{
    if ((!arena && n) || (!descs && n) || nthreads < 1) return -1;
    const uint32_t maxlen = max_verified_len(descs, n);
    uint8_t* S = (uint8_t*)malloc((size_t)ora_sender_buffer_size(maxlen));
    if (!S) return -1;
    ora_build_sender_buffer(S, maxlen);
    if ((uint32_t)nthreads > n) nthreads = n ? (int)n : 1;
    verify_job* jobs = (verify_job*)calloc((size_t)nthreads, sizeof(verify_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) {
        free(S); free(jobs); free(th);
        return -1;
    }
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].arena = arena;
        jobs[t].arena_bytes = arena_bytes;
        jobs[t].descs = descs;
        jobs[t].begin = (uint32_t)(((uint64_t)n * t) / nthreads);
        jobs[t].end = (uint32_t)(((uint64_t)n * (t + 1)) / nthreads);
        jobs[t].results = results;
        jobs[t].conn_first_fail = conn_first_fail;
        jobs[t].n_conns = n_conns;
        jobs[t].S = S;
    }
    if (nthreads == 1) {
        verify_worker(&jobs[0]);
    } else {
        for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, verify_worker, &jobs[t]);
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    }
    if (counters) {
        for (int t = 0; t < nthreads; ++t) {
            counters->bytes_checked += jobs[t].counters.bytes_checked;
            counters->bytes_ok += jobs[t].counters.bytes_ok;
            counters->buffers_checked += jobs[t].counters.buffers_checked;
            counters->buffers_failed += jobs[t].counters.buffers_failed;
            counters->mismatched_bytes += jobs[t].counters.mismatched_bytes;
        }
    }
    free(S); free(jobs); free(th);
    return 0;
}

uint64_t ora_fnv1a64(const uint8_t* p, size_t n)
{
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

static int64_t ora_i64le(const uint8_t* p)
{
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) v |= (uint64_t)p[b] << (8 * b);
    return (int64_t)v;
}

void ora_media_stream_verify(const uint8_t* arena, uint64_t arena_bytes, const ora_desc* descs, uint32_t n,
                             ora_dgram_record* records, ora_result* results, ora_counters* counters)
{
    uint32_t maxlen = 0;
    for (uint32_t i = 0; i < n; ++i) maxlen = descs[i].length > maxlen ? descs[i].length : maxlen;
    uint8_t* S = (uint8_t*)malloc((size_t)ora_sender_buffer_size(maxlen));
    if (!S) return;
    ora_build_sender_buffer(S, maxlen);
    for (uint32_t i = 0; i < n; ++i) {
        const ora_desc* d = &descs[i];
        const uint32_t completed = d->length;
        ora_dgram_record rec;
        memset(&rec, 0, sizeof(rec));
        rec.completed_bytes = completed;
        ora_result r;
        memset(&r, 0, sizeof(r));
        const uint8_t* buf = arena + d->byte_offset;
        if (d->byte_offset > arena_bytes || arena_bytes - d->byte_offset < completed) {
            rec.kind = 5;
        } else if (completed == 0) {
            rec.kind = 2;                                   /* zero-byte datagram, :158-167 */
        } else if (completed < 2) {                         /* < c_udpDatagramProtocolHeaderFlagLength */
            rec.kind = 3;
        } else {
            rec.flag = (uint16_t)(buf[0] | (buf[1] << 8));  /* *reinterpret_cast<unsigned short*>(m_buffer) */
            if (rec.flag == 0x0000)
                rec.kind = completed < 26 ? 3 : 0;           /* c_udpDatagramDataHeaderLength */
            else if (rec.flag == 0x1000)
                rec.kind = completed < 39 ? 3 : 1;           /* c_udpDatagramConnectionIdHeaderLength */
            else
                rec.kind = 4;
        }
        if (rec.kind == 0) {
            rec.sequence_number = ora_i64le(buf + 2);
            rec.sender_qpc = ora_i64le(buf + 8);
            rec.sender_qpf = ora_i64le(buf + 16);
            const uint32_t transferred = completed - 26;
            ora_verify_buffer(S, buf, 26, 0, transferred, &r);
            if (counters) {
                counters->bytes_checked += transferred;
                counters->buffers_checked += 1;
                if (r.pass) {
                    counters->bytes_ok += transferred;
                } else {
                    counters->buffers_failed += 1;
                    counters->mismatched_bytes += r.mismatch_bytes;
                }
            }
        } else {
            r.flags = rec.kind == 5 ? 1 : 2;
        }
        if (records) records[i] = rec;
        if (results) results[i] = r;
    }
    free(S);
}

/* g_senderSharedBuffer as the reference keeps it: built once per process (InitOnceIoPatternCallback),
 * here for buffers up to 1 MiB. */
#define ORA_HOOK_MAX_BUFFER (1u << 20)
static uint8_t* g_hook_sender;
static pthread_once_t g_hook_once = PTHREAD_ONCE_INIT;
static void build_hook_sender(void)
{
    g_hook_sender = (uint8_t*)malloc((size_t)ora_sender_buffer_size(ORA_HOOK_MAX_BUFFER));
    if (g_hook_sender) ora_build_sender_buffer(g_hook_sender, ORA_HOOK_MAX_BUFFER);
}

int ora_batch_verifier(void* ctx, const uint8_t* arena, uint64_t arena_bytes, const ora_desc* descs, uint32_t n,
                       ora_result* results)
{
    (void)ctx;
    pthread_once(&g_hook_once, build_hook_sender);
    if (!g_hook_sender || max_verified_len(descs, n) > ORA_HOOK_MAX_BUFFER)
        return ora_verify_batch(arena, arena_bytes, descs, n, results, NULL, NULL, 0, 1);
    for (uint32_t i = 0; i < n; ++i) {
        const ora_desc* d = &descs[i];
        if (desc_bad(d, arena_bytes)) {
            memset(&results[i], 0, sizeof(results[i]));
            results[i].flags = 1;
            continue;
        }
        ora_verify_buffer(g_hook_sender, arena + d->byte_offset, d->skip_head, d->expected_pattern_offset,
                          d->length - d->skip_head, &results[i]);
    }
    return 0;
}
