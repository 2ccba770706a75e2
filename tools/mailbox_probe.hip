// mailbox_probe.hip — the PCIe primitives under the SYNC mailbox (cts_verify_mapped), measured on
// their own: (1) a chain of dependent 16-B system-scope loads from host-coherent pinned memory (GPU
// clock: one round trip each); (2) host <-> GPU ping-pong through that memory (host clock: the
// fixed cost of a posted job without any verify work); (3) the same ping-pong with a 64 KiB read of
// pinned host memory by P workgroups between poll and answer (what a SYNC verify has to pay).
// Prints one JSON line per measurement.   build: make tools/mailbox_probe   run: tools/mailbox_probe
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define HIP_OK(x)                                                                                        \
    do {                                                                                                 \
        const hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                          \
            std::fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(e_));              \
            std::exit(1);                                                                                \
        }                                                                                                \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void chain_kernel(const uint64_t* p, int n, uint64_t* out)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(p), (short)0, 4096, 0x00020000);
    uint32_t off = 0;
    const uint64_t t0 = wall_clock64();
    for (int i = 0; i < n; ++i) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0u, 1 | 16);
        off = (v[0] + 16u * (uint32_t)i) & 0x3F0u;  // dependent: the next address needs this value
    }
    const uint64_t t1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = off;
    }
}

// lane 0 of block 0 polls seq; all blocks read `bytes` of data (bytes / P each) once it appears;
// every block answers with its own tagged word, the host waits for all P
// seq_words / ack_words: each block's seq word and ack word sit that many uint64 apart (0: one shared seq)
__global__ void pingpong_kernel(const uint64_t* seq, uint64_t* ack, const uint8_t* data, uint32_t bytes, int iters,
                                uint32_t seq_words = 0, uint32_t ack_words = 2)
{
    __shared__ uint32_t go;
    const uint32_t P = gridDim.x;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(seq + blockIdx.x * seq_words), (short)0, 16, 0x00020000);
    const uint32_t per = bytes / P;
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(data + (size_t)blockIdx.x * per), (short)0, (int)per, 0x00020000);
    for (int i = 1; i <= iters; ++i) {
        if (threadIdx.x == 0) {
            const uint64_t start = wall_clock64();
            go = i;
            for (;;) {
                const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 0u, 0u, 1 | 16);
                if ((int)v[0] >= i) break;
                if (wall_clock64() - start > 200000000ull) {  // 2 s without the word: give up (every wave exits)
                    go = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
        if (go == 0) return;
        uint32_t acc = 0;
        for (uint32_t o = threadIdx.x * 16u; o < per; o += blockDim.x * 16u) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rd, o, 0u, 1 | 16);
            acc |= v[0] ^ v[1] ^ v[2] ^ v[3];
        }
        acc = __syncthreads_or(acc != 0x12345678u);
        if (threadIdx.x == 0)
            __hip_atomic_store(ack + blockIdx.x * ack_words, (uint64_t)i | ((uint64_t)acc << 32), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
    }
}

// bandwidth of 16-B loads of pinned host memory by cache policy (aux): every lane reads 16 B per step
template <int AUX>
__global__ void bw_kernel(const uint8_t* data, uint64_t bytes, uint32_t* sink)
{
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(data), (short)0, 0x7FFFFFFF, 0x00020000);
    uint32_t acc = 0;
    for (uint64_t o = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16u; o < bytes; o += (uint64_t)gridDim.x * blockDim.x * 16u) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (uint32_t)o, 0u, AUX);
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <int AUX>
static void bw(const char* name, const uint8_t* d, uint64_t bytes, uint32_t* sink)
{
    hipEvent_t a, b;
    HIP_OK(hipEventCreate(&a));
    HIP_OK(hipEventCreate(&b));
    bw_kernel<AUX><<<1024, 256>>>(d, bytes, sink);
    HIP_OK(hipEventRecord(a));
    for (int i = 0; i < 5; ++i) bw_kernel<AUX><<<1024, 256>>>(d, bytes, sink);
    HIP_OK(hipEventRecord(b));
    HIP_OK(hipEventSynchronize(b));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"probe\": \"host_read_bw\", \"policy\": \"%s\", \"GBps\": %.2f}\n", name, 5.0 * bytes / (ms * 1e6));
    std::fflush(stdout);
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    uint64_t *hseq = nullptr, *hack = nullptr, *dout = nullptr;
    uint8_t* hdata = nullptr;
    const unsigned fl = hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent;
    if (hipHostMalloc((void**)&hseq, 4096, fl) != hipSuccess || hipHostMalloc((void**)&hack, 64 * 16, fl) != hipSuccess ||
        hipHostMalloc((void**)&hdata, 1 << 20, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess ||
        hipMalloc((void**)&dout, 16) != hipSuccess)
        return 1;
    std::memset(hseq, 0, 4096);
    std::memset(hack, 0, 64 * 16);
    std::memset(hdata, 1, 1 << 20);
    uint64_t *dseq, *dack;
    uint8_t* ddata;
    HIP_OK(hipHostGetDevicePointer((void**)&dseq, hseq, 0));
    HIP_OK(hipHostGetDevicePointer((void**)&dack, hack, 0));
    HIP_OK(hipHostGetDevicePointer((void**)&ddata, hdata, 0));
    // (0) bandwidth by load policy over 256 MiB of pinned (non-coherent, like a recv container) and coherent memory
    {
        uint8_t *big = nullptr, *dbig = nullptr, *bigc = nullptr, *dbigc = nullptr;
        uint32_t* sink = nullptr;
        const uint64_t B = 256ull << 20;
        if (hipHostMalloc((void**)&big, B, hipHostMallocMapped | hipHostMallocPortable) == hipSuccess &&
            hipHostMalloc((void**)&bigc, B, fl) == hipSuccess && hipMalloc((void**)&sink, 64) == hipSuccess) {
            std::memset(big, 3, B);
            std::memset(bigc, 3, B);
            HIP_OK(hipHostGetDevicePointer((void**)&dbig, big, 0));
            HIP_OK(hipHostGetDevicePointer((void**)&dbigc, bigc, 0));
            bw<0>("default", dbig, B, sink);
            bw<2>("nt", dbig, B, sink);
            bw<16>("sc1", dbig, B, sink);
            bw<1>("sc0", dbig, B, sink);
            bw<17>("sc0_sc1", dbig, B, sink);
            bw<0>("coherent_default", dbigc, B, sink);
            bw<17>("coherent_sc0_sc1", dbigc, B, sink);
            HIP_OK(hipHostFree(big));
            HIP_OK(hipHostFree(bigc));
            HIP_OK(hipFree(sink));
        }
    }
    // (1) dependent load chain
    for (int n : {100, 1000}) {
        chain_kernel<<<1, 64>>>(dseq, n, dout);
        uint64_t h[2];
        HIP_OK(hipMemcpy(h, dout, 16, hipMemcpyDeviceToHost));
        std::printf("{\"probe\": \"dependent_16B_sys_load\", \"loads\": %d, \"us_per_load\": %.3f}\n", n, h[0] / 100.0 / n);
    }
    // (2)/(3) ping-pong
    for (uint32_t bytes : {0u, 4096u, 65536u})
        for (uint32_t P : {1u, 4u, 16u, 64u}) {
            if (bytes == 0 && P > 1) continue;
            const int iters = 2000;
            std::memset(hack, 0, 64 * 16);
            __atomic_store_n(hseq, 0ull, __ATOMIC_SEQ_CST);
            hipStream_t s;
            HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            pingpong_kernel<<<P, 256, 0, s>>>(dseq, dack, ddata, bytes, iters);
            double t0 = 0;
            bool ok = true;
            for (int i = 1; i <= iters && ok; ++i) {
                if (i == 101) t0 = now_us();
                __atomic_store_n(hseq, (uint64_t)i, __ATOMIC_RELEASE);
                const double ts = now_us();
                for (uint32_t b = 0; b < P; ++b)
                    while ((uint32_t)__atomic_load_n(hack + 2 * b, __ATOMIC_ACQUIRE) != (uint32_t)i)
                        if (now_us() - ts > 2e6) {
                            ok = false;
                            break;
                        }
            }
            const double t1 = now_us();
            if (!ok) {  // let the grid finish: feed it every remaining ticket
                __atomic_store_n(hseq, (uint64_t)iters, __ATOMIC_RELEASE);
            }
            HIP_OK(hipStreamSynchronize(s));
            HIP_OK(hipStreamDestroy(s));
            std::printf("{\"probe\": \"pingpong\", \"bytes\": %u, \"workgroups\": %u, \"us_per_round\": %.3f, \"ok\": %d}\n",
                        bytes, P, (t1 - t0) / (iters - 100), ok ? 1 : 0);
            std::fflush(stdout);
            if (!ok) return 2;
        }
    // (5) 16 workgroups, 64 KiB or nothing: one shared seq line vs a line per workgroup (the host writes
    //     16 copies), and acks 16 B apart (4 per line) vs a line per workgroup
    for (uint32_t bytes : {0u, 65536u})
        for (uint32_t seq_words : {0u, 8u})
            for (uint32_t ack_words : {2u, 8u}) {
                const uint32_t P = 16;
                const int iters = 2000;
                std::memset(hack, 0, 64 * 16);
                for (uint32_t b = 0; b < P; ++b) __atomic_store_n(hseq + b * seq_words, 0ull, __ATOMIC_SEQ_CST);
                hipStream_t s;
                HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                pingpong_kernel<<<P, 256, 0, s>>>(dseq, dack, ddata, bytes, iters, seq_words, ack_words);
                double t0 = 0;
                bool ok = true;
                for (int i = 1; i <= iters && ok; ++i) {
                    if (i == 101) t0 = now_us();
                    for (uint32_t b = 0; b < (seq_words ? P : 1u); ++b)
                        __atomic_store_n(hseq + b * seq_words, (uint64_t)i, __ATOMIC_RELEASE);
                    const double ts = now_us();
                    for (uint32_t b = 0; b < P; ++b)
                        while ((uint32_t)__atomic_load_n(hack + ack_words * b, __ATOMIC_ACQUIRE) != (uint32_t)i)
                            if (now_us() - ts > 2e6) {
                                ok = false;
                                break;
                            }
                }
                const double t1 = now_us();
                if (!ok)
                    for (uint32_t b = 0; b < P; ++b) __atomic_store_n(hseq + b * seq_words, (uint64_t)iters, __ATOMIC_RELEASE);
                HIP_OK(hipStreamSynchronize(s));
                HIP_OK(hipStreamDestroy(s));
                std::printf("{\"probe\": \"pingpong_lines\", \"bytes\": %u, \"workgroups\": %u, \"seq_line_per_wg\": %d, "
                            "\"ack_line_per_wg\": %d, \"us_per_round\": %.3f, \"ok\": %d}\n",
                            bytes, P, seq_words ? 1 : 0, ack_words == 8 ? 1 : 0, (t1 - t0) / (iters - 100), ok ? 1 : 0);
                std::fflush(stdout);
                if (!ok) return 2;
            }
    // (4) the same ping-pong with the job word in device memory the host writes through its mapping
    //     (fine-grained / uncached VRAM behind the BAR): the GPU polls HBM instead of host memory
    for (const unsigned flag : {(unsigned)hipDeviceMallocUncached, (unsigned)hipDeviceMallocFinegrained}) {
        const char* fname = flag == hipDeviceMallocUncached ? "uncached" : "finegrained";
        uint64_t* vseq = nullptr;
        if (hipExtMallocWithFlags((void**)&vseq, 4096, flag) != hipSuccess) {
            std::printf("{\"probe\": \"pingpong_vram\", \"alloc\": \"%s\", \"error\": \"alloc\"}\n", fname);
            continue;
        }
        hipPointerAttribute_t at{};
        const bool attr_ok = hipPointerGetAttributes(&at, vseq) == hipSuccess;
        std::printf("{\"probe\": \"pingpong_vram\", \"alloc\": \"%s\", \"host_pointer\": \"%p\", \"attr_ok\": %d}\n", fname,
                    attr_ok ? at.hostPointer : nullptr, attr_ok ? 1 : 0);
        std::fflush(stdout);
        uint64_t* hv = attr_ok && at.hostPointer ? static_cast<uint64_t*>(at.hostPointer) : vseq;
        __atomic_store_n(hv, 0ull, __ATOMIC_SEQ_CST);  // faults here if the BAR is not mapped for the host
        std::printf("{\"probe\": \"pingpong_vram\", \"alloc\": \"%s\", \"host_write\": \"ok\"}\n", fname);
        std::fflush(stdout);
        for (uint32_t bytes : {0u, 65536u})
            for (uint32_t P : {1u, 16u}) {
                if (bytes == 0 && P > 1) continue;
                const int iters = 2000;
                std::memset(hack, 0, 64 * 16);
                __atomic_store_n(hv, 0ull, __ATOMIC_SEQ_CST);
                hipStream_t s;
                HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                pingpong_kernel<<<P, 256, 0, s>>>(vseq, dack, ddata, bytes, iters);
                double t0 = 0;
                bool ok = true;
                for (int i = 1; i <= iters && ok; ++i) {
                    if (i == 101) t0 = now_us();
                    __atomic_store_n(hv, (uint64_t)i, __ATOMIC_SEQ_CST);
                    const double ts = now_us();
                    for (uint32_t b = 0; b < P; ++b)
                        while ((uint32_t)__atomic_load_n(hack + 2 * b, __ATOMIC_ACQUIRE) != (uint32_t)i)
                            if (now_us() - ts > 2e6) {
                                ok = false;
                                break;
                            }
                }
                const double t1 = now_us();
                if (!ok) __atomic_store_n(hv, (uint64_t)iters, __ATOMIC_SEQ_CST);
                HIP_OK(hipStreamSynchronize(s));
                HIP_OK(hipStreamDestroy(s));
                std::printf("{\"probe\": \"pingpong_vram\", \"alloc\": \"%s\", \"bytes\": %u, \"workgroups\": %u, "
                            "\"us_per_round\": %.3f, \"ok\": %d}\n",
                            fname, bytes, P, (t1 - t0) / (iters - 100), ok ? 1 : 0);
                std::fflush(stdout);
                if (!ok) return 2;
            }
        HIP_OK(hipFree(vseq));
    }
    return 0;
}
