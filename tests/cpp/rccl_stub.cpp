// rccl_stub.cpp — a host-only stand-in for the five RCCL entry points cts_counters_allreduce (cts_collective.cpp)
// resolves with dlsym, built as a shared library by tests/test_host_sanitizers.py and loaded through
// $CTS_RCCL_LIBRARY. "Device" buffers are host memory (the fake HIP of tests/cpp/counters_fold.cpp). It keeps
// RCCL's contract where the engine could get it wrong: ncclCommInitAll refuses duplicate devices, an all-reduce
// of a multi-rank clique outside ncclGroupStart/End fails (one thread would deadlock on the real one), and a
// group must hold exactly one op per rank of every clique it touches, each with the same count and type.
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

struct ncclComm {
    int clique;
    int rank;
    int nranks;
};

namespace {
struct Op {
    const void* send;
    void* recv;
    size_t count;
    ncclDataType_t type;
    ncclRedOp_t op;
    ncclComm_t comm;
};
std::mutex mu;
int depth = 0;
int next_clique = 0;
std::vector<Op> pending;
int live_comms = 0;
}  // namespace

extern "C" {

ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist)
{
    if (std::getenv("STUB_RCCL_FAIL_INIT") != nullptr) return ncclSystemError;
    if (comm == nullptr || ndev <= 0 || devlist == nullptr) return ncclInvalidArgument;
    for (int i = 0; i < ndev; ++i)
        for (int j = 0; j < i; ++j)
            if (devlist[i] == devlist[j]) return ncclInvalidUsage;  // "Duplicate GPU detected"
    std::lock_guard<std::mutex> lk(mu);
    const int c = next_clique++;
    for (int i = 0; i < ndev; ++i) {
        comm[i] = new ncclComm{c, i, ndev};
        ++live_comms;
    }
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm)
{
    if (comm == nullptr) return ncclInvalidArgument;
    std::lock_guard<std::mutex> lk(mu);
    delete comm;
    --live_comms;
    return ncclSuccess;
}

ncclResult_t ncclGroupStart()
{
    std::lock_guard<std::mutex> lk(mu);
    ++depth;
    return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t type, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t)
{
    if (comm == nullptr || send == nullptr || recv == nullptr) return ncclInvalidArgument;
    if (type != ncclUint64 || op != ncclSum) return ncclInvalidArgument;  // all the engine ever asks for
    std::lock_guard<std::mutex> lk(mu);
    if (depth == 0 && comm->nranks > 1) return ncclInvalidUsage;
    pending.push_back(Op{send, recv, count, type, op, comm});
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd()
{
    std::lock_guard<std::mutex> lk(mu);
    if (depth == 0) return ncclInvalidUsage;
    if (--depth > 0) return ncclSuccess;
    std::map<int, std::vector<Op>> by_clique;
    for (const Op& o : pending) by_clique[o.comm->clique].push_back(o);
    pending.clear();
    for (auto& kv : by_clique) {
        std::vector<Op>& ops = kv.second;
        if ((int)ops.size() != ops[0].comm->nranks) return ncclInvalidUsage;
        std::vector<bool> seen(ops.size(), false);
        for (const Op& o : ops) {
            if (seen[o.comm->rank] || o.count != ops[0].count) return ncclInvalidUsage;
            seen[o.comm->rank] = true;
        }
        std::vector<uint64_t> sum(ops[0].count, 0);
        for (const Op& o : ops)
            for (size_t i = 0; i < o.count; ++i) sum[i] += static_cast<const uint64_t*>(o.send)[i];
        for (const Op& o : ops) std::memcpy(o.recv, sum.data(), sum.size() * sizeof(uint64_t));
    }
    return ncclSuccess;
}

// test hook: communicators created and not destroyed
int stub_rccl_live_comms()
{
    std::lock_guard<std::mutex> lk(mu);
    return live_comms;
}

}  // extern "C"
