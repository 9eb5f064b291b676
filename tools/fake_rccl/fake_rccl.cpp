// fake_rccl.cpp — a TEST DOUBLE of the RCCL entry points libkarma_hip.so binds
// (ncclGetUniqueId, ncclCommInitRank, ncclCommDestroy, ncclGetErrorString,
// ncclAllReduce, ncclAllGather, ncclSend, ncclRecv, ncclGroupStart/End), for
// running the library's real communicator code (csrc/comm.hip) with several
// ranks as threads of ONE process on ONE GPU, which real RCCL refuses
// (duplicate devices).  Never on the product path: tests load it in a child
// process through LD_LIBRARY_PATH (libkarma_hip.so's RUNPATH comes after it),
// built as librccl.so.1 by `make -C karma_amd/csrc fake_rccl`.
//
// Semantics, host-staged and blocking (results are what RCCL computes; timing
// is not):
//   * a communicator is the set of ranks that called ncclCommInitRank with one
//     unique id; init returns once all of them have joined;
//   * a collective synchronises the caller's stream (its inputs are complete),
//     stages the send buffer through host memory, meets the other ranks, and
//     writes the receive buffer before returning;
//   * inside ncclGroupStart/End, sends and receives are queued and run at the
//     outermost ncclGroupEnd: all sends first (into per (source, destination)
//     FIFO mailboxes), then the receives, each taking the oldest message from
//     its peer: the k-th send from a to b meets the k-th receive on b from a,
//     as in NCCL.  A receive whose message has a different size fails with
//     ncclInvalidUsage (the peers disagree about the exchange).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unistd.h>
#include <vector>

namespace {

struct Shared {
    int n = 0;
    std::mutex m;
    std::condition_variable cv;
    int joined = 0, refs = 0;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<std::vector<uint8_t>> slot;                            // per-rank payload of a collective
    std::map<std::pair<int, int>, std::deque<std::vector<uint8_t>>> box;  // (src, dst) -> messages
};

std::mutex g_reg_m;
std::map<std::string, std::shared_ptr<Shared>> g_reg;  // open communicators by unique id
std::atomic<uint64_t> g_ids{0};

// a rank waits until all n ranks have arrived (generation barrier)
void barrier(Shared& s, std::unique_lock<std::mutex>& lk) {
    const uint64_t g = s.gen;
    if (++s.arrived == s.n) {
        s.arrived = 0;
        ++s.gen;
        s.cv.notify_all();
    } else {
        s.cv.wait(lk, [&] { return s.gen != g; });
    }
}

size_t dt_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

template <typename T>
void reduce_into(T* acc, const T* x, size_t n, ncclRedOp_t op) {
    for (size_t i = 0; i < n; ++i) {
        switch (op) {
            case ncclSum: acc[i] = acc[i] + x[i]; break;
            case ncclProd: acc[i] = acc[i] * x[i]; break;
            case ncclMax: acc[i] = acc[i] > x[i] ? acc[i] : x[i]; break;
            case ncclMin: acc[i] = acc[i] < x[i] ? acc[i] : x[i]; break;
            default: break;
        }
    }
}

bool reduce_bytes(uint8_t* acc, const uint8_t* x, size_t count, ncclDataType_t t, ncclRedOp_t op) {
    switch (t) {
        case ncclInt8: reduce_into((int8_t*)acc, (const int8_t*)x, count, op); return true;
        case ncclUint8: reduce_into(acc, x, count, op); return true;
        case ncclInt32: reduce_into((int32_t*)acc, (const int32_t*)x, count, op); return true;
        case ncclUint32: reduce_into((uint32_t*)acc, (const uint32_t*)x, count, op); return true;
        case ncclInt64: reduce_into((int64_t*)acc, (const int64_t*)x, count, op); return true;
        case ncclUint64: reduce_into((uint64_t*)acc, (const uint64_t*)x, count, op); return true;
        case ncclFloat32: reduce_into((float*)acc, (const float*)x, count, op); return true;
        case ncclFloat64: reduce_into((double*)acc, (const double*)x, count, op); return true;
        default: return false;
    }
}

struct P2p {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
    ncclComm_t comm;
    hipStream_t stream;
};
thread_local int t_depth = 0;
thread_local std::vector<P2p> t_ops;

}  // namespace

struct ncclComm {
    std::shared_ptr<Shared> sh;
    int rank = 0;
};

namespace {

bool to_host(std::vector<uint8_t>& h, const void* src, size_t bytes, hipStream_t s) {
    if (hipStreamSynchronize(s) != hipSuccess) return false;
    h.resize(bytes);
    return bytes == 0 || hipMemcpy(h.data(), src, bytes, hipMemcpyDefault) == hipSuccess;
}

ncclResult_t run_ops(std::vector<P2p>& ops) {
    for (auto& o : ops)
        if (hipStreamSynchronize(o.stream) != hipSuccess) return ncclUnhandledCudaError;
    for (auto& o : ops) {  // sends first: nothing here waits for a peer
        if (!o.send) continue;
        std::vector<uint8_t> h(o.bytes);
        if (o.bytes && hipMemcpy(h.data(), o.buf, o.bytes, hipMemcpyDefault) != hipSuccess)
            return ncclUnhandledCudaError;
        Shared& s = *o.comm->sh;
        std::lock_guard<std::mutex> lk(s.m);
        s.box[{o.comm->rank, o.peer}].push_back(std::move(h));
        s.cv.notify_all();
    }
    for (auto& o : ops) {
        if (o.send) continue;
        Shared& s = *o.comm->sh;
        std::vector<uint8_t> h;
        {
            std::unique_lock<std::mutex> lk(s.m);
            auto& q = s.box[{o.peer, o.comm->rank}];
            if (!s.cv.wait_for(lk, std::chrono::seconds(120), [&] { return !q.empty(); })) {
                std::fprintf(stderr, "fake_rccl: rank %d timed out waiting for a message from %d\n", o.comm->rank,
                             o.peer);
                return ncclSystemError;
            }
            h = std::move(q.front());
            q.pop_front();
        }
        if (h.size() != o.bytes) {
            std::fprintf(stderr, "fake_rccl: rank %d expected %zu bytes from %d, the send held %zu\n", o.comm->rank,
                         o.bytes, o.peer, h.size());
            return ncclInvalidUsage;
        }
        if (o.bytes && hipMemcpy(o.buf, h.data(), o.bytes, hipMemcpyDefault) != hipSuccess)
            return ncclUnhandledCudaError;
    }
    return ncclSuccess;
}

ncclResult_t p2p(bool send, void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
    const size_t sz = dt_size(t);
    if (!comm || !sz || peer < 0 || peer >= comm->sh->n || (count && !buf)) return ncclInvalidArgument;
    P2p o{send, buf, count * sz, peer, comm, s};
    if (t_depth > 0) {
        t_ops.push_back(o);
        return ncclSuccess;
    }
    std::vector<P2p> one{o};
    return run_ops(one);
}

}  // namespace

extern "C" {

// marker for tests: the process runs this fake, not RCCL
int fake_rccl_marker(void) { return 0x7ACE; }

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (fake_rccl)";
        case ncclUnhandledCudaError: return "unhandled HIP error (fake_rccl)";
        case ncclSystemError: return "system error (fake_rccl)";
        case ncclInvalidArgument: return "invalid argument (fake_rccl)";
        case ncclInvalidUsage: return "invalid usage (fake_rccl)";
        default: return "error (fake_rccl)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id->internal, 0, NCCL_UNIQUE_ID_BYTES);
    std::snprintf(id->internal, NCCL_UNIQUE_ID_BYTES, "fake_rccl:%d:%llu", (int)getpid(),
                  (unsigned long long)g_ids.fetch_add(1));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    const std::string key(id.internal, strnlen(id.internal, NCCL_UNIQUE_ID_BYTES));
    std::shared_ptr<Shared> sh;
    {
        std::lock_guard<std::mutex> lk(g_reg_m);
        auto& e = g_reg[key];
        if (!e) {
            e = std::make_shared<Shared>();
            e->n = nranks;
            e->slot.resize(nranks);
        }
        sh = e;
    }
    if (sh->n != nranks) return ncclInvalidUsage;
    std::unique_lock<std::mutex> lk(sh->m);
    ++sh->joined;
    ++sh->refs;
    sh->cv.notify_all();
    if (!sh->cv.wait_for(lk, std::chrono::seconds(120), [&] { return sh->joined >= sh->n; })) return ncclSystemError;
    lk.unlock();
    {
        std::lock_guard<std::mutex> lk2(g_reg_m);
        auto it = g_reg.find(key);
        if (it != g_reg.end() && it->second == sh) g_reg.erase(it);  // complete: the id is spent
    }
    auto* c = new ncclComm();
    c->sh = sh;
    c->rank = rank;
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t s) {
    const size_t sz = dt_size(t), bytes = count * sz;
    if (!comm || !sz || (count && (!send || !recv))) return ncclInvalidArgument;
    Shared& sh = *comm->sh;
    std::vector<uint8_t> mine;
    if (!to_host(mine, send, bytes, s)) return ncclUnhandledCudaError;
    std::vector<uint8_t> acc;
    {
        std::unique_lock<std::mutex> lk(sh.m);
        sh.slot[comm->rank] = std::move(mine);
        barrier(sh, lk);
        acc = sh.slot[0];
        bool ok = true;
        for (int r = 1; r < sh.n; ++r) ok = ok && reduce_bytes(acc.data(), sh.slot[r].data(), count, t, op);
        barrier(sh, lk);  // every rank has read the slots
        if (!ok) return ncclInvalidArgument;
    }
    if (bytes && hipMemcpy(recv, acc.data(), bytes, hipMemcpyDefault) != hipSuccess) return ncclUnhandledCudaError;
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t s) {
    const size_t sz = dt_size(t), bytes = count * sz;
    if (!comm || !sz || (count && (!send || !recv))) return ncclInvalidArgument;
    Shared& sh = *comm->sh;
    std::vector<uint8_t> mine;
    if (!to_host(mine, send, bytes, s)) return ncclUnhandledCudaError;
    std::vector<uint8_t> all(bytes * sh.n);
    {
        std::unique_lock<std::mutex> lk(sh.m);
        sh.slot[comm->rank] = std::move(mine);
        barrier(sh, lk);
        bool ok = true;
        for (int r = 0; r < sh.n; ++r) {
            if (sh.slot[r].size() != bytes) ok = false;
            else if (bytes) std::memcpy(all.data() + r * bytes, sh.slot[r].data(), bytes);
        }
        barrier(sh, lk);
        if (!ok) return ncclInvalidUsage;  // the ranks disagree about the size
    }
    if (bytes && hipMemcpy(recv, all.data(), bytes * sh.n, hipMemcpyDefault) != hipSuccess)
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
    return p2p(true, const_cast<void*>(buf), count, t, peer, comm, s);
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
    return p2p(false, buf, count, t, peer, comm, s);
}

ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    std::vector<P2p> ops;
    ops.swap(t_ops);
    return run_ops(ops);
}

}  // extern "C"
