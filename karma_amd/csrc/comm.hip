// comm.hip — the library's own RCCL communicator (SURVEY.md §8(b) threading row,
// §8(e)): one communicator per device and process, bound to a karma_ctx, every
// collective enqueued on that context's stream.  The multi-GPU build has two
// exchange steps and they are the only users:
//   * k-mer columns: MAX-allreduce of the presence bytes, all-gather of the
//     exception keys (kmer.py:146-179 is a global sorted union);
//   * shared-read graph: all-to-all-v of pre-reduced (key, count) pairs to the
//     owner of contig a, all-gather of the owners' readset totals.
// The unique id travels between processes through the caller's bootstrap
// (karma_amd/hostgroup.py: a TCP star on the launcher's MASTER_ADDR).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "comm_group.h"
#include "karma_internal.h"

struct karma_comm {
    karma_ctx* ctx = nullptr;
    ncclComm_t nc = nullptr;
    int world = 1, rank = 0;
    size_t scalar_bytes = 64;       // max(64, 8 * world): host scalars one call may reduce
    int32_t* scratch = nullptr;     // device: barrier word / host-scalar staging (scalar_bytes; host side:
                                    // the context's mapped buffer, ctx_mapped)
    int64_t* counts_dev = nullptr;  // device: all-to-all count exchange (2 * world int64)
    // the context's mapped slot for host scalars: a side-stream communicator
    // (KARMA_COMM_SIDE) has its own, so its scalars never alias the main one's
    int scalar_slot = karma::kMapCommScalar;
};

namespace {

#define KARMA_NCCL(expr)                                                                                \
    do {                                                                                                \
        ++::karma::t_hip_calls;                                                                         \
        ncclResult_t _r = (expr);                                                                       \
        if (_r != ncclSuccess) {                                                                        \
            ::karma::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, ncclGetErrorString(_r));    \
            return KARMA_ERR_COMM;                                                                      \
        }                                                                                               \
    } while (0)

int dtype_of(int dt, ncclDataType_t* out, size_t* size) {
    switch (dt) {
        case KARMA_DT_U8: *out = ncclUint8; *size = 1; return KARMA_OK;
        case KARMA_DT_I32: *out = ncclInt32; *size = 4; return KARMA_OK;
        case KARMA_DT_I64: *out = ncclInt64; *size = 8; return KARMA_OK;
        case KARMA_DT_U64: *out = ncclUint64; *size = 8; return KARMA_OK;
        case KARMA_DT_F64: *out = ncclFloat64; *size = 8; return KARMA_OK;
        default: karma::set_error("unknown karma dtype %d", dt); return KARMA_ERR_ARG;
    }
}

int op_of(int op, ncclRedOp_t* out) {
    switch (op) {
        case KARMA_OP_SUM: *out = ncclSum; return KARMA_OK;
        case KARMA_OP_MAX: *out = ncclMax; return KARMA_OK;
        case KARMA_OP_MIN: *out = ncclMin; return KARMA_OK;
        default: karma::set_error("unknown karma reduction op %d", op); return KARMA_ERR_ARG;
    }
}

int comm_begin(karma_comm* c) {
    KARMA_CHECK(c && c->ctx, KARMA_ERR_ARG, "null karma_comm");
    return karma::ctx_begin(c->ctx);
}


}  // namespace

using namespace karma;

namespace {
int group_rc(int rc, const NcclGroup& g) {
    if (rc != KARMA_OK) set_error("%s", g.err);
    return rc;
}

// Host scalars in and out through mapped host memory, moved by a one-block
// kernel: a copy launch to or from host memory waits for free CUs and, to
// host, for the L2 write-back, both slow beside the running profile kernel
// (a 72-byte readback took 0.24 ms there); a kernel writing mapped memory does not.
__global__ void copy_words_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}
}  // namespace

extern "C" {

int karma_comm_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

int karma_comm_unique_id(uint8_t* id) {
    KARMA_CHECK(id, KARMA_ERR_ARG, "null id buffer");
    ncclUniqueId u;
    KARMA_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    return KARMA_OK;
}

int karma_comm_create_ex(karma_ctx* ctx, const uint8_t* id, int world, int rank, int flags, karma_comm** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(id && out && world >= 1 && rank >= 0 && rank < world, KARMA_ERR_ARG,
                "karma_comm_create: bad arguments (world %d, rank %d)", world, rank);
    KARMA_CHECK(world <= 1024, KARMA_ERR_ARG, "karma_comm_create: world %d above 1024", world);
    KARMA_CHECK((flags & ~KARMA_COMM_SIDE) == 0, KARMA_ERR_ARG, "karma_comm_create: unknown flags %d", flags);
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    auto* c = new karma_comm();
    c->ctx = ctx;
    c->world = world;
    c->rank = rank;
    c->scalar_slot = (flags & KARMA_COMM_SIDE) ? kMapSideScalar : kMapCommScalar;
    ncclResult_t r = ncclCommInitRank(&c->nc, world, u, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank(world %d, rank %d): %s", world, rank, ncclGetErrorString(r));
        delete c;
        return KARMA_ERR_COMM;
    }
    c->scalar_bytes = std::max<size_t>(64, 8 * (size_t)world);
    void* p = nullptr;
    int rc = ctx_alloc(ctx, c->scalar_bytes, &p);
    if (rc == KARMA_OK) {
        c->scratch = static_cast<int32_t*>(p);
        rc = ctx_alloc(ctx, 16 * (size_t)world, &p);
        c->counts_dev = static_cast<int64_t*>(p);
    }
    if (rc != KARMA_OK) {
        ncclCommDestroy(c->nc);
        ctx_free(ctx, c->scratch);
        ctx_free(ctx, c->counts_dev);
        delete c;
        return rc;
    }
    *out = c;
    return KARMA_OK;
}

int karma_comm_create(karma_ctx* ctx, const uint8_t* id, int world, int rank, karma_comm** out) {
    return karma_comm_create_ex(ctx, id, world, rank, 0, out);
}

int karma_comm_destroy(karma_comm* c) {
    if (!c) return KARMA_OK;
    if (c->ctx) {
        hipSetDevice(c->ctx->device);
        hipStreamSynchronize(c->ctx->stream);
        ctx_free(c->ctx, c->scratch);
        ctx_free(c->ctx, c->counts_dev);
    }
    if (c->nc) ncclCommDestroy(c->nc);
    delete c;
    return KARMA_OK;
}

int karma_comm_info(karma_comm* c, int* world, int* rank) {
    KARMA_CHECK(c, KARMA_ERR_ARG, "null karma_comm");
    if (world) *world = c->world;
    if (rank) *rank = c->rank;
    return KARMA_OK;
}

int karma_comm_allreduce(karma_comm* c, void* buf_dev, int64_t count, int dtype, int op) {
    KARMA_TRY(comm_begin(c));
    KARMA_CHECK(count >= 0 && (buf_dev || count == 0), KARMA_ERR_ARG, "karma_comm_allreduce: bad buffer");
    ncclDataType_t t;
    size_t sz;
    ncclRedOp_t o;
    KARMA_TRY(dtype_of(dtype, &t, &sz));
    KARMA_TRY(op_of(op, &o));
    if (count == 0) return KARMA_OK;
    KARMA_NCCL(ncclAllReduce(buf_dev, buf_dev, (size_t)count, t, o, c->nc, c->ctx->stream));
    return KARMA_OK;
}

int karma_comm_allreduce_host(karma_comm* c, void* buf_host, int64_t count, int dtype, int op) {
    KARMA_TRY(comm_begin(c));
    ncclDataType_t t;
    size_t sz;
    ncclRedOp_t o;
    KARMA_TRY(dtype_of(dtype, &t, &sz));
    KARMA_TRY(op_of(op, &o));
    KARMA_CHECK(buf_host && count >= 1 && (size_t)count * sz <= c->scalar_bytes, KARMA_ERR_ARG,
                "karma_comm_allreduce_host: 1..%zu bytes of host scalars", c->scalar_bytes);
    const size_t bytes = (size_t)count * sz;
    const int words = (int)((bytes + 7) / 8);
    void *hm = nullptr, *dm = nullptr;
    KARMA_TRY(ctx_mapped(c->ctx, c->scalar_slot, (size_t)words * 8, &hm, &dm));
    std::memcpy(hm, buf_host, bytes);
    ++t_hip_calls;
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(64), 0, c->ctx->stream, static_cast<const uint64_t*>(dm),
                       reinterpret_cast<uint64_t*>(c->scratch), words);
    KARMA_HIP(hipGetLastError());
    KARMA_NCCL(ncclAllReduce(c->scratch, c->scratch, (size_t)count, t, o, c->nc, c->ctx->stream));
    ++t_hip_calls;
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(64), 0, c->ctx->stream,
                       reinterpret_cast<const uint64_t*>(c->scratch), static_cast<uint64_t*>(dm), words);
    KARMA_HIP(hipGetLastError());
    KARMA_HIP(hipStreamSynchronize(c->ctx->stream));
    std::memcpy(buf_host, hm, bytes);
    return KARMA_OK;
}

int karma_comm_barrier(karma_comm* c) {
    int32_t one = 1;
    return karma_comm_allreduce_host(c, &one, 1, KARMA_DT_I32, KARMA_OP_SUM);
}

int karma_comm_allgather(karma_comm* c, const void* send_dev, void* recv_dev, int64_t bytes_per_rank) {
    KARMA_TRY(comm_begin(c));
    KARMA_CHECK(bytes_per_rank >= 0 && (bytes_per_rank == 0 || (send_dev && recv_dev)), KARMA_ERR_ARG,
                "karma_comm_allgather: bad buffers");
    if (bytes_per_rank == 0) return KARMA_OK;
    KARMA_NCCL(ncclAllGather(send_dev, recv_dev, (size_t)bytes_per_rank, ncclUint8, c->nc, c->ctx->stream));
    return KARMA_OK;
}

int karma_comm_exchange_counts(karma_comm* c, const int64_t* send_host, int64_t* recv_host) {
    KARMA_TRY(comm_begin(c));
    KARMA_CHECK(send_host && recv_host, KARMA_ERR_ARG, "karma_comm_exchange_counts: null argument");
    const int W = c->world;
    void *hm = nullptr, *dm = nullptr;
    KARMA_TRY(ctx_mapped(c->ctx, kMapCommCounts, 16 * (size_t)W, &hm, &dm));
    int64_t* pin = static_cast<int64_t*>(hm);
    std::memcpy(pin, send_host, 8 * (size_t)W);
    ++t_hip_calls;
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(64), 0, c->ctx->stream, static_cast<const uint64_t*>(dm),
                       reinterpret_cast<uint64_t*>(c->counts_dev), W);
    KARMA_HIP(hipGetLastError());
    {
        NcclGroup g;
        KARMA_TRY(group_rc(g.start(), g));
        for (int r = 0; r < W; ++r) {
            KARMA_GROUP_ADD(g, ncclSend(c->counts_dev + r, 1, ncclInt64, r, c->nc, c->ctx->stream));
            KARMA_GROUP_ADD(g, ncclRecv(c->counts_dev + W + r, 1, ncclInt64, r, c->nc, c->ctx->stream));
        }
        KARMA_TRY(group_rc(g.end(), g));
    }
    ++t_hip_calls;
    hipLaunchKernelGGL(copy_words_kernel, dim3(1), dim3(64), 0, c->ctx->stream,
                       reinterpret_cast<const uint64_t*>(c->counts_dev + W), static_cast<uint64_t*>(dm) + W, W);
    KARMA_HIP(hipGetLastError());
    KARMA_HIP(hipStreamSynchronize(c->ctx->stream));
    std::memcpy(recv_host, pin + W, 8 * (size_t)W);
    return KARMA_OK;
}

int karma_comm_alltoallv(karma_comm* c, const void* send_dev, const int64_t* send_off, void* recv_dev,
                         const int64_t* recv_off) {
    KARMA_TRY(comm_begin(c));
    const int W = c->world;
    {
        char msg[160];
        KARMA_CHECK(alltoallv_args_ok(W, c->rank, send_dev, send_off, recv_dev, recv_off, msg, sizeof msg),
                    KARMA_ERR_ARG, "karma_comm_alltoallv: %s", msg);
    }
    const uint8_t* s = static_cast<const uint8_t*>(send_dev);
    uint8_t* d = static_cast<uint8_t*>(recv_dev);
    {
        NcclGroup g;
        KARMA_TRY(group_rc(g.start(), g));
        for (int r = 0; r < W; ++r) {
            if (r == c->rank) continue;
            const size_t sb = (size_t)(send_off[r + 1] - send_off[r]), rb = (size_t)(recv_off[r + 1] - recv_off[r]);
            if (sb) KARMA_GROUP_ADD(g, ncclSend(s + send_off[r], sb, ncclUint8, r, c->nc, c->ctx->stream));
            if (rb) KARMA_GROUP_ADD(g, ncclRecv(d + recv_off[r], rb, ncclUint8, r, c->nc, c->ctx->stream));
        }
        KARMA_TRY(group_rc(g.end(), g));
    }
    const size_t own = (size_t)(send_off[c->rank + 1] - send_off[c->rank]);
    if (own)
        KARMA_HIP(hipMemcpyAsync(d + recv_off[c->rank], s + send_off[c->rank], own, hipMemcpyDeviceToDevice,
                                 c->ctx->stream));
    return KARMA_OK;
}

int karma_comm_alltoallv_kv(karma_comm* c, const void* send_a, const void* send_b, const int64_t* send_off,
                            void* recv_a, void* recv_b, const int64_t* recv_off) {
    KARMA_TRY(comm_begin(c));
    const int W = c->world;
    {
        char msg[160];
        KARMA_CHECK(alltoallv_args_ok(W, c->rank, send_a, send_off, recv_a, recv_off, msg, sizeof msg) &&
                        alltoallv_args_ok(W, c->rank, send_b, send_off, recv_b, recv_off, msg, sizeof msg),
                    KARMA_ERR_ARG, "karma_comm_alltoallv_kv: %s", msg);
    }
    const uint8_t *sa = static_cast<const uint8_t*>(send_a), *sb_ = static_cast<const uint8_t*>(send_b);
    uint8_t *da = static_cast<uint8_t*>(recv_a), *db = static_cast<uint8_t*>(recv_b);
    {
        // per peer: part a, then part b, in the same order on both sides
        NcclGroup g;
        KARMA_TRY(group_rc(g.start(), g));
        for (int r = 0; r < W; ++r) {
            if (r == c->rank) continue;
            const size_t sn = (size_t)(send_off[r + 1] - send_off[r]), rn = (size_t)(recv_off[r + 1] - recv_off[r]);
            if (sn) {
                KARMA_GROUP_ADD(g, ncclSend(sa + send_off[r], sn, ncclUint8, r, c->nc, c->ctx->stream));
                KARMA_GROUP_ADD(g, ncclSend(sb_ + send_off[r], sn, ncclUint8, r, c->nc, c->ctx->stream));
            }
            if (rn) {
                KARMA_GROUP_ADD(g, ncclRecv(da + recv_off[r], rn, ncclUint8, r, c->nc, c->ctx->stream));
                KARMA_GROUP_ADD(g, ncclRecv(db + recv_off[r], rn, ncclUint8, r, c->nc, c->ctx->stream));
            }
        }
        KARMA_TRY(group_rc(g.end(), g));
    }
    const size_t own = (size_t)(send_off[c->rank + 1] - send_off[c->rank]);
    if (own) {
        KARMA_HIP(hipMemcpyAsync(da + recv_off[c->rank], sa + send_off[c->rank], own, hipMemcpyDeviceToDevice,
                                 c->ctx->stream));
        KARMA_HIP(hipMemcpyAsync(db + recv_off[c->rank], sb_ + send_off[c->rank], own, hipMemcpyDeviceToDevice,
                                 c->ctx->stream));
    }
    return KARMA_OK;
}

}  // extern "C"
