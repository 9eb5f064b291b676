// comm_group.h — grouped RCCL point-to-point sections that cannot be left open,
// and the all-to-all-v argument check (comm.hip).  Host code only; unit-tested
// without a GPU against a scripted NCCL (tests/test_comm_group_cpu.py,
// comm_group_test.cpp).
#pragma once
#include <rccl/rccl.h>

#include <cstdint>
#include <cstdio>

namespace karma {

// Every argument is validated before start(); inside the group a failing call
// is recorded and the rest are skipped, and ncclGroupEnd() runs on every path
// (end(), or the destructor on an early return), so no error leaves a group
// open: the next NCCL call on this thread would silently join it, a hang on
// the other ranks rather than an error.
struct NcclGroup {
    ncclResult_t first = ncclSuccess;
    bool started = false;
    char err[192] = {0};

    int start() {
        ncclResult_t r = ncclGroupStart();
        if (r != ncclSuccess) {
            std::snprintf(err, sizeof err, "ncclGroupStart -> %s", ncclGetErrorString(r));
            return -9;  // KARMA_ERR_COMM
        }
        started = true;
        return 0;
    }
    // run `call` unless an earlier call of the group failed
    template <typename F>
    void add(F&& call, const char* expr, int line) {
        if (first != ncclSuccess) return;
        ncclResult_t r = call();
        if (r != ncclSuccess) {
            first = r;
            std::snprintf(err, sizeof err, "comm.hip:%d %s -> %s", line, expr, ncclGetErrorString(r));
        }
    }
    int end() {
        if (!started) return first == ncclSuccess ? 0 : -9;
        started = false;
        ncclResult_t r = ncclGroupEnd();
        if (first != ncclSuccess) return -9;
        if (r != ncclSuccess) {
            std::snprintf(err, sizeof err, "ncclGroupEnd -> %s", ncclGetErrorString(r));
            return -9;
        }
        return 0;
    }
    ~NcclGroup() {
        if (started) ncclGroupEnd();
    }
};
#define KARMA_GROUP_ADD(g, expr) (g).add([&] { return (expr); }, #expr, __LINE__)

// all-to-all-v offsets: W + 1 non-decreasing byte offsets per side, buffers
// present when non-empty, and this rank's own slice the same size on both
// sides (it is copied, not sent).  Checked before any group starts.
inline bool alltoallv_args_ok(int W, int rank, const void* send, const int64_t* so, const void* recv,
                              const int64_t* ro, char* msg, size_t n) {
    if (!so || !ro) return std::snprintf(msg, n, "null offsets"), false;
    if (W < 1 || rank < 0 || rank >= W) return std::snprintf(msg, n, "bad rank %d of %d", rank, W), false;
    if (so[0] < 0 || ro[0] < 0) return std::snprintf(msg, n, "negative offset"), false;
    for (int r = 0; r < W; ++r)
        if (so[r + 1] < so[r] || ro[r + 1] < ro[r]) return std::snprintf(msg, n, "offsets must not decrease"), false;
    if ((!send && so[W] != so[0]) || (!recv && ro[W] != ro[0])) return std::snprintf(msg, n, "null buffer"), false;
    const int64_t s = so[rank + 1] - so[rank], r = ro[rank + 1] - ro[rank];
    if (s != r)
        return std::snprintf(msg, n, "own slice %lld != %lld bytes", (long long)s, (long long)r), false;
    return true;
}

}  // namespace karma
