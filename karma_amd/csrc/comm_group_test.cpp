// Host unit test of comm_group.h (no GPU, no RCCL library): the NCCL entry
// points are scripted here, so error paths that need a failing transport can
// be driven on the CPU.  Built by `make -C karma_amd/csrc comm_group_test`,
// run by tests/test_comm_group_cpu.py.  Exit status 0 = every case passed.
#include <cstdio>
#include <cstring>

#include "comm_group.h"

namespace {
int g_starts = 0, g_ends = 0, g_calls = 0, g_fail_at = -1;
ncclResult_t g_end_rc = ncclSuccess;
int g_bad = 0;

#define EXPECT(c)                                                  \
    do {                                                           \
        if (!(c)) {                                                \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
            ++g_bad;                                               \
        }                                                          \
    } while (0)

void reset(int fail_at, ncclResult_t end_rc = ncclSuccess) {
    g_starts = g_ends = g_calls = 0;
    g_fail_at = fail_at;
    g_end_rc = end_rc;
}
ncclResult_t p2p() { return g_calls++ == g_fail_at ? ncclRemoteError : ncclSuccess; }

// the shape of karma_comm_alltoallv's group: W peers, a send and a recv each
int exchange(int W) {
    karma::NcclGroup g;
    int rc = g.start();
    if (rc) return rc;
    for (int r = 0; r < W; ++r) {
        KARMA_GROUP_ADD(g, p2p());
        KARMA_GROUP_ADD(g, p2p());
    }
    return g.end();
}
// an early return after start() without end(): the destructor closes the group
int early_return() {
    karma::NcclGroup g;
    if (g.start()) return -9;
    KARMA_GROUP_ADD(g, p2p());
    return -1;
}
}  // namespace

extern "C" {
ncclResult_t ncclGroupStart() {
    ++g_starts;
    return ncclSuccess;
}
ncclResult_t ncclGroupEnd() {
    ++g_ends;
    return g_end_rc;
}
const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "scripted error"; }
}

int main() {
    reset(-1);
    EXPECT(exchange(8) == 0 && g_starts == 1 && g_ends == 1 && g_calls == 16);
    for (int at : {0, 1, 5, 15}) {  // a failing send/recv: the rest skipped, the group still closed
        reset(at);
        EXPECT(exchange(8) == -9);
        EXPECT(g_starts == 1 && g_ends == 1);
        EXPECT(g_calls == at + 1);
    }
    reset(-1, ncclInternalError);  // ncclGroupEnd itself failing
    EXPECT(exchange(4) == -9 && g_ends == 1);
    reset(-1);
    EXPECT(early_return() == -1 && g_starts == 1 && g_ends == 1);

    char msg[160];
    int64_t so[4] = {0, 8, 24, 24}, ro[4] = {0, 16, 24, 40};
    int x = 0;
    // rank 1's own slice: 16 sent, 8 received -> refused before any group starts
    EXPECT(!karma::alltoallv_args_ok(3, 1, &x, so, &x, ro, msg, sizeof msg) && std::strstr(msg, "own slice"));
    EXPECT(!karma::alltoallv_args_ok(3, 2, &x, so, &x, ro, msg, sizeof msg));  // own slice 0 vs 16 bytes
    int64_t so2[4] = {0, 8, 24, 40}, ro2[4] = {0, 4, 20, 36};
    EXPECT(karma::alltoallv_args_ok(3, 1, &x, so2, &x, ro2, msg, sizeof msg));
    int64_t dec[4] = {0, 8, 4, 40};
    EXPECT(!karma::alltoallv_args_ok(3, 0, &x, dec, &x, ro2, msg, sizeof msg) && std::strstr(msg, "decrease"));
    EXPECT(!karma::alltoallv_args_ok(3, 0, nullptr, so2, &x, ro2, msg, sizeof msg) && std::strstr(msg, "null"));
    EXPECT(!karma::alltoallv_args_ok(3, 0, &x, nullptr, &x, ro2, msg, sizeof msg));
    EXPECT(!karma::alltoallv_args_ok(3, 3, &x, so2, &x, ro2, msg, sizeof msg));
    std::printf("%s (%d failures)\n", g_bad ? "FAILED" : "ok", g_bad);
    return g_bad ? 1 : 0;
}
