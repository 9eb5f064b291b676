// Launch cost on the GPU box (diagnostic): a chain of K small dependent
// kernels per "step", R steps back to back.
//   stream   K hipLaunchKernelGGL per step on one stream
//   fork     the same with a fork/join through a second stream (2 events per step)
//   graph    the step captured once (hipStreamBeginCapture), one hipGraphLaunch per step
//   graphf   the fork/join step captured once
// Prints host microseconds per step (enqueue only) and wall microseconds per
// step (enqueue + device, synchronised at the end), so the device-side gap
// between dependent kernels is wall / K minus the kernel's own time.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

__global__ void tiny(unsigned* p, int i) {
    if (threadIdx.x == 0) atomicAdd(p + (blockIdx.x & 63), (unsigned)i);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? std::atoi(argv[1]) : 16;
    const int R = argc > 2 ? std::atoi(argv[2]) : 400;
    const int G = argc > 3 ? std::atoi(argv[3]) : 256;  // blocks per kernel
    unsigned* d = nullptr;
    CK(hipMalloc(&d, 64 * 4));
    hipStream_t s, s2;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t ea, eb;
    CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
    auto step = [&](bool fork) {
        for (int k = 0; k < K; ++k) {
            if (fork && k == K / 4) {
                CK(hipEventRecord(ea, s));
                CK(hipStreamWaitEvent(s2, ea, 0));
                for (int j = 0; j < 3; ++j) hipLaunchKernelGGL(tiny, dim3(G), dim3(64), 0, s2, d, j);
                CK(hipEventRecord(eb, s2));
            }
            if (fork && k == K / 2) CK(hipStreamWaitEvent(s, eb, 0));
            hipLaunchKernelGGL(tiny, dim3(G), dim3(64), 0, s, d, k);
        }
    };
    for (int mode = 0; mode < 4; ++mode) {
        const bool fork = mode & 1, graph = mode & 2;
        hipGraphExec_t ge = nullptr;
        if (graph) {
            hipGraph_t g;
            CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            step(fork);
            CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphDestroy(g));
        }
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipDeviceSynchronize());
            const double t0 = now_us();
            for (int r = 0; r < R; ++r) {
                if (graph) CK(hipGraphLaunch(ge, s));
                else step(fork);
            }
            const double t1 = now_us();
            CK(hipStreamSynchronize(s));
            const double t2 = now_us();
            std::printf("%-7s K=%d G=%d rep %d: host %.2f us/step, wall %.2f us/step (%.2f us per kernel)\n",
                        graph ? (fork ? "graphf" : "graph") : (fork ? "fork" : "stream"), K, G, rep, (t1 - t0) / R,
                        (t2 - t0) / R, (t2 - t0) / R / (K + (fork ? 3 : 0)));
        }
        if (ge) CK(hipGraphExecDestroy(ge));
    }
    return 0;
}
