// Row-write patterns for the profile (diagnostic, GPU box), 200k rows of 8.7 KB,
// next to hipMemsetAsync of the same bytes, in one process:
//   stream   the grid writes one linear stream (thread t: 16-byte unit t + k*threads)
//   wave     one wave per row, rows c = blockIdx*8 + wave + k*stride (the profile's order)
//   waveB    the same with the profile's buffer stores (sc1 nt)
//   waveS    the same with a pause between rows (the profile counts a contig
//            between two rows: ~half of its time); pause p = p x s_sleep 32
//   waveT    one wave per row, the next row from a per-XCD ticket (rows in
//            flight stay a contiguous window)
// Build: hipcc -O3 --offload-arch=gfx950 write_bw6.hip -o write_bw6
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512) stream_k(d2* __restrict__ out, long n2) {
    const long T = (long)gridDim.x * blockDim.x;
    for (long j = (long)blockIdx.x * blockDim.x + threadIdx.x; j < n2; j += T)
        __builtin_nontemporal_store(d2{1.0, (double)j}, out + j);
}

template <int MODE>
__global__ void __launch_bounds__(512) wave_k(double* __restrict__ out, long rows, int M, int pause,
                                              unsigned long long* __restrict__ tickets) {
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long waves = (long)gridDim.x * 8;
    long c = (long)blockIdx.x * 8 + w;
    const int x = blockIdx.x & 7;  // blocks go to the XCDs round-robin
    const long per = (rows + 7) / 8, lo = x * per;
    if (MODE == 3) c = lo + (long)__builtin_amdgcn_readfirstlane(
                                (int)(lane == 0 ? atomicAdd(tickets + 32 * x, 1ull) : 0ull));
    for (; MODE == 3 ? (c < lo + per && c < rows) : c < rows;) {
        long nxt = c + waves;
        if (MODE == 3) {
            unsigned long long t = 0;
            if (lane == 0) t = atomicAdd(tickets + 32 * x, 1ull);
            nxt = lo + (long)__builtin_amdgcn_readfirstlane((int)t);
        }
        if (MODE == 2)
            for (int p = 0; p < pause; ++p) __builtin_amdgcn_s_sleep(32);  // ~0.85 us each
        d2* row = reinterpret_cast<d2*>(out + c * M);
        if (MODE == 1) {
            const unsigned long long u = (unsigned long long)row;
            const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<void*>(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(u >> 32))
                                         << 32) |
                                        (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u)),
                0, M * 8, 0x00020000);
            for (int j = lane; j < M / 2; j += 64) {
                const u32x4 v = {1u, 2u, (unsigned)j, 3u};
                __builtin_amdgcn_raw_buffer_store_b128(v, rr, j * 16, 0, 18);
            }
        } else {
            for (int j = lane; j < M / 2; j += 64) __builtin_nontemporal_store(d2{1.0, (double)j}, row + j);
        }
        c = nxt;
    }
}

int main() {
    const long rows = 200000, M = 1088;
    const long bytes = rows * M * 8;
    double* out;
    unsigned long long* tickets;
    if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&tickets, 8 * 32 * 8) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        const int reps = 10;
        float tot = 0;
        for (int r = 0; r < reps; ++r) {
            hipMemsetAsync(tickets, 0, 8 * 32 * 8);
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            tot += ms;
        }
        const float ms = tot / reps;
        printf("%-28s %.4f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    char nm[64];
    for (int rep = 0; rep < 2; ++rep) {
        run("memset", [&] { hipMemsetAsync(out, 0, bytes); });
        for (int bpc : {1, 2, 4}) {
            snprintf(nm, sizeof nm, "stream %d blk/CU", bpc);
            run(nm, [&] { stream_k<<<cus * bpc, 512>>>(reinterpret_cast<d2*>(out), bytes / 16); });
        }
        for (int bpc : {2, 3, 4}) {
            snprintf(nm, sizeof nm, "wave %d blk/CU", bpc);
            run(nm, [&] { wave_k<0><<<cus * bpc, 512>>>(out, rows, (int)M, 0, tickets); });
            snprintf(nm, sizeof nm, "waveB %d blk/CU", bpc);
            run(nm, [&] { wave_k<1><<<cus * bpc, 512>>>(out, rows, (int)M, 0, tickets); });
            snprintf(nm, sizeof nm, "waveT %d blk/CU", bpc);
            run(nm, [&] { wave_k<3><<<cus * bpc, 512>>>(out, rows, (int)M, 0, tickets); });
        }
        for (int p : {0, 3, 6, 10}) {
            snprintf(nm, sizeof nm, "waveS 3 blk/CU pause %d", p);
            run(nm, [&] { wave_k<2><<<cus * 3, 512>>>(out, rows, (int)M, p, tickets); });
        }
    }
    return 0;
}
