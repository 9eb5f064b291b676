// What lets hipMemsetAsync write 1.74 GB at ~6.5 TB/s when a grid-stride
// non-temporal stream of the same bytes gets ~5.5 (write_bw6)?  Linear
// streams over the profile's byte count with each cache policy of a 16-byte
// buffer store (aux bits: 1 sc0, 2 nt, 16 sc1), plain and non-temporal
// global stores, block sizes and blocks per CU; then the profile's row order
// (one wave per 8.7 KB row) with the best policies.  Diagnostic, GPU box.
// Build: hipcc -O3 --offload-arch=gfx950 write_bw7.hip -o write_bw7
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(void* p, unsigned bytes) {
    const unsigned long long u = (unsigned long long)p;
    return __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                                (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u)),
        0, (int)bytes, 0x00020000);
}

// AUX >= 0: buffer store with that policy; -1 plain global; -2 non-temporal global
template <int AUX>
__global__ void stream_k(u32x4* __restrict__ out, long n16) {
    const long T = (long)gridDim.x * blockDim.x;
    const __amdgpu_buffer_rsrc_t rr = rsrc(out, (unsigned)(n16 * 16 > 0xFFFFFFFFl ? 0xFFFFFFFFu : n16 * 16));
    for (long j = (long)blockIdx.x * blockDim.x + threadIdx.x; j < n16; j += T) {
        const u32x4 v = {1u, (unsigned)j, 2u, 3u};
        if (AUX >= 0) __builtin_amdgcn_raw_buffer_store_b128(v, rr, (int)(j * 16), 0, AUX);
        else if (AUX == -1) out[j] = v;
        else __builtin_nontemporal_store(v, out + j);
    }
}

template <int AUX>
__global__ void __launch_bounds__(512) rows_k(double* __restrict__ out, long rows, int M) {
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long waves = (long)gridDim.x * 8;
    for (long c = (long)blockIdx.x * 8 + w; c < rows; c += waves) {
        double* row = out + c * M;
        const __amdgpu_buffer_rsrc_t rr = rsrc(row, M * 8);
        for (int j = lane; j < M / 2; j += 64) {
            const u32x4 v = {1u, 2u, (unsigned)j, 3u};
            if (AUX >= 0) __builtin_amdgcn_raw_buffer_store_b128(v, rr, j * 16, 0, AUX);
            else reinterpret_cast<u32x4*>(row)[j] = v;
        }
    }
}

int main() {
    const long rows = 200000, M = 1088;
    const long bytes = rows * M * 8, n16 = bytes / 16;
    u32x4* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        const int reps = 10;
        (void)hipEventRecord(a);
        for (int r = 0; r < reps; ++r) launch();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        printf("%-34s %.4f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
        fflush(stdout);
    };
    char nm[80];
    for (int rep = 0; rep < 2; ++rep) {
        run("memset", [&] { (void)hipMemsetAsync(out, 0, bytes); });
        for (int bs : {256, 512, 1024}) {
            for (int bpc : {1, 2}) {
                const int g = cus * bpc;
#define S(AUXV, LBL)                                                               \
    snprintf(nm, sizeof nm, "stream %-9s bs %4d x%d/CU", LBL, bs, bpc);           \
    run(nm, [&] { stream_k<AUXV><<<g, bs>>>(out, n16); });
                S(-1, "plain") S(-2, "nt") S(0, "buf") S(2, "buf nt") S(16, "buf sc1") S(18, "buf sc1nt")
                S(1, "buf sc0") S(3, "buf sc0nt")
#undef S
            }
        }
        for (int bpc : {2, 3}) {
            snprintf(nm, sizeof nm, "rows plain x%d/CU", bpc);
            run(nm, [&] { rows_k<-1><<<cus * bpc, 512>>>(reinterpret_cast<double*>(out), rows, (int)M); });
            snprintf(nm, sizeof nm, "rows buf x%d/CU", bpc);
            run(nm, [&] { rows_k<0><<<cus * bpc, 512>>>(reinterpret_cast<double*>(out), rows, (int)M); });
            snprintf(nm, sizeof nm, "rows buf sc1nt x%d/CU", bpc);
            run(nm, [&] { rows_k<18><<<cus * bpc, 512>>>(reinterpret_cast<double*>(out), rows, (int)M); });
            snprintf(nm, sizeof nm, "rows buf sc1 x%d/CU", bpc);
            run(nm, [&] { rows_k<16><<<cus * bpc, 512>>>(reinterpret_cast<double*>(out), rows, (int)M); });
        }
    }
    return 0;
}
