// Row-write patterns for the profile (diagnostic, GPU box), 8.7 KB rows:
//   wave   one wave per row, rows c = blockIdx*8 + wave + k*stride (the profile today)
//   block8 a 512-thread block writes its 8 consecutive rows as one flat 70 KB region
//   block1 a 512-thread block writes one row at a time, rows c = blockIdx + k*grid
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(512) wave_rows(double* __restrict__ out, long rows, int M) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long waves = (long)gridDim.x * 8;
    for (long c = (long)blockIdx.x * 8 + w; c < rows; c += waves) {
        d2* row = reinterpret_cast<d2*>(out + c * M);
        for (int j = lane; j < M / 2; j += 64) __builtin_nontemporal_store(d2{1.0, (double)j}, row + j);
    }
}

__global__ void __launch_bounds__(512) block8_rows(double* __restrict__ out, long rows, int M) {
    const long groups = (rows + 7) / 8;
    for (long g = blockIdx.x; g < groups; g += gridDim.x) {
        const long r0 = g * 8, nr = rows - r0 < 8 ? rows - r0 : 8;
        d2* base = reinterpret_cast<d2*>(out + r0 * M);
        const int n2 = (int)(nr * M / 2);
        for (int j = threadIdx.x; j < n2; j += 512) __builtin_nontemporal_store(d2{1.0, (double)j}, base + j);
        __syncthreads();
    }
}

__global__ void __launch_bounds__(512) block1_rows(double* __restrict__ out, long rows, int M) {
    for (long c = blockIdx.x; c < rows; c += gridDim.x) {
        d2* row = reinterpret_cast<d2*>(out + c * M);
        for (int j = threadIdx.x; j < M / 2; j += 512) __builtin_nontemporal_store(d2{1.0, (double)j}, row + j);
        __syncthreads();
    }
}

int main() {
    const long rows = 200000, M = 1088;
    const long bytes = rows * M * 8;
    double* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(a);
        const int reps = 10;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        printf("%-24s %.4f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    for (int rep = 0; rep < 2; ++rep)
        for (int bpc : {1, 2, 4}) {
            const int g = cus * bpc;
            char nm[64];
            snprintf(nm, sizeof nm, "wave   %d blk/CU", bpc);
            run(nm, [&] { wave_rows<<<g, 512>>>(out, rows, (int)M); });
            snprintf(nm, sizeof nm, "block8 %d blk/CU", bpc);
            run(nm, [&] { block8_rows<<<g, 512>>>(out, rows, (int)M); });
            snprintf(nm, sizeof nm, "block1 %d blk/CU", bpc);
            run(nm, [&] { block1_rows<<<g, 512>>>(out, rows, (int)M); });
        }
    run("hipMemsetAsync", [&] { hipMemsetAsync(out, 0, bytes); });
    return 0;
}
