// Does the written data change the write rate? (diagnostic, GPU box)
// Same rows, same stores; values: 0 zeros, 1 one constant, 2 index-derived
// doubles (every 16 B different), 3 small quotients like the profile's.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int D>
__global__ void __launch_bounds__(512) rows_kernel(double* __restrict__ out, long rows, int M) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const long waves = (long)gridDim.x * 8;
    for (long c = (long)blockIdx.x * 8 + w; c < rows; c += waves) {
        d2* row = reinterpret_cast<d2*>(out + c * M);
        for (int j = lane; j < M / 2; j += 64) {
            d2 v;
            if (D == 0) v = {0.0, 0.0};
            if (D == 1) v = {1.0, 1.0};
            if (D == 2) {
                const unsigned long h = (unsigned long)(c * 1088 + 2 * j) * 0x9E3779B97F4A7C15ull;
                v.x = (double)(h >> 11);
                v.y = (double)((h * 0xBF58476D1CE4E5B9ull) >> 11);
            }
            if (D == 3) {
                const unsigned h = (unsigned)((c * 131 + j * 7) & 15);
                v.x = (double)h / 797.0;
                v.y = (double)(h ^ 5) / 797.0;
            }
            __builtin_nontemporal_store(v, row + j);
        }
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
        printf("%-22s %.4f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    const int g = cus * 4;
    for (int rep = 0; rep < 2; ++rep) {
        run("zeros", [&] { rows_kernel<0><<<g, 512>>>(out, rows, (int)M); });
        run("ones", [&] { rows_kernel<1><<<g, 512>>>(out, rows, (int)M); });
        run("hashed doubles", [&] { rows_kernel<2><<<g, 512>>>(out, rows, (int)M); });
        run("small quotients", [&] { rows_kernel<3><<<g, 512>>>(out, rows, (int)M); });
    }
    return 0;
}
