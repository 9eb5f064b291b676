// Write-bandwidth ceiling for the profile's output (1.74 GB of f64 rows):
// grid-stride 16-byte stores, non-temporal or plain, and per-wave rows of the
// profile's shape.  Diagnostic only: tools/micro/write_bw (GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ void __launch_bounds__(256) stream_kernel(d2* __restrict__ out, long n2) {
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) {
        d2 v = {1.0, 2.0};
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}

// one wave per row of M doubles (rows c = wave, wave + waves, ...), as the profile writes
template <bool NT>
__global__ void __launch_bounds__(256) rows_kernel(double* __restrict__ out, long rows, int M) {
    const int lane = threadIdx.x & 63;
    const long waves = (long)gridDim.x * 4;
    for (long c = (long)blockIdx.x * 4 + (threadIdx.x >> 6); c < rows; c += waves) {
        d2* row = reinterpret_cast<d2*>(out + c * M);
        for (int j = lane; j < M / 2; j += 64) {
            d2 v = {1.0, (double)j};
            if (NT) __builtin_nontemporal_store(v, row + j);
            else row[j] = v;
        }
    }
}

int main(int argc, char** argv) {
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
        const int reps = 20;
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        ms /= reps;
        printf("%-28s %.4f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    for (int bpc : {1, 2, 4, 8}) {
        const int g = cus * bpc;
        char nm[64];
        snprintf(nm, sizeof nm, "stream NT  %d blk/CU", bpc);
        run(nm, [&] { stream_kernel<true><<<g, 256>>>(reinterpret_cast<d2*>(out), bytes / 16); });
        snprintf(nm, sizeof nm, "stream st  %d blk/CU", bpc);
        run(nm, [&] { stream_kernel<false><<<g, 256>>>(reinterpret_cast<d2*>(out), bytes / 16); });
        snprintf(nm, sizeof nm, "rows NT    %d blk/CU", bpc);
        run(nm, [&] { rows_kernel<true><<<g, 256>>>(out, rows, (int)M); });
        snprintf(nm, sizeof nm, "rows st    %d blk/CU", bpc);
        run(nm, [&] { rows_kernel<false><<<g, 256>>>(out, rows, (int)M); });
    }
    run("hipMemsetAsync", [&] { hipMemsetAsync(out, 0, bytes); });
    hipFree(out);
    return 0;
}
