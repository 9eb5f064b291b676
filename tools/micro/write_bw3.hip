// Which part of the profile's row phase slows its writes (diagnostic, GPU box).
// Rows as write_bw2 (512-thread blocks, 4 per CU, one wave per 8.7 KB row,
// values from an LDS histogram through an LDS quotient table), plus, by flag:
//   1  a per-row 8-byte total stored by lane 0 to a separate array
//   2  the quotient table rebuilt per row with f64 divisions
//   4  the error test of write_row_wave (a branch per store)
//   8  one scalar-addressed load per row (the next row's offsets)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int F>
__global__ void __launch_bounds__(512) rows_kernel(double* __restrict__ out, long rows, int M, long* __restrict__ tot,
                                                   int* __restrict__ err, const long* __restrict__ offs) {
    __shared__ unsigned cnt[8][576];
    __shared__ double lut[8][64];
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long waves = (long)gridDim.x * 8;
    for (int j = lane; j < 576; j += 64) cnt[w][j] = (j * 7) & 0x3F003F;
    lut[w][lane] = lane * 0.5;
    long klen = 800;
    for (long c = (long)blockIdx.x * 8 + w; c < rows; c += waves) {
        if (F & 8) klen = offs[c + 1] - offs[c];
        if (F & 2) {
            lut[w][lane] = lane ? (double)lane / (double)klen : 0.0;
            __builtin_amdgcn_wave_barrier();
        }
        d2* row = reinterpret_cast<d2*>(out + c * M);
        for (int j = lane; j < M / 2; j += 64) {
            const unsigned ab = cnt[w][j];
            cnt[w][j] = ab;
            const unsigned a = ab & 0xFFFF, b = ab >> 16;
            if ((F & 4) && (a | b) && klen == 0) *err = 1;
            d2 v;
            v.x = lut[w][a & 63];
            v.y = lut[w][b & 63];
            __builtin_nontemporal_store(v, row + j);
        }
        if ((F & 1) && lane == 0) tot[c] = c;
    }
}

int main() {
    const long rows = 200000, M = 1088;
    const long bytes = rows * M * 8;
    double* out;
    long *tot, *offs;
    int* err;
    if (hipMalloc(&out, bytes) != hipSuccess || hipMalloc(&tot, rows * 8) != hipSuccess ||
        hipMalloc(&offs, (rows + 1) * 8) != hipSuccess || hipMalloc(&err, 4) != hipSuccess)
        return 1;
    hipMemset(offs, 0, (rows + 1) * 8);
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
        printf("%-20s %.4f ms  %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    const int g = cus * 4;
#define V(F) run("flags " #F, [&] { rows_kernel<F><<<g, 512>>>(out, rows, (int)M, tot, err, offs); })
    V(0); V(1); V(2); V(4); V(8); V(15);
    V(0); V(1); V(2); V(4); V(8); V(15);
    return 0;
}
