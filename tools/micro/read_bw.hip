// Read patterns of the classify kernel (diagnostic, GPU box): 2.47 GB of
// records, 16-byte loads.
//   chunk   one wave per 64 KB chunk, 4 KB per step (classify today), 256-thread blocks
//   istep   the same steps interleaved: step s of wave w at (s * W + w) * 4 KB
//   stream  grid-stride 16-byte loads, 1 or 4 blocks of 256 per CU
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) chunk_read(const u32x4* __restrict__ in, long n16, unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long chunks = n16 / 4096;  // 64 KB
    const long waves = (long)gridDim.x * 4;
    unsigned acc = 0;
    for (long c = (long)blockIdx.x * 4 + (threadIdx.x >> 6); c < chunks; c += waves) {
        const u32x4* p = in + c * 4096;
        for (int s = 0; s < 16; ++s) {
            u32x4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(p + s * 256 + u * 64 + lane);
#pragma unroll
            for (int u = 0; u < 4; ++u) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) istep_read(const u32x4* __restrict__ in, long n16, unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long steps = n16 / 256;  // 4 KB steps
    const long waves = (long)gridDim.x * 4;
    unsigned acc = 0;
    for (long st = (long)blockIdx.x * 4 + (threadIdx.x >> 6); st < steps; st += waves) {
        const u32x4* p = in + st * 256;
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(p + u * 64 + lane);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc ^= v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) stream_read(const u32x4* __restrict__ in, long n16, unsigned* __restrict__ sink) {
    const long stride = (long)gridDim.x * 256;
    unsigned acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        const u32x4 v = __builtin_nontemporal_load(in + i);
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const long bytes = 2469497688L & ~65535L;
    const long n16 = bytes / 16;
    u32x4* in;
    unsigned* sink;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipMemset(in, 1, bytes);
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
    for (int rep = 0; rep < 2; ++rep) {
        run("chunk  16 blk/CU", [&] { chunk_read<<<cus * 16, 256>>>(in, n16, sink); });
        run("istep  16 blk/CU", [&] { istep_read<<<cus * 16, 256>>>(in, n16, sink); });
        run("stream 1 blk/CU", [&] { stream_read<<<cus, 256>>>(in, n16, sink); });
        run("stream 4 blk/CU", [&] { stream_read<<<cus * 4, 256>>>(in, n16, sink); });
        run("stream 16 blk/CU", [&] { stream_read<<<cus * 16, 256>>>(in, n16, sink); });
    }
    return 0;
}
