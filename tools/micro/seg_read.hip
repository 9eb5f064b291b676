// FETCH_SIZE calibration for the code reduce's access shape (VERDICT r05 item
// 4): is code_seg_reduce_kernel's 213 MiB of FETCH per launch its 207 MB of
// codes read once, or half of a 2x re-read (the guide's x2 correction is
// calibrated for wide contiguous streams only)?  Known byte counts, two shapes:
//   stream  grid-stride 16-byte loads over the whole buffer (the guide's
//           calibrated shape: FETCH_SIZE = 1/2 of the bytes)
//   runs    the reduce's shape: runs of L 16-byte granules, one run per
//           1 KB region of the buffer (its start 16-byte aligned at a hashed
//           offset), a wave takes 64 runs per batch and reads them as one
//           stream of 64 consecutive granules per load instruction (lane j:
//           granule j of the batch's concatenated runs), 16 loads in flight
// Bytes read: stream = the buffer; runs = runs x L x 16.  Each kernel prints
// its time; FETCH_SIZE per dispatch comes from rocprofv3 --pmc FETCH_SIZE.
// Usage: seg_read [L]   (hipcc --offload-arch=gfx950 -O3 -o seg_read seg_read.hip)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) stream_read(const u32x4* __restrict__ in, long n16, unsigned* __restrict__ sink) {
    const long stride = (long)gridDim.x * 256;
    unsigned acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        const u32x4 v = in[i];
        acc ^= v.x + v.y + v.z + v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// run r: granules [r * 64 + off(r), + L) of the buffer (1 KB regions), off <= 64 - L
__device__ __forceinline__ long run_start(long r, int L) {
    const unsigned h = (unsigned)(r * 2654435761u) >> 16;
    return r * 64 + (long)(h % (unsigned)(64 - L + 1));
}

__global__ void __launch_bounds__(1024) runs_read(const u32x4* __restrict__ in, long n_runs, int L,
                                                  unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * 16 + (threadIdx.x >> 6), waves = (long)gridDim.x * 16;
    unsigned acc = 0;
    for (long b = wave * 64; b < n_runs; b += waves * 64) {
        const long nb = min(64L, n_runs - b);
        const long T = nb * L;  // granules of the batch
        for (long j0 = 0; j0 < T; j0 += 64 * 16) {
            u32x4 e[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const long j = j0 + 64 * u + lane;
                if (j < T) {
                    const long r = b + j / L;
                    e[u] = in[run_start(r, L) + j % L];
                }
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (j0 + 64 * u + lane < T) acc ^= e[u].x + e[u].y + e[u].z + e[u].w;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// the back segments' shape: 128-byte aligned segments at random 128-byte slots,
// 8 lanes per segment (8 segments per load instruction), 8 loads in flight
__global__ void __launch_bounds__(1024) seg128_read(const u32x4* __restrict__ in, long n_segs, long n_slots,
                                                    unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * 16 + (threadIdx.x >> 6), waves = (long)gridDim.x * 16;
    unsigned acc = 0;
    for (long s0 = wave * 64; s0 < n_segs; s0 += waves * 64) {
        u32x4 v[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const long sg = s0 + 8 * t + (lane >> 3);
            const long slot = (long)((unsigned)(sg * 2654435761u) % (unsigned)n_slots);
            v[t] = sg < n_segs ? in[slot * 8 + (lane & 7)] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) acc ^= v[t].x + v[t].y + v[t].z + v[t].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int L = argc > 1 ? atoi(argv[1]) : 7;
    const long bytes = 2L << 30;  // 2 GiB: well past the 256 MiB Infinity Cache
    const long n16 = bytes / 16, n_runs = n16 / 64;
    u32x4* in;
    unsigned* sink;
    hipMalloc(&in, bytes);
    hipMalloc(&sink, 4);
    hipMemset(in, 1, bytes);
    int cu = 0;
    hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        float ms = 0;
        hipEventRecord(a);
        stream_read<<<cu * 8, 256>>>(in, n16, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("stream: %.1f MB in %.3f ms = %.0f GB/s\n", bytes / 1e6, ms, bytes / ms / 1e6);
        hipEventRecord(a);
        runs_read<<<cu, 1024>>>(in, n_runs, L, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        const double rb = (double)n_runs * L * 16;
        printf("runs L=%d: %.1f MB in %.3f ms = %.0f GB/s\n", L, rb / 1e6, ms, rb / ms / 1e6);
        const long n_segs = bytes / 128 / 8;  // 1/8 of the slots, ~ the codes' 207 MB at 2 GiB
        hipEventRecord(a);
        seg128_read<<<cu, 1024>>>(in, n_segs, bytes / 128, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("seg128: %.1f MB in %.3f ms = %.0f GB/s\n", n_segs * 128 / 1e6, ms, n_segs * 128 / ms / 1e6);
    }
    hipFree(in);
    hipFree(sink);
    return 0;
}
