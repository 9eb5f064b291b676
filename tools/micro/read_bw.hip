// Read patterns of the classify kernel (diagnostic, GPU box): 2.47 GB of
// records, 16-byte loads.
//   chunk   one wave per 64 KB chunk, 4 KB per step (classify today), 256-thread blocks
//   istep   the same steps interleaved: step s of wave w at (s * W + w) * 4 KB
//   stream  grid-stride 16-byte loads, 1 or 4 blocks of 256 per CU
//   one     classify's exact shape: one wave per 64 KB chunk (no loop), grid
//           chunks / 4, 4 waves per SIMD, the next 4 KB step loaded before the
//           current one is consumed; "one+w" also writes 1 KB per 3 steps into
//           the chunk's own output region (classify's 8.4% of writes)
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

// W: 0 read only; 1 nt store every 3rd step; 2 plain store; 3 buffer store
// with cache policy AUX (sc1|nt = 18, as the profile rows); 4 the chunk's
// writes held back and written together at its end (one 5 KB burst)
template <int W, int AUX = 0>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))
one_chunk(const u32x4* __restrict__ in, long n16, u32x4* __restrict__ out, unsigned* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    const long c = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if ((c + 1) * 4096 > n16) return;
    const u32x4* p = in + c * 4096;
    u32x4* o = out + c * 344;  // 16 steps / 3 * 64 lanes, rounded up
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(o, 0, 344 * 16, 0x00020000);
    unsigned acc = 0;
    u32x4 v[4], nx[4], held[5];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(p + u * 64 + lane);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        if (s + 1 < 16) {
#pragma unroll
            for (int u = 0; u < 4; ++u) nx[u] = __builtin_nontemporal_load(p + (s + 1) * 256 + u * 64 + lane);
        }
        u32x4 w = v[0] ^ v[1] ^ v[2] ^ v[3];
        acc ^= w.x + w.y + w.z + w.w;
        if (s % 3 == 2) {
            if (W == 1) __builtin_nontemporal_store(w, o + (s / 3) * 64 + lane);
            if (W == 2) o[(s / 3) * 64 + lane] = w;
            if (W == 3) __builtin_amdgcn_raw_buffer_store_b128(w, rs, ((s / 3) * 64 + lane) * 16, 0, AUX);
            if (W == 4) held[s / 3] = w;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = nx[u];
    }
    if (W == 4) {
#pragma unroll
        for (int i = 0; i < 5; ++i) __builtin_nontemporal_store(held[i], o + i * 64 + lane);
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const long bytes = 2469497688L & ~65535L;
    const long n16 = bytes / 16;
    u32x4* in;
    u32x4* out;
    unsigned* sink;
    if (hipMalloc(&in, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
    if (hipMalloc(&out, (n16 / 4096 + 1) * 344 * 16) != hipSuccess) return 1;
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
        const int ob = (int)((n16 / 4096 + 3) / 4);
        run("one    chunks/4", [&] { one_chunk<0><<<ob, 256>>>(in, n16, out, sink); });
        run("one+w  nt", [&] { one_chunk<1><<<ob, 256>>>(in, n16, out, sink); });
        run("one+w  plain", [&] { one_chunk<2><<<ob, 256>>>(in, n16, out, sink); });
        run("one+w  buf sc1|nt", [&] { one_chunk<3, 18><<<ob, 256>>>(in, n16, out, sink); });
        run("one+w  buf nt", [&] { one_chunk<3, 2><<<ob, 256>>>(in, n16, out, sink); });
        run("one+w  buf sc0|sc1", [&] { one_chunk<3, 17><<<ob, 256>>>(in, n16, out, sink); });
        run("one+w  end burst", [&] { one_chunk<4><<<ob, 256>>>(in, n16, out, sink); });
    }
    return 0;
}
