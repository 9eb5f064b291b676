// sort.hip — the library's own device sort, scan and reduce-by-key (gfx950).
//
// The low-volume paths around the hot pipeline (unsorted records, the generic
// sort-reduce behind bucket overflows, big reads and the relabelled list, the
// exception k-mer keys, the consumers' edge orders, the contig store's word
// offsets, the eq path's scans) sorted and scanned with hipCUB/rocPRIM until
// round 4.  These are their replacements:
//   scan_excl     exclusive prefix sum in ONE launch: a decoupled look-back,
//                 each tile publishing its aggregate at once and its inclusive
//                 prefix as soon as the tiles before it have theirs (tile order
//                 from an atomic ticket, so every predecessor a tile waits for
//                 is already running);
//   radix_sort    stable LSD radix sort of u32/u64 keys with u32 values, 8-bit
//                 digits: per pass a digit histogram per 4,096-key tile, one
//                 scan of the digit-major counts, and a scatter that ranks each
//                 key inside its tile by wave-level digit matches (9 ballots)
//                 and per-wave running counts in LDS (no cross-wave atomics,
//                 so equal digits keep their input order);
//   reduce_sorted the groups of equal adjacent keys of a sorted array: summed
//                 counts and the smallest "first" value (through the sort's
//                 permutation), compacted in two launches.
#include <algorithm>

#include "karma_internal.h"

using namespace karma;

namespace {

// ---- look-back scan ------------------------------------------------------------
constexpr int kST = 256, kSPer = 16, kSTile = kST * kSPer;
constexpr uint64_t kAgg = 1ull << 62, kPre = 2ull << 62, kVal = kAgg - 1;

__device__ __forceinline__ int64_t wave_incl_sum(int64_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// exclusive block scan of one value per thread; *total = the block's sum
__device__ __forceinline__ int64_t block_excl(int64_t v, int64_t* lds_w, int64_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t inc = wave_incl_sum(v);
    if (lane == 63) lds_w[wave] = inc;
    __syncthreads();
    int64_t before = 0, all = 0;
    for (int w = 0; w < kST / 64; ++w) {
        const int64_t s = lds_w[w];
        before += w < wave ? s : 0;
        all += s;
    }
    *total = all;
    __syncthreads();
    return before + inc - v;
}

// inputs of the scan: an array, or the pair count of each eq class
template <typename T>
struct ArrayIn {
    const T* __restrict__ p;
    __device__ int64_t operator()(int64_t i) const { return (int64_t)p[i]; }
};
struct PairCountIn {  // m (m - 1) / 2 for class i of m members, 0 when skipped (and for i = C)
    const int64_t* __restrict__ off;
    const uint8_t* __restrict__ skip;
    int64_t C;
    __device__ int64_t operator()(int64_t i) const {
        if (i >= C) return 0;
        const int64_t m = off[i + 1] - off[i];
        return (skip && skip[i]) ? 0 : m * (m - 1) / 2;
    }
};

// compact eq classes (karma_graph_eq_compact): the member count in bits 0-6,
// the size token "1" in bit 7, unpacked into skip as the sizes are scanned
struct SizeIn {
    const uint8_t* __restrict__ sz;
    uint8_t* __restrict__ skip;
    int64_t C;
    __device__ int64_t operator()(int64_t i) const {
        if (i >= C) return 0;
        const uint32_t v = sz[i];
        skip[i] = (uint8_t)(v >> 7);
        return v & 0x7Fu;
    }
};

template <typename In>
__global__ void __launch_bounds__(kST) scan_lb_kernel(In in, int64_t n, int64_t* __restrict__ out,
                                                      uint64_t* __restrict__ st, unsigned* __restrict__ ticket) {
    __shared__ int64_t lds_w[kST / 64];
    __shared__ int64_t tile_s, excl_s;
    if (threadIdx.x == 0) tile_s = atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t tile = tile_s;
    const int64_t t0 = tile * kSTile;
    // thread t holds items t0 + t * kSPer .. + kSPer - 1 (contiguous)
    int64_t v[kSPer];
    int64_t s = 0;
#pragma unroll
    for (int i = 0; i < kSPer; ++i) {
        const int64_t p = t0 + (int64_t)threadIdx.x * kSPer + i;
        v[i] = p < n ? in(p) : 0;
        s += v[i];
    }
    int64_t total;
    const int64_t x = block_excl(s, lds_w, &total);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        if (tile == 0) {
            if (lane == 0) {
                __hip_atomic_store(&st[0], kPre | (uint64_t)total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                excl_s = 0;
            }
        } else {
            if (lane == 0)
                __hip_atomic_store(&st[tile], kAgg | (uint64_t)total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            int64_t excl = 0;
            for (int64_t top = tile - 1;; top -= 64) {
                const int64_t idx = top - lane;  // lane 0: the nearest predecessor
                uint64_t w;
                unsigned long long pre, none;
                for (;;) {
                    w = idx >= 0 ? __hip_atomic_load(&st[idx], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) : kPre;
                    pre = __ballot((w & ~kVal) == kPre);
                    none = __ballot((w & ~kVal) == 0);
                    const unsigned long long need = pre ? (pre & (~pre + 1)) * 2 - 1 : ~0ull;
                    if (!(none & need)) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                const int first = pre ? __ffsll((long long)pre) - 1 : 64;
                int64_t y = lane <= first ? (int64_t)(w & kVal) : 0;
                for (int o = 32; o > 0; o >>= 1) y += __shfl_xor(y, o);
                excl += y;
                if (pre) break;
            }
            if (lane == 0) {
                __hip_atomic_store(&st[tile], kPre | (uint64_t)(excl + total), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
                excl_s = excl;
            }
        }
    }
    __syncthreads();
    int64_t r = excl_s + x;
#pragma unroll
    for (int i = 0; i < kSPer; ++i) {
        const int64_t p = t0 + (int64_t)threadIdx.x * kSPer + i;
        if (p < n) out[p] = r;
        r += v[i];
    }
}

// ---- radix sort ------------------------------------------------------------------
constexpr int kRT = 256, kRPer = 16, kRTile = kRT * kRPer, kRW = kRT / 64;

// lanes whose digit equals this lane's (d < 512), among the wave's active lanes
__device__ __forceinline__ unsigned long long match9(uint32_t d) {
    unsigned long long m = __ballot(1);
#pragma unroll
    for (int b = 0; b < 9; ++b) {
        const bool bit = (d >> b) & 1u;
        const unsigned long long bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

// per tile: digit counts, one LDS add per distinct digit of a wave's 64 keys
template <typename K>
__global__ void __launch_bounds__(kRT) radix_hist_kernel(const K* __restrict__ keys, int64_t n, int shift,
                                                         int64_t nb, int64_t* __restrict__ cnt) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t c0 = (int64_t)blockIdx.x * kRTile + (int64_t)wave * (kRTile / kRW);
    for (int i = 0; i < kRPer; ++i) {
        const int64_t j = c0 + (int64_t)i * 64 + lane;
        const bool ok = j < n;
        const uint32_t d = ok ? (uint32_t)((keys[j] >> shift) & 255u) : 256u;
        const unsigned long long m = match9(d);
        if (ok && lane == __ffsll((long long)m) - 1) atomicAdd(&h[d], (uint32_t)__popcll(m));
    }
    __syncthreads();
    cnt[(int64_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// Each wave takes a contiguous quarter of the tile, 64 keys at a time, so the
// tile's order is (wave, step, lane); a key's rank inside the tile is its
// wave's base for the digit (the counts of the waves before) plus the running
// count of its digit in its wave.
template <typename K>
__global__ void __launch_bounds__(kRT) radix_scatter_kernel(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                            int64_t n, int shift, int64_t nb,
                                                            const int64_t* __restrict__ off, K* __restrict__ kout,
                                                            uint32_t* __restrict__ vout) {
    __shared__ uint32_t wc[kRW][256];
    __shared__ int64_t boff[256];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int w = 0; w < kRW; ++w) wc[w][threadIdx.x] = 0;
    boff[threadIdx.x] = off[(int64_t)threadIdx.x * nb + blockIdx.x];
    __syncthreads();
    const int64_t c0 = (int64_t)blockIdx.x * kRTile + (int64_t)wave * (kRTile / kRW);
    const unsigned long long lt = (1ull << lane) - 1ull;
    K k[kRPer];
    uint32_t rk[kRPer];
#pragma unroll
    for (int i = 0; i < kRPer; ++i) {
        const int64_t j = c0 + (int64_t)i * 64 + lane;
        const bool ok = j < n;
        k[i] = ok ? kin[j] : K(0);
        const uint32_t d = ok ? (uint32_t)((k[i] >> shift) & 255u) : 256u;
        const unsigned long long m = match9(d);
        const int leader = __ffsll((long long)m) - 1;
        uint32_t old = 0;
        if (ok && lane == leader) {
            old = wc[wave][d];
            wc[wave][d] = old + (uint32_t)__popcll(m);
        }
        old = (uint32_t)__shfl((int)old, leader, 64);
        rk[i] = old + (uint32_t)__popcll(m & lt);
    }
    __syncthreads();
    {  // wave bases per digit (thread = digit)
        uint32_t s = 0;
        for (int w = 0; w < kRW; ++w) {
            const uint32_t c = wc[w][threadIdx.x];
            wc[w][threadIdx.x] = s;
            s += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRPer; ++i) {
        const int64_t j = c0 + (int64_t)i * 64 + lane;
        if (j >= n) continue;
        const uint32_t d = (uint32_t)((k[i] >> shift) & 255u);
        const int64_t pos = boff[d] + wc[wave][d] + rk[i];
        kout[pos] = k[i];
        if (vout) vout[pos] = vin ? vin[j] : (uint32_t)j;
    }
}

// ---- reduce by key on sorted keys -------------------------------------------------
constexpr int kGT = 1024;

__device__ __forceinline__ bool head_at(const uint64_t* __restrict__ k, int64_t i) { return i == 0 || k[i - 1] != k[i]; }

__global__ void __launch_bounds__(kGT) heads_count_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                          int64_t* __restrict__ blk) {
    const int64_t i = (int64_t)blockIdx.x * kGT + threadIdx.x;
    const int c = __syncthreads_count(i < n && head_at(keys, i));
    if (threadIdx.x == 0) blk[blockIdx.x] = c;
}

// Group g's head writes the key, the summed counts (counts[perm[i]], or 1
// each) and the smallest first (first[perm[i]], or perm[i] itself), at the
// number of heads before it (blocks before: blk; inside: ballots).
__global__ void __launch_bounds__(kGT) heads_write_kernel(const uint64_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ perm,
                                                          const int64_t* __restrict__ cin,
                                                          const uint64_t* __restrict__ fin, int64_t n,
                                                          const int64_t* __restrict__ blk,
                                                          uint64_t* __restrict__ uk, int64_t* __restrict__ uc,
                                                          uint64_t* __restrict__ uf, int64_t* __restrict__ n_out) {
    __shared__ int64_t wsum[kGT / 64];
    __shared__ int64_t base_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t b = 0;
    for (int64_t j = threadIdx.x; j < (int64_t)blockIdx.x; j += kGT) b += blk[j];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) b += __shfl_xor(b, d, 64);
    if (lane == 0) wsum[wave] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t s = 0;
        for (int w = 0; w < kGT / 64; ++w) s += wsum[w];
        base_s = s;
    }
    const int64_t i = (int64_t)blockIdx.x * kGT + threadIdx.x;
    const bool h = i < n && head_at(keys, i);
    const unsigned long long m = __ballot(h);
    __syncthreads();
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int64_t before = 0, total = 0;
    for (int w = 0; w < kGT / 64; ++w) {
        if (w < wave) before += wsum[w];
        total += wsum[w];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_out = base_s + total;
    if (!h) return;
    const int64_t o = base_s + before + __popcll(m & ((1ull << lane) - 1ull));
    const uint64_t k = keys[i];
    auto src = [&](int64_t j) -> int64_t { return perm ? (int64_t)perm[j] : j; };
    int64_t c = 0;
    uint64_t f = ~0ull;
    for (int64_t j = i; j < n && keys[j] == k; ++j) {
        const int64_t s = src(j);
        c += cin ? cin[s] : 1;
        const uint64_t fv = fin ? fin[s] : (uint64_t)s;
        f = fv < f ? fv : f;
    }
    uk[o] = k;
    if (uc) uc[o] = c;
    if (uf) uf[o] = f;
}

}  // namespace

namespace karma {

template <typename In>
static int scan_excl(karma_ctx* ctx, In in, int64_t* out, int64_t n) {
    if (n <= 0) return KARMA_OK;
    const int64_t tiles = ceil_div(n, kSTile);
    DevArray<uint64_t> st;
    KARMA_TRY(st.alloc(ctx, tiles + 1));
    KARMA_HIP(hipMemsetAsync(st.ptr, 0, (tiles + 1) * 8, ctx->stream));
    KARMA_LAUNCH(ctx, "scan", scan_lb_kernel<In>, tiles, kST, 0, in, n, out, st.ptr,
                 reinterpret_cast<unsigned*>(st.ptr + tiles));
    return KARMA_OK;
}

int scan_excl_i64(karma_ctx* ctx, const int64_t* in, int64_t* out, int64_t n) {
    return scan_excl(ctx, ArrayIn<int64_t>{in}, out, n);
}

int scan_excl_u32(karma_ctx* ctx, const uint32_t* in, int64_t* out, int64_t n) {
    return scan_excl(ctx, ArrayIn<uint32_t>{in}, out, n);
}

// off[c] = members of the compact classes before c (c <= C), skip[c] = bit 7
int scan_excl_sizes(karma_ctx* ctx, const uint8_t* sizes, uint8_t* skip, int64_t C, int64_t* off) {
    return scan_excl(ctx, SizeIn{sizes, skip, C}, off, C + 1);
}

// out[c] = pairs of the eq classes before c (c <= C; out[C] = all pairs)
int scan_excl_pairs(karma_ctx* ctx, const int64_t* off, const uint8_t* skip, int64_t C, int64_t* out) {
    return scan_excl(ctx, PairCountIn{off, skip, C}, out, C + 1);
}

template <typename K>
static int radix_sort(karma_ctx* ctx, const K* kin, const uint32_t* vin, int64_t n, int key_bits, K* kout,
                      uint32_t* vout) {
    KARMA_CHECK(n >= 0 && n < (int64_t(1) << 32), KARMA_ERR_ARG, "radix_sort: %lld keys", (long long)n);
    KARMA_CHECK(key_bits >= 1 && key_bits <= (int)(8 * sizeof(K)), KARMA_ERR_ARG, "radix_sort: %d key bits",
                key_bits);
    if (n == 0) return KARMA_OK;
    const int passes = (key_bits + 7) / 8;
    const int64_t nb = ceil_div(n, kRTile);
    DevArray<K> kt;
    DevArray<uint32_t> vt;
    DevArray<int64_t> cnt, off;
    KARMA_TRY(kt.alloc(ctx, passes > 1 ? n : 1));
    if (vout) KARMA_TRY(vt.alloc(ctx, passes > 1 ? n : 1));
    KARMA_TRY(cnt.alloc(ctx, 256 * nb));
    KARMA_TRY(off.alloc(ctx, 256 * nb));
    const K* ks = kin;
    const uint32_t* vs = vin;
    for (int p = 0; p < passes; ++p) {
        // the last pass lands in the output: passes - 1 - p even -> out
        const bool to_out = ((passes - 1 - p) & 1) == 0;
        K* kd = to_out ? kout : kt.ptr;
        uint32_t* vd = vout ? (to_out ? vout : vt.ptr) : nullptr;
        KARMA_LAUNCH(ctx, "radix_hist", radix_hist_kernel<K>, nb, kRT, 0, ks, n, 8 * p, nb, cnt.ptr);
        KARMA_TRY(scan_excl_i64(ctx, cnt.ptr, off.ptr, 256 * nb));
        KARMA_LAUNCH(ctx, "radix_scatter", radix_scatter_kernel<K>, nb, kRT, 0, ks, (p == 0 ? vin : vs), n, 8 * p, nb,
                     off.ptr, kd, vd);
        ks = kd;
        vs = vd;
    }
    return KARMA_OK;
}

int radix_sort_u64(karma_ctx* ctx, const uint64_t* kin, const uint32_t* vin, int64_t n, int key_bits,
                   uint64_t* kout, uint32_t* vout) {
    return radix_sort<uint64_t>(ctx, kin, vin, n, key_bits, kout, vout);
}

int radix_sort_u32(karma_ctx* ctx, const uint32_t* kin, const uint32_t* vin, int64_t n, int key_bits,
                   uint32_t* kout, uint32_t* vout) {
    return radix_sort<uint32_t>(ctx, kin, vin, n, key_bits, kout, vout);
}

int reduce_sorted(karma_ctx* ctx, const uint64_t* keys, const uint32_t* perm, const int64_t* cin,
                  const uint64_t* fin, int64_t n, uint64_t* uk, int64_t* uc, uint64_t* uf, int64_t* n_out_dev) {
    if (n <= 0) {
        KARMA_HIP(hipMemsetAsync(n_out_dev, 0, 8, ctx->stream));
        return KARMA_OK;
    }
    const int64_t nb = ceil_div(n, kGT);
    DevArray<int64_t> blk;
    KARMA_TRY(blk.alloc(ctx, nb));
    KARMA_LAUNCH(ctx, "reduce_heads", heads_count_kernel, nb, kGT, 0, keys, n, blk.ptr);
    KARMA_LAUNCH(ctx, "reduce_write", heads_write_kernel, nb, kGT, 0, keys, perm, cin, fin, n, blk.ptr, uk, uc, uf,
                 n_out_dev);
    return KARMA_OK;
}

}  // namespace karma
