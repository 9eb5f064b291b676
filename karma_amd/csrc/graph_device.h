// graph_device.h — device helpers of the read-record graph pipeline
// (graph_sets.hip): the per-read sort/dedup network, the generic walk of reads
// with more than 8 records, a 32-bit mix hash and an LDS bitonic sort.
// Included inside an anonymous namespace.
#pragma once

constexpr int kMaxFast = 8;          // register fast path: reads with <= 8 records
constexpr uint32_t kEmpty = 0xFFFFFFFFu;


// ---- per-read pair walk -------------------------------------------------------
// A read's contigs (<= 8 records, else it is a "big read") sorted by a fixed
// network; keep[p] marks the first copy of each distinct contig and rank[p] is
// its index among the kept ones, so the read emits u - rank[p] entries
// (p, q >= p) with first contig m[p] (u = number of distinct contigs).
struct ReadSet {
    uint32_t m[kMaxFast];
    bool keep[kMaxFast];
    uint32_t rank[kMaxFast];
    uint32_t u;
};

__device__ __forceinline__ void sort_dedup(ReadSet& s) {
#define CE(x, y)                                                       \
    {                                                                  \
        uint32_t lo_ = min(s.m[x], s.m[y]), hi_ = max(s.m[x], s.m[y]); \
        s.m[x] = lo_;                                                  \
        s.m[y] = hi_;                                                  \
    }
    // Batcher odd-even merge sort network, 8 inputs, 19 comparators
    CE(0, 1) CE(2, 3) CE(4, 5) CE(6, 7)
    CE(0, 2) CE(1, 3) CE(4, 6) CE(5, 7)
    CE(1, 2) CE(5, 6)
    CE(0, 4) CE(1, 5) CE(2, 6) CE(3, 7)
    CE(2, 4) CE(3, 5)
    CE(1, 2) CE(3, 4) CE(5, 6)
#undef CE
    uint32_t u = 0;
#pragma unroll
    for (int p = 0; p < kMaxFast; ++p) {
        s.keep[p] = s.m[p] != kEmpty && (p == 0 || s.m[p] != s.m[p - 1]);
        s.rank[p] = u;
        u += s.keep[p] ? 1u : 0u;
    }
    s.u = u;
}


// Arbitrary read size (reads with more than 8 records; rare), O(m^3) over
// global memory, one thread per read.
// contig ids relabelled by map (a bijection of [0, N); the identity below)
template <typename Map, typename Emit>
__device__ inline void read_pairs_slow(karma::RecIn rec, int64_t A, int64_t i, Map map, Emit emit) {
    int64_t end = i + 1;
    while (end < A && rec.cont(end)) ++end;
    for (int64_t p = i; p < end; ++p) {
        const uint32_t c = map(rec.contig(p));
        bool dup = false;
        for (int64_t q = i; q < p && !dup; ++q) dup = map(rec.contig(q)) == c;
        if (dup) continue;
        for (int64_t q = i; q < end; ++q) {
            const uint32_t d = map(rec.contig(q));
            if (d < c) continue;
            bool first = true;
            for (int64_t r = i; r < q && first; ++r) first = map(rec.contig(r)) != d;
            if (first) emit(c, d);
        }
    }
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// Bitonic sort of (key, val) pairs in LDS, n a power of two.  Thread t
// compares elements i = 2t - (t mod stride) and i + stride, so for strides
// <= 64 the lanes of one wave touch only their own 128 elements
// ([2 * t0, 2 * t0 + 128) for the wave's first t0): those steps need the
// wave's LDS ordering only, and block barriers are left to the strides >= 128
// (a 1024-key sort: 6 block barriers instead of 55).
__device__ __forceinline__ void wave_lds_order() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ inline void lds_bitonic(uint32_t* keys, uint32_t* vals, int n) {
    auto step = [&](int size, int stride) {
        for (int t = threadIdx.x; t < n / 2; t += blockDim.x) {
            const int i = 2 * t - (t & (stride - 1));
            const int j = i + stride;
            const bool up = (i & size) == 0;
            const uint32_t ki = keys[i], kj = keys[j];
            if ((ki > kj) == up) {
                keys[i] = kj;
                keys[j] = ki;
                const uint32_t v = vals[i];
                vals[i] = vals[j];
                vals[j] = v;
            }
        }
    };
    for (int size = 2; size <= n; size <<= 1) {
        int stride = size >> 1;
        for (; stride >= 128; stride >>= 1) {
            step(size, stride);
            __syncthreads();
        }
        for (; stride > 0; stride >>= 1) {
            step(size, stride);
            wave_lds_order();
        }
        if (size >= 128) __syncthreads();  // the next size starts with a cross-wave stride
    }
    __syncthreads();
}

// ---- decoupled look-back offsets ------------------------------------------------
// Lists written back to back in one array (the final kernel's buckets, the eq
// path's segment runs): block b's offset is the sum of the lists of blocks < b,
// found by a decoupled look-back (one wave): the block publishes its own size
// at once (kLbAgg), reads its predecessors' words
// 64 at a time from the nearest down, and stops at the first that carries an
// inclusive prefix (kLbPre); block 0 (and the virtual block -1) carry one.
// Predecessors were dispatched first and publish before they wait, so every
// wave's spin ends.
constexpr uint64_t kLbAgg = 1ull << 62, kLbPre = 2ull << 62, kLbVal = kLbAgg - 1;

__device__ inline int64_t lookback_offset(uint64_t* lb, int b, int64_t total, int lane) {
    if (b == 0) {
        if (lane == 0) __hip_atomic_store(&lb[0], kLbPre | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&lb[b], kLbAgg | (uint64_t)total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t excl = 0;
    for (int top = b - 1;; top -= 64) {
        const int idx = top - lane;  // lane 0: the nearest predecessor
        uint64_t v;
        unsigned long long pre, none;
        for (;;) {
            v = idx >= 0 ? __hip_atomic_load(&lb[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbPre;
            pre = __ballot((v & ~kLbVal) == kLbPre);
            none = __ballot((v & ~kLbVal) == 0);
            const unsigned long long need = pre ? (pre & (~pre + 1)) * 2 - 1 : ~0ull;  // lanes up to the first prefix
            if (!(none & need)) break;
            __builtin_amdgcn_s_sleep(1);
        }
        const int first = pre ? __ffsll((long long)pre) - 1 : 64;
        int64_t x = lane <= first ? (int64_t)(v & kLbVal) : 0;
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        excl += x;
        if (pre) break;
    }
    if (lane == 0)
        __hip_atomic_store(&lb[b], kLbPre | (uint64_t)(excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}
