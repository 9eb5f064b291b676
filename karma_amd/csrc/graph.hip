// graph.hip — contig x contig shared-read graph for gfx950.
//
// Reference (lmfaber/karma) being replaced:
//   ReadGraph.from_contigs          karma/read_graph.py:19-50  (O(N^2) readset intersections)
//   Contig readsets                 karma/contig.py:4-35       (QNAME set per contig)
//   ReadGraph.update_graph          karma/read_graph.py:192-221
//   ReadGraph.from_equivalence_classes karma/read_graph.py:61-148
//
// Read-record path (the hot one):
//   records {u32 read, u32 contig}, grouped by read (SAM order)
//   K1 graph_count    : per read, dedup its contig set S, count pairs a<=b of S
//                       per (bucket of a, block)        -> hist[bucket][block]
//   scan              : exclusive scan of hist (bucket-major)
//   K3 graph_scatter  : same walk, writes 32-bit entries (a_local << bbits | b)
//                       into the bucket-partitioned array (one write per pair)
//   K4 bucket_reduce  : one block per bucket, LDS open-addressing hash (key ->
//                       count), then LDS bitonic sort -> sorted unique (a,b,count)
//   assemble          : concatenate buckets -> globally sorted (a << 32 | b, count)
// The diagonal (a, a) counts |readset(a)| (the normaliser), so one mechanism
// yields both the shared counts and the totals.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <memory>
#include <cstdlib>

#include "karma_internal.h"

using namespace karma;

struct karma_edges {
    karma_ctx* ctx = nullptr;
    int64_t E = 0, n_contigs = 0;
    DevArray<uint32_t> a, b;
    DevArray<int64_t> s;
    DevArray<double> w;
    DevArray<uint64_t> first;
    DevArray<int64_t> totals;
    bool has_first = false;
};

namespace {

constexpr int kWT = 1024;            // walk threads per block
constexpr int kWalkTile = 4096;      // records per block-chunk granule
// <= 256 walk blocks (32 per XCD): blocks x buckets x 128-B open write lines
// (~1.6 MB per XCD at 391 buckets) stay inside the XCD's 4 MB L2
constexpr int kMaxWalkBlocks = 256;
constexpr int kMaxFast = 8;          // register fast path: reads with <= 8 records
constexpr int kReduceBlock = 512;
constexpr int kTableCap = 8192;      // LDS hash slots per bucket block (64 KB)
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

struct Geo {
    int bw;      // log2 bucket width (contigs per bucket)
    int bbits;   // bits of b
    int64_t n_buckets;
};

int make_geo(int64_t N, Geo* g) {
    KARMA_CHECK(N >= 1 && N <= (int64_t(1) << 24), KARMA_ERR_ARG, "n_contigs %lld out of range [1, 2^24]",
                (long long)N);
    int bbits = 1;
    while ((int64_t(1) << bbits) < N) ++bbits;
    // ~<= 512 coarse buckets: few enough that every block's open write lines
    // (blocks x buckets x 128 B) stay in its XCD's L2, few enough distinct
    // pairs per bucket for one LDS hash table
    int target = 512;
    if (const char* v = getenv("KARMA_BUCKETS_TARGET")) target = std::max(1, atoi(v));
    int bw = 4;
    while ((N >> bw) > target) ++bw;
    KARMA_CHECK(bw + bbits <= 31, KARMA_ERR_ARG, "n_contigs too large for 32-bit entries");
    g->bw = bw;
    g->bbits = bbits;
    g->n_buckets = (N + (int64_t(1) << bw) - 1) >> bw;
    return KARMA_OK;
}

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
template <typename Emit>
__device__ void read_pairs_slow(const uint2* __restrict__ rec, int64_t A, int64_t i, Emit emit) {
    const uint32_t rid = rec[i].x;
    int64_t end = i;
    while (end < A && rec[end].x == rid) ++end;
    for (int64_t p = i; p < end; ++p) {
        const uint32_t c = rec[p].y;
        bool dup = false;
        for (int64_t q = i; q < p && !dup; ++q) dup = rec[q].y == c;
        if (dup) continue;
        for (int64_t q = i; q < end; ++q) {
            const uint32_t d = rec[q].y;
            if (d < c) continue;
            bool first = true;
            for (int64_t r = i; r < q && first; ++r) first = rec[r].y != d;
            if (first) emit(c, d);
        }
    }
}

// COUNT=true : entries per (bucket, block) + order/contig checks + big-read list
// COUNT=false: writes the 32-bit entries (a_local << bbits | b) at bucket-major
//              positions; one LDS cursor reservation per (read, bucket run).
// Every wave walks its own contiguous record range in tiles of 256 records plus
// an 8-record halo (so the <= 9 records a read needs are one unconditional LDS
// gather), with the next tile's loads in flight; waves of a block share only
// the per-bucket counters, so the main loop has no block barrier.
constexpr int kWaveTile = 256;
constexpr int kHalo = kMaxFast;

template <bool COUNT>
__global__ void __launch_bounds__(kWT) walk_kernel(const uint2* __restrict__ rec, int64_t A, int64_t chunk, int bw,
                                                   int bbits, int B, int nblk, uint32_t* __restrict__ hist,
                                                   const int64_t* __restrict__ offs, uint32_t* __restrict__ entries,
                                                   int* __restrict__ flags, uint32_t N, int64_t* __restrict__ big_list,
                                                   unsigned* __restrict__ big_n) {
    constexpr int WPB = kWT / 64;
    constexpr int PER = kWaveTile / 64;
    __shared__ uint2 wrec[WPB][kWaveTile + kHalo];
    __shared__ uint16_t wstart[WPB][kWaveTile];
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];
    unsigned long long* cursor = reinterpret_cast<unsigned long long*>(dyn);  // !COUNT
    uint32_t* cnt = reinterpret_cast<uint32_t*>(dyn);                          // COUNT

    const int64_t blk = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int b = threadIdx.x; b < B; b += blockDim.x) {
        if (COUNT) cnt[b] = 0;
        else cursor[b] = (unsigned long long)offs[(int64_t)b * (nblk + 1) + blk];
    }
    __syncthreads();
    const int64_t blo = blk * chunk, bhi = min(A, blo + chunk);
    const int64_t wchunk = (bhi - blo + WPB - 1) / WPB;
    const int64_t lo = min(bhi, blo + wave * wchunk), hi = min(bhi, lo + wchunk);
    const uint32_t wmask = (1u << bw) - 1u;
    uint2* tr = wrec[wave];
    uint16_t* st_list = wstart[wave];
    int bad_order = 0, bad_contig = 0;

    auto ld = [&](int64_t g) -> uint2 {
        if (g >= A) return make_uint2(kEmpty, kEmpty);
        const unsigned long long v = __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(rec + g));
        return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
    };
    uint2 nxt[PER], nxt_h = make_uint2(kEmpty, kEmpty);
    auto prefetch = [&](int64_t t0) {
        // tile records t0 .. t0+255 (owned if < hi) and halo t0+256 .. +263
#pragma unroll
        for (int u = 0; u < PER; ++u) nxt[u] = (t0 < hi) ? ld(t0 + u * 64 + lane) : make_uint2(kEmpty, kEmpty);
        nxt_h = (t0 < hi && lane < kHalo) ? ld(t0 + kWaveTile + lane) : make_uint2(kEmpty, kEmpty);
    };
    uint32_t prev = lo > 0 ? rec[lo - 1].x : 0u;
    bool has_prev = lo > 0;
    prefetch(lo);
    for (int64_t ts = lo; ts < hi; ts += kWaveTile) {
        const int tn = (int)min<int64_t>(kWaveTile, hi - ts);
#pragma unroll
        for (int u = 0; u < PER; ++u) tr[u * 64 + lane] = nxt[u];
        if (lane < kHalo) tr[kWaveTile + lane] = nxt_h;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        prefetch(ts + kWaveTile);
        // a record past the owned range belongs to the next tile/wave even if
        // it lies in this tile's slots (tn < 256): mask it out of the starts
        int ns = 0;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = u * 64 + lane;
            const uint2 r = tr[j];
            bool s = false;
            if (j < tn) {
                const bool hp = j > 0 || has_prev;
                const uint32_t p = j > 0 ? tr[j - 1].x : prev;
                if (COUNT) {
                    if (hp && p > r.x) bad_order = 1;
                    if (r.y >= N) bad_contig = 1;
                }
                s = !hp || p != r.x;
            }
            const unsigned long long bal = __ballot(s);
            if (s) st_list[ns + __popcll(bal & ((1ull << lane) - 1ull))] = (uint16_t)j;
            ns += __popcll(bal);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int s = lane; s < ns; s += 64) {
            const int j0 = st_list[s];
            // records j0 .. j0+8 are in the tile or its halo (j0 <= 255)
            uint2 r[kMaxFast + 1];
#pragma unroll
            for (int t = 0; t <= kMaxFast; ++t) r[t] = tr[j0 + t];
            const uint32_t rid = r[0].x;
            ReadSet rs;
            bool v = true;
#pragma unroll
            for (int t = 0; t < kMaxFast; ++t) {
                v = v && (t == 0 || r[t].x == rid);
                rs.m[t] = v ? r[t].y : kEmpty;
            }
            const bool big = v && r[kMaxFast].x == rid;
            if (big) {
                if (COUNT) big_list[atomicAdd(big_n, 1u)] = ts + j0;
                continue;
            }
            sort_dedup(rs);
            uint32_t run_b = kEmpty, run_n = 0;
            unsigned long long base[kMaxFast];
            if (COUNT) {
#pragma unroll
                for (int p = 0; p < kMaxFast; ++p) {
                    if (rs.keep[p] && rs.m[p] < N) {
                        const uint32_t b = rs.m[p] >> bw;
                        if (b != run_b) {
                            if (run_n) atomicAdd(&cnt[run_b], run_n);
                            run_b = b;
                            run_n = 0;
                        }
                        run_n += rs.u - rs.rank[p];
                    }
                }
                if (run_n) atomicAdd(&cnt[run_b], run_n);
            } else {
                // reserve per run of one bucket, then write each element's entries
                uint32_t rb = kEmpty, rn = 0;
                int rp0 = 0;
#pragma unroll
                for (int p = 0; p <= kMaxFast; ++p) {
                    const bool valid = p < kMaxFast && rs.keep[p] && rs.m[p] < N;
                    const uint32_t b = valid ? (rs.m[p] >> bw) : kEmpty;
                    if (p == kMaxFast || (valid && b != rb)) {
                        if (rn) {
                            unsigned long long pos = atomicAdd(&cursor[rb], (unsigned long long)rn);
#pragma unroll
                            for (int q = 0; q < kMaxFast; ++q) {
                                if (q >= rp0 && q < p && rs.keep[q] && rs.m[q] < N) {
                                    base[q] = pos;
                                    pos += rs.u - rs.rank[q];
                                }
                            }
                        }
                        if (valid) {
                            rb = b;
                            rn = 0;
                            rp0 = p;
                        }
                    }
                    if (valid) rn += rs.u - rs.rank[p];
                }
#pragma unroll
                for (int p = 0; p < kMaxFast; ++p) {
                    if (!(rs.keep[p] && rs.m[p] < N)) continue;
                    const uint32_t hi_key = (rs.m[p] & wmask) << bbits;
                    unsigned long long pos = base[p];
#pragma unroll
                    for (int q = p; q < kMaxFast; ++q) {
                        if (rs.keep[q] && rs.m[q] < N) entries[pos++] = hi_key | rs.m[q];
                    }
                }
            }
        }
        prev = tr[tn - 1].x;
        has_prev = true;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (COUNT) {
        if (bad_order) flags[0] = 1;
        if (bad_contig) flags[1] = 1;
        __syncthreads();
        for (int b = threadIdx.x; b < B; b += blockDim.x) hist[(int64_t)b * (nblk + 1) + blk] = cnt[b];
    }
}

// Reads with more than 8 records: one thread per read, the virtual last block
// column of the histogram (global atomics; rare).
template <bool SCATTER>
__global__ void big_reads_kernel(const uint2* __restrict__ rec, int64_t A, const int64_t* __restrict__ big_list,
                                 int64_t n_big, int bw, int bbits, int nblk, uint32_t* __restrict__ hist,
                                 unsigned long long* __restrict__ cursor, uint32_t* __restrict__ entries, uint32_t N) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_big) return;
    const uint32_t wmask = (1u << bw) - 1u;
    read_pairs_slow(rec, A, big_list[k], [&](uint32_t a, uint32_t b) {
        if (b >= N) return;
        const uint32_t bucket = a >> bw;
        if (SCATTER) entries[atomicAdd(&cursor[bucket], 1ull)] = ((a & wmask) << bbits) | b;
        else atomicAdd(&hist[(int64_t)bucket * (nblk + 1) + nblk], 1u);
    });
}

__global__ void big_cursor_kernel(const int64_t* __restrict__ offs, int B, int nblk,
                                  unsigned long long* __restrict__ cursor) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < B) cursor[b] = (unsigned long long)offs[(int64_t)b * (nblk + 1) + nblk];
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// Bitonic sort of (key, val) pairs in LDS, n = power of two <= kTableCap.
__device__ void lds_bitonic(uint32_t* keys, uint32_t* vals, int n) {
    for (int size = 2; size <= n; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
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
            __syncthreads();
        }
    }
}

// ---- bucket reduction ----------------------------------------------------------
// LDS open-addressing table (key -> count) of kTableCap slots.  A block inserts
// at most kIter keys between capacity checks, so it never fills up: past
// kTableCap - kIter distinct keys it raises the bucket's overflow flag and the
// bucket goes to the generic sort-reduce path.
constexpr int64_t kIter = 4 * kReduceBlock;
constexpr int64_t kSlice = 131072;  // entries per slice block (load balance)

struct Table {
    uint32_t* keys;
    uint32_t* vals;
    int* nuniq;
    __device__ void init() {
        for (int t = threadIdx.x; t < kTableCap; t += blockDim.x) {
            keys[t] = kEmpty;
            vals[t] = 0;
        }
        if (threadIdx.x == 0) *nuniq = 0;
    }
    __device__ __forceinline__ void insert(uint32_t key, uint32_t c) {
        uint32_t h = hash32(key) & (kTableCap - 1);
        while (true) {
            const uint32_t k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (k == key) {
                atomicAdd(&vals[h], c);
                return;
            }
            if (k == kEmpty) {
                const uint32_t old = atomicCAS(&keys[h], kEmpty, key);
                if (old == kEmpty || old == key) {
                    if (old == kEmpty) atomicAdd(nuniq, 1);
                    atomicAdd(&vals[h], c);
                    return;
                }
            }
            h = (h + 1) & (kTableCap - 1);
        }
    }
    // compact occupied slots to the front; returns their number (all threads)
    __device__ int compact(int* cnt) {
        if (threadIdx.x == 0) *cnt = 0;
        __syncthreads();
        uint32_t my_k[kTableCap / kReduceBlock], my_v[kTableCap / kReduceBlock];
#pragma unroll
        for (int u = 0; u < kTableCap / kReduceBlock; ++u) {
            const int t = u * kReduceBlock + threadIdx.x;
            my_k[u] = keys[t];
            my_v[u] = vals[t];
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kTableCap / kReduceBlock; ++u) {
            if (my_k[u] != kEmpty) {
                const int pos = atomicAdd(cnt, 1);
                keys[pos] = my_k[u];
                vals[pos] = my_v[u];
            }
        }
        __syncthreads();
        return *cnt;
    }
};

// sorted (global key, count) list of a bucket into its slot region
__device__ void emit_sorted(Table& t, int n, int64_t bucket, int bw, int bbits, uint64_t* __restrict__ out_keys,
                           int64_t* __restrict__ out_counts, int64_t* __restrict__ out_n) {
    int p2 = 1;
    while (p2 < n) p2 <<= 1;
    for (int i = n + threadIdx.x; i < p2; i += blockDim.x) {
        t.keys[i] = kEmpty;
        t.vals[i] = 0;
    }
    __syncthreads();
    lds_bitonic(t.keys, t.vals, p2);
    const uint32_t bmask = (1u << bbits) - 1u;
    const uint64_t abase = (uint64_t)bucket << bw;
    uint64_t* ok = out_keys + bucket * (int64_t)kTableCap;
    int64_t* oc = out_counts + bucket * (int64_t)kTableCap;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t k = t.keys[i];
        ok[i] = ((abase + (k >> bbits)) << 32) | (k & bmask);
        oc[i] = (int64_t)t.vals[i];
    }
    if (threadIdx.x == 0) out_n[bucket] = n;
}

// One block per slice [s, e) of a bucket's entries.  A bucket with one slice
// is finalised here; otherwise the slice's partial (key, count) list goes to
// part_* for bucket_merge_kernel.
__global__ void __launch_bounds__(kReduceBlock) slice_reduce_kernel(
    const uint32_t* __restrict__ entries, const int64_t* __restrict__ sl_bucket, const int64_t* __restrict__ sl_lo,
    const int64_t* __restrict__ sl_hi, const uint8_t* __restrict__ single, int bw, int bbits,
    uint64_t* __restrict__ out_keys, int64_t* __restrict__ out_counts, int64_t* __restrict__ out_n,
    uint32_t* __restrict__ part_keys, uint32_t* __restrict__ part_cnt, int* __restrict__ part_n,
    uint8_t* __restrict__ overflow) {
    __shared__ uint32_t keys[kTableCap];
    __shared__ uint32_t vals[kTableCap];
    __shared__ int nuniq, cnt, ovf;
    Table t{keys, vals, &nuniq};
    const int64_t sl = blockIdx.x, bucket = sl_bucket[sl], s = sl_lo[sl], e = sl_hi[sl];
    t.init();
    if (threadIdx.x == 0) ovf = 0;
    __syncthreads();
    // 16-byte loads (4 entries per lane), the next iteration's loads issued
    // before the current one is inserted
    const int64_t a0 = s & ~int64_t(3);
    auto load4 = [&](int64_t base) -> uint4 {
        const int64_t i = base + 4 * threadIdx.x;
        return i < e ? *reinterpret_cast<const uint4*>(entries + i) : make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
    };
    uint4 nxt = load4(a0);
    for (int64_t base = a0; base < e; base += kIter) {
        if (nuniq > kTableCap - kIter) {
            if (threadIdx.x == 0) ovf = 1;
            break;
        }
        const uint4 cur = nxt;
        nxt = load4(base + kIter);
        const uint32_t v[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t i = base + 4 * threadIdx.x + u;
            if (i >= s && i < e) t.insert(v[u], 1u);
        }
        __syncthreads();
    }
    __syncthreads();
    if (ovf) {
        if (threadIdx.x == 0) overflow[bucket] = 1;
        return;
    }
    const int n = t.compact(&cnt);
    if (single[sl]) {
        emit_sorted(t, n, bucket, bw, bbits, out_keys, out_counts, out_n);
    } else {
        uint32_t* pk = part_keys + sl * (int64_t)kTableCap;
        uint32_t* pc = part_cnt + sl * (int64_t)kTableCap;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            pk[i] = keys[i];
            pc[i] = vals[i];
        }
        if (threadIdx.x == 0) part_n[sl] = n;
    }
}

// One block per multi-slice bucket: merge its slices' partial lists.
__global__ void __launch_bounds__(kReduceBlock) bucket_merge_kernel(
    const int64_t* __restrict__ mb_bucket, const int64_t* __restrict__ mb_s0, const int64_t* __restrict__ mb_s1,
    int bw, int bbits, const uint32_t* __restrict__ part_keys, const uint32_t* __restrict__ part_cnt,
    const int* __restrict__ part_n, uint64_t* __restrict__ out_keys, int64_t* __restrict__ out_counts,
    int64_t* __restrict__ out_n, uint8_t* __restrict__ overflow) {
    __shared__ uint32_t keys[kTableCap];
    __shared__ uint32_t vals[kTableCap];
    __shared__ int nuniq, cnt;
    Table t{keys, vals, &nuniq};
    const int64_t bucket = mb_bucket[blockIdx.x], s0 = mb_s0[blockIdx.x], s1 = mb_s1[blockIdx.x];
    if (overflow[bucket]) return;  // a slice overflowed: generic path
    t.init();
    __syncthreads();
    // insert the partial lists in chunks of <= kIter keys with the same
    // capacity test as the slice kernel
    for (int64_t sl = s0; sl < s1; ++sl) {
        const int n = part_n[sl];
        for (int c0 = 0; c0 < n; c0 += (int)kIter) {
            if (nuniq > kTableCap - kIter) {
                __syncthreads();
                if (threadIdx.x == 0) overflow[bucket] = 1;
                return;
            }
            const int c1 = min(n, c0 + (int)kIter);
            for (int i = c0 + threadIdx.x; i < c1; i += blockDim.x)
                t.insert(part_keys[sl * (int64_t)kTableCap + i], part_cnt[sl * (int64_t)kTableCap + i]);
            __syncthreads();
        }
    }
    const int n = t.compact(&cnt);
    emit_sorted(t, n, bucket, bw, bbits, out_keys, out_counts, out_n);
}

// Copies each bucket's sorted list (from its slot region or an overflow buffer)
// to its final offset.
__global__ void assemble_kernel(const uint64_t* const* __restrict__ src_k, const int64_t* const* __restrict__ src_c,
                                const int64_t* __restrict__ n_per, const int64_t* __restrict__ dst_off,
                                uint64_t* __restrict__ keys, int64_t* __restrict__ counts) {
    const int64_t b = blockIdx.x;
    const int64_t n = n_per[b], d = dst_off[b];
    const uint64_t* sk = src_k[b];
    const int64_t* sc = src_c[b];
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
        keys[d + t] = sk[t];
        counts[d + t] = sc[t];
    }
}

__global__ void fill_ptrs_kernel(const uint64_t* base_k, const int64_t* base_c, int64_t n_buckets, int64_t stride,
                                 const uint64_t** pk, const int64_t** pc) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n_buckets) {
        pk[b] = base_k + b * stride;
        pc[b] = base_c + b * stride;
    }
}

// bucket b gets entries of every block: hist[b][*]; bstart = exclusive scan of bucket totals
__global__ void bucket_bounds_kernel(const int64_t* __restrict__ offs, int64_t n_buckets, int64_t n_blocks,
                                     int64_t total, int64_t* __restrict__ bstart) {
    int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n_buckets) bstart[b] = offs[b * n_blocks];
    if (b == n_buckets) bstart[b] = total;
}

// Overflowed bucket -> u64 global keys (generic path input)
__global__ void widen_kernel(const uint32_t* __restrict__ entries, int64_t s, int64_t n, uint64_t abase, int bbits,
                             uint64_t* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t k = entries[s + i];
        out[i] = ((abase + (k >> bbits)) << 32) | (k & ((1u << bbits) - 1u));
    }
}

__global__ void fill_ones_kernel(int64_t* __restrict__ v, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = 1;
}

// ---- generic sort + reduce (low-volume paths) ----------------------------------
__global__ void iota_kernel(uint32_t* __restrict__ v, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}

__global__ void gather_kernel(const uint32_t* __restrict__ idx, const int64_t* __restrict__ c_in,
                              const uint64_t* __restrict__ f_in, int64_t n, int64_t* __restrict__ c_out,
                              uint64_t* __restrict__ f_out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t j = idx[i];
        c_out[i] = c_in ? c_in[j] : 1;
        if (f_out) f_out[i] = f_in ? f_in[j] : (uint64_t)j;
    }
}

struct MinOp {
    __device__ __forceinline__ uint64_t operator()(const uint64_t& a, const uint64_t& b) const { return a < b ? a : b; }
};

// ---- eq classes -----------------------------------------------------------------
__global__ void eq_totals_kernel(const int64_t* __restrict__ cls_off, const uint32_t* __restrict__ members,
                                 const int64_t* __restrict__ counts, int64_t n_classes, uint32_t n_contigs,
                                 unsigned long long* __restrict__ totals, int64_t* __restrict__ pair_cnt,
                                 const uint8_t* __restrict__ skip, int* __restrict__ bad) {
    int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_classes) return;
    const int64_t s = cls_off[c], e = cls_off[c + 1], m = e - s;
    const unsigned long long cnt = (unsigned long long)counts[c];
    for (int64_t t = s; t < e; ++t) {
        const uint32_t x = members[t];
        if (x >= n_contigs) {
            *bad = 1;
            continue;
        }
        atomicAdd(&totals[x], cnt);  // two's complement: exact for negative counts too
    }
    pair_cnt[c] = (skip && skip[c]) ? 0 : m * (m - 1) / 2;
}

__global__ void eq_emit_kernel(const int64_t* __restrict__ cls_off, const uint32_t* __restrict__ members,
                               const int64_t* __restrict__ counts, const int64_t* __restrict__ pair_off,
                               int64_t n_classes, int64_t P, uint64_t* __restrict__ keys, int64_t* __restrict__ cnt_out) {
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    // class = last c with pair_off[c] <= p
    int64_t lo = 0, hi = n_classes;
    while (hi - lo > 1) {
        int64_t mid = (lo + hi) >> 1;
        if (pair_off[mid] <= p) lo = mid;
        else hi = mid;
    }
    // skip empty classes that share the offset
    int64_t c = lo;
    const int64_t t = p - pair_off[c];
    const int64_t s = cls_off[c], m = cls_off[c + 1] - s;
    // combinations order: row i holds pairs (i, i+1..m-1); cum(i) = i*m - i*(i+1)/2
    int64_t il = 0, ih = m - 1;
    while (ih - il > 1) {
        int64_t mid = (il + ih) >> 1;
        if (mid * m - mid * (mid + 1) / 2 <= t) il = mid;
        else ih = mid;
    }
    const int64_t i = il, j = i + 1 + (t - (i * m - i * (i + 1) / 2));
    const uint32_t a = members[s + i], b = members[s + j];
    const uint32_t lo2 = min(a, b), hi2 = max(a, b);
    keys[p] = ((uint64_t)lo2 << 32) | hi2;
    cnt_out[p] = counts[c];
}

// ---- finalize --------------------------------------------------------------------
__global__ void diag_totals_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts, int64_t n,
                                   int64_t* __restrict__ totals) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint64_t k = keys[i];
        const uint32_t a = (uint32_t)(k >> 32), b = (uint32_t)k;
        if (a == b) totals[a] = counts[i];
    }
}

__global__ void edge_flags_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts, int64_t n,
                                  int mode, int64_t* __restrict__ flags) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint64_t k = keys[i];
        const bool diag = (uint32_t)(k >> 32) == (uint32_t)k;
        flags[i] = (counts[i] != 0 && !(diag && mode == KARMA_MODE_READS)) ? 1 : 0;
    }
}

__global__ void edge_write_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts,
                                  const uint64_t* __restrict__ first, const int64_t* __restrict__ flags,
                                  const int64_t* __restrict__ pos, int64_t n, const int64_t* __restrict__ totals,
                                  uint32_t* __restrict__ ea, uint32_t* __restrict__ eb, int64_t* __restrict__ es,
                                  double* __restrict__ ew, uint64_t* __restrict__ ef, int* __restrict__ zero_div) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flags[i]) return;
    const int64_t o = pos[i];
    const uint64_t k = keys[i];
    const uint32_t a = (uint32_t)(k >> 32), b = (uint32_t)k;
    const int64_t s = counts[i], ta = totals[a], tb = totals[b];
    ea[o] = a;
    eb[o] = b;
    es[o] = s;
    if (ef) ef[o] = first[i];
    if (ta == 0 || tb == 0) {
        *zero_div = 1;
        ew[o] = 0.0;
        return;
    }
    // read_graph.py:39-42 / :128-130: ((s / tA) + (s / tB)) / 2, IEEE binary64, no FMA
    const double x = __ddiv_rn((double)s, (double)ta);
    const double y = __ddiv_rn((double)s, (double)tb);
    ew[o] = __dadd_rn(x, y) * 0.5;
}

int scan_i64(karma_ctx* ctx, const int64_t* in, int64_t* out, int64_t n) {
    size_t tb = 0;
    KARMA_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, ctx->stream));
    DevArray<uint8_t> tmp;
    KARMA_TRY(tmp.alloc(ctx, tb));
    KARMA_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.ptr, tb, in, out, n, ctx->stream));
    return KARMA_OK;
}

__global__ void u32_to_i64_kernel(const uint32_t* __restrict__ in, int64_t* __restrict__ out, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = in[i];
}

int grid1(int64_t n, int block = 256) { return (int)std::max<int64_t>(1, ceil_div(n, block)); }

// Records path into a pair list (records already on the device, grouped by read).
int records_to_pairs(karma_ctx* ctx, const uint2* rec, int64_t A, int64_t N, karma_pairs* out) {
    Geo g;
    KARMA_TRY(make_geo(N, &g));
    const int B = (int)g.n_buckets;
    constexpr int kTileCount = kWalkTile;
    // persistent-style grid: <= 1024 blocks, each a contiguous run of whole tiles
    int64_t nblk = std::max<int64_t>(1, std::min<int64_t>(kMaxWalkBlocks, ceil_div(A, kTileCount)));
    const int64_t chunk = std::max<int64_t>(kTileCount, ceil_div(ceil_div(A, nblk), kTileCount) * kTileCount);
    nblk = std::max<int64_t>(1, ceil_div(A, chunk));
    const int64_t H = (int64_t)B * (nblk + 1);  // last column: reads with > 8 records
    DevArray<uint32_t> hist;
    DevArray<int64_t> hist64, offs, bstart, big_list;
    DevArray<int> flags;
    DevArray<unsigned> big_n;
    KARMA_TRY(hist.alloc(ctx, H));
    KARMA_TRY(hist64.alloc(ctx, H + 1));
    KARMA_TRY(offs.alloc(ctx, H + 1));
    KARMA_TRY(bstart.alloc(ctx, g.n_buckets + 1));
    KARMA_TRY(flags.alloc(ctx, 2));
    KARMA_TRY(big_n.alloc(ctx, 1));
    KARMA_TRY(big_list.alloc(ctx, A / (kMaxFast + 1) + 1));
    KARMA_HIP(hipMemsetAsync(flags.ptr, 0, 8, ctx->stream));
    KARMA_HIP(hipMemsetAsync(big_n.ptr, 0, 4, ctx->stream));
    KARMA_HIP(hipMemsetAsync(hist.ptr, 0, H * 4, ctx->stream));
    if (A > 0)
        KARMA_LAUNCH(ctx, "graph_count", walk_kernel<true>, nblk, kWT, B * 4, rec, A, chunk, g.bw, g.bbits, B,
                     (int)nblk, hist.ptr, (const int64_t*)nullptr, (uint32_t*)nullptr, flags.ptr, (uint32_t)N,
                     big_list.ptr, big_n.ptr);
    int hflags[2];
    unsigned n_big = 0;
    KARMA_HIP(hipMemcpyAsync(hflags, flags.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipMemcpyAsync(&n_big, big_n.ptr, 4, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_CHECK(!hflags[0], KARMA_ERR_UNSORTED, "records are not grouped by read (read ids decrease)");
    KARMA_CHECK(!hflags[1], KARMA_ERR_ARG, "a record's contig index is >= n_contigs (%lld)", (long long)N);
    if (n_big)
        KARMA_LAUNCH(ctx, "graph_big_count", big_reads_kernel<false>, grid1(n_big, 64), 64, 0, rec, A, big_list.ptr,
                     (int64_t)n_big, g.bw, g.bbits, (int)nblk, hist.ptr, (unsigned long long*)nullptr,
                     (uint32_t*)nullptr, (uint32_t)N);
    KARMA_LAUNCH(ctx, "hist_widen", u32_to_i64_kernel, grid1(H), 256, 0, hist.ptr, hist64.ptr, H);
    KARMA_HIP(hipMemsetAsync(hist64.ptr + H, 0, 8, ctx->stream));
    KARMA_TRY(scan_i64(ctx, hist64.ptr, offs.ptr, H + 1));
    int64_t total = 0;
    KARMA_HIP(hipMemcpyAsync(&total, offs.ptr + H, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_LAUNCH(ctx, "bucket_bounds", bucket_bounds_kernel, grid1(g.n_buckets + 1), 256, 0, offs.ptr, g.n_buckets,
                 nblk + 1, total, bstart.ptr);
    DevArray<uint32_t> entries;
    KARMA_TRY(entries.alloc(ctx, total + 4));  // +4: 16-byte loads past the end
    if (A > 0)
        KARMA_LAUNCH(ctx, "graph_scatter", walk_kernel<false>, nblk, kWT, B * 8, rec, A, chunk, g.bw, g.bbits, B,
                     (int)nblk, (uint32_t*)nullptr, offs.ptr, entries.ptr, flags.ptr, (uint32_t)N, (int64_t*)nullptr,
                     (unsigned*)nullptr);
    if (n_big) {
        DevArray<unsigned long long> cur;
        KARMA_TRY(cur.alloc(ctx, B));
        KARMA_LAUNCH(ctx, "big_cursor", big_cursor_kernel, grid1(B), 256, 0, offs.ptr, B, (int)nblk, cur.ptr);
        KARMA_LAUNCH(ctx, "graph_big_scatter", big_reads_kernel<true>, grid1(n_big, 64), 64, 0, rec, A, big_list.ptr,
                     (int64_t)n_big, g.bw, g.bbits, (int)nblk, (uint32_t*)nullptr, cur.ptr, entries.ptr, (uint32_t)N);
    }
    // per-bucket reduction
    DevArray<uint64_t> slot_k;
    DevArray<int64_t> slot_c, n_per;
    DevArray<uint8_t> ovf;
    KARMA_TRY(slot_k.alloc(ctx, g.n_buckets * kTableCap));
    KARMA_TRY(slot_c.alloc(ctx, g.n_buckets * kTableCap));
    KARMA_TRY(n_per.alloc(ctx, g.n_buckets + 1));
    KARMA_TRY(ovf.alloc(ctx, g.n_buckets));
    KARMA_HIP(hipMemsetAsync(ovf.ptr, 0, g.n_buckets, ctx->stream));
    KARMA_HIP(hipMemsetAsync(n_per.ptr + g.n_buckets, 0, 8, ctx->stream));
    {
        // slices of <= kSlice entries; buckets with one slice finish in the slice kernel
        std::vector<int64_t> hb(g.n_buckets + 1);
        KARMA_HIP(hipMemcpyAsync(hb.data(), bstart.ptr, (g.n_buckets + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        std::vector<int64_t> sb, slo, shi, mb, m0, m1;
        std::vector<uint8_t> single;
        for (int64_t b = 0; b < g.n_buckets; ++b) {
            const int64_t len = hb[b + 1] - hb[b];
            const int64_t ns = std::max<int64_t>(1, ceil_div(len, kSlice));
            const int64_t first = (int64_t)sb.size();
            for (int64_t k = 0; k < ns; ++k) {
                sb.push_back(b);
                slo.push_back(hb[b] + len * k / ns);
                shi.push_back(hb[b] + len * (k + 1) / ns);
                single.push_back(ns == 1);
            }
            if (ns > 1) {
                mb.push_back(b);
                m0.push_back(first);
                m1.push_back(first + ns);
            }
        }
        const int64_t NS = (int64_t)sb.size(), NM = (int64_t)mb.size();
        DevArray<int64_t> d_sl;  // [sb | slo | shi | mb | m0 | m1]
        DevArray<uint8_t> d_single;
        DevArray<uint32_t> part_k, part_c;
        DevArray<int> part_n;
        KARMA_TRY(d_sl.alloc(ctx, 3 * NS + 3 * NM + 1));
        KARMA_TRY(d_single.alloc(ctx, NS));
        KARMA_TRY(part_k.alloc(ctx, (NM ? NS : 1) * (int64_t)kTableCap));
        KARMA_TRY(part_c.alloc(ctx, (NM ? NS : 1) * (int64_t)kTableCap));
        KARMA_TRY(part_n.alloc(ctx, NS));
        std::vector<int64_t> packed_tab;
        packed_tab.reserve(3 * NS + 3 * NM);
        for (auto* v : {&sb, &slo, &shi, &mb, &m0, &m1}) packed_tab.insert(packed_tab.end(), v->begin(), v->end());
        KARMA_HIP(hipMemcpyAsync(d_sl.ptr, packed_tab.data(), packed_tab.size() * 8, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(d_single.ptr, single.data(), NS, hipMemcpyHostToDevice, ctx->stream));
        KARMA_LAUNCH(ctx, "graph_bucket_reduce", slice_reduce_kernel, NS, kReduceBlock, 0, entries.ptr, d_sl.ptr,
                     d_sl.ptr + NS, d_sl.ptr + 2 * NS, d_single.ptr, g.bw, g.bbits, slot_k.ptr, slot_c.ptr, n_per.ptr,
                     part_k.ptr, part_c.ptr, part_n.ptr, ovf.ptr);
        if (NM)
            KARMA_LAUNCH(ctx, "graph_bucket_merge", bucket_merge_kernel, NM, kReduceBlock, 0, d_sl.ptr + 3 * NS,
                         d_sl.ptr + 3 * NS + NM, d_sl.ptr + 3 * NS + 2 * NM, g.bw, g.bbits, part_k.ptr, part_c.ptr,
                         part_n.ptr, slot_k.ptr, slot_c.ptr, n_per.ptr, ovf.ptr);
        KARMA_HIP(hipStreamSynchronize(ctx->stream));  // tables above die at scope end
    }
    std::vector<uint8_t> hovf(g.n_buckets);
    KARMA_HIP(hipMemcpyAsync(hovf.data(), ovf.ptr, g.n_buckets, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    // source pointer table
    DevArray<const uint64_t*> pk;
    DevArray<const int64_t*> pc;
    KARMA_TRY(pk.alloc(ctx, g.n_buckets));
    KARMA_TRY(pc.alloc(ctx, g.n_buckets));
    KARMA_LAUNCH(ctx, "bucket_ptrs", fill_ptrs_kernel, grid1(g.n_buckets), 256, 0, slot_k.ptr, slot_c.ptr,
                 g.n_buckets, (int64_t)kTableCap, pk.ptr, pc.ptr);
    // overflowed buckets: generic sort-reduce of their entries
    std::vector<std::unique_ptr<DevArray<uint64_t>>> ovk;
    std::vector<std::unique_ptr<DevArray<int64_t>>> ovc;
    std::vector<int64_t> hbstart;
    bool any_ovf = std::any_of(hovf.begin(), hovf.end(), [](uint8_t v) { return v != 0; });
    if (any_ovf) {
        hbstart.resize(g.n_buckets + 1);
        KARMA_HIP(hipMemcpyAsync(hbstart.data(), bstart.ptr, (g.n_buckets + 1) * 8, hipMemcpyDeviceToHost,
                                 ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        for (int64_t b = 0; b < g.n_buckets; ++b) {
            if (!hovf[b]) continue;
            const int64_t s = hbstart[b], n = hbstart[b + 1] - s;
            DevArray<uint64_t> wide;
            DevArray<int64_t> ones;
            KARMA_TRY(wide.alloc(ctx, n));
            KARMA_TRY(ones.alloc(ctx, n));
            KARMA_LAUNCH(ctx, "bucket_widen", widen_kernel, grid1(n), 256, 0, entries.ptr, s, n,
                         (uint64_t)b << g.bw, g.bbits, wide.ptr);
            KARMA_LAUNCH(ctx, "fill_ones", fill_ones_kernel, grid1(n), 256, 0, ones.ptr, n);
            ovk.emplace_back(new DevArray<uint64_t>());
            ovc.emplace_back(new DevArray<int64_t>());
            int64_t nu = 0;
            KARMA_TRY(sort_reduce_pairs(ctx, wide.ptr, ones.ptr, nullptr, n, 64, *ovk.back(), *ovc.back(), nullptr,
                                        &nu));
            const uint64_t* kp = ovk.back()->ptr;
            const int64_t* cp = ovc.back()->ptr;
            KARMA_HIP(hipMemcpyAsync(pk.ptr + b, &kp, sizeof kp, hipMemcpyHostToDevice, ctx->stream));
            KARMA_HIP(hipMemcpyAsync(pc.ptr + b, &cp, sizeof cp, hipMemcpyHostToDevice, ctx->stream));
            KARMA_HIP(hipMemcpyAsync(n_per.ptr + b, &nu, 8, hipMemcpyHostToDevice, ctx->stream));
            KARMA_HIP(hipStreamSynchronize(ctx->stream));
        }
    }
    DevArray<int64_t> dst;
    KARMA_TRY(dst.alloc(ctx, g.n_buckets + 1));
    KARMA_TRY(scan_i64(ctx, n_per.ptr, dst.ptr, g.n_buckets + 1));
    int64_t U = 0;
    KARMA_HIP(hipMemcpyAsync(&U, dst.ptr + g.n_buckets, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_TRY(out->keys.alloc(ctx, U));
    KARMA_TRY(out->counts.alloc(ctx, U));
    KARMA_LAUNCH(ctx, "bucket_assemble", assemble_kernel, g.n_buckets, 256, 0, pk.ptr, pc.ptr, n_per.ptr, dst.ptr,
                 out->keys.ptr, out->counts.ptr);
    out->n = U;
    out->n_contigs = N;
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

__global__ void interleave_kernel(const uint32_t* __restrict__ rid, const uint32_t* __restrict__ cid, int64_t n,
                                  uint2* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = make_uint2(rid[i], cid[i]);
}

__global__ void deinterleave_kernel(const uint2* __restrict__ in, int64_t n, uint32_t* __restrict__ rid,
                                    uint32_t* __restrict__ cid) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        rid[i] = in[i].x;
        cid[i] = in[i].y;
    }
}

}  // namespace

namespace karma {

int sort_reduce_pairs(karma_ctx* ctx, const uint64_t* keys_in, const int64_t* counts_in, const uint64_t* first_in,
                      int64_t n, int key_bits, DevArray<uint64_t>& keys_out, DevArray<int64_t>& counts_out,
                      DevArray<uint64_t>* first_out, int64_t* n_out) {
    KARMA_CHECK(n < (int64_t(1) << 31), KARMA_ERR_ARG, "sort_reduce_pairs: %lld items exceed 2^31", (long long)n);
    if (n == 0) {
        KARMA_TRY(keys_out.alloc(ctx, 0));
        KARMA_TRY(counts_out.alloc(ctx, 0));
        if (first_out) KARMA_TRY(first_out->alloc(ctx, 0));
        *n_out = 0;
        return KARMA_OK;
    }
    DevArray<uint64_t> ks;
    DevArray<uint32_t> idx, idx_s;
    DevArray<int64_t> cs;
    DevArray<uint64_t> fs;
    KARMA_TRY(ks.alloc(ctx, n));
    KARMA_TRY(idx.alloc(ctx, n));
    KARMA_TRY(idx_s.alloc(ctx, n));
    KARMA_TRY(cs.alloc(ctx, n));
    if (first_out) KARMA_TRY(fs.alloc(ctx, n));
    KARMA_LAUNCH(ctx, "iota", iota_kernel, grid1(n), 256, 0, idx.ptr, n);
    size_t tb = 0;
    KARMA_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys_in, ks.ptr, idx.ptr, idx_s.ptr, (int)n, 0, key_bits,
                                                 ctx->stream));
    DevArray<uint8_t> tmp;
    KARMA_TRY(tmp.alloc(ctx, tb));
    KARMA_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.ptr, tb, keys_in, ks.ptr, idx.ptr, idx_s.ptr, (int)n, 0, key_bits,
                                                 ctx->stream));
    KARMA_LAUNCH(ctx, "gather", gather_kernel, grid1(n), 256, 0, idx_s.ptr, counts_in, first_in, n, cs.ptr,
                 first_out ? fs.ptr : (uint64_t*)nullptr);
    DevArray<uint64_t> uk;
    DevArray<int64_t> uc, nruns;
    KARMA_TRY(uk.alloc(ctx, n));
    KARMA_TRY(uc.alloc(ctx, n));
    KARMA_TRY(nruns.alloc(ctx, 1));
    size_t tb2 = 0;
    KARMA_HIP(hipcub::DeviceReduce::ReduceByKey(nullptr, tb2, ks.ptr, uk.ptr, cs.ptr, uc.ptr, nruns.ptr,
                                                hipcub::Sum(), (int)n, ctx->stream));
    DevArray<uint8_t> tmp2;
    KARMA_TRY(tmp2.alloc(ctx, tb2));
    KARMA_HIP(hipcub::DeviceReduce::ReduceByKey(tmp2.ptr, tb2, ks.ptr, uk.ptr, cs.ptr, uc.ptr, nruns.ptr,
                                                hipcub::Sum(), (int)n, ctx->stream));
    DevArray<uint64_t> uf, uk2;
    if (first_out) {
        KARMA_TRY(uf.alloc(ctx, n));
        KARMA_TRY(uk2.alloc(ctx, n));
        size_t tb3 = 0;
        KARMA_HIP(hipcub::DeviceReduce::ReduceByKey(nullptr, tb3, ks.ptr, uk2.ptr, fs.ptr, uf.ptr, nruns.ptr, MinOp(),
                                                    (int)n, ctx->stream));
        DevArray<uint8_t> tmp3;
        KARMA_TRY(tmp3.alloc(ctx, tb3));
        KARMA_HIP(hipcub::DeviceReduce::ReduceByKey(tmp3.ptr, tb3, ks.ptr, uk2.ptr, fs.ptr, uf.ptr, nruns.ptr,
                                                    MinOp(), (int)n, ctx->stream));
    }
    int64_t U = 0;
    KARMA_HIP(hipMemcpyAsync(&U, nruns.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_TRY(keys_out.alloc(ctx, U));
    KARMA_TRY(counts_out.alloc(ctx, U));
    KARMA_HIP(hipMemcpyAsync(keys_out.ptr, uk.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    KARMA_HIP(hipMemcpyAsync(counts_out.ptr, uc.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    if (first_out) {
        KARMA_TRY(first_out->alloc(ctx, U));
        KARMA_HIP(hipMemcpyAsync(first_out->ptr, uf.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    *n_out = U;
    return KARMA_OK;
}

}  // namespace karma

extern "C" {

int karma_graph_records(karma_ctx* ctx, const uint32_t* records, int64_t A, int64_t N, int flags, int is_device,
                        karma_pairs** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && (records || A == 0) && A >= 0, KARMA_ERR_ARG, "karma_graph_records: bad arguments");
    KARMA_CHECK(A < (int64_t(1) << 40), KARMA_ERR_ARG, "too many records");
    auto* p = new karma_pairs();
    p->ctx = ctx;
    DevArray<uint2> own;
    const uint2* rec = reinterpret_cast<const uint2*>(records);
    int rc = KARMA_OK;
    if (!is_device || flags == KARMA_REC_UNSORTED) {
        if ((rc = own.alloc(ctx, A))) {
            delete p;
            return rc;
        }
        if (A) {
            KARMA_HIP(hipMemcpyAsync(own.ptr, records, A * 8, is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                     ctx->stream));
        }
        rec = own.ptr;
    }
    if (flags == KARMA_REC_UNSORTED && A > 1) {
        KARMA_CHECK(A < (int64_t(1) << 31), KARMA_ERR_ARG, "unsorted path limited to 2^31 records");
        DevArray<uint32_t> rid, cid, rid2, cid2;
        if ((rc = rid.alloc(ctx, A)) || (rc = cid.alloc(ctx, A)) || (rc = rid2.alloc(ctx, A)) ||
            (rc = cid2.alloc(ctx, A))) {
            delete p;
            return rc;
        }
        KARMA_LAUNCH(ctx, "deinterleave", deinterleave_kernel, grid1(A), 256, 0, own.ptr, A, rid.ptr, cid.ptr);
        size_t tb = 0;
        KARMA_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, rid.ptr, rid2.ptr, cid.ptr, cid2.ptr, (int)A, 0, 32,
                                                     ctx->stream));
        DevArray<uint8_t> tmp;
        if ((rc = tmp.alloc(ctx, tb))) {
            delete p;
            return rc;
        }
        KARMA_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.ptr, tb, rid.ptr, rid2.ptr, cid.ptr, cid2.ptr, (int)A, 0, 32,
                                                     ctx->stream));
        KARMA_LAUNCH(ctx, "interleave", interleave_kernel, grid1(A), 256, 0, rid2.ptr, cid2.ptr, A, own.ptr);
    }
    rc = records_to_pairs(ctx, rec, A, N, p);
    if (rc) {
        delete p;
        return rc;
    }
    *out = p;
    return KARMA_OK;
}

int karma_graph_eq(karma_ctx* ctx, const int64_t* cls_off, const uint32_t* members, const int64_t* counts,
                   const uint8_t* pair_skip, int64_t C, int64_t N, int is_device, karma_pairs** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && cls_off && C >= 0 && N >= 0 && N < (int64_t(1) << 32), KARMA_ERR_ARG,
                "karma_graph_eq: bad arguments");
    int64_t n_mem = 0;
    if (is_device) {
        KARMA_HIP(hipMemcpyAsync(&n_mem, cls_off + C, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
    } else {
        n_mem = cls_off[C];
    }
    DevArray<int64_t> d_off, d_cnt;
    DevArray<uint32_t> d_mem;
    DevArray<uint8_t> d_skip;
    KARMA_TRY(d_off.alloc(ctx, C + 1));
    KARMA_TRY(d_cnt.alloc(ctx, C));
    KARMA_TRY(d_mem.alloc(ctx, n_mem));
    KARMA_TRY(d_skip.alloc(ctx, C));
    const hipMemcpyKind kind = is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    KARMA_HIP(hipMemcpyAsync(d_off.ptr, cls_off, (C + 1) * 8, kind, ctx->stream));
    if (C) KARMA_HIP(hipMemcpyAsync(d_cnt.ptr, counts, C * 8, kind, ctx->stream));
    if (n_mem) KARMA_HIP(hipMemcpyAsync(d_mem.ptr, members, n_mem * 4, kind, ctx->stream));
    if (C) {
        if (pair_skip) KARMA_HIP(hipMemcpyAsync(d_skip.ptr, pair_skip, C, kind, ctx->stream));
        else KARMA_HIP(hipMemsetAsync(d_skip.ptr, 0, C, ctx->stream));
    }
    auto* p = new karma_pairs();
    p->ctx = ctx;
    p->n_contigs = N;
    std::unique_ptr<karma_pairs> guard(p);
    KARMA_TRY(p->totals.alloc(ctx, N));
    p->has_totals = true;
    if (N) KARMA_HIP(hipMemsetAsync(p->totals.ptr, 0, N * 8, ctx->stream));
    DevArray<int64_t> pc, poff;
    DevArray<int> bad;
    KARMA_TRY(pc.alloc(ctx, C + 1));
    KARMA_TRY(poff.alloc(ctx, C + 1));
    KARMA_TRY(bad.alloc(ctx, 1));
    KARMA_HIP(hipMemsetAsync(bad.ptr, 0, 4, ctx->stream));
    KARMA_HIP(hipMemsetAsync(pc.ptr + C, 0, 8, ctx->stream));
    if (C)
        KARMA_LAUNCH(ctx, "eq_totals", eq_totals_kernel, grid1(C), 256, 0, d_off.ptr, d_mem.ptr, d_cnt.ptr, C,
                     (uint32_t)N, (unsigned long long*)p->totals.ptr, pc.ptr, d_skip.ptr, bad.ptr);
    KARMA_TRY(scan_i64(ctx, pc.ptr, poff.ptr, C + 1));
    int64_t P = 0;
    int hbad = 0;
    KARMA_HIP(hipMemcpyAsync(&P, poff.ptr + C, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipMemcpyAsync(&hbad, bad.ptr, 4, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_CHECK(!hbad, KARMA_ERR_ARG, "eq class member index >= n_contigs");
    DevArray<uint64_t> keys;
    DevArray<int64_t> cnts;
    KARMA_TRY(keys.alloc(ctx, P));
    KARMA_TRY(cnts.alloc(ctx, P));
    if (P)
        KARMA_LAUNCH(ctx, "eq_emit", eq_emit_kernel, grid1(P), 256, 0, d_off.ptr, d_mem.ptr, d_cnt.ptr, poff.ptr, C,
                     P, keys.ptr, cnts.ptr);
    int key_bits = 32;
    while (key_bits < 64 && (int64_t(1) << (key_bits - 32)) < N) ++key_bits;
    KARMA_TRY(sort_reduce_pairs(ctx, keys.ptr, cnts.ptr, nullptr, P, key_bits, p->keys, p->counts, &p->first, &p->n));
    p->has_first = true;
    *out = guard.release();
    return KARMA_OK;
}

int karma_pairs_merge(karma_ctx* ctx, const uint64_t* keys, const int64_t* counts, int64_t n, int is_device,
                      karma_pairs** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && n >= 0 && (n == 0 || (keys && counts)), KARMA_ERR_ARG, "karma_pairs_merge: bad arguments");
    auto* p = new karma_pairs();
    p->ctx = ctx;
    std::unique_ptr<karma_pairs> guard(p);
    DevArray<uint64_t> k;
    DevArray<int64_t> c;
    const uint64_t* kp = keys;
    const int64_t* cp = counts;
    if (!is_device && n) {
        KARMA_TRY(k.alloc(ctx, n));
        KARMA_TRY(c.alloc(ctx, n));
        KARMA_HIP(hipMemcpyAsync(k.ptr, keys, n * 8, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(c.ptr, counts, n * 8, hipMemcpyHostToDevice, ctx->stream));
        kp = k.ptr;
        cp = c.ptr;
    }
    KARMA_TRY(sort_reduce_pairs(ctx, kp, cp, nullptr, n, 64, p->keys, p->counts, nullptr, &p->n));
    *out = guard.release();
    return KARMA_OK;
}

int karma_pairs_destroy(karma_pairs* p) {
    if (!p) return KARMA_OK;
    hipSetDevice(p->ctx->device);
    delete p;
    return KARMA_OK;
}

int karma_pairs_count(karma_pairs* p, int64_t* n) {
    KARMA_CHECK(p && n, KARMA_ERR_ARG, "null argument");
    *n = p->n;
    return KARMA_OK;
}

int karma_pairs_device(karma_pairs* p, const uint64_t** keys, const int64_t** counts) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    if (keys) *keys = p->keys.ptr;
    if (counts) *counts = p->counts.ptr;
    return KARMA_OK;
}

int karma_pairs_get(karma_pairs* p, uint64_t* keys, int64_t* counts, uint64_t* first, int is_device) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    KARMA_TRY(ctx_begin(p->ctx));
    const hipMemcpyKind kind = is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (p->n) {
        if (keys) KARMA_HIP(hipMemcpyAsync(keys, p->keys.ptr, p->n * 8, kind, p->ctx->stream));
        if (counts) KARMA_HIP(hipMemcpyAsync(counts, p->counts.ptr, p->n * 8, kind, p->ctx->stream));
        if (first && p->has_first) KARMA_HIP(hipMemcpyAsync(first, p->first.ptr, p->n * 8, kind, p->ctx->stream));
    }
    KARMA_HIP(hipStreamSynchronize(p->ctx->stream));
    return KARMA_OK;
}

int karma_pairs_split(karma_pairs* p, const int64_t* bounds, int nranks, int64_t* starts) {
    KARMA_CHECK(p && bounds && starts && nranks >= 1, KARMA_ERR_ARG, "bad arguments");
    KARMA_TRY(ctx_begin(p->ctx));
    std::vector<uint64_t> hk(p->n);
    if (p->n) {
        KARMA_HIP(hipMemcpyAsync(hk.data(), p->keys.ptr, p->n * 8, hipMemcpyDeviceToHost, p->ctx->stream));
        KARMA_HIP(hipStreamSynchronize(p->ctx->stream));
    }
    for (int r = 0; r <= nranks; ++r) {
        const uint64_t lim = (uint64_t)bounds[r] << 32;
        starts[r] = std::lower_bound(hk.begin(), hk.end(), lim) - hk.begin();
    }
    return KARMA_OK;
}

int karma_pairs_totals(karma_pairs* p, int64_t* totals_dev, int64_t N) {
    KARMA_CHECK(p && totals_dev && N >= 0, KARMA_ERR_ARG, "bad arguments");
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    if (N) KARMA_HIP(hipMemsetAsync(totals_dev, 0, N * 8, ctx->stream));
    if (p->n)
        KARMA_LAUNCH(ctx, "diag_totals", diag_totals_kernel, grid1(p->n), 256, 0, p->keys.ptr, p->counts.ptr, p->n,
                     totals_dev);
    return KARMA_OK;
}

int karma_edges_from_pairs(karma_ctx* ctx, karma_pairs* p, int mode, const int64_t* totals_dev, int64_t N,
                           karma_edges** out, int64_t* n_edges) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(p && out && n_edges && N >= 0, KARMA_ERR_ARG, "karma_edges_from_pairs: bad arguments");
    KARMA_CHECK(mode == KARMA_MODE_READS || mode == KARMA_MODE_EQ, KARMA_ERR_ARG, "bad mode");
    auto* e = new karma_edges();
    e->ctx = ctx;
    e->n_contigs = N;
    std::unique_ptr<karma_edges> guard(e);
    KARMA_TRY(e->totals.alloc(ctx, N));
    const int64_t* tot = totals_dev;
    if (!tot) {
        if (mode == KARMA_MODE_EQ) {
            KARMA_CHECK(p->has_totals && p->n_contigs == N, KARMA_ERR_STATE, "eq pair list without totals");
            if (N) KARMA_HIP(hipMemcpyAsync(e->totals.ptr, p->totals.ptr, N * 8, hipMemcpyDeviceToDevice, ctx->stream));
        } else {
            KARMA_TRY(karma_pairs_totals(p, e->totals.ptr, N));
        }
    } else if (N) {
        KARMA_HIP(hipMemcpyAsync(e->totals.ptr, tot, N * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    const int64_t n = p->n;
    DevArray<int64_t> flags, pos;
    DevArray<int> zd;
    KARMA_TRY(flags.alloc(ctx, n + 1));
    KARMA_TRY(pos.alloc(ctx, n + 1));
    KARMA_TRY(zd.alloc(ctx, 1));
    KARMA_HIP(hipMemsetAsync(zd.ptr, 0, 4, ctx->stream));
    KARMA_HIP(hipMemsetAsync(flags.ptr + n, 0, 8, ctx->stream));
    if (n) KARMA_LAUNCH(ctx, "edge_flags", edge_flags_kernel, grid1(n), 256, 0, p->keys.ptr, p->counts.ptr, n, mode, flags.ptr);
    KARMA_TRY(scan_i64(ctx, flags.ptr, pos.ptr, n + 1));
    int64_t E = 0;
    KARMA_HIP(hipMemcpyAsync(&E, pos.ptr + n, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_TRY(e->a.alloc(ctx, E));
    KARMA_TRY(e->b.alloc(ctx, E));
    KARMA_TRY(e->s.alloc(ctx, E));
    KARMA_TRY(e->w.alloc(ctx, E));
    e->has_first = p->has_first;
    if (e->has_first) KARMA_TRY(e->first.alloc(ctx, E));
    if (n)
        KARMA_LAUNCH(ctx, "edge_weights", edge_write_kernel, grid1(n), 256, 0, p->keys.ptr, p->counts.ptr,
                     p->has_first ? p->first.ptr : (const uint64_t*)nullptr, flags.ptr, pos.ptr, n, e->totals.ptr,
                     e->a.ptr, e->b.ptr, e->s.ptr, e->w.ptr, e->has_first ? e->first.ptr : (uint64_t*)nullptr, zd.ptr);
    int hz = 0;
    KARMA_HIP(hipMemcpyAsync(&hz, zd.ptr, 4, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_CHECK(!hz, KARMA_ERR_ZERO_DIV, "division by zero: a shared count over a zero total");
    e->E = E;
    *n_edges = E;
    *out = guard.release();
    return KARMA_OK;
}

int karma_edges_destroy(karma_edges* e) {
    if (!e) return KARMA_OK;
    hipSetDevice(e->ctx->device);
    delete e;
    return KARMA_OK;
}

int karma_edges_get(karma_edges* e, uint32_t* a, uint32_t* b, int64_t* s, double* w, uint64_t* first, int is_device) {
    KARMA_CHECK(e, KARMA_ERR_ARG, "null edges");
    KARMA_TRY(ctx_begin(e->ctx));
    const hipMemcpyKind kind = is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    hipStream_t st = e->ctx->stream;
    if (e->E) {
        if (a) KARMA_HIP(hipMemcpyAsync(a, e->a.ptr, e->E * 4, kind, st));
        if (b) KARMA_HIP(hipMemcpyAsync(b, e->b.ptr, e->E * 4, kind, st));
        if (s) KARMA_HIP(hipMemcpyAsync(s, e->s.ptr, e->E * 8, kind, st));
        if (w) KARMA_HIP(hipMemcpyAsync(w, e->w.ptr, e->E * 8, kind, st));
        if (first && e->has_first) KARMA_HIP(hipMemcpyAsync(first, e->first.ptr, e->E * 8, kind, st));
    }
    KARMA_HIP(hipStreamSynchronize(st));
    return KARMA_OK;
}

int karma_edges_totals(karma_edges* e, int64_t* totals, int is_device) {
    KARMA_CHECK(e && (totals || !e->n_contigs), KARMA_ERR_ARG, "bad arguments");
    KARMA_TRY(ctx_begin(e->ctx));
    if (e->n_contigs)
        KARMA_HIP(hipMemcpyAsync(totals, e->totals.ptr, e->n_contigs * 8,
                                 is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, e->ctx->stream));
    KARMA_HIP(hipStreamSynchronize(e->ctx->stream));
    return KARMA_OK;
}

}  // extern "C"
