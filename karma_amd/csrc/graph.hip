// graph.hip — contig x contig shared-read graph for gfx950.
//
// Reference (lmfaber/karma) being replaced:
//   ReadGraph.from_contigs          karma/read_graph.py:19-50  (O(N^2) readset intersections)
//   Contig readsets                 karma/contig.py:4-35       (QNAME set per contig)
//   ReadGraph.update_graph          karma/read_graph.py:192-221
//   ReadGraph.from_equivalence_classes karma/read_graph.py:61-148
//
// This file: the C ABI of the graph paths, the equivalence-class path, the
// generic sort + reduce, and the edge finalisation (weights).  The read-record
// pipeline (the hot one) is graph_sets.hip.  The diagonal (a, a) of a pair
// list counts |readset(a)| (the normaliser), so one mechanism yields both the
// shared counts and the totals.
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
    // between karma_edges_begin and _end: the pair list (caller-owned until
    // _end), the per-block edge counts and the mode
    const karma_pairs* src = nullptr;
    DevArray<int64_t> blk;
    int mode = 0;
    bool open = false;
    // karma_edges_end without a count: the write kernel's status words
    // (zero-total flag, edge count, merge order flag) wait in blk past the
    // per-block counts until the first read of the edges
    bool pending = false;
    int64_t n_blk = 0;
};

namespace {


// ---- generic sort + reduce (low-volume paths) ----------------------------------
// ---- finalize --------------------------------------------------------------------
// A list may hold runs of equal adjacent keys (karma_pairs::dups): the first
// element of a run stands for it, with the run's summed count.  On a sorted
// unique list every run has one element.
__device__ __forceinline__ bool group_head(const uint64_t* __restrict__ keys, int64_t i, uint64_t k) {
    return i == 0 || keys[i - 1] != k;
}
__device__ __forceinline__ int64_t group_sum(const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts,
                                             int64_t n, int64_t i, uint64_t k) {
    int64_t c = counts[i];
    for (int64_t j = i + 1; j < n && keys[j] == k; ++j) c += counts[j];
    return c;
}

__global__ void diag_totals_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts, int64_t n,
                                   int64_t* __restrict__ totals) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint64_t k = keys[i];
        const uint32_t a = (uint32_t)(k >> 32), b = (uint32_t)k;
        if (a == b && group_head(keys, i, k)) totals[a] = group_sum(keys, counts, n, i, k);
    }
}

// ---- compaction in two launches ----------------------------------------------------
// A count kernel writes each 1024-element block's number of kept elements; the
// write kernel places block j at the sum of the counts before it (read by the
// whole block: <= a few thousand words) and an element at that base plus its
// rank among the block's kept elements (ballots, then the waves before).  No
// scan launches, no host round trip.
constexpr int kET = 1024;

struct BlockPlace {
    int64_t base;    // kept elements of the blocks before this one
    int64_t rank;    // this thread's rank among the block's kept elements
    int64_t total;   // kept elements of this block
};

__device__ __forceinline__ BlockPlace block_place(const int64_t* __restrict__ blk_cnt, bool keep) {
    __shared__ int64_t wsum[kET / 64];
    __shared__ int64_t base_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t b = 0;
    for (int64_t j = threadIdx.x; j < (int64_t)blockIdx.x; j += kET) b += blk_cnt[j];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) b += __shfl_xor(b, d, 64);
    if (lane == 0) wsum[wave] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int w = 0; w < kET / 64; ++w) t += wsum[w];
        base_s = t;
    }
    const uint64_t m = __ballot(keep);
    const int64_t r = __popcll(m & ((1ull << lane) - 1ull));
    __syncthreads();  // base_s is set; wsum is free again
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    BlockPlace p;
    p.base = base_s;
    p.rank = r;
    p.total = 0;
    for (int w = 0; w < kET / 64; ++w) {
        if (w == wave) p.rank += p.total;
        p.total += wsum[w];
    }
    return p;
}

// The edge stage: edges_count_kernel flags the keys that are edges (count !=
// 0; the diagonal is not an edge of the readset graph), writing the diagonal
// totals on the way when the pair list owns them; edges_write_kernel writes
// (a, b, s, w) of each edge at its place.
__device__ __forceinline__ bool edge_flag(uint64_t k, int64_t c, int mode) {
    const bool diag = (uint32_t)(k >> 32) == (uint32_t)k;
    return c != 0 && !(diag && mode == KARMA_MODE_READS);
}

// With totals (n_tot entries, n >= 1) the kernel writes every entry itself, so
// no memset precedes it: the diagonal group of contig a writes its sum, and
// the first key of each contig a zeroes a when it is not the diagonal and the
// contigs between the previous contig and a; the grid zeroes those before the
// first contig and after the last (the keys are sorted by a, and (a, a) is
// the smallest key of a).
__global__ void __launch_bounds__(kET) edges_count_kernel(const uint64_t* __restrict__ keys,
                                                          const int64_t* __restrict__ counts, int64_t n, int mode,
                                                          int64_t* __restrict__ totals, int64_t n_tot,
                                                          int64_t* __restrict__ blk_cnt, int64_t* __restrict__ st) {
    const int64_t i = (int64_t)blockIdx.x * kET + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 3) st[threadIdx.x] = 0;  // the write kernel's status words
    if (totals) {
        const int64_t a_first = (int64_t)(keys[0] >> 32), a_last = (int64_t)(keys[n - 1] >> 32);
        const int64_t stride = (int64_t)gridDim.x * kET;
        for (int64_t c = i; c < min(a_first, n_tot); c += stride) totals[c] = 0;
        for (int64_t c = a_last + 1 + i; c < n_tot; c += stride) totals[c] = 0;
    }
    bool f = false;
    if (i < n) {
        const uint64_t k = keys[i];
        const uint32_t a = (uint32_t)(k >> 32);
        const bool in_tot = totals && (int64_t)a < n_tot;
        if (totals && i > 0) {
            const uint32_t pa = (uint32_t)(keys[i - 1] >> 32);
            // contigs without keys between the previous contig and this one
            // (none when pa == a), up to n_tot also when a itself is past it
            const uint32_t lim = (int64_t)a < n_tot ? a : (uint32_t)n_tot;
            for (uint32_t c = pa + 1; c < lim; ++c) totals[c] = 0;
            if (in_tot && pa != a && a != (uint32_t)k) totals[a] = 0;
        } else if (in_tot && a != (uint32_t)k) {
            totals[a] = 0;  // the first contig has no diagonal
        }
        if (group_head(keys, i, k)) {
            const int64_t c = group_sum(keys, counts, n, i, k);
            if (in_tot && a == (uint32_t)k) totals[a] = c;
            f = edge_flag(k, c, mode);
        }
    }
    const int cnt = __syncthreads_count(f);
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = cnt;
}

__global__ void __launch_bounds__(kET) edges_write_kernel(
    const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts, const uint64_t* __restrict__ first,
    int64_t n, int mode, const int64_t* __restrict__ totals, const int64_t* __restrict__ blk_cnt,
    uint32_t* __restrict__ ea, uint32_t* __restrict__ eb, int64_t* __restrict__ es, double* __restrict__ ew,
    uint64_t* __restrict__ ef, int64_t* __restrict__ st, const int64_t* __restrict__ bad) {
    const int64_t i = (int64_t)blockIdx.x * kET + threadIdx.x;
    uint64_t k = 0;
    int64_t c = 0;
    bool f = false;
    if (i < n) {
        k = keys[i];
        if (group_head(keys, i, k)) {
            c = group_sum(keys, counts, n, i, k);
            f = edge_flag(k, c, mode);
        }
    }
    const BlockPlace pl = block_place(blk_cnt, f);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        st[1] = pl.base + pl.total;  // the edge count
        st[2] = bad ? *bad : 0;      // the order check of the merge that made the list
    }
    if (!f) return;
    const int64_t o = pl.base + pl.rank;
    const uint32_t a = (uint32_t)(k >> 32), bb = (uint32_t)k;
    const int64_t ta = totals[a], tb = totals[bb];
    ea[o] = a;
    eb[o] = bb;
    es[o] = c;
    if (ef) ef[o] = first[i];
    if (ta == 0 || tb == 0) {
        reinterpret_cast<int*>(st)[0] = 1;
        ew[o] = 0.0;
        return;
    }
    // read_graph.py:39-42 / :128-130: ((s / tA) + (s / tB)) / 2, IEEE binary64, no FMA
    const double x = __ddiv_rn((double)c, (double)ta);
    const double y = __ddiv_rn((double)c, (double)tb);
    ew[o] = __dadd_rn(x, y) * 0.5;
}

// Sum of the counts of equal adjacent keys (a merged list: a key occurs at
// most once per run): the first of each group is kept and sums its group.
__global__ void __launch_bounds__(kET) group_count_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                                          int64_t* __restrict__ blk_cnt) {
    const int64_t i = (int64_t)blockIdx.x * kET + threadIdx.x;
    const bool head = i < n && (i == 0 || keys[i] != keys[i - 1]);
    const int cnt = __syncthreads_count(head);
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = cnt;
}

__global__ void __launch_bounds__(kET) group_sum_kernel(const uint64_t* __restrict__ keys,
                                                        const int64_t* __restrict__ counts, int64_t n,
                                                        const int64_t* __restrict__ blk_cnt,
                                                        uint64_t* __restrict__ ko, int64_t* __restrict__ co,
                                                        int64_t* __restrict__ n_out) {
    const int64_t i = (int64_t)blockIdx.x * kET + threadIdx.x;
    uint64_t k = 0;
    bool head = false;
    if (i < n) {
        k = keys[i];
        head = i == 0 || keys[i - 1] != k;
    }
    const BlockPlace pl = block_place(blk_cnt, head);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_out = pl.base + pl.total;
    if (!head) return;
    int64_t c = counts[i];
    for (int64_t j = i + 1; j < n && keys[j] == k; ++j) c += counts[j];
    ko[pl.base + pl.rank] = k;
    co[pl.base + pl.rank] = c;
}


int grid1(int64_t n, int block = 256) { return (int)std::max<int64_t>(1, ceil_div(n, block)); }

// ---- eq edges in the reference's insertion order -------------------------------
// read_graph.py:96-131 adds edge (u, v) to the intermediate graph at the pair's
// first emission, from its lower endpoint u; the copy cls(incoming_graph_data=)
// keeps that order per node.  The edge list is sorted by (a, b); each edge's
// place inside its run of equal a is its rank by first emission (distinct per
// pair).  A block takes 256 consecutive edges; the runs they belong to are
// streamed through LDS in chunks, and every thread counts the smaller first
// emissions of its own run.  Outputs are the (a, b, w) arrays in that order.
constexpr int kOrdT = 256, kOrdChunk = 4096;
__global__ void __launch_bounds__(kOrdT) eq_order_kernel(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                        const double* __restrict__ w,
                                                        const uint64_t* __restrict__ first, int64_t E,
                                                        uint32_t* __restrict__ oa, uint32_t* __restrict__ ob,
                                                        double* __restrict__ ow) {
    __shared__ uint64_t sf[kOrdChunk];
    __shared__ int64_t span[2];
    const int64_t t0 = (int64_t)blockIdx.x * kOrdT, i = t0 + threadIdx.x;
    const int64_t t1 = min(E, t0 + kOrdT);
    const bool own = i < E;
    const uint32_t ai = own ? a[i] : 0u;
    const uint64_t fi = own ? first[i] : 0ull;
    // the run of a[i]: [lo, hi)
    int64_t lo = 0, hi = 0;
    if (own) {
        int64_t l = 0, h = i;  // first index with a == ai
        while (l < h) {
            const int64_t m = (l + h) >> 1;
            if (a[m] < ai) l = m + 1;
            else h = m;
        }
        lo = l;
        l = i + 1, h = E;  // first index with a > ai
        while (l < h) {
            const int64_t m = (l + h) >> 1;
            if (a[m] <= ai) l = m + 1;
            else h = m;
        }
        hi = l;
    }
    if (threadIdx.x == 0) span[0] = lo;                 // the block's first edge opens the span
    if (i == t1 - 1) span[1] = hi;                      // ... its last one closes it
    __syncthreads();
    const int64_t s0 = span[0], s1 = span[1];
    int64_t rank = 0;
    for (int64_t c0 = s0; c0 < s1; c0 += kOrdChunk) {
        const int64_t c1 = min(s1, c0 + kOrdChunk);
        __syncthreads();
        for (int64_t j = c0 + threadIdx.x; j < c1; j += kOrdT) sf[j - c0] = first[j];
        __syncthreads();
        const int64_t j0 = max(lo, c0), j1 = min(hi, c1);
        for (int64_t j = j0; j < j1; ++j) rank += sf[j - c0] < fi ? 1 : 0;
    }
    if (own) {
        const int64_t pos = lo + rank;
        oa[pos] = ai;
        ob[pos] = b[i];
        ow[pos] = w[i];
    }
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

// rank boundaries of a sorted pair list: first key with a >= bounds[r]
__global__ void split_kernel(const uint64_t* __restrict__ keys, int64_t n, const int64_t* __restrict__ bounds, int nb,
                             int64_t* __restrict__ starts) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nb) return;
    const uint64_t lim = (uint64_t)bounds[r] << 32;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < lim) lo = mid + 1;
        else hi = mid;
    }
    starts[r] = lo;
}

// The exchange's split and wire format in one launch: block 0's first nb
// threads search the owners' bounds (first key with a >= bounds[r]); every
// thread interleaves (key, count) pairs.
__global__ void split_kc_kernel(const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts, int64_t n,
                                const int64_t* __restrict__ bounds, int nb, int64_t* __restrict__ starts,
                                longlong2* __restrict__ kc) {
    if (blockIdx.x == 0 && (int)threadIdx.x < nb) {
        const uint64_t lim = (uint64_t)bounds[threadIdx.x] << 32;
        int64_t lo = 0, hi = n;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < lim) lo = mid + 1;
            else hi = mid;
        }
        starts[threadIdx.x] = lo;
    }
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        kc[i] = make_longlong2((long long)keys[i], (long long)counts[i]);
}

// (key, count) pairs <-> separate key and count arrays (the exchange's wire format)
__global__ void interleave_kc_kernel(const uint64_t* __restrict__ k, const int64_t* __restrict__ c, int64_t n,
                                     longlong2* __restrict__ kc) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        kc[i] = make_longlong2((long long)k[i], (long long)c[i]);
}

__global__ void deinterleave_kc_kernel(const longlong2* __restrict__ kc, int64_t n, uint64_t* __restrict__ k,
                                       int64_t* __restrict__ c) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const longlong2 v = kc[i];
        k[i] = (uint64_t)v.x;
        c[i] = (int64_t)v.y;
    }
}

// ---- owner merge of W sorted runs: one ranking pass ------------------------------
// Element j of run r (key k) lands at j + sum over the other runs s of the
// number of their elements that precede it: < k for s > r, <= k for s < r
// (stable, so equal keys from different runs end up adjacent in run order).
// A block takes a tile of kMergeTile consecutive elements of one run.  For each
// other run, the counts of the tile's first and last keys bound the counts of
// every key in between: that window of run s is searched once per block (two
// global binary searches), staged in LDS when it fits, and each element's
// count is a short search inside it.  The same pass flags a descent inside a
// run.  Replaces a merge tree of W - 1 pairwise merges (2 launches each).
constexpr int kMergeMaxRuns = 64;
constexpr int kMergeLds = 6144;      // staged window keys per block (48 KB)
// elements per block (4 per thread).  A window that does not fit the stage is
// searched in global memory; halving the tile so that 8 runs' windows fit
// measured slower (0.103 vs 0.076 ms for 1.6M pairs: twice the window searches)
constexpr int kMergeTile = 1024;
struct RunOffs {
    int64_t o[kMergeMaxRuns + 1];    // run offsets
    int64_t t[kMergeMaxRuns + 1];    // first tile of each run (prefix of ceil(len / tile))
};

// number of elements of sorted run [lo, hi) preceding key k (<= k when le, else < k)
template <typename KeyAt>
__device__ __forceinline__ int64_t count_before(KeyAt key_at, int64_t lo, int64_t hi, uint64_t k, bool le) {
    int64_t n = hi - lo, base = lo;
    while (n > 0) {
        const int64_t half = n >> 1;
        const uint64_t m = key_at(base + half);
        const bool before = le ? m <= k : m < k;
        base = before ? base + half + 1 : base;
        n = before ? n - half - 1 : half;
    }
    return base;
}

// The window bounds of every (tile, other run): one thread per bound, all in
// one round (searched inside merge_rank_kernel, 14 dependent binary searches
// per block made each block a chain of global-load latencies; beside the
// profile kernel, with few free CU slots, 1.6M pairs took 0.28 ms).
__device__ __forceinline__ int tile_run(const RunOffs& R, int nr, int64_t tile) {
    int lo = 0, hi = nr - 1;  // the last run r with R.t[r] <= tile
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (R.t[mid] <= tile) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// A group of kMG lanes per bound, searching kMG ways at once: each round probes
// kMG evenly spaced keys of the remaining range and keeps the stretch between
// the last probe before the key and the first after it, so a run of n keys
// takes log_kMG(n) dependent loads (5 for 200k at kMG = 16) instead of a
// thread's log2(n) (18).  64 lanes per bound took 3 rounds but 4x the loads:
// slower for the weak-scaled merge's 1.6M keys (0.029 against 0.014 ms).
constexpr int kMG = 16;
__global__ void __launch_bounds__(256) merge_bounds_kernel(const uint64_t* __restrict__ keys,
                                                           const longlong2* __restrict__ kc, RunOffs R, int nr,
                                                           int64_t tiles, int64_t* __restrict__ wb,
                                                           int64_t* __restrict__ bad) {
    const int lane = threadIdx.x & 63, g = lane & (kMG - 1);
    const unsigned long long gmask = ((1ull << kMG) - 1ull) << (lane & ~(kMG - 1));
    const int64_t q = ((int64_t)blockIdx.x * 256 + threadIdx.x) / kMG;
    if (q == 0 && g == 0) *bad = 0;  // merge_rank_kernel (next on the stream) flags a descent inside a run
    auto key_at = [&](int64_t i) -> uint64_t { return kc ? (uint64_t)kc[i].x : keys[i]; };
    int64_t lo = 0, hi = 0;
    uint64_t k = 0;
    bool le = false, search = false;  // search: a bound this group writes
    if (q < tiles * nr * 2) {
        const int64_t tile = q / (2 * nr);
        const int sr = (int)((q >> 1) % nr);
        const int r = tile_run(R, nr, tile);
        if (sr != r) {
            search = true;
            const int64_t t0 = R.o[r] + (tile - R.t[r]) * kMergeTile;
            const int64_t t1 = min(R.o[r + 1], t0 + kMergeTile);
            k = key_at((q & 1) ? t1 - 1 : t0);
            le = sr < r;
            lo = R.o[sr];  // the answer (keys of run sr before k) lies in [lo, hi]
            hi = R.o[sr + 1];
        }
    }
    // every group of the wave runs the same number of rounds (ballots are wave-wide)
    for (;;) {
        const bool more = hi - lo > kMG;
        if (!__ballot(more)) break;
        const int64_t step = (hi - lo + kMG - 1) / kMG;
        const int64_t p = min(hi - 1, lo + (int64_t)(g + 1) * step - 1);
        const bool before = more && (le ? key_at(p) <= k : key_at(p) < k);
        const int c = __popcll(__ballot(before) & gmask);  // probes before the key: a prefix of the group
        if (more) {
            const int64_t nlo = c ? min(hi, lo + (int64_t)c * step) : lo;
            const int64_t nhi = c < kMG ? min(hi, lo + (int64_t)(c + 1) * step - 1) : hi;
            lo = nlo;
            hi = nhi;
        }
    }
    const int64_t p = lo + g;
    const bool before = p < hi && (le ? key_at(p) <= k : key_at(p) < k);
    const int64_t ans = lo + __popcll(__ballot(before) & gmask);
    if (search && g == 0) wb[q] = ans;
}

__global__ void __launch_bounds__(256) merge_rank_kernel(const uint64_t* __restrict__ keys,
                                                         const int64_t* __restrict__ counts,
                                                         const longlong2* __restrict__ kc, RunOffs R, int nr,
                                                         const int64_t* __restrict__ wb, uint64_t* __restrict__ ko,
                                                         int64_t* __restrict__ co, int64_t* __restrict__ bad) {
    __shared__ int64_t wlo[kMergeMaxRuns], whi[kMergeMaxRuns];  // window of run s: [wlo, whi] (counts)
    __shared__ int wbase[kMergeMaxRuns];                        // its LDS slot (-1: searched in place)
    __shared__ uint64_t wkeys[kMergeLds];
    auto key_at = [&](int64_t i) -> uint64_t { return kc ? (uint64_t)kc[i].x : keys[i]; };
    const int64_t tile = blockIdx.x;
    const int r = tile_run(R, nr, tile);
    const int64_t t0 = R.o[r] + (tile - R.t[r]) * kMergeTile;
    const int64_t t1 = min(R.o[r + 1], t0 + kMergeTile);
    if (threadIdx.x < 2 * nr && (threadIdx.x >> 1) != r) {
        const int64_t c = wb[tile * nr * 2 + threadIdx.x];
        if (threadIdx.x & 1) whi[threadIdx.x >> 1] = c;
        else wlo[threadIdx.x >> 1] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int used = 0;
        for (int sr = 0; sr < nr; ++sr) {
            if (sr == r) continue;
            if (whi[sr] < wlo[sr]) whi[sr] = wlo[sr];  // an unsorted run (flagged below): stay in bounds
            const int64_t len = whi[sr] - wlo[sr];
            if (used + len <= kMergeLds) {
                wbase[sr] = used;
                used += (int)len;
            } else {
                wbase[sr] = -1;
            }
        }
    }
    __syncthreads();
    for (int sr = 0; sr < nr; ++sr) {
        if (sr == r || wbase[sr] < 0) continue;
        const int64_t lo = wlo[sr];
        const int len = (int)(whi[sr] - lo);
        for (int i = threadIdx.x; i < len; i += blockDim.x) wkeys[wbase[sr] + i] = key_at(lo + i);
    }
    __syncthreads();
    for (int64_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) {
        uint64_t k;
        int64_t c;
        if (kc) {
            const longlong2 v = kc[i];
            k = (uint64_t)v.x;
            c = (int64_t)v.y;
        } else {
            k = keys[i];
            c = counts[i];
        }
        if (i > R.o[r] && key_at(i - 1) > k) *bad = 1;
        int64_t pos = i - R.o[r];
        for (int sr = 0; sr < nr; ++sr) {
            if (sr == r) continue;
            const int64_t lo = wlo[sr], hi = whi[sr];
            int64_t cnt;
            if (wbase[sr] >= 0) {
                const uint64_t* w = wkeys + wbase[sr] - lo;  // w[x] = key of element x of the window
                cnt = count_before([&](int64_t x) { return w[x]; }, lo, hi, k, sr < r);
            } else {
                cnt = count_before(key_at, lo, hi, k, sr < r);
            }
            pos += cnt - R.o[sr];
        }
        ko[pos] = k;
        co[pos] = c;
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
    // the library's radix sort (sort.hip) with the input positions as values,
    // then one reduce-by-key pass through that permutation
    DevArray<uint64_t> ks;
    DevArray<uint32_t> perm;
    KARMA_TRY(ks.alloc(ctx, n));
    KARMA_TRY(perm.alloc(ctx, n));
    KARMA_TRY(radix_sort_u64(ctx, keys_in, nullptr, n, key_bits, ks.ptr, perm.ptr));
    DevArray<uint64_t> uk, uf;
    DevArray<int64_t> uc, nruns;
    KARMA_TRY(uk.alloc(ctx, n));
    KARMA_TRY(uc.alloc(ctx, n));
    if (first_out) KARMA_TRY(uf.alloc(ctx, n));
    KARMA_TRY(nruns.alloc(ctx, 1));
    KARMA_TRY(reduce_sorted(ctx, ks.ptr, perm.ptr, counts_in, first_in, n, uk.ptr, uc.ptr,
                            first_out ? uf.ptr : nullptr, nruns.ptr));
    int64_t* hp = nullptr;
    KARMA_TRY(ctx_pinned(ctx, 8, reinterpret_cast<void**>(&hp)));
    KARMA_HIP(hipMemcpyAsync(hp, nruns.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    const int64_t U = *hp;
    KARMA_TRY(keys_out.alloc(ctx, U));
    KARMA_TRY(counts_out.alloc(ctx, U));
    KARMA_HIP(hipMemcpyAsync(keys_out.ptr, uk.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    KARMA_HIP(hipMemcpyAsync(counts_out.ptr, uc.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    if (first_out) {
        KARMA_TRY(first_out->alloc(ctx, U));
        KARMA_HIP(hipMemcpyAsync(first_out->ptr, uf.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    *n_out = U;  // the copies are stream-ordered; temporaries return to the stream's free list
    return KARMA_OK;
}

}  // namespace karma

struct karma_graph_job {
    karma_pairs* p = nullptr;
    karma::DevArray<uint2> own;      // copied / read-sorted records, read by the kernels until _end
    karma::DevArray<uint32_t> ownw;  // copied flagged records (KARMA_REC_FLAGGED)
    karma::SetsJob* sets = nullptr;  // open compact-path call (null: p already complete)
    ~karma_graph_job() {
        if (sets) karma::sets_free(sets);
        delete p;
    }
};

extern "C" {

int karma_graph_records_begin(karma_ctx* ctx, const uint32_t* records, int64_t A, int64_t N, int flags, int is_device,
                              karma_graph_job** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && (records || A == 0) && A >= 0, KARMA_ERR_ARG, "karma_graph_records: bad arguments");
    KARMA_CHECK(A < (int64_t(1) << 40), KARMA_ERR_ARG, "too many records");
    KARMA_CHECK(flags == KARMA_REC_SORTED || flags == KARMA_REC_UNSORTED || flags == KARMA_REC_FLAGGED, KARMA_ERR_ARG,
                "karma_graph_records: unknown record format %d", flags);
    // held until the job owns it, so every early return (KARMA_HIP / KARMA_CHECK) frees it
    std::unique_ptr<karma_pairs> ph(new karma_pairs());
    ph->ctx = ctx;
    DevArray<uint2> own;
    DevArray<uint32_t> ownw;
    const uint2* rec = reinterpret_cast<const uint2*>(records);
    int rc = KARMA_OK;
    if (flags == KARMA_REC_FLAGGED) {
        // one u32 per record; the classify kernel streams 16-byte loads
        const uint32_t* w = records;
        if (!is_device || (reinterpret_cast<uintptr_t>(w) & 15)) {
            if ((rc = ownw.alloc(ctx, std::max<int64_t>(A, 1)))) return rc;
            if (A)
                KARMA_HIP(hipMemcpyAsync(ownw.ptr, records, A * 4,
                                         is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, ctx->stream));
            w = ownw.ptr;
        }
        karma_pairs* p = ph.get();
        auto* job = new karma_graph_job();
        job->p = ph.release();
        job->ownw.swap(ownw);
        RecIn in;
        in.fw = w;
        rc = N > sets_max_contigs() ? records_to_pairs_sets(ctx, in, A, N, p) : sets_begin(ctx, in, A, N, &job->sets);
        if (rc) {
            delete job;
            return rc;
        }
        *out = job;
        return KARMA_OK;
    }
    if (!is_device || flags == KARMA_REC_UNSORTED) {
        if ((rc = own.alloc(ctx, A))) return rc;
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
            (rc = cid2.alloc(ctx, A))) return rc;
        KARMA_LAUNCH(ctx, "deinterleave", deinterleave_kernel, grid1(A), 256, 0, own.ptr, A, rid.ptr, cid.ptr);
        // grouped by read: the library's radix sort on the read ids (sort.hip)
        if ((rc = radix_sort_u32(ctx, rid.ptr, cid.ptr, A, 32, rid2.ptr, cid2.ptr))) return rc;
        KARMA_LAUNCH(ctx, "interleave", interleave_kernel, grid1(A), 256, 0, rid2.ptr, cid2.ptr, A, own.ptr);
    }
    if (reinterpret_cast<uintptr_t>(rec) & 15) {  // the set pipeline streams 16-byte loads
        if (!own.ptr) {
            if ((rc = own.alloc(ctx, A))) return rc;
            KARMA_HIP(hipMemcpyAsync(own.ptr, rec, A * 8, hipMemcpyDeviceToDevice, ctx->stream));
            rec = own.ptr;
        }
    }
    karma_pairs* p = ph.get();
    auto* job = new karma_graph_job();
    job->p = ph.release();
    job->own.swap(own);
    RecIn in;
    in.pr = rec;
    if (N > sets_max_contigs()) {  // wide path: runs to completion here
        rc = records_to_pairs_sets(ctx, in, A, N, p);
    } else {
        rc = sets_begin(ctx, in, A, N, &job->sets);
    }
    if (rc) {
        delete job;
        return rc;
    }
    *out = job;
    return KARMA_OK;
}

int karma_graph_records_end(karma_graph_job* job, karma_pairs** out) {
    KARMA_CHECK(job && out, KARMA_ERR_ARG, "karma_graph_records_end: null argument");
    KARMA_TRY(ctx_begin(job->p->ctx));
    int rc = KARMA_OK;
    if (job->sets) {
        SetsJob* sj = job->sets;
        job->sets = nullptr;
        rc = sets_end(sj, job->p);
    }
    if (rc) {
        delete job;
        return rc;
    }
    *out = job->p;
    job->p = nullptr;
    delete job;
    return KARMA_OK;
}

int karma_graph_records(karma_ctx* ctx, const uint32_t* records, int64_t A, int64_t N, int flags, int is_device,
                        karma_pairs** out) {
    karma_graph_job* job = nullptr;
    KARMA_TRY(karma_graph_records_begin(ctx, records, A, N, flags, is_device, &job));
    return karma_graph_records_end(job, out);
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

// A list with runs of equal adjacent keys (karma_pairs::dups) to a sorted
// unique one: group counts + group sums (two launches), one synchronisation,
// and the order check of the merge that made it.
static int compact_pairs(karma_pairs* p) {
    if (!p->dups) return KARMA_OK;
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    const int64_t n = p->n;
    DevArray<uint64_t> k;
    DevArray<int64_t> c, nout;
    KARMA_TRY(k.alloc(ctx, n));
    KARMA_TRY(c.alloc(ctx, n));
    KARMA_TRY(nout.alloc(ctx, 1));
    KARMA_HIP(hipMemsetAsync(nout.ptr, 0, 8, ctx->stream));
    if (n) {
        const int64_t nb = ceil_div(n, kET);
        DevArray<int64_t> blk;
        KARMA_TRY(blk.alloc(ctx, nb));
        KARMA_LAUNCH(ctx, "merge_groups", group_count_kernel, nb, kET, 0, p->keys.ptr, n, blk.ptr);
        KARMA_LAUNCH(ctx, "merge_sum", group_sum_kernel, nb, kET, 0, p->keys.ptr, p->counts.ptr, n, blk.ptr, k.ptr,
                     c.ptr, nout.ptr);
    }
    int64_t* hp = nullptr;
    KARMA_TRY(ctx_pinned(ctx, 16, reinterpret_cast<void**>(&hp)));
    KARMA_HIP(hipMemcpyAsync(hp, nout.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipMemcpyAsync(hp + 1, p->bad.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_CHECK(!hp[1], KARMA_ERR_UNSORTED, "karma_pairs_merge_runs: a run is not sorted by key");
    p->keys.swap(k);
    p->counts.swap(c);
    p->n = hp[0];
    p->dups = false;
    return KARMA_OK;
}

static int merge_runs_impl(karma_ctx* ctx, const uint64_t* keys, const int64_t* counts, const int64_t* kc,
                           const int64_t* run_off, int n_runs, int is_device, karma_pairs** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && run_off && n_runs >= 1, KARMA_ERR_ARG, "karma_pairs_merge_runs: bad arguments");
    std::vector<int64_t> off(run_off, run_off + n_runs + 1);
    KARMA_CHECK(off[0] == 0, KARMA_ERR_ARG, "karma_pairs_merge_runs: run_off[0] must be 0");
    for (int r = 0; r < n_runs; ++r)
        KARMA_CHECK(off[r] <= off[r + 1], KARMA_ERR_ARG, "karma_pairs_merge_runs: run offsets decrease");
    const int64_t n = off[n_runs];
    KARMA_CHECK(n == 0 || (keys && counts) || kc, KARMA_ERR_ARG, "karma_pairs_merge_runs: null keys or counts");
    KARMA_CHECK(n < (int64_t(1) << 31), KARMA_ERR_ARG, "karma_pairs_merge_runs: %lld items exceed 2^31", (long long)n);
    auto* p = new karma_pairs();
    p->ctx = ctx;
    std::unique_ptr<karma_pairs> guard(p);
    DevArray<uint64_t> kb[2];
    DevArray<int64_t> cb[2];
    const uint64_t* sk = keys;
    const int64_t* sc = counts;
    if (!is_device && n) {
        KARMA_TRY(kb[1].alloc(ctx, n));
        KARMA_TRY(cb[1].alloc(ctx, n));
        KARMA_HIP(hipMemcpyAsync(kb[1].ptr, keys, n * 8, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(cb[1].ptr, counts, n * 8, hipMemcpyHostToDevice, ctx->stream));
        sk = kb[1].ptr;
        sc = cb[1].ptr;
    }
    // st (mapped host memory, written by the kernels): [0] unique keys
    // (ReduceByKey's run count), [1] order violation
    void *hst = nullptr, *dst_ = nullptr;
    KARMA_TRY(ctx_mapped(ctx, kMapMerge, 16, &hst, &dst_));
    std::memset(hst, 0, 16);
    int64_t* const st = static_cast<int64_t*>(dst_);
    if (n_runs <= kMergeMaxRuns) {
        // one ranking pass into merged order (reads the interleaved wire format directly)
        RunOffs R{};
        for (int r = 0; r <= n_runs; ++r) R.o[r] = off[r];
        KARMA_TRY(kb[0].alloc(ctx, n));
        KARMA_TRY(cb[0].alloc(ctx, n));
        int64_t tiles = 0;
        for (int r = 0; r < n_runs; ++r) {
            R.t[r] = tiles;
            tiles += ceil_div(off[r + 1] - off[r], kMergeTile);
        }
        R.t[n_runs] = tiles;
        const bool lazy = is_device != 0;
        int64_t* badp = st + 1;
        if (lazy) {
            KARMA_TRY(p->bad.alloc(ctx, 1));
            badp = p->bad.ptr;
            if (!tiles) KARMA_HIP(hipMemsetAsync(badp, 0, 8, ctx->stream));
        }
        if (tiles) {
            DevArray<int64_t> wb;
            KARMA_TRY(wb.alloc(ctx, tiles * n_runs * 2));
            KARMA_LAUNCH(ctx, "merge_bounds", merge_bounds_kernel, ceil_div(tiles * n_runs * 2, 256 / kMG), 256, 0, sk,
                         reinterpret_cast<const longlong2*>(kc), R, n_runs, tiles, wb.ptr, badp);
            KARMA_LAUNCH(ctx, "merge_rank", merge_rank_kernel, tiles, 256, 0, sk, sc,
                         reinterpret_cast<const longlong2*>(kc), R, n_runs, wb.ptr, kb[0].ptr, cb[0].ptr, badp);
        }
        if (lazy) {
            // merged order, equal keys adjacent: the edge stage sums the groups
            // itself; other accessors compact first (compact_pairs).  No host
            // synchronisation here.
            p->keys.swap(kb[0]);
            p->counts.swap(cb[0]);
            p->n = n;
            p->dups = true;
            *out = guard.release();
            return KARMA_OK;
        }
        sk = kb[0].ptr;
        sc = cb[0].ptr;
    } else {
        // more than kMergeMaxRuns runs: the ranking merge on groups of up to
        // kMergeMaxRuns consecutive runs, level by level, ping-pong buffers
        if (kc && n) {  // interleaved device input: split once into the merge's first buffers
            KARMA_TRY(kb[1].alloc(ctx, n));
            KARMA_TRY(cb[1].alloc(ctx, n));
            KARMA_LAUNCH(ctx, "merge_split", deinterleave_kc_kernel, std::min<int64_t>(grid1(n), 4096), 256, 0,
                         reinterpret_cast<const longlong2*>(kc), n, kb[1].ptr, cb[1].ptr);
            sk = kb[1].ptr;
            sc = cb[1].ptr;
        }
        KARMA_TRY(kb[0].alloc(ctx, n));
        KARMA_TRY(cb[0].alloc(ctx, n));
        if (!kb[1].ptr) {
            KARMA_TRY(kb[1].alloc(ctx, n));
            KARMA_TRY(cb[1].alloc(ctx, n));
        }
        DevArray<int64_t> scratch;  // merge_bounds_kernel clears its flag word: a throwaway one here
        KARMA_TRY(scratch.alloc(ctx, 1));
        int dst = 0;
        for (std::vector<int64_t> o = off; o.size() > 2; dst ^= 1) {
            const int nr_all = (int)o.size() - 1;
            std::vector<int64_t> next{0};
            for (int g0 = 0; g0 < nr_all; g0 += kMergeMaxRuns) {
                const int g1 = std::min(nr_all, g0 + kMergeMaxRuns);
                const int64_t base = o[g0], len = o[g1] - base;
                next.push_back(o[g1]);
                if (!len) continue;
                if (g1 - g0 == 1) {  // a lone run: carried over
                    KARMA_HIP(hipMemcpyAsync(kb[dst].ptr + base, sk + base, len * 8, hipMemcpyDeviceToDevice,
                                             ctx->stream));
                    KARMA_HIP(hipMemcpyAsync(cb[dst].ptr + base, sc + base, len * 8, hipMemcpyDeviceToDevice,
                                             ctx->stream));
                    continue;
                }
                RunOffs R{};
                const int nr = g1 - g0;
                int64_t tiles = 0;
                for (int r = 0; r <= nr; ++r) R.o[r] = o[g0 + r] - base;
                for (int r = 0; r < nr; ++r) {
                    R.t[r] = tiles;
                    tiles += ceil_div(R.o[r + 1] - R.o[r], kMergeTile);
                }
                R.t[nr] = tiles;
                DevArray<int64_t> wb;
                KARMA_TRY(wb.alloc(ctx, tiles * nr * 2));
                KARMA_LAUNCH(ctx, "merge_bounds", merge_bounds_kernel, ceil_div(tiles * nr * 2, 256 / kMG), 256, 0,
                             sk + base, (const longlong2*)nullptr, R, nr, tiles, wb.ptr, scratch.ptr);
                KARMA_LAUNCH(ctx, "merge_rank", merge_rank_kernel, tiles, 256, 0, sk + base, sc + base,
                             (const longlong2*)nullptr, R, nr, wb.ptr, kb[dst].ptr + base, cb[dst].ptr + base, st + 1);
            }
            o.swap(next);
            sk = kb[dst].ptr;
            sc = cb[dst].ptr;
        }
    }
    // equal keys (from different runs, or repeated in one) are now adjacent
    KARMA_TRY(p->keys.alloc(ctx, n));
    KARMA_TRY(p->counts.alloc(ctx, n));
    if (n) {
        const int64_t nb = ceil_div(n, kET);
        DevArray<int64_t> blk;
        KARMA_TRY(blk.alloc(ctx, nb));
        KARMA_LAUNCH(ctx, "merge_groups", group_count_kernel, nb, kET, 0, sk, n, blk.ptr);
        KARMA_LAUNCH(ctx, "merge_sum", group_sum_kernel, nb, kET, 0, sk, sc, n, blk.ptr, p->keys.ptr, p->counts.ptr,
                     st);
    }
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    const volatile int64_t* h = static_cast<const volatile int64_t*>(hst);
    KARMA_CHECK(!h[1], KARMA_ERR_UNSORTED, "karma_pairs_merge_runs: a run is not sorted by key");
    p->n = h[0];
    *out = guard.release();
    return KARMA_OK;
}

int karma_pairs_merge_runs(karma_ctx* ctx, const uint64_t* keys, const int64_t* counts, const int64_t* run_off,
                           int n_runs, int is_device, karma_pairs** out) {
    return merge_runs_impl(ctx, keys, counts, nullptr, run_off, n_runs, is_device, out);
}

int karma_pairs_merge_runs_kc(karma_ctx* ctx, const int64_t* kc_dev, const int64_t* run_off, int n_runs,
                              karma_pairs** out) {
    return merge_runs_impl(ctx, nullptr, nullptr, kc_dev, run_off, n_runs, 1, out);
}

int karma_pairs_get_kc(karma_pairs* p, int64_t* kc_dev) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    KARMA_TRY(compact_pairs(p));
    KARMA_CHECK(p && (kc_dev || p->n == 0), KARMA_ERR_ARG, "karma_pairs_get_kc: bad arguments");
    KARMA_TRY(ctx_begin(p->ctx));
    if (p->n)
        KARMA_LAUNCH(p->ctx, "pairs_interleave", interleave_kc_kernel, std::min<int64_t>(grid1(p->n), 4096), 256, 0,
                     p->keys.ptr, p->counts.ptr, p->n, reinterpret_cast<longlong2*>(kc_dev));
    return KARMA_OK;
}

int karma_pairs_destroy(karma_pairs* p) {
    if (!p) return KARMA_OK;
    hipSetDevice(p->ctx->device);
    delete p;
    return KARMA_OK;
}

int karma_pairs_rebind(karma_pairs* p, karma_ctx* ctx) {
    KARMA_CHECK(p && ctx, KARMA_ERR_ARG, "null argument");
    KARMA_CHECK(p->ctx->device == ctx->device, KARMA_ERR_ARG, "pairs and context are on different devices");
    KARMA_TRY(ctx_begin(p->ctx));
    KARMA_HIP(hipStreamSynchronize(p->ctx->stream));
    p->ctx = ctx;
    return KARMA_OK;
}

int karma_pairs_count(karma_pairs* p, int64_t* n) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    KARMA_TRY(compact_pairs(p));
    KARMA_CHECK(p && n, KARMA_ERR_ARG, "null argument");
    *n = p->n;
    return KARMA_OK;
}

int karma_pairs_device(karma_pairs* p, const uint64_t** keys, const int64_t** counts) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    KARMA_TRY(compact_pairs(p));
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    if (keys) *keys = p->keys.ptr;
    if (counts) *counts = p->counts.ptr;
    return KARMA_OK;
}

int karma_pairs_get(karma_pairs* p, uint64_t* keys, int64_t* counts, uint64_t* first, int is_device) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    KARMA_TRY(compact_pairs(p));
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    KARMA_TRY(ctx_begin(p->ctx));
    const hipMemcpyKind kind = is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (p->n) {
        if (keys) KARMA_HIP(hipMemcpyAsync(keys, p->keys.ptr, p->n * 8, kind, p->ctx->stream));
        if (counts) KARMA_HIP(hipMemcpyAsync(counts, p->counts.ptr, p->n * 8, kind, p->ctx->stream));
        if (first && p->has_first) KARMA_HIP(hipMemcpyAsync(first, p->first.ptr, p->n * 8, kind, p->ctx->stream));
    }
    if (!is_device) KARMA_HIP(hipStreamSynchronize(p->ctx->stream));  // device copies stay stream-ordered
    return KARMA_OK;
}

int karma_graph_split_hint(karma_ctx* ctx, const int64_t* bounds, int nranks) {
    KARMA_CHECK(ctx && nranks >= 0 && (bounds || nranks == 0), KARMA_ERR_ARG, "karma_graph_split_hint: bad arguments");
    ctx->split_bounds.assign(bounds, bounds + (nranks ? nranks + 1 : 0));
    return KARMA_OK;
}

int karma_pairs_split(karma_pairs* p, const int64_t* bounds, int nranks, int64_t* starts) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null pairs");
    KARMA_TRY(compact_pairs(p));
    KARMA_CHECK(p && bounds && starts && nranks >= 1, KARMA_ERR_ARG, "bad arguments");
    if (p->split_bounds.size() == (size_t)nranks + 1 &&
        std::equal(p->split_bounds.begin(), p->split_bounds.end(), bounds)) {
        std::memcpy(starts, p->split_starts.data(), (nranks + 1) * 8);  // found by the job's final kernel
        return KARMA_OK;
    }
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    // binary searches on the device; bounds and starts live in mapped host
    // memory (no copy launches: beside a running profile kernel those waited
    // for free CUs, 0.24 ms in the 8-rank emulation)
    const int nb = nranks + 1;
    void *hb = nullptr, *db = nullptr;
    KARMA_TRY(ctx_mapped(ctx, kMapSplit, 2 * nb * 8, &hb, &db));
    int64_t* h = static_cast<int64_t*>(hb);
    int64_t* d = static_cast<int64_t*>(db);
    std::memcpy(h, bounds, nb * 8);
    KARMA_LAUNCH(ctx, "pairs_split", split_kernel, grid1(nb, 64), 64, 0, p->keys.ptr, p->n, d, nb, d + nb);
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    std::memcpy(starts, h + nb, nb * 8);
    return KARMA_OK;
}

int karma_pairs_split_kc(karma_pairs* p, const int64_t* bounds, int nranks, int64_t* starts, int64_t* kc_dev) {
    KARMA_CHECK(p && bounds && starts && nranks >= 1 && nranks < 1024, KARMA_ERR_ARG, "bad arguments");
    KARMA_TRY(compact_pairs(p));
    KARMA_CHECK(kc_dev || p->n == 0, KARMA_ERR_ARG, "karma_pairs_split_kc: null wire buffer");
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    const int nb = nranks + 1;
    void *hb = nullptr, *db = nullptr;
    KARMA_TRY(ctx_mapped(ctx, kMapSplit, 2 * nb * 8, &hb, &db));
    int64_t* h = static_cast<int64_t*>(hb);
    int64_t* d = static_cast<int64_t*>(db);
    std::memcpy(h, bounds, nb * 8);
    const int grid = (int)std::min<int64_t>(std::max<int64_t>(1, ceil_div(p->n, 256)), 4096);
    KARMA_LAUNCH(ctx, "pairs_split_kc", split_kc_kernel, grid, std::max(256, ((nb + 63) / 64) * 64), 0, p->keys.ptr,
                 p->counts.ptr, p->n, d, nb, d + nb, reinterpret_cast<longlong2*>(kc_dev));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    std::memcpy(starts, h + nb, nb * 8);
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

// The edge stage in two halves.  _begin sets the totals (the caller's, the eq
// totals, or zeros that the count kernel fills with the list's diagonal) and
// launches the count kernel; _end launches the write kernel and synchronises.
// Between the two the caller may all-gather the totals (the owners' readset
// sizes, karma_edges_begin's totals_dev).
static int edges_begin_impl(karma_ctx* ctx, karma_pairs* p, int mode, const int64_t* totals_dev, int64_t N,
                            karma_edges** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(p && out && N >= 0, KARMA_ERR_ARG, "karma_edges: bad arguments");
    KARMA_CHECK(mode == KARMA_MODE_READS || mode == KARMA_MODE_EQ, KARMA_ERR_ARG, "bad mode");
    KARMA_CHECK(!p->dups || !p->has_first, KARMA_ERR_STATE, "karma_edges: an eq list with unsummed groups");
    auto* e = new karma_edges();
    e->ctx = ctx;
    e->n_contigs = N;
    e->src = p;
    e->mode = mode;
    std::unique_ptr<karma_edges> guard(e);
    KARMA_TRY(e->totals.alloc(ctx, N));
    bool diag_here = false;
    if (!totals_dev) {
        if (mode == KARMA_MODE_EQ) {
            KARMA_CHECK(p->has_totals && p->n_contigs == N, KARMA_ERR_STATE, "eq pair list without totals");
            if (N) KARMA_HIP(hipMemcpyAsync(e->totals.ptr, p->totals.ptr, N * 8, hipMemcpyDeviceToDevice, ctx->stream));
        } else {  // the diagonal counts, written by the edge count kernel (with the zeros when the list is not empty)
            if (N && !p->n) KARMA_HIP(hipMemsetAsync(e->totals.ptr, 0, N * 8, ctx->stream));
            diag_here = true;
        }
    } else if (N) {
        KARMA_HIP(hipMemcpyAsync(e->totals.ptr, totals_dev, N * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    const int64_t n = p->n;
    e->n_blk = std::max<int64_t>(1, ceil_div(n, kET));
    KARMA_TRY(e->blk.alloc(ctx, e->n_blk + 3));
    if (n)
        KARMA_LAUNCH(ctx, "edge_count", edges_count_kernel, ceil_div(n, kET), kET, 0, p->keys.ptr, p->counts.ptr, n,
                     mode, diag_here ? e->totals.ptr : (int64_t*)nullptr, N, e->blk.ptr, e->blk.ptr + e->n_blk);
    else
        KARMA_HIP(hipMemsetAsync(e->blk.ptr + e->n_blk, 0, 3 * 8, ctx->stream));
    e->open = true;
    *out = guard.release();
    return KARMA_OK;
}

// The deferred half of karma_edges_end (n_edges = NULL): the status words
// from device memory, one synchronisation, the same checks.
static int edges_resolve(karma_edges* e) {
    if (!e->pending) return KARMA_OK;
    karma_ctx* ctx = e->ctx;
    KARMA_TRY(ctx_begin(ctx));
    void* hpin = nullptr;
    KARMA_TRY(ctx_pinned(ctx, 24, &hpin));
    KARMA_HIP(hipMemcpyAsync(hpin, e->blk.ptr + e->n_blk, 24, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    e->pending = false;
    e->blk.release();
    const int64_t* hs = static_cast<const int64_t*>(hpin);
    KARMA_CHECK(!hs[2], KARMA_ERR_UNSORTED, "karma_pairs_merge_runs: a run is not sorted by key");
    KARMA_CHECK(!(int)hs[0], KARMA_ERR_ZERO_DIV, "division by zero: a shared count over a zero total");
    e->E = hs[1];
    return KARMA_OK;
}

static int edges_end_impl(karma_edges* e, int64_t* n_edges) {
    KARMA_CHECK(e && e->open, KARMA_ERR_STATE, "karma_edges_end: no open edge stage");
    karma_ctx* ctx = e->ctx;
    KARMA_TRY(ctx_begin(ctx));
    const karma_pairs* p = e->src;
    e->open = false;
    const int64_t n = p->n;
    if (!n_edges) {  // deferred: the write kernel's status words stay on the device
        KARMA_TRY(e->a.alloc(ctx, n));
        KARMA_TRY(e->b.alloc(ctx, n));
        KARMA_TRY(e->s.alloc(ctx, n));
        KARMA_TRY(e->w.alloc(ctx, n));
        e->has_first = p->has_first;
        if (e->has_first) KARMA_TRY(e->first.alloc(ctx, n));
        if (n)
            KARMA_LAUNCH(ctx, "edge_weights", edges_write_kernel, ceil_div(n, kET), kET, 0, p->keys.ptr, p->counts.ptr,
                         p->has_first ? p->first.ptr : (const uint64_t*)nullptr, n, e->mode, e->totals.ptr,
                         e->blk.ptr, e->a.ptr, e->b.ptr, e->s.ptr, e->w.ptr,
                         e->has_first ? e->first.ptr : (uint64_t*)nullptr, e->blk.ptr + e->n_blk,
                         p->dups ? (const int64_t*)p->bad.ptr : (const int64_t*)nullptr);
        e->src = nullptr;
        e->pending = true;
        e->E = -1;
        return KARMA_OK;
    }
    // st (mapped host memory, written by the write kernel): 0 zero-division
    // flag, 1 edge count, 2 the list's merge order check
    void *hst = nullptr, *dst_ = nullptr;
    KARMA_TRY(ctx_mapped(ctx, kMapEdges, 24, &hst, &dst_));
    std::memset(hst, 0, 24);
    int64_t* const st = static_cast<int64_t*>(dst_);
    // edges <= pairs: written before the count is known on the host
    KARMA_TRY(e->a.alloc(ctx, n));
    KARMA_TRY(e->b.alloc(ctx, n));
    KARMA_TRY(e->s.alloc(ctx, n));
    KARMA_TRY(e->w.alloc(ctx, n));
    e->has_first = p->has_first;
    if (e->has_first) KARMA_TRY(e->first.alloc(ctx, n));
    if (n)
        KARMA_LAUNCH(ctx, "edge_weights", edges_write_kernel, ceil_div(n, kET), kET, 0, p->keys.ptr, p->counts.ptr,
                     p->has_first ? p->first.ptr : (const uint64_t*)nullptr, n, e->mode, e->totals.ptr, e->blk.ptr,
                     e->a.ptr, e->b.ptr, e->s.ptr, e->w.ptr, e->has_first ? e->first.ptr : (uint64_t*)nullptr, st,
                     p->dups ? (const int64_t*)p->bad.ptr : (const int64_t*)nullptr);
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    e->blk.release();
    e->src = nullptr;
    const volatile int64_t* hs = static_cast<const volatile int64_t*>(hst);
    KARMA_CHECK(!hs[2], KARMA_ERR_UNSORTED, "karma_pairs_merge_runs: a run is not sorted by key");
    KARMA_CHECK(!(int)hs[0], KARMA_ERR_ZERO_DIV, "division by zero: a shared count over a zero total");
    e->E = hs[1];
    *n_edges = e->E;
    return KARMA_OK;
}

}  // extern "C"

namespace karma {
// karma_step: the device address of a pending edge stage's three status words
// (zero-total flag, edge count, merge order), which the caller copies out in
// stream order and checks later; the edges are then no longer pending.
const int64_t* edges_take_pending(karma_edges* e) {
    if (!e || !e->pending) return nullptr;
    e->pending = false;
    return e->blk.ptr + e->n_blk;
}
}  // namespace karma

extern "C" {

int karma_edges_from_pairs(karma_ctx* ctx, karma_pairs* p, int mode, const int64_t* totals_dev, int64_t N,
                           karma_edges** out, int64_t* n_edges) {
    KARMA_CHECK(out && n_edges, KARMA_ERR_ARG, "karma_edges_from_pairs: bad arguments");
    karma_edges* e = nullptr;
    KARMA_TRY(edges_begin_impl(ctx, p, mode, totals_dev, N, &e));
    std::unique_ptr<karma_edges> guard(e);
    KARMA_TRY(edges_end_impl(e, n_edges));
    *out = guard.release();
    return KARMA_OK;
}

int karma_edges_begin(karma_ctx* ctx, karma_pairs* p, int mode, int64_t N, karma_edges** out, int64_t** totals_dev) {
    KARMA_CHECK(out && totals_dev, KARMA_ERR_ARG, "karma_edges_begin: bad arguments");
    KARMA_TRY(edges_begin_impl(ctx, p, mode, nullptr, N, out));
    *totals_dev = (*out)->totals.ptr;
    return KARMA_OK;
}

int karma_edges_end(karma_edges* e, int64_t* n_edges) { return edges_end_impl(e, n_edges); }

int karma_edges_count(karma_edges* e, int64_t* n_edges) {
    KARMA_CHECK(e && n_edges && !e->open, KARMA_ERR_STATE, "karma_edges_count: no finished edge stage");
    KARMA_TRY(edges_resolve(e));
    *n_edges = e->E;
    return KARMA_OK;
}

// An edge stage still pending (karma_edges_end without a count) has its
// zero-total and merge-order words unread: they are read here (one wait) and
// an error is reported on stderr and returned, not dropped.
int karma_edges_destroy(karma_edges* e) {
    if (!e) return KARMA_OK;
    hipSetDevice(e->ctx->device);
    int rc = KARMA_OK;
    if (e->pending) {
        rc = edges_resolve(e);
        if (rc) std::fprintf(stderr, "karma_edges_destroy: a deferred edge stage reported: %s\n", karma_last_error());
    }
    delete e;
    return rc;
}

int karma_edges_get(karma_edges* e, uint32_t* a, uint32_t* b, int64_t* s, double* w, uint64_t* first, int is_device) {
    KARMA_CHECK(e, KARMA_ERR_ARG, "null edges");
    KARMA_TRY(ctx_begin(e->ctx));
    KARMA_TRY(edges_resolve(e));
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

// karma_edges_get and karma_edges_totals in one synchronisation
int karma_edges_get_all(karma_edges* e, uint32_t* a, uint32_t* b, int64_t* s, double* w, uint64_t* first,
                        int64_t* totals, int is_device) {
    KARMA_CHECK(e && (totals || !e->n_contigs), KARMA_ERR_ARG, "bad arguments");
    KARMA_TRY(ctx_begin(e->ctx));
    KARMA_TRY(edges_resolve(e));
    const hipMemcpyKind kind = is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    hipStream_t st = e->ctx->stream;
    if (e->n_contigs) KARMA_HIP(hipMemcpyAsync(totals, e->totals.ptr, e->n_contigs * 8, kind, st));
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

int karma_edges_get_ordered(karma_edges* e, uint32_t* a, uint32_t* b, double* w, int is_device) {
    KARMA_CHECK(e && a && b && w, KARMA_ERR_ARG, "bad arguments");
    KARMA_TRY(ctx_begin(e->ctx));
    KARMA_TRY(edges_resolve(e));
    KARMA_CHECK(e->has_first, KARMA_ERR_STATE, "karma_edges_get_ordered: not an equivalence-class edge stage");
    karma_ctx* ctx = e->ctx;
    const hipMemcpyKind kind = is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (e->E) {
        DevArray<uint32_t> oa, ob;
        DevArray<double> ow;
        KARMA_TRY(oa.alloc(ctx, e->E));
        KARMA_TRY(ob.alloc(ctx, e->E));
        KARMA_TRY(ow.alloc(ctx, e->E));
        KARMA_LAUNCH(ctx, "eq_order", eq_order_kernel, (int)ceil_div(e->E, kOrdT), kOrdT, 0, e->a.ptr, e->b.ptr,
                     e->w.ptr, e->first.ptr, e->E, oa.ptr, ob.ptr, ow.ptr);
        KARMA_HIP(hipMemcpyAsync(a, oa.ptr, e->E * 4, kind, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(b, ob.ptr, e->E * 4, kind, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(w, ow.ptr, e->E * 8, kind, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));  // before the scratch returns to the cache
    }
    return KARMA_OK;
}

int karma_edges_totals(karma_edges* e, int64_t* totals, int is_device) {
    KARMA_CHECK(e && (totals || !e->n_contigs), KARMA_ERR_ARG, "bad arguments");
    KARMA_TRY(ctx_begin(e->ctx));
    KARMA_TRY(edges_resolve(e));
    if (e->n_contigs)
        KARMA_HIP(hipMemcpyAsync(totals, e->totals.ptr, e->n_contigs * 8,
                                 is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, e->ctx->stream));
    KARMA_HIP(hipStreamSynchronize(e->ctx->stream));
    return KARMA_OK;
}

}  // extern "C"
