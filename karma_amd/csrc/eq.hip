// eq.hip — the eq-class graph (the path karma.py:240 calls,
// /root/reference/karma/read_graph.py:61-148) on hand-written gfx950 kernels:
// per-contig totals (read_graph.py:86-92), every unordered pair of every class
// whose size token is not "1" weighted by the class count (:96-114), summed per
// distinct pair, with the pair's first emission index (the intermediate
// graph's edge order, read_graph.py:120).  No library sort or reduce.
//
// Data are small next to the records path (config 3: 519k classes of at most 4
// members, 977k members, 617k pairs), so the design is about launch count,
// balance and hiding the host->device copies of the inputs:
//   1. one look-back scan of the classes' pair counts (m (m - 1) / 2, fused
//      into the scan's loads): class pair offsets = first-emission indices;
//   2. eq_rank     one thread per class (a block per class above kSmallM
//                  members): every pair's key, class, and rank among the pairs
//                  of its lower contig a (one returning atomic on a's count);
//   3. a scan of the per-contig counts (segment offsets) and eq_place: every
//      pair to segment start + rank -- a counting sort by a, no comparisons;
//   4. seg_reduce  a block takes a run of whole segments (<= kSegCap entries,
//                  snapped to segment starts), ranks every entry inside its
//                  segment by (b, position) in LDS, and sums equal (a, b) keys
//                  (counts: i64 adds in key order; first: min).  A run longer
//                  than kSegCap (one contig with > kSeg pairs as lower id) is
//                  sorted in global memory by a block-wide merge sort instead;
//                  the run's distinct keys go to their final place after the
//                  runs before it (decoupled look-back, runs in ticket order);
//   eq_totals      per-contig totals, one thread per member, u64 atomics, on
//                  the fork stream beside 2-5.
// Host inputs go up on the fork stream in the order the kernels need them;
// one readback sizes the scratch (the pair total, while the members and counts
// are still being copied) and one reads the distinct-key total at the end.
#include <memory>

#include "karma_internal.h"

using karma::ceil_div;

namespace {

#include "graph_device.h"

constexpr int kEqT = 256;      // threads of the per-class kernels
constexpr int64_t kSmallM = 32;  // classes above this size: a block each
constexpr int kRT = 512;         // seg_reduce threads
constexpr int kSeg = 1024;       // target entries per seg_reduce block (48 KB of LDS: 3 blocks per CU, one round)
constexpr int kSegCap = 2 * kSeg;  // LDS capacity of one block's run (runs snap to segment starts)

// pair t (combinations order) of a class of m members -> (i, j), i < j:
// row i holds (i, i+1..m-1); pairs before row i: i*m - i*(i+1)/2
__device__ __forceinline__ void pair_ij(int64_t t, int64_t m, int64_t* i, int64_t* j) {
    int64_t lo = 0, hi = m - 1;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (mid * m - mid * (mid + 1) / 2 <= t) lo = mid;
        else hi = mid;
    }
    *i = lo;
    *j = lo + 1 + (t - (lo * m - lo * (lo + 1) / 2));
}

struct EqIn {
    const int64_t* off;
    const uint32_t* mem;
    const int64_t* cnt;
    const uint8_t* skip;
    int64_t C;
    uint32_t N;
    int64_t n_mem;  // members readable: a class past it fails the call (bad |= 2), nothing reads beyond
};

// ---- 1. each pair's rank inside its lower contig's segment ------------------------
// Pair t of class c (t = poff[c] + its combinations index) gets its key, its
// class and its rank among the pairs whose lower contig is a (a returning
// atomic on segcnt[a]; every pair's three words are written, a pair with a
// member >= N as a sentinel the placement skips, the call then fails).
struct Pairs3 {
    uint64_t* key;
    uint32_t* rank;
    uint32_t* cls;
    int64_t cap;  // entries allocated
};

__device__ __forceinline__ void rank_pair(uint32_t xi, uint32_t xj, uint32_t N, uint32_t c, int64_t t,
                                          uint32_t* __restrict__ segcnt, Pairs3 P3, int* __restrict__ bad) {
    if (t >= P3.cap) {  // more pairs than the speculative capacity: the call runs again, sized
        bad[1] = 1;
        return;
    }
    const uint32_t a = min(xi, xj), b = max(xi, xj);
    if (b >= N) {
        *bad = 1;
        P3.rank[t] = ~0u;
        return;
    }
    P3.key[t] = ((uint64_t)a << 32) | b;
    P3.rank[t] = atomicAdd(&segcnt[a], 1u);
    P3.cls[t] = c;
}

__global__ void __launch_bounds__(kEqT) eq_rank_kernel(EqIn in, const int64_t* __restrict__ poff,
                                                       uint32_t* __restrict__ segcnt, Pairs3 P3,
                                                       uint32_t* __restrict__ big, unsigned* __restrict__ n_big,
                                                       int* __restrict__ bad) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && in.off[in.C] != in.n_mem) atomicOr(bad, 2);
    for (int64_t c = (int64_t)blockIdx.x * kEqT + threadIdx.x; c < in.C; c += (int64_t)gridDim.x * kEqT) {
        const int64_t s = in.off[c], e = in.off[c + 1], m = e - s;
        if (s < 0 || e < s || e > in.n_mem) {  // offsets past the members (or decreasing ones)
            atomicOr(bad, 2);
            // the class's pair slots as sentinels the placement skips (never left unwritten)
            for (int64_t t = poff[c]; t < min(poff[c + 1], P3.cap); ++t) P3.rank[t] = ~0u;
            continue;
        }
        if (m < 2 || (in.skip && in.skip[c])) continue;
        if (m > kSmallM) {
            big[atomicAdd(n_big, 1u)] = (uint32_t)c;
            continue;
        }
        int64_t t = poff[c];
        for (int64_t i = s; i + 1 < e; ++i) {
            const uint32_t xi = in.mem[i];
            for (int64_t j = i + 1; j < e; ++j, ++t) rank_pair(xi, in.mem[j], in.N, (uint32_t)c, t, segcnt, P3, bad);
        }
    }
}

__global__ void __launch_bounds__(kEqT) eq_rank_big_kernel(EqIn in, const int64_t* __restrict__ poff,
                                                           uint32_t* __restrict__ segcnt, Pairs3 P3,
                                                           const uint32_t* __restrict__ big,
                                                           const unsigned* __restrict__ n_big, int* __restrict__ bad) {
    const unsigned nb = *n_big;
    for (unsigned q = blockIdx.x; q < nb; q += gridDim.x) {
        const int64_t c = big[q], s = in.off[c], m = in.off[c + 1] - s, P = m * (m - 1) / 2;
        for (int64_t t = threadIdx.x; t < P; t += kEqT) {
            int64_t i, j;
            pair_ij(t, m, &i, &j);
            rank_pair(in.mem[s + i], in.mem[s + j], in.N, (uint32_t)c, poff[c] + t, segcnt, P3, bad);
        }
    }
}

// ---- per-contig totals (read_graph.py:86-92), beside the pair pipeline -----------
// One thread per member, its class by binary search over the class offsets.
__global__ void __launch_bounds__(kEqT) eq_totals_kernel(EqIn in, int64_t n_mem,
                                                         unsigned long long* __restrict__ totals,
                                                         int* __restrict__ bad) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && in.off[in.C] != in.n_mem) atomicOr(bad, 2);
    for (int64_t j = (int64_t)blockIdx.x * kEqT + threadIdx.x; j < n_mem; j += (int64_t)gridDim.x * kEqT) {
        int64_t lo = 0, hi = in.C;  // the last class with off[c] <= j
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (in.off[mid] <= j) lo = mid;
            else hi = mid;
        }
        const uint32_t x = in.mem[j];
        if (x >= in.N) *bad = 1;
        else atomicAdd(&totals[x], (unsigned long long)in.cnt[lo]);  // two's complement: exact for negative counts
    }
}

// ---- 2. every pair into its segment (a counting sort by a) -----------------------
struct Entries {
    uint64_t* key;    // a << 32 | b, a <= b
    int64_t* cnt;
    uint64_t* first;  // global emission index (class pair offset + combinations index)
};
struct Placed {       // a pair in its segment: key, emission index, class
    uint64_t* key;
    uint32_t* ref;
    uint32_t* cls;
};

__global__ void __launch_bounds__(kEqT) eq_place_kernel(const int64_t* __restrict__ P_dev, Pairs3 P3,
                                                        const int64_t* __restrict__ segoff, Placed E) {
    const int64_t P = min(*P_dev, P3.cap);
    for (int64_t t = (int64_t)blockIdx.x * kEqT + threadIdx.x; t < P; t += (int64_t)gridDim.x * kEqT) {
        const uint32_t r = P3.rank[t];
        if (r == ~0u) continue;
        const uint64_t k = P3.key[t];
        const int64_t slot = segoff[k >> 32] + r;
        E.key[slot] = k;
        E.ref[slot] = (uint32_t)t;
        E.cls[slot] = P3.cls[t];
    }
}

// ---- block-wide scans ---------------------------------------------------------------
// exclusive scan of one value per thread; returns the block total in *total
template <int T>
__device__ int64_t block_scan_excl(int64_t v, int64_t* lds_w, int64_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) lds_w[w] = x;
    __syncthreads();
    int64_t base = 0, tot = 0;
    for (int i = 0; i < T / 64; ++i) {
        const int64_t s = lds_w[i];
        if (i < w) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// ---- 4. sort + reduce of whole segments, one block per run -------------------------
// Run r takes the entries [lo(r), lo(r + 1)), lo(r) = the first segment start
// at or after r * kSeg (segments never straddle two runs).  One 32-lane group
// per bound probes 32 segment offsets per round (200k contigs: 4 dependent
// loads instead of 18).
__device__ __forceinline__ int64_t run_start_g(const int64_t* __restrict__ segoff, int64_t N, int64_t P, int64_t r,
                                               int g) {
    const int64_t target = r * kSeg;
    const bool done = target >= P;
    int64_t lo = 0, hi = N;  // first a with segoff[a] >= target (segoff[N] = P >= target)
    const int lane = threadIdx.x & 63;
    const unsigned long long gm = 0xFFFFFFFFull << (lane & 32);
    for (;;) {
        const bool more = !done && hi - lo > 32;
        if (!(__ballot(more) & gm)) break;
        const int64_t step = (hi - lo + 31) / 32;
        const int64_t p = min(hi, lo + (int64_t)(g + 1) * step) - 1;
        const bool below = more && segoff[p] < target;
        const int c = __popcll(__ballot(below) & gm);
        if (more) {
            lo = min(hi, lo + (int64_t)c * step);
            hi = c < 32 ? min(hi, lo + step) : hi;
        }
    }
    const int64_t p = lo + g;
    const bool below = !done && p < hi && segoff[p] < target;
    const int64_t a = lo + __popcll(__ballot(below) & gm);
    return done ? P : segoff[a];
}

// Distinct keys of a sorted run, summed: position p of the run holds key(p),
// its class count cnt_at(p) and emission index ref_at(p).  Writes them to the
// staging arrays at [r0, r0 + u) and returns u (every thread).
template <typename KeyAt, typename CntAt, typename RefAt>
__device__ int64_t reduce_sorted_run(int64_t r0, int64_t n, KeyAt key_at, CntAt cnt_at, RefAt ref_at, Entries st,
                                     int64_t* lds_w) {
    int64_t u_total = 0, base_u = 0;
    for (int64_t c0 = 0; c0 < n; c0 += kRT) {
        const int64_t p = c0 + threadIdx.x;
        const bool head = p < n && (p == 0 || key_at(p) != key_at(p - 1));
        int64_t chunk_u;
        const int64_t pos = base_u + block_scan_excl<kRT>(head ? 1 : 0, lds_w, &chunk_u);
        if (head) {
            const uint64_t k = key_at(p);
            int64_t sum = 0;
            uint64_t f = ~0ull;
            for (int64_t q = p; q < n && key_at(q) == k; ++q) {
                sum += cnt_at(q);
                f = min(f, (uint64_t)ref_at(q));
            }
            st.key[r0 + pos] = k;
            st.cnt[r0 + pos] = sum;
            st.first[r0 + pos] = f;
        }
        base_u += chunk_u;
    }
    u_total = base_u;
    return u_total;
}

// Runs are taken in ticket order; each run's distinct keys go straight to
// their final place, after the runs before it (decoupled look-back), so no
// scan or compaction launch follows.  The last run writes the total.
__global__ void __launch_bounds__(kRT) seg_reduce_kernel(const int64_t* __restrict__ segoff, int64_t N,
                                                         int64_t n_runs, Placed in, const int64_t* __restrict__ cnt,
                                                         Entries st, uint64_t* __restrict__ gk0,
                                                         uint64_t* __restrict__ gk1, uint32_t* __restrict__ gi0,
                                                         uint32_t* __restrict__ gi1, uint64_t* __restrict__ lb,
                                                         unsigned* __restrict__ ticket, Entries out,
                                                         int64_t* __restrict__ n_out) {
    __shared__ uint64_t skey[kSegCap];
    __shared__ uint32_t sidx[kSegCap];
    __shared__ uint64_t okey[kSegCap];
    __shared__ uint32_t oidx[kSegCap];
    __shared__ int64_t lds_w[kRT / 64];
    __shared__ int64_t r_s, r0_s, r1_s, base_s;
    if (threadIdx.x == 0) r_s = atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t r = r_s;
    // the placed pairs (segoff[N]): fewer than P when a member id is out of
    // range (those pairs are not placed; the call then fails)
    const int64_t P = segoff[N];
    if (threadIdx.x < 64) {
        const int64_t b = run_start_g(segoff, N, P, r + (threadIdx.x >> 5), threadIdx.x & 31);
        if (threadIdx.x == 0) r0_s = b;
        if (threadIdx.x == 32) r1_s = b;
    }
    __syncthreads();
    const int64_t r0 = r0_s, r1 = r1_s;
    const int64_t n = r1 - r0;
    int64_t u = 0;
    if (n <= kSegCap) {
        for (int64_t p = threadIdx.x; p < n; p += kRT) {
            skey[p] = in.key[r0 + p];
            sidx[p] = (uint32_t)p;
        }
        __syncthreads();
        // the run is grouped by a (counting sort): rank each entry inside its
        // segment by (b, position); a segment is found by binary search on a
        for (int64_t p = threadIdx.x; p < n; p += kRT) {
            const uint64_t k = skey[p];
            const uint32_t a = (uint32_t)(k >> 32);
            int64_t lo = 0, hi = p;  // first index with the same a
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if ((uint32_t)(skey[mid] >> 32) >= a) hi = mid;
                else lo = mid + 1;
            }
            int64_t rank = lo;
            for (int64_t q = lo; q < n; ++q) {
                const uint64_t kq = skey[q];
                if ((uint32_t)(kq >> 32) != a) break;
                rank += (kq < k || (kq == k && q < p)) ? 1 : 0;
            }
            okey[rank] = k;
            oidx[rank] = (uint32_t)p;
        }
        __syncthreads();
        // each entry's class count and emission index into LDS in sorted order
        // (independent gathers, all in flight; the group sums then read LDS)
        int64_t* scnt = reinterpret_cast<int64_t*>(skey);
        uint32_t* sref = sidx;
        for (int64_t p = threadIdx.x; p < n; p += kRT) {
            const int64_t e = r0 + (int64_t)oidx[p];
            scnt[p] = cnt[in.cls[e]];
            sref[p] = in.ref[e];
        }
        __syncthreads();
        u = reduce_sorted_run(
            r0, n, [&](int64_t p) { return okey[p]; }, [&](int64_t p) { return scnt[p]; },
            [&](int64_t p) { return sref[p]; }, st, lds_w);
    } else {
        // a run with a segment of > kSeg entries: bottom-up merge sort of
        // (key, index) in global scratch (stable merge ranks), then the same reduce
        uint64_t *ka = gk0 + r0, *kb = gk1 + r0;
        uint32_t *ia = gi0 + r0, *ib = gi1 + r0;
        for (int64_t p = threadIdx.x; p < n; p += kRT) {
            ka[p] = in.key[r0 + p];
            ia[p] = (uint32_t)p;
        }
        __syncthreads();
        for (int64_t w = 1; w < n; w <<= 1) {
            for (int64_t p = threadIdx.x; p < n; p += kRT) {
                const int64_t pair0 = (p / (2 * w)) * (2 * w), mid = min(pair0 + w, n), end = min(pair0 + 2 * w, n);
                const uint64_t k = ka[p];
                int64_t pos;
                if (p < mid) {  // left run: right elements < k come first
                    int64_t lo = mid, hi = end;
                    while (lo < hi) {
                        const int64_t m = (lo + hi) >> 1;
                        if (ka[m] < k) lo = m + 1;
                        else hi = m;
                    }
                    pos = pair0 + (p - pair0) + (lo - mid);
                } else {  // right run: left elements <= k come first
                    int64_t lo = pair0, hi = mid;
                    while (lo < hi) {
                        const int64_t m = (lo + hi) >> 1;
                        if (ka[m] <= k) lo = m + 1;
                        else hi = m;
                    }
                    pos = pair0 + (p - mid) + (lo - pair0);
                }
                kb[pos] = k;
                ib[pos] = ia[p];
            }
            __threadfence_block();
            __syncthreads();
            uint64_t* tk = ka;
            ka = kb;
            kb = tk;
            uint32_t* ti = ia;
            ia = ib;
            ib = ti;
        }
        u = reduce_sorted_run(
            r0, n, [&](int64_t p) { return ka[p]; }, [&](int64_t p) { return cnt[in.cls[r0 + (int64_t)ia[p]]]; },
            [&](int64_t p) { return in.ref[r0 + (int64_t)ia[p]]; }, st, lds_w);
    }
    // 5. the run's distinct keys after those of the runs before it
    if (threadIdx.x < 64) {
        const int64_t o = lookback_offset(lb, (int)r, u, (int)threadIdx.x);
        if (threadIdx.x == 0) base_s = o;
    }
    __syncthreads();  // base known; the staged keys visible to the whole block
    const int64_t base = base_s;
    if (r == n_runs - 1 && threadIdx.x == 0) *n_out = base + u;
    for (int64_t p = threadIdx.x; p < u; p += kRT) {
        out.key[base + p] = st.key[r0 + p];
        out.cnt[base + p] = st.cnt[r0 + p];
        out.first[base + p] = st.first[r0 + p];
    }
}

// compact inputs: u32 counts widened on the device
__global__ void widen_counts_kernel(const uint32_t* __restrict__ in, int64_t n, int64_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

int grid_of(int64_t n, int block) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(karma::ceil_div(n, block), 1 << 20));
}

}  // namespace

using namespace karma;

namespace {

// One pass of karma_graph_eq.  cap > 0: the pair scratch is sized speculatively
// (the context's previous pair total) and nothing waits for the pair total;
// *P_out > cap then means the pass must run again with cap = *P_out.  cap = 0:
// one readback of the pair total sizes the scratch.
// Compact host inputs (karma_graph_eq_compact): sizes (member count | size
// token "1" << 7) and u32 counts; n_mem their summed sizes.
struct EqCompact {
    const uint8_t* sizes = nullptr;
    const uint32_t* counts32 = nullptr;
    int64_t n_mem = 0;
};

int graph_eq_run(karma_ctx* ctx, const int64_t* cls_off, const uint32_t* members, const int64_t* counts,
                 const uint8_t* pair_skip, int64_t C, int64_t N, int is_device, int64_t cap, int64_t* P_out,
                 karma_pairs** out, const EqCompact& cq = EqCompact{}) {
    hipStream_t const ms = ctx->stream;
    int64_t* hp = nullptr;  // pinned: [0] pairs, [1] distinct keys, [2] bad member flag, [3] over capacity
    KARMA_TRY(ctx_pinned(ctx, 32, reinterpret_cast<void**>(&hp)));
    const bool compact = cq.sizes != nullptr;
    int64_t n_mem = 0;
    if (compact) {
        n_mem = cq.n_mem;
    } else if (is_device) {
        KARMA_HIP(hipMemcpyAsync(hp, cls_off + C, 8, hipMemcpyDeviceToHost, ms));
        KARMA_HIP(hipStreamSynchronize(ms));
        n_mem = hp[0];
    } else {
        n_mem = cls_off[C];
    }
    KARMA_CHECK(n_mem >= 0, KARMA_ERR_ARG, "karma_graph_eq: negative member count");
    auto* p = new karma_pairs();
    p->ctx = ctx;
    p->n_contigs = N;
    std::unique_ptr<karma_pairs> guard(p);
    KARMA_TRY(p->totals.alloc(ctx, N));
    p->has_totals = true;
    p->has_first = true;
    // one zeroed block: segcnt (N + 1 u32) | counters (n_big, bad)
    const int64_t seg_words = (N + 2) / 2;
    DevArray<int64_t> zero, poff, segoff;
    DevArray<uint32_t> big;
    KARMA_TRY(zero.alloc(ctx, seg_words + 1 + 4));
    KARMA_TRY(poff.alloc(ctx, C + 1));
    KARMA_TRY(segoff.alloc(ctx, N + 1));
    KARMA_TRY(big.alloc(ctx, std::max<int64_t>(C, 1)));
    uint32_t* segcnt = reinterpret_cast<uint32_t*>(zero.ptr);
    int64_t* ctr = zero.ptr + seg_words + 1;
    unsigned* n_big = reinterpret_cast<unsigned*>(ctr);
    int* bad = reinterpret_cast<int*>(ctr + 1);
    // Host inputs go up on the fork stream in the order the kernels need them
    // (class offsets, members, counts) while the main stream computes with
    // what has arrived; the totals run on the fork stream beside the pair
    // pipeline.  Every buffer is the main stream's (allocator), so the fork
    // stream first waits for the main stream's earlier work.
    DevArray<int64_t> d_off, d_cnt;
    DevArray<uint32_t> d_mem, d_c32;
    DevArray<uint8_t> d_skip, d_sz;
    const int64_t* off = cls_off;
    const uint32_t* mem = members;
    const int64_t* cnt = counts;
    const uint8_t* skip = pair_skip;
    hipStream_t xs = ms;
    hipEvent_t* ev = ctx->xfer_ev;
    if (!is_device) {
        KARMA_TRY(ctx_fork(ctx));
        for (int i = 0; i < 4; ++i)
            if (!ev[i]) KARMA_HIP(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
        xs = ctx->fork_use ? ctx->fork_use : ctx->fork_stream;
        KARMA_TRY(d_off.alloc(ctx, C + 1));
        KARMA_TRY(d_cnt.alloc(ctx, std::max<int64_t>(C, 1)));
        KARMA_TRY(d_mem.alloc(ctx, std::max<int64_t>(n_mem, 1)));
        if (pair_skip || compact) KARMA_TRY(d_skip.alloc(ctx, std::max<int64_t>(C, 1)));
        if (compact) {
            KARMA_TRY(d_sz.alloc(ctx, std::max<int64_t>(C, 1)));
            KARMA_TRY(d_c32.alloc(ctx, std::max<int64_t>(C, 1)));
        }
        KARMA_HIP(hipEventRecord(ev[0], ms));
        KARMA_HIP(hipStreamWaitEvent(xs, ev[0], 0));
        KARMA_HIP(hipMemsetAsync(zero.ptr, 0, (seg_words + 1 + 4) * 8, xs));
        if (compact) {  // 1 byte per class instead of 9 (offset + skip)
            if (C) KARMA_HIP(hipMemcpyAsync(d_sz.ptr, cq.sizes, C, hipMemcpyHostToDevice, xs));
        } else {
            KARMA_HIP(hipMemcpyAsync(d_off.ptr, cls_off, (C + 1) * 8, hipMemcpyHostToDevice, xs));
            if (pair_skip && C) KARMA_HIP(hipMemcpyAsync(d_skip.ptr, pair_skip, C, hipMemcpyHostToDevice, xs));
        }
        KARMA_HIP(hipEventRecord(ev[1], xs));
        off = d_off.ptr;
        skip = pair_skip || compact ? d_skip.ptr : nullptr;
        mem = d_mem.ptr;
        cnt = d_cnt.ptr;
        KARMA_HIP(hipStreamWaitEvent(ms, ev[1], 0));
        // the class offsets and skip flags from the sizes, in one scan
        if (compact) KARMA_TRY(scan_excl_sizes(ctx, d_sz.ptr, d_skip.ptr, C, d_off.ptr));
    } else {
        KARMA_HIP(hipMemsetAsync(zero.ptr, 0, (seg_words + 1 + 4) * 8, ms));
    }
    // pair offsets of the classes (first-emission indices), one launch
    KARMA_TRY(scan_excl_pairs(ctx, off, skip, C, poff.ptr));
    KARMA_HIP(hipMemcpyAsync(hp, poff.ptr + C, 8, hipMemcpyDeviceToHost, ms));
    if (!is_device) {
        if (n_mem) KARMA_HIP(hipMemcpyAsync(d_mem.ptr, members, n_mem * 4, hipMemcpyHostToDevice, xs));
        KARMA_HIP(hipEventRecord(ev[2], xs));
    }
    const EqIn in{off, mem, cnt, skip, C, (uint32_t)N, n_mem};
    const int bg = std::max(1, ctx->cu_count);
    // the pair total sizes the scratch: the one readback before the end
    // (none when the previous call's total is taken as the capacity)
    const bool spec = cap > 0;
    if (!spec) {
        KARMA_HIP(hipStreamSynchronize(ms));
        cap = hp[0];
        KARMA_CHECK(cap >= 0 && cap < (int64_t(1) << 32), KARMA_ERR_ARG, "karma_graph_eq: %lld pairs exceed 2^32",
                    (long long)cap);
    }
    const int64_t P = cap;  // scratch entries
    KARMA_TRY(p->keys.alloc(ctx, std::max<int64_t>(P, 1)));
    KARMA_TRY(p->counts.alloc(ctx, std::max<int64_t>(P, 1)));
    KARMA_TRY(p->first.alloc(ctx, std::max<int64_t>(P, 1)));
    const int cg = grid_of(C, kEqT);
    DevArray<uint64_t> pk, ek, sk, sf, gk0, gk1;
    DevArray<uint32_t> pr, pcl, er, ecl, gi0, gi1;
    DevArray<int64_t> sc;
    DevArray<uint64_t> lb;  // n_runs look-back words | ticket | distinct-key total
    const int64_t n_runs = ceil_div(std::max<int64_t>(P, 1), kSeg);
    Placed E{nullptr, nullptr, nullptr};
    if (!is_device) KARMA_HIP(hipStreamWaitEvent(ms, ev[2], 0));  // members
    if (P) {
        KARMA_TRY(pk.alloc(ctx, P));
        KARMA_TRY(pr.alloc(ctx, P));
        KARMA_TRY(pcl.alloc(ctx, P));
        KARMA_TRY(ek.alloc(ctx, P));
        KARMA_TRY(er.alloc(ctx, P));
        KARMA_TRY(ecl.alloc(ctx, P));
        E = Placed{ek.ptr, er.ptr, ecl.ptr};
        KARMA_TRY(sk.alloc(ctx, P));
        KARMA_TRY(sc.alloc(ctx, P));
        KARMA_TRY(sf.alloc(ctx, P));
        KARMA_TRY(gk0.alloc(ctx, P));
        KARMA_TRY(gk1.alloc(ctx, P));
        KARMA_TRY(gi0.alloc(ctx, P));
        KARMA_TRY(gi1.alloc(ctx, P));
        KARMA_TRY(lb.alloc(ctx, n_runs + 2));
        const Pairs3 P3{pk.ptr, pr.ptr, pcl.ptr, P};
        KARMA_LAUNCH(ctx, "eq_rank", eq_rank_kernel, cg, kEqT, 0, in, poff.ptr, segcnt, P3, big.ptr, n_big, bad);
        KARMA_LAUNCH(ctx, "eq_rank", eq_rank_big_kernel, bg, kEqT, 0, in, poff.ptr, segcnt, P3, big.ptr, n_big, bad);
        KARMA_TRY(scan_excl_u32(ctx, segcnt, segoff.ptr, N + 1));
        KARMA_LAUNCH(ctx, "eq_place", eq_place_kernel, grid_of(P, kEqT), kEqT, 0, poff.ptr + C, P3, segoff.ptr, E);
    }
    // the counts go up while the pair kernels run; then the totals beside them
    if (!is_device) {
        if (compact) {
            if (C) {
                KARMA_HIP(hipMemcpyAsync(d_c32.ptr, cq.counts32, C * 4, hipMemcpyHostToDevice, xs));
                ctx->stream = xs;
                KARMA_LAUNCH(ctx, "eq_widen", widen_counts_kernel, grid_of(C, 256), 256, 0, d_c32.ptr, C, d_cnt.ptr);
                ctx->stream = ms;
            }
        } else if (C) {
            KARMA_HIP(hipMemcpyAsync(d_cnt.ptr, counts, C * 8, hipMemcpyHostToDevice, xs));
        }
        KARMA_HIP(hipEventRecord(ev[3], xs));
    }
    {
        ctx->stream = xs;
        if (N) KARMA_HIP(hipMemsetAsync(p->totals.ptr, 0, N * 8, xs));
        if (n_mem || compact)  // (compact: also checks the sizes' sum against n_mem)
            KARMA_LAUNCH(ctx, "eq_totals", eq_totals_kernel, grid_of(n_mem, kEqT), kEqT, 0, in, n_mem,
                         (unsigned long long*)p->totals.ptr, bad);
        ctx->stream = ms;
        if (!is_device) KARMA_HIP(hipEventRecord(ev[0], xs));  // totals done (ev[0] reused)
    }
    if (P) {
        if (!is_device) KARMA_HIP(hipStreamWaitEvent(ms, ev[3], 0));  // counts
        // runs of whole segments; a run over kSegCap (one long segment) sorts in global scratch
        const Entries S{sk.ptr, sc.ptr, sf.ptr}, O{p->keys.ptr, p->counts.ptr, p->first.ptr};
        KARMA_HIP(hipMemsetAsync(lb.ptr, 0, (n_runs + 2) * 8, ms));
        int64_t* n_out = reinterpret_cast<int64_t*>(lb.ptr + n_runs + 1);
        KARMA_LAUNCH(ctx, "seg_reduce", seg_reduce_kernel, n_runs, kRT, 0, segoff.ptr, N, n_runs, E, cnt, S, gk0.ptr,
                     gk1.ptr, gi0.ptr, gi1.ptr, lb.ptr, reinterpret_cast<unsigned*>(lb.ptr + n_runs), O, n_out);
        KARMA_HIP(hipMemcpyAsync(hp + 1, n_out, 8, hipMemcpyDeviceToHost, ms));
    } else {
        hp[1] = 0;
    }
    if (!is_device) KARMA_HIP(hipStreamWaitEvent(ms, ev[0], 0));  // totals
    KARMA_HIP(hipMemcpyAsync(hp + 2, bad, 4, hipMemcpyDeviceToHost, ms));
    KARMA_HIP(hipMemcpyAsync(hp + 3, bad + 1, 4, hipMemcpyDeviceToHost, ms));
    KARMA_HIP(hipStreamSynchronize(ms));
    *P_out = hp[0];
    KARMA_CHECK(hp[0] >= 0 && hp[0] < (int64_t(1) << 32), KARMA_ERR_ARG, "karma_graph_eq: %lld pairs exceed 2^32",
                (long long)hp[0]);
    KARMA_CHECK(!((int)hp[2] & 2), KARMA_ERR_ARG, "eq class offsets / sizes disagree with the member count (%lld)",
                (long long)n_mem);
    KARMA_CHECK(!(int)hp[2], KARMA_ERR_ARG, "eq class member index >= n_contigs");
    if (spec && hp[0] > cap) return KARMA_OK;  // *out untouched: run again, sized
    p->n = hp[1];
    *out = guard.release();
    return KARMA_OK;
}

}  // namespace

// The next call's speculative pair capacity: this call's total + 1/8, not the
// largest ever seen (one large call would otherwise size -- and launch -- every
// later small call's scratch at its size).
static int64_t eq_next_cap(int64_t P) { return P + P / 8; }

extern "C" {

int karma_graph_eq(karma_ctx* ctx, const int64_t* cls_off, const uint32_t* members, const int64_t* counts,
                   const uint8_t* pair_skip, int64_t C, int64_t N, int is_device, karma_pairs** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && cls_off && C >= 0 && N >= 0 && N < (int64_t(1) << 32), KARMA_ERR_ARG,
                "karma_graph_eq: bad arguments");
    // the previous call's pair total (+ 1/8) as the scratch capacity: a
    // stream of similar calls never waits for the pair total
    const int64_t cap = ctx->eq_pair_cap;
    int64_t P = 0;
    *out = nullptr;
    KARMA_TRY(graph_eq_run(ctx, cls_off, members, counts, pair_skip, C, N, is_device, cap, &P, out));
    if (!*out) KARMA_TRY(graph_eq_run(ctx, cls_off, members, counts, pair_skip, C, N, is_device, 0, &P, out));
    ctx->eq_pair_cap = eq_next_cap(P);
    return KARMA_OK;
}

int karma_graph_eq_compact(karma_ctx* ctx, const uint8_t* sizes, const uint32_t* members, int64_t n_members,
                           const uint32_t* counts, int64_t C, int64_t N, karma_pairs** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && (sizes || C == 0) && (counts || C == 0) && (members || n_members == 0) && C >= 0 &&
                    n_members >= 0 && N >= 0 && N < (int64_t(1) << 32),
                KARMA_ERR_ARG, "karma_graph_eq_compact: bad arguments");
    EqCompact cq;
    static const uint8_t none = 0;
    cq.sizes = C ? sizes : &none;
    cq.counts32 = counts;
    cq.n_mem = n_members;  // the sizes' sum is checked on the device (eq_rank)
    const int64_t cap = ctx->eq_pair_cap;
    int64_t P = 0;
    *out = nullptr;
    KARMA_TRY(graph_eq_run(ctx, nullptr, members, nullptr, nullptr, C, N, 0, cap, &P, out, cq));
    if (!*out) KARMA_TRY(graph_eq_run(ctx, nullptr, members, nullptr, nullptr, C, N, 0, 0, &P, out, cq));
    ctx->eq_pair_cap = eq_next_cap(P);
    return KARMA_OK;
}

}  // extern "C"
