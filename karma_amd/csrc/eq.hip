// eq.hip — the eq-class graph (the path karma.py:240 calls,
// /root/reference/karma/read_graph.py:61-148) on hand-written gfx950 kernels:
// per-contig totals (read_graph.py:86-92), every unordered pair of every class
// whose size token is not "1" weighted by the class count (:96-114), summed per
// distinct pair, with the pair's first emission index (the intermediate
// graph's edge order, read_graph.py:120).  No library sort or reduce.
//
// Data are small next to the records path (config 3: 519k classes, 977k
// members, 617k pairs), so the design is about launch count and balance:
//   1. eq_count    one thread per class (a block per class above kSmallM
//                  members): totals (u64 atomics), the class's pair count,
//                  and per contig a the number of pairs whose lower id is a;
//   2. two exclusive scans (single-launch look-back, sort.hip): class pair
//      offsets (first-emission indices) and contig segment offsets;
//   3. eq_scatter  the same walk writes every pair into the segment of its
//                  lower contig: a counting sort by a, no comparisons;
//   4. seg_reduce  a block takes a run of whole segments (<= kSegCap entries,
//                  snapped to segment starts), ranks every entry inside its
//                  segment by (b, position) in LDS, and sums equal (a, b) keys
//                  (counts: i64 adds in key order; first: min).  A run longer
//                  than kSegCap (one contig with > kSeg pairs as lower id) is
//                  sorted in global memory by a block-wide merge sort instead;
//   5. seg_compact every block places its distinct keys after the ones of the
//                  blocks before it (a scan of the per-block counts).
// One host synchronisation reads the pair total (to size the scratch) and one
// the distinct-key total at the end.
#include <memory>

#include "karma_internal.h"

using karma::ceil_div;

namespace {

constexpr int kEqT = 256;      // threads of the per-class kernels
constexpr int64_t kSmallM = 32;  // classes above this size: a block each
constexpr int kRT = 512;         // seg_reduce threads
constexpr int kSeg = 2048;       // target entries per seg_reduce block
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
};

// ---- 1. totals, pair counts, segment sizes ----------------------------------------
__global__ void __launch_bounds__(kEqT) eq_count_kernel(EqIn in, unsigned long long* __restrict__ totals,
                                                        int64_t* __restrict__ pc, uint32_t* __restrict__ segcnt,
                                                        uint32_t* __restrict__ big, unsigned* __restrict__ n_big,
                                                        int* __restrict__ bad) {
    for (int64_t c = (int64_t)blockIdx.x * kEqT + threadIdx.x; c < in.C; c += (int64_t)gridDim.x * kEqT) {
        const int64_t s = in.off[c], e = in.off[c + 1], m = e - s;
        const bool sk = in.skip[c] != 0;
        pc[c] = sk ? 0 : m * (m - 1) / 2;
        if (m > kSmallM) {
            big[atomicAdd(n_big, 1u)] = (uint32_t)c;
            continue;
        }
        const unsigned long long k = (unsigned long long)in.cnt[c];
        for (int64_t t = s; t < e; ++t) {
            const uint32_t x = in.mem[t];
            if (x >= in.N) *bad = 1;
            else atomicAdd(&totals[x], k);  // two's complement: exact for negative counts too
        }
        if (sk) continue;
        for (int64_t i = s; i + 1 < e; ++i) {
            const uint32_t xi = in.mem[i];
            for (int64_t j = i + 1; j < e; ++j) {
                const uint32_t xj = in.mem[j];
                if (max(xi, xj) < in.N) atomicAdd(&segcnt[min(xi, xj)], 1u);
            }
        }
    }
}

__global__ void __launch_bounds__(kEqT) eq_count_big_kernel(EqIn in, unsigned long long* __restrict__ totals,
                                                            uint32_t* __restrict__ segcnt,
                                                            const uint32_t* __restrict__ big,
                                                            const unsigned* __restrict__ n_big, int* __restrict__ bad) {
    const unsigned nb = *n_big;
    for (unsigned q = blockIdx.x; q < nb; q += gridDim.x) {
        const int64_t c = big[q], s = in.off[c], m = in.off[c + 1] - s;
        const unsigned long long k = (unsigned long long)in.cnt[c];
        for (int64_t t = threadIdx.x; t < m; t += kEqT) {
            const uint32_t x = in.mem[s + t];
            if (x >= in.N) *bad = 1;
            else atomicAdd(&totals[x], k);
        }
        if (in.skip[c]) continue;
        const int64_t P = m * (m - 1) / 2;
        for (int64_t t = threadIdx.x; t < P; t += kEqT) {
            int64_t i, j;
            pair_ij(t, m, &i, &j);
            const uint32_t xi = in.mem[s + i], xj = in.mem[s + j];
            if (max(xi, xj) < in.N) atomicAdd(&segcnt[min(xi, xj)], 1u);
        }
    }
}

// ---- 3. counting sort of the pairs by lower contig --------------------------------
struct Entries {
    uint64_t* key;    // a << 32 | b, a <= b
    int64_t* cnt;
    uint64_t* first;  // global emission index (class pair offset + combinations index)
};

__device__ __forceinline__ void put_pair(uint32_t xi, uint32_t xj, int64_t k, uint64_t first,
                                         const int64_t* __restrict__ segoff, uint32_t* __restrict__ cursor,
                                         Entries E) {
    const uint32_t a = min(xi, xj), b = max(xi, xj);
    const int64_t slot = segoff[a] + (int64_t)(atomicSub(&cursor[a], 1u) - 1u);
    E.key[slot] = ((uint64_t)a << 32) | b;
    E.cnt[slot] = k;
    E.first[slot] = first;
}

__global__ void __launch_bounds__(kEqT) eq_scatter_kernel(EqIn in, const int64_t* __restrict__ poff,
                                                          const int64_t* __restrict__ segoff,
                                                          uint32_t* __restrict__ cursor, Entries E) {
    for (int64_t c = (int64_t)blockIdx.x * kEqT + threadIdx.x; c < in.C; c += (int64_t)gridDim.x * kEqT) {
        const int64_t s = in.off[c], e = in.off[c + 1], m = e - s;
        if (m > kSmallM || in.skip[c] || m < 2) continue;
        const int64_t k = in.cnt[c];
        uint64_t f = (uint64_t)poff[c];
        for (int64_t i = s; i + 1 < e; ++i) {
            const uint32_t xi = in.mem[i];
            for (int64_t j = i + 1; j < e; ++j, ++f) put_pair(xi, in.mem[j], k, f, segoff, cursor, E);
        }
    }
}

__global__ void __launch_bounds__(kEqT) eq_scatter_big_kernel(EqIn in, const int64_t* __restrict__ poff,
                                                              const int64_t* __restrict__ segoff,
                                                              uint32_t* __restrict__ cursor, Entries E,
                                                              const uint32_t* __restrict__ big,
                                                              const unsigned* __restrict__ n_big) {
    const unsigned nb = *n_big;
    for (unsigned q = blockIdx.x; q < nb; q += gridDim.x) {
        const int64_t c = big[q], s = in.off[c], m = in.off[c + 1] - s;
        if (in.skip[c]) continue;
        const int64_t k = in.cnt[c], P = m * (m - 1) / 2;
        for (int64_t t = threadIdx.x; t < P; t += kEqT) {
            int64_t i, j;
            pair_ij(t, m, &i, &j);
            put_pair(in.mem[s + i], in.mem[s + j], k, (uint64_t)(poff[c] + t), segoff, cursor, E);
        }
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
// Block r takes the entries [lo(r), lo(r + 1)), lo(r) = the first segment start
// at or after r * kSeg (segments never straddle two blocks).
__device__ __forceinline__ int64_t run_start(const int64_t* __restrict__ segoff, int64_t N, int64_t P, int64_t r) {
    const int64_t target = r * kSeg;
    if (target >= P) return P;
    int64_t lo = 0, hi = N;  // first a with segoff[a] >= target (segoff[N] = P >= target)
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (segoff[mid] >= target) hi = mid;
        else lo = mid + 1;
    }
    return segoff[lo];
}

// Distinct keys of a sorted run, summed: position p of the run holds
// key(p) / the original entry index idx(p).  Writes them to the staging
// arrays at [r0, r0 + u) and returns u (every thread).
template <typename KeyAt, typename IdxAt>
__device__ int64_t reduce_sorted_run(int64_t r0, int64_t n, KeyAt key_at, IdxAt idx_at, Entries in, Entries st,
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
                const int64_t e = idx_at(q);
                sum += in.cnt[e];
                f = min(f, in.first[e]);
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

__global__ void __launch_bounds__(kRT) seg_reduce_kernel(const int64_t* __restrict__ segoff, int64_t N, int64_t P,
                                                         Entries in, Entries st, uint64_t* __restrict__ gk0,
                                                         uint64_t* __restrict__ gk1, uint32_t* __restrict__ gi0,
                                                         uint32_t* __restrict__ gi1,
                                                         int64_t* __restrict__ run_u) {
    __shared__ uint64_t skey[kSegCap];
    __shared__ uint32_t sidx[kSegCap];
    __shared__ uint64_t okey[kSegCap];
    __shared__ uint32_t oidx[kSegCap];
    __shared__ int64_t lds_w[kRT / 64];
    const int64_t r = blockIdx.x;
    const int64_t r0 = run_start(segoff, N, P, r), r1 = run_start(segoff, N, P, r + 1);
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
        u = reduce_sorted_run(
            r0, n, [&](int64_t p) { return okey[p]; }, [&](int64_t p) { return r0 + (int64_t)oidx[p]; }, in, st,
            lds_w);
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
            r0, n, [&](int64_t p) { return ka[p]; }, [&](int64_t p) { return r0 + (int64_t)ia[p]; }, in, st, lds_w);
    }
    if (threadIdx.x == 0) run_u[r] = u;
}

// ---- 5. distinct keys to their final positions ---------------------------------------
__global__ void __launch_bounds__(kRT) seg_compact_kernel(const int64_t* __restrict__ segoff, int64_t N, int64_t P,
                                                          const int64_t* __restrict__ run_base, Entries st,
                                                          Entries out) {
    const int64_t r = blockIdx.x;
    const int64_t r0 = run_start(segoff, N, P, r), base = run_base[r], u = run_base[r + 1] - base;
    for (int64_t p = threadIdx.x; p < u; p += kRT) {
        out.key[base + p] = st.key[r0 + p];
        out.cnt[base + p] = st.cnt[r0 + p];
        out.first[base + p] = st.first[r0 + p];
    }
}

int grid_of(int64_t n, int block) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(karma::ceil_div(n, block), 1 << 20));
}

}  // namespace

namespace karma {

// out[i] = in[0] + ... + in[i - 1] for i < n: the single-launch look-back
// scans of sort.hip
int scan_excl_device(karma_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, DevArray<int64_t>&) {
    return scan_excl_i64(ctx, in, out, n);
}
int scan_excl_device(karma_ctx* ctx, const uint32_t* in, int64_t* out, int64_t n, DevArray<int64_t>&) {
    return scan_excl_u32(ctx, in, out, n);
}


}  // namespace karma

using namespace karma;

extern "C" {

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
    KARMA_CHECK(n_mem >= 0, KARMA_ERR_ARG, "karma_graph_eq: negative member count");
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
    p->has_first = true;

    // one zeroed block: segcnt (N + 1) | counters (n_big, bad)
    const int64_t seg_words = (N + 2) / 2;  // u32 x (N + 1), in 8-byte words
    DevArray<int64_t> zero;
    KARMA_TRY(zero.alloc(ctx, seg_words + 1 + 4));
    KARMA_HIP(hipMemsetAsync(zero.ptr, 0, (seg_words + 1 + 4) * 8, ctx->stream));
    if (N) KARMA_HIP(hipMemsetAsync(p->totals.ptr, 0, N * 8, ctx->stream));
    uint32_t* segcnt = reinterpret_cast<uint32_t*>(zero.ptr);
    int64_t* ctr = zero.ptr + seg_words + 1;
    unsigned* n_big = reinterpret_cast<unsigned*>(ctr);
    int* bad = reinterpret_cast<int*>(ctr + 1);
    DevArray<int64_t> pc, poff, segoff, sums;
    DevArray<uint32_t> big;
    KARMA_TRY(pc.alloc(ctx, C + 1));
    KARMA_TRY(poff.alloc(ctx, C + 1));
    KARMA_TRY(segoff.alloc(ctx, N + 1));
    KARMA_TRY(big.alloc(ctx, C));
    KARMA_HIP(hipMemsetAsync(pc.ptr + C, 0, 8, ctx->stream));
    const EqIn in{d_off.ptr, d_mem.ptr, d_cnt.ptr, d_skip.ptr, C, (uint32_t)N};
    const int cg = grid_of(C, kEqT), bg = std::max(1, ctx->cu_count);
    if (C) {
        KARMA_LAUNCH(ctx, "eq_count", eq_count_kernel, cg, kEqT, 0, in, (unsigned long long*)p->totals.ptr, pc.ptr,
                     segcnt, big.ptr, n_big, bad);
        KARMA_LAUNCH(ctx, "eq_count", eq_count_big_kernel, bg, kEqT, 0, in, (unsigned long long*)p->totals.ptr, segcnt,
                     big.ptr, n_big, bad);
    }
    KARMA_TRY(scan_excl_device(ctx, pc.ptr, poff.ptr, C + 1, sums));
    KARMA_TRY(scan_excl_device(ctx, segcnt, segoff.ptr, N + 1, sums));
    // the pair total sizes the scratch: one readback (with the member check)
    int64_t* hp = nullptr;
    KARMA_TRY(ctx_pinned(ctx, 16, reinterpret_cast<void**>(&hp)));
    KARMA_HIP(hipMemcpyAsync(hp, poff.ptr + C, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipMemcpyAsync(hp + 1, bad, 4, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    const int64_t P = hp[0];
    KARMA_CHECK(!(int)hp[1], KARMA_ERR_ARG, "eq class member index >= n_contigs");
    KARMA_CHECK(P < (int64_t(1) << 32), KARMA_ERR_ARG, "karma_graph_eq: %lld pairs exceed 2^32", (long long)P);
    KARMA_TRY(p->keys.alloc(ctx, P));
    KARMA_TRY(p->counts.alloc(ctx, P));
    KARMA_TRY(p->first.alloc(ctx, P));
    if (P == 0) {
        p->n = 0;
        *out = guard.release();
        return KARMA_OK;
    }
    DevArray<uint64_t> ek, ef, sk, sf, gk0, gk1;
    DevArray<int64_t> ec, sc, run_u;
    DevArray<uint32_t> gi0, gi1;
    KARMA_TRY(ek.alloc(ctx, P));
    KARMA_TRY(ec.alloc(ctx, P));
    KARMA_TRY(ef.alloc(ctx, P));
    KARMA_TRY(sk.alloc(ctx, P));
    KARMA_TRY(sc.alloc(ctx, P));
    KARMA_TRY(sf.alloc(ctx, P));
    const Entries E{ek.ptr, ec.ptr, ef.ptr}, S{sk.ptr, sc.ptr, sf.ptr}, O{p->keys.ptr, p->counts.ptr, p->first.ptr};
    KARMA_LAUNCH(ctx, "eq_scatter", eq_scatter_kernel, cg, kEqT, 0, in, poff.ptr, segoff.ptr, segcnt, E);
    KARMA_LAUNCH(ctx, "eq_scatter", eq_scatter_big_kernel, bg, kEqT, 0, in, poff.ptr, segoff.ptr, segcnt, E, big.ptr,
                 n_big);
    // runs of whole segments; a run over kSegCap (one long segment) sorts in
    // global scratch, which is only allocated when the host-side bound allows it
    const int64_t n_runs = ceil_div(P, kSeg);
    DevArray<int64_t> run_base;
    KARMA_TRY(run_u.alloc(ctx, n_runs + 1));
    KARMA_TRY(run_base.alloc(ctx, n_runs + 1));
    KARMA_HIP(hipMemsetAsync(run_u.ptr + n_runs, 0, 8, ctx->stream));
    KARMA_TRY(gk0.alloc(ctx, P));
    KARMA_TRY(gk1.alloc(ctx, P));
    KARMA_TRY(gi0.alloc(ctx, P));
    KARMA_TRY(gi1.alloc(ctx, P));
    KARMA_LAUNCH(ctx, "seg_reduce", seg_reduce_kernel, n_runs, kRT, 0, segoff.ptr, N, P, E, S, gk0.ptr, gk1.ptr,
                 gi0.ptr, gi1.ptr, run_u.ptr);
    KARMA_TRY(scan_excl_device(ctx, run_u.ptr, run_base.ptr, n_runs + 1, sums));
    KARMA_LAUNCH(ctx, "seg_compact", seg_compact_kernel, n_runs, kRT, 0, segoff.ptr, N, P, run_base.ptr, S, O);
    KARMA_HIP(hipMemcpyAsync(hp, run_base.ptr + n_runs, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    p->n = hp[0];
    *out = guard.release();
    return KARMA_OK;
}

}  // extern "C"
