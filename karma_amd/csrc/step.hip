// step.hip — one rank's step of the sharded build as one native call
// (the work is read_graph.py:19-50 + kmer.py:199-264).
//
// A step is: the records job (classify .. final kernel) on the main stream;
// the presence pass, the column set's exchange (several ranks) and the column
// table on the side stream beside it; the dense profile on the side stream
// beside the graph's tail; the owners' split, the key/count all-to-all-v, the
// owner's merge, the edge stage around the totals all-gather on the main
// stream.  karma_amd/distributed.py drove this sequence from Python (35 HIP
// calls and two host waits per step, ~40 us of Python between them); here it
// is one C ABI call, and a step that needs no host decision waits for nothing.
//
// Two paths:
//   synchronous  every case (several ranks over RCCL, keep = outputs read
//                back, the per-kernel timing pass): the host waits where a
//                size must reach it -- the column count M, the records job's
//                control block, the all-to-all's counts.
//   deferred     (KARMA_STEP_DEFER; one process: one GPU, or one rank's share
//                of an emulated W-rank job) nothing waits: the profile reads M
//                from the column table on the device (launched for the
//                plan's capacity kmer_m_cap), the records job keeps its
//                control block on the device, the tail kernels take their
//                sizes from device memory, and a one-block status kernel
//                copies every word the host would have checked (order and
//                range errors, relabel vote, pair capacity, big reads, bucket
//                overflow, merge order, zero totals) into a ring in mapped host
//                memory.  The host reads entry i at most two steps later (or
//                at karma_step_sync); a step whose words call for the general
//                path is run again synchronously (the same work the
//                synchronous path would have done), an error is returned.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <thread>
#include <vector>

#include "karma_internal.h"

using namespace karma;

namespace {

constexpr int kRing = 64;  // status entries in the mapped slot (64 B each)
constexpr int kLag = 3;    // deferred steps the host may have in flight (two main streams alternate)

// One deferred step's status, written by step_status_kernel (seq last).
struct StepStatus {
    uint64_t seq;
    int64_t slow;   // bits: 1 relabel, 2 pair capacity, 4 big reads, 8 bucket overflow, 16 exchange slots,
                    // 32 another rank's step needs the general path
    int64_t err;    // bits: 1 unsorted records, 2 contig range, 4 partition check, 8 zero total, 16 merge order
    int64_t U;      // pairs of the local list
    int64_t E;      // edges
    int64_t pad[3];
};
static_assert(sizeof(StepStatus) == 64, "status entry");

#ifndef KARMA_EDGE_THREADS
#define KARMA_EDGE_THREADS 512  // with 512-thread final blocks (graph_sets.hip kFT), profiles/r06/measurements.md (r06t)
#endif
constexpr int kET = KARMA_EDGE_THREADS;  // edge-stage tile (elements per block round)
constexpr int kMaxRuns = 64;

// ---- edge stage on device-sized lists ----------------------------------------
// The tile loops take the list length from device memory, so the host
// launches them without knowing it: a fixed grid strides over the tiles.
__device__ __forceinline__ bool is_head(const uint64_t* __restrict__ k, int64_t i, uint64_t key) {
    return i == 0 || k[i - 1] != key;
}
__device__ __forceinline__ int64_t run_sum(const uint64_t* __restrict__ k, const int64_t* __restrict__ c, int64_t n,
                                           int64_t i, uint64_t key) {
    int64_t s = c[i];
    for (int64_t j = i + 1; j < n && k[j] == key; ++j) s += c[j];
    return s;
}

// Tile counts of edges (non-zero off-diagonal keys) and the totals: the
// diagonal group of contig a writes |readset(a)|, every other entry is zeroed
// (contigs between keys by the key after the gap, those before the first and
// after the last key by the grid).  st[0..2] cleared for the write kernel.
__global__ void __launch_bounds__(kET) step_edge_count_kernel(const uint64_t* __restrict__ keys,
                                                              const int64_t* __restrict__ counts,
                                                              const int64_t* __restrict__ n_dev, int64_t n_tot,
                                                              int64_t* __restrict__ totals,
                                                              int64_t* __restrict__ tile_cnt,
                                                              int64_t* __restrict__ st) {
    const int64_t n = *n_dev;
    if (blockIdx.x == 0 && threadIdx.x < 3) st[threadIdx.x] = 0;
    const int64_t stride = (int64_t)gridDim.x * kET, gid = (int64_t)blockIdx.x * kET + threadIdx.x;
    const int64_t a_first = n ? (int64_t)(keys[0] >> 32) : n_tot;
    const int64_t a_last = n ? (int64_t)(keys[n - 1] >> 32) : n_tot;
    for (int64_t c = gid; c < min(a_first, n_tot); c += stride) totals[c] = 0;
    for (int64_t c = a_last + 1 + gid; c < n_tot; c += stride) totals[c] = 0;
    const int64_t tiles = (n + kET - 1) / kET;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t i = t * kET + threadIdx.x;
        bool f = false;
        if (i < n) {
            const uint64_t k = keys[i];
            const uint32_t a = (uint32_t)(k >> 32), b = (uint32_t)k;
            if (i > 0) {
                const uint32_t pa = (uint32_t)(keys[i - 1] >> 32);
                const uint32_t lim = (int64_t)a < n_tot ? a : (uint32_t)n_tot;
                for (uint32_t c = pa + 1; c < lim; ++c) totals[c] = 0;
                if ((int64_t)a < n_tot && pa != a && a != b) totals[a] = 0;
            } else if ((int64_t)a < n_tot && a != b) {
                totals[a] = 0;
            }
            if (is_head(keys, i, k) && (int64_t)b < n_tot) {  // b >= n_tot: reported by the write kernel
                const int64_t s = run_sum(keys, counts, n, i, k);
                if (a == b) totals[a] = s;
                else f = s != 0;
            }
        }
        const int cnt = __syncthreads_count(f);
        if (threadIdx.x == 0) tile_cnt[t] = cnt;
    }
}

// Each tile's edges at the sum of the earlier tiles' counts plus their rank in
// the tile (ballots, then the waves before); w = (s/ta + s/tb)/2 in IEEE
// binary64 without contraction (read_graph.py:39-42).  st[0] zero-total flag,
// st[1] a key past the contig range (no edge), st[2] the edge count (all
// cleared by the count kernel, earlier on the stream).
__global__ void __launch_bounds__(kET) step_edge_write_kernel(
    const uint64_t* __restrict__ keys, const int64_t* __restrict__ counts, const int64_t* __restrict__ n_dev,
    const int64_t* __restrict__ totals, const int64_t* __restrict__ tile_cnt, uint32_t* __restrict__ ea,
    uint32_t* __restrict__ eb, int64_t* __restrict__ es, double* __restrict__ ew, int64_t* __restrict__ st,
    int64_t n_tot) {
    __shared__ int64_t wsum[kET / 64];
    __shared__ int64_t base_s;
    const int64_t n = *n_dev;
    const int64_t tiles = (n + kET - 1) / kET;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (blockIdx.x == 0 && tiles == 0 && threadIdx.x == 0) st[2] = 0;
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        int64_t b = 0;
        for (int64_t j = threadIdx.x; j < t; j += kET) b += tile_cnt[j];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) b += __shfl_xor(b, d, 64);
        if (lane == 0) wsum[wave] = b;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t s = 0;
            for (int w = 0; w < kET / 64; ++w) s += wsum[w];
            base_s = s;
        }
        const int64_t i = t * kET + threadIdx.x;
        uint64_t k = 0;
        int64_t c = 0;
        bool f = false;
        if (i < n) {
            k = keys[i];
            const uint32_t a = (uint32_t)(k >> 32), bb = (uint32_t)k;
            if ((int64_t)bb >= n_tot) {
                st[1] = 1;
            } else if (a != bb && is_head(keys, i, k)) {
                c = run_sum(keys, counts, n, i, k);
                f = c != 0;
            }
        }
        const uint64_t m = __ballot(f);
        __syncthreads();  // base_s is set, wsum free
        if (lane == 0) wsum[wave] = __popcll(m);
        __syncthreads();
        int64_t before = 0, total = 0;
        for (int w = 0; w < kET / 64; ++w) {
            if (w < wave) before += wsum[w];
            total += wsum[w];
        }
        const int64_t base = base_s;
        if (t == tiles - 1 && threadIdx.x == 0) st[2] = base + total;
        if (f) {
            const int64_t o = base + before + __popcll(m & ((1ull << lane) - 1ull));
            const uint32_t a = (uint32_t)(k >> 32), bb = (uint32_t)k;
            const int64_t ta = totals[a], tb = totals[bb];
            ea[o] = a;
            eb[o] = bb;
            es[o] = c;
            if (ta == 0 || tb == 0) {
                st[0] = 1;
                ew[o] = 0.0;
            } else {
                const double x = __ddiv_rn((double)c, (double)ta);
                const double y = __ddiv_rn((double)c, (double)tb);
                ew[o] = __dadd_rn(x, y) * 0.5;
            }
        }
        __syncthreads();  // wsum / base_s reused by the next tile
    }
}

// ---- owner merge of W sorted runs, sizes on the device ---------------------------
// The runs are the owners' slices of one rank's list (an emulated exchange:
// this rank's own W slices stand in for the W received ones), their offsets
// computed in every block from the final kernel's bucket offsets (dst) and
// in-bucket split counts (split_loc), as SetsJob::finish does on the host.
// One kernel: each tile (kMT elements of one run) finds its window in every
// other run with 16-lane groups probing 16 keys per round (a run of 200k keys:
// 5 dependent loads), stages the windows in LDS, and places every element at
// its rank in its own run plus its rank in each other run (stable: equal keys
// of different runs end up adjacent, in run order).
#ifndef KARMA_MARK_ONE
#define KARMA_MARK_ONE 2  // deferred batches on one main stream (SetsJob::launch positions)
#endif
#ifndef KARMA_MARK_TWO
#define KARMA_MARK_TWO 4  // deferred batches alternating two main streams (5, after the final kernel: 8-rank
                          // strong preview 0.196 against 0.188 ms with the binned classify)
#endif
#ifndef KARMA_MARK_ONE_FLAGGED
#define KARMA_MARK_ONE_FLAGGED 2  // ... on flagged records too.  3 (at once, beside classify, which reads half the
                                  // bytes and is VALU-bound) measured 0.849 against 0.860 ms at config 3 (three
                                  // reps each; after classify 0.928, after the final kernel 0.911), but then
                                  // neither kernel's live time is its own (classify 0.65 ms live beside the
                                  // profile): not kept for 1 %, profiles/r06/measurements.md (r06h)
#endif
constexpr int kMarkOne = KARMA_MARK_ONE, kMarkTwo = KARMA_MARK_TWO, kMarkOneFlagged = KARMA_MARK_ONE_FLAGGED;
constexpr int64_t kAltMaxRecords = int64_t(1) << 27;  // batches below this alternate main streams
constexpr int kMT = 1024;       // tile elements (one round of tiles at the 8-rank preview's ~300k keys)
constexpr int kMLds = 8192;     // staged window keys
constexpr int kMFast = 8;       // up to this many runs: every element's searches run in lockstep
constexpr int kMG = 16;         // lanes per bound search
struct RunSrc {
    int nr, B, bw;
    int64_t b[kMaxRuns + 1];     // owner bounds (contig ids)
    int64_t slot = 0;            // > 0: runs are all-to-all slots of this many words (length first)
    int64_t* n_out = nullptr;    // the merged length (device), or null
};

__device__ __forceinline__ int64_t count_below(const uint64_t* __restrict__ a, int64_t lo, int64_t hi, uint64_t k,
                                               bool le) {
    int64_t n = hi - lo, base = lo;
    while (n > 0) {
        const int64_t half = n >> 1;
        const uint64_t m = a[base + half];
        const bool before = le ? m <= k : m < k;
        base = before ? base + half + 1 : base;
        n = before ? n - half - 1 : half;
    }
    return base;
}

__global__ void __launch_bounds__(256) step_merge_kernel(const uint64_t* __restrict__ keys,
                                                         const int64_t* __restrict__ counts,
                                                         const int64_t* __restrict__ dst,
                                                         const int64_t* __restrict__ split_loc, RunSrc rs,
                                                         uint64_t* __restrict__ ko, int64_t* __restrict__ co,
                                                         int64_t* __restrict__ bad) {
    __shared__ int64_t ro[kMaxRuns + 1], re[kMaxRuns + 1], rt[kMaxRuns + 1];
    __shared__ int64_t wlo[kMaxRuns], whi[kMaxRuns];
    __shared__ int wbase[kMaxRuns];
    __shared__ int all_fit;
    __shared__ uint64_t wkeys[kMLds];
    const int nr = rs.nr;
    const int64_t U = rs.slot > 0 ? 0 : dst[rs.B];
    if (rs.slot == 0 && threadIdx.x <= (unsigned)nr) {
        const int64_t bd = rs.b[threadIdx.x];
        const int64_t b = bd >> rs.bw;
        ro[threadIdx.x] = bd <= 0 ? 0 : (b < rs.B ? dst[b] + split_loc[threadIdx.x] : U);
    }
    __syncthreads();
    // run r = [ro[r], re[r]): consecutive slices of one list, or (rs.slot > 0)
    // the padded slots of an all-to-all, the length in the slot's first word
    if (threadIdx.x < (unsigned)nr) {
        const int r = threadIdx.x;
        if (rs.slot > 0) {
            const uint64_t h = keys[(int64_t)r * rs.slot];
            if (h >> 62) {  // a slice outgrew its slot (bit 63) or the sender's step needs the general path (62)
                atomicOr(reinterpret_cast<unsigned long long*>(bad), (h >> 63 ? 2ull : 0ull) | (h >> 62 & 1 ? 4ull : 0ull));
            }
            ro[r] = (int64_t)r * rs.slot + 1;
            re[r] = ro[r] + (int64_t)min<uint64_t>(h & ~(3ull << 62), (uint64_t)(rs.slot - 1));
        } else {
            re[r] = ro[r + 1];
        }
    }
    __syncthreads();
    if (rs.n_out && blockIdx.x == 0 && threadIdx.x == 0) {
        int64_t tot = 0;
        for (int r = 0; r < nr; ++r) tot += re[r] - ro[r];
        *rs.n_out = tot;  // the merged list's length, for the edge stage
    }
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int r = 0; r < nr; ++r) {
            rt[r] = t;
            t += (re[r] - ro[r] + kMT - 1) / kMT;
        }
        rt[nr] = t;
    }
    __syncthreads();
    const int64_t tiles = rt[nr];
    const int lane = threadIdx.x & 63, g = lane & (kMG - 1), grp = threadIdx.x / kMG;
    const unsigned long long gmask = ((1ull << kMG) - 1ull) << (lane & ~(kMG - 1));
    for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        int r = 0;
        while (r + 1 < nr && rt[r + 1] <= tile) ++r;
        const int64_t t0 = ro[r] + (tile - rt[r]) * kMT, t1 = min(re[r], t0 + kMT);
        // window bounds: search q covers run q >> 1, (q & 1) ? last key : first key
        for (int q0 = 0; q0 < 2 * nr; q0 += 256 / kMG) {
            const int q = q0 + grp;
            const int sr = q >> 1;
            const bool search = q < 2 * nr && sr != r;
            int64_t lo = search ? ro[sr] : 0, hi = search ? re[sr] : 0;
            const uint64_t k = search ? keys[(q & 1) ? t1 - 1 : t0] : 0;
            const bool le = sr < r;
            // a run wholly before or after the key needs no search (the
            // emulated exchange's runs are disjoint owner slices)
            if (hi > lo) {
                const uint64_t f = keys[lo], l = keys[hi - 1];
                if (le ? l <= k : l < k) lo = hi;
                else if (le ? f > k : f >= k) hi = lo;
            }
            for (;;) {  // every group of the wave runs the same rounds (ballots are wave-wide)
                const bool more = hi - lo > kMG;
                if (!__ballot(more)) break;
                const int64_t step = (hi - lo + kMG - 1) / kMG;
                const int64_t p = min(hi - 1, lo + (int64_t)(g + 1) * step - 1);
                const bool before = more && (le ? keys[p] <= k : keys[p] < k);
                const int c = __popcll(__ballot(before) & gmask);
                if (more) {
                    const int64_t nlo = c ? min(hi, lo + (int64_t)c * step) : lo;
                    const int64_t nhi = c < kMG ? min(hi, lo + (int64_t)(c + 1) * step - 1) : hi;
                    lo = nlo;
                    hi = nhi;
                }
            }
            const int64_t p = lo + g;
            const bool before = p < hi && (le ? keys[p] <= k : keys[p] < k);
            const int64_t ans = lo + __popcll(__ballot(before) & gmask);
            if (search && g == 0) {
                if (q & 1) whi[sr] = ans;
                else wlo[sr] = ans;
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int used = 0, fit = 1;
            for (int sr = 0; sr < nr; ++sr) {
                if (sr == r) continue;
                if (whi[sr] < wlo[sr]) whi[sr] = wlo[sr];
                const int64_t len = whi[sr] - wlo[sr];
                if (used + len <= kMLds) {
                    wbase[sr] = used;
                    used += (int)len;
                } else {
                    wbase[sr] = -1;
                    fit = 0;
                }
            }
            all_fit = fit && nr <= kMFast;
        }
        __syncthreads();
        for (int sr = 0; sr < nr; ++sr) {
            if (sr == r || wbase[sr] < 0) continue;
            const int64_t lo = wlo[sr];
            const int len = (int)(whi[sr] - lo);
            for (int i = threadIdx.x; i < len; i += blockDim.x) wkeys[wbase[sr] + i] = keys[lo + i];
        }
        __syncthreads();
        if (all_fit) {
            // every window staged, <= kMFast runs: the element's binary
            // searches of all runs advance together (independent LDS loads in
            // flight instead of one dependent chain per run)
            int b[kMFast], n[kMFast], maxn = 0;
            int64_t adj = 0;
#pragma unroll
            for (int sr = 0; sr < kMFast; ++sr) {
                const bool on = sr < nr && sr != r;
                b[sr] = on ? wbase[sr] : 0;
                n[sr] = on ? (int)(whi[sr] - wlo[sr]) : 0;
                maxn = max(maxn, n[sr]);
                if (on) adj += wlo[sr] - wbase[sr] - ro[sr];
            }
            const int nit = 32 - __clz(maxn);  // halving steps until every window is empty
            // the tile's loads first (kMT / 256 elements per thread, all in flight)
            constexpr int kPer = kMT / 256;
            uint64_t kv[kPer], kp[kPer];
            int64_t cv[kPer];
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int64_t i = t0 + threadIdx.x + (int64_t)u * 256;
                const bool ok = i < t1;
                kv[u] = ok ? keys[i] : 0;
                kp[u] = ok && i > ro[r] ? keys[i - 1] : 0;
                cv[u] = ok ? counts[i] : 0;
            }
#pragma unroll
            for (int u = 0; u < kPer; ++u) {
                const int64_t i = t0 + threadIdx.x + (int64_t)u * 256;
                if (i >= t1) break;
                const uint64_t k = kv[u];
                if (kp[u] > k) atomicOr(reinterpret_cast<unsigned long long*>(bad), 1ull);
                int bb[kMFast], nn[kMFast];
#pragma unroll
                for (int sr = 0; sr < kMFast; ++sr) {
                    bb[sr] = b[sr];
                    nn[sr] = n[sr];
                }
                for (int it = 0; it < nit; ++it) {
#pragma unroll
                    for (int sr = 0; sr < kMFast; ++sr) {
                        const int half = nn[sr] >> 1;
                        const uint64_t m = wkeys[min(bb[sr] + half, kMLds - 1)];
                        const bool before = nn[sr] > 0 && (sr < r ? m <= k : m < k);
                        bb[sr] = before ? bb[sr] + half + 1 : bb[sr];
                        nn[sr] = before ? nn[sr] - half - 1 : half;
                    }
                }
                int64_t pos = i - ro[r] + adj;
#pragma unroll
                for (int sr = 0; sr < kMFast; ++sr) pos += bb[sr];
                ko[pos] = k;
                co[pos] = cv[u];
            }
            __syncthreads();  // the windows are rebuilt for the next tile
            continue;
        }
        for (int64_t i = t0 + threadIdx.x; i < t1; i += blockDim.x) {
            const uint64_t k = keys[i];
            if (i > ro[r] && keys[i - 1] > k) atomicOr(reinterpret_cast<unsigned long long*>(bad), 1ull);
            int64_t pos = i - ro[r];
            for (int sr = 0; sr < nr; ++sr) {
                if (sr == r) continue;
                const int64_t lo = wlo[sr], hi = whi[sr];
                int64_t cnt;
                if (wbase[sr] >= 0) {
                    const uint64_t* w = wkeys + wbase[sr] - lo;
                    cnt = count_below(w, lo, hi, k, sr < r);
                } else {
                    cnt = count_below(keys, lo, hi, k, sr < r);
                }
                pos += cnt - ro[sr];
            }
            ko[pos] = k;
            co[pos] = counts[i];
        }
        __syncthreads();  // the windows are rebuilt for the next tile
    }
}

// ---- the exchange's send slots, sized on the device ----------------------------
// Owner r's slice of this rank's list (offsets from the final kernel's bucket
// offsets and split counts, as in step_merge_kernel) into slot r of a padded
// all-to-all: word 0 the length, bit 63 set in every slot when any slice
// outgrew its slot (so every receiver sees the same flag and every rank runs
// the step again), then up to slot - 1 keys (counts in the same layout).
__global__ void __launch_bounds__(256) step_pack_kernel(const uint64_t* __restrict__ keys,
                                                        const int64_t* __restrict__ counts,
                                                        const int64_t* __restrict__ dst,
                                                        const int64_t* __restrict__ split_loc, RunSrc rs, int64_t slot,
                                                        uint64_t* __restrict__ sk, int64_t* __restrict__ sc,
                                                        const int* __restrict__ flags,
                                                        const unsigned* __restrict__ counters,
                                                        const uint8_t* __restrict__ ovf) {
    __shared__ int64_t ro[kMaxRuns + 1];
    __shared__ int over, slow;
    const int nr = rs.nr;
    const int64_t U = dst[rs.B];
    if (threadIdx.x <= (unsigned)nr) {
        const int64_t bd = rs.b[threadIdx.x];
        const int64_t b = bd >> rs.bw;
        ro[threadIdx.x] = bd <= 0 ? 0 : (b < rs.B ? dst[b] + split_loc[threadIdx.x] : U);
    }
    if (threadIdx.x == 0) {
        over = 0;
        slow = counters[3] || flags[2] || counters[0];  // the status kernel's slow words, less the slots
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)nr && ro[threadIdx.x + 1] - ro[threadIdx.x] > slot - 1) over = 1;
    if (blockIdx.x == 0)
        for (int b = threadIdx.x; b < rs.B; b += blockDim.x)
            if (ovf[b]) slow = 1;
    __syncthreads();
    // the slot's first word: the slice length; bit 63: some slice of this
    // sender outgrew its slot; bit 62: this sender's step needs the general
    // path.  Every rank receives every sender's word, so every rank learns
    // that the step runs again (no separate all-reduce of the verdict).
    if (blockIdx.x == 0 && threadIdx.x < (unsigned)nr) {
        const int r = threadIdx.x;
        sk[(int64_t)r * slot] = (uint64_t)(ro[r + 1] - ro[r]) | ((uint64_t)over << 63) | ((uint64_t)slow << 62);
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < U; i += (int64_t)gridDim.x * 256) {
        int r = 0;
        while (r + 1 < nr && ro[r + 1] <= i) ++r;
        const int64_t j = i - ro[r];
        if (j < slot - 1) {
            sk[(int64_t)r * slot + 1 + j] = keys[i];
            sc[(int64_t)r * slot + 1 + j] = counts[i];
        }
    }
}

// Every word a host would have checked after a deferred step, into the ring
// entry (seq written last, released to the host).  With several processes the
// merge's word carries the other ranks' verdicts (step_pack_kernel), so every
// rank's entry asks for the same re-runs and the collectives stay matched.
// ctrl (n_ctrl words): the records job's control block when it was the
// step's own (SetsDeferred::ctrl): zeroed once every word is read, for the
// next records job of this tail (no clearing launch ahead of its classify).
// flags, counters, ovf and dst point into ctrl then, so none of the four (nor
// ctrl) is __restrict__; every read of them is staged into LDS (any_ovf,
// words[]) ahead of the __syncthreads that precedes the clear, and must stay so.
__global__ void step_status_kernel(const int* flags, const unsigned* counters, const uint8_t* ovf, int B,
                                   const int64_t* dst, int64_t* __restrict__ merge_bad,
                                   const int64_t* __restrict__ est, StepStatus* __restrict__ out, uint64_t seq,
                                   int64_t* ctrl, int64_t n_ctrl) {
    __shared__ int any_ovf;
    __shared__ int64_t words[4];
    if (threadIdx.x == 0) any_ovf = 0;
    __syncthreads();
    for (int b = threadIdx.x; b < B; b += blockDim.x)
        if (ovf[b]) any_ovf = 1;
    if (threadIdx.x == 0) {
        words[0] = (int64_t)flags[0] | (int64_t)flags[1] << 8 | (int64_t)flags[2] << 16 | (int64_t)flags[3] << 24;
        words[1] = (int64_t)(counters[0] != 0) | (int64_t)(counters[3] != 0) << 1;
        words[2] = dst[B];
    }
    __syncthreads();
    if (ctrl)
        for (int64_t i = threadIdx.x; i < n_ctrl; i += blockDim.x) ctrl[i] = 0;
    if (threadIdx.x != 0) return;
    const int fw = (int)words[0];
    const int f0 = fw & 255, f1 = (fw >> 8) & 255, f2 = (fw >> 16) & 255, f3 = (fw >> 24) & 255;
    const bool c0 = words[1] & 1, c3 = (words[1] >> 1) & 1;
    int64_t slow = 0, err = 0;
    if (c3) slow |= 1;
    if (f2) slow |= 2;
    if (c0) slow |= 4;
    if (any_ovf) slow |= 8;
    if (f0) err |= 1;
    if (f1) err |= 2;
    if (f3) err |= 4;
    if (est[0]) err |= 8;
    if (est[1]) err |= 2;  // a key past the contig range
    if (merge_bad) {
        if (*merge_bad & 1) err |= 16;
        if (*merge_bad & 2) slow |= 16;  // the exchange's slots were too small
        if (*merge_bad & 4) slow |= 32;  // another rank's step needs the general path
        *merge_bad = 0;  // cleared for the next step's merge (stream order)
    }
    out->slow = slow;
    out->err = err;
    out->U = words[2];
    out->E = est[2];
    __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

struct karma_step {
    karma_ctx* ctx = nullptr;
    karma_comm* comm = nullptr;   // main-stream communicator (NULL: one process)
    karma_comm* scomm = nullptr;  // side-stream communicator (column set exchange)
    int kmode = 0, world = 1, rank = 0, nranks = 1, emulate = 0;
    int64_t n_glob = 0, c_lo = 0, n_loc = 0;
    std::vector<int64_t> bounds;  // owner bounds: nranks + 1 contig ids
    bool exchange = false;        // a split / merge happens (world > 1 or emulation)
    hipStream_t main_s = nullptr, side_s = nullptr;
    // deferred steps alternate between main_s and alt_s: nothing ties step
    // i + 1's records job to step i's tail, so the next batch's classify runs
    // beside this batch's merge and edge stage (a stream of batches)
    hipStream_t alt_s = nullptr;
    // with two main streams, the odd batches' presence, column table and
    // profile go to side_alt_s (one side stream made every batch's column
    // table wait for the previous batch's profile); the general-read branch
    // then stays on the main stream, so no two busy streams share one of the
    // process's 4 hardware queues
    hipStream_t side_alt_s = nullptr;
    int sides = 2;                // KARMA_STEP_SIDES=1: one side stream (A/B)
    int streams = 0;              // KARMA_STEP_STREAMS: 1 / 2 main streams (0: by the batch's size)
    hipEvent_t ev = nullptr;      // side -> main join: the last deferred step's profile (one main stream)
    bool ev_set = false;
    bool join = false;            // KARMA_STEP_JOIN=1: join (A/B; measured slower, see run_deferred)
    // the profile (persistent; rows of n_loc x M, dense)
    DevArray<double> prof;
    // outputs of the last synchronous step
    karma_kmer_plan* plan = nullptr;
    karma_pairs* local = nullptr;
    karma_pairs* merged = nullptr;
    karma_edges* edges = nullptr;
    int64_t M = -1, E = -1, pairs_local = -1, entries = -1;
    // deferred steps
    struct Pending {
        uint64_t seq;
        karma_contigs* store;
        const uint32_t* rec;
        int64_t A;
        bool flg;  // KARMA_STEP_FLAGGED records
    };
    std::deque<Pending> pending;
    uint64_t seq = 0;
    StepStatus* ring_h = nullptr;  // mapped host memory (ring_mem): per step its status words ...
    StepStatus* ring_d = nullptr;
    int64_t* mring_h = nullptr;    // ... and its column count, written by its column table
    int64_t* mring_d = nullptr;
    int sticky_sync = 0;           // deferred steps to run synchronously after a slow one
    // deferred steps' device buffers, one set per main stream (kept across
    // steps: identical shapes reuse them)
    DevArray<int64_t> m_ring;      // per ring entry: the step's column count, written by its column table
    // per side stream: the k-mer plan's presence bitmap block, zero between
    // plans (ctx->plan_zeroed; the column table kernel clears it after use)
    DevArray<uint32_t> plan_zero[2];
    struct Tail {
        DevArray<double> prof;         // the step's profile
        DevArray<uint64_t> mk, sk, rk;  // merged keys; the exchange's send and receive slots
        DevArray<int64_t> mc, mbad, tot, tile_cnt, est, sc, rc, nm;
        DevArray<uint32_t> ea, eb;
        DevArray<int64_t> es;
        DevArray<double> ew;
        DevArray<int64_t> ctrl;        // the records job's control block, kept zero by the status kernel
        void release() {
            ctrl.release();
            prof.release();
            sk.release();
            rk.release();
            sc.release();
            rc.release();
            nm.release();
            mk.release();
            mc.release();
            mbad.release();
            tot.release();
            tile_cnt.release();
            est.release();
            ea.release();
            eb.release();
            es.release();
            ew.release();
        }
    } tail[2];
    uint64_t prof_seq = 0;         // the deferred step whose profile is the newest (0: a synchronous one)
    int prof_par = 0;              // its buffer: tail[prof_par].prof
    int64_t prof_M = -1;           // M of the profile in `prof` (-1: not known yet)
    // status words of synchronous steps whose edge count was not read
    // (count = false): copied out in stream order, checked when their event
    // has passed (or at karma_step_sync)
    int64_t* graves_h = nullptr;  // pinned, kRing x 4 words
    hipEvent_t grave_ev[kRing] = {};
    std::deque<int> graves;
    int grave_next = 0;
    // counters
    int64_t n_sync = 0, n_deferred = 0, n_redone = 0;
    // host time inside karma_step_run, and the part spent waiting for the
    // device (a deferred step's status kLag steps back, synchronous readbacks
    // excluded)
    int64_t run_ns = 0, wait_ns = 0;
    // several processes: deferred steps once every rank's store is known to
    // be ACGT-only (no exception k-mers to exchange) and the exchange's slot
    // size is known from a synchronous step (the largest slice + 25 %)
    karma_contigs* acgt_store = nullptr;
    int64_t kc = 0;
    bool defer_ranks = true;      // KARMA_STEP_DEFER_RANKS=0: synchronous steps with several processes
    // several processes, two main streams: every deferred step's exchange and
    // edge stage (all of the main communicator's operations) on one exchange
    // stream, side_alt_s (idle then: the column exchange keeps to side_s), so
    // batch i + 1's records job runs beside batch i's collectives.  Events
    // hand the records job's lists to it (ev_rec), return them before the
    // same main stream's next records job reuses them (ev_tail[par]), and
    // order the communicator's operations across the exchange stream and the
    // synchronous steps' main stream (ev_tail, ev_sync).
    bool xstream = true;          // KARMA_STEP_XSTREAM=0: one main stream with several processes
    hipEvent_t ev_rec = nullptr, ev_sync = nullptr, ev_tail[2] = {};
    bool tail_set[2] = {}, sync_set = false;
    int tail_last = -1;
    // One communicator (no distinct side communicator passed, the default):
    // every collective of a step -- the presence all-gather included -- is
    // issued on ONE stream in the same order on every rank: the exchange
    // stream for deferred steps, and a synchronous step's side-stream column
    // exchange only after every earlier collective has completed.  No two
    // collectives are ever in flight at once, the usage RCCL guarantees to be
    // deadlock-free.  With a distinct side communicator (KARMA_STEP_SIDE_COMM=1
    // in karma_amd/comm.py) the presence all-gather runs on the side stream
    // beside the main communicator's operations (round 4's mode).
    bool one_comm = true;
    hipEvent_t ev_pres = nullptr, ev_pres2 = nullptr, ev_pre = nullptr;
    // deferred steps by mode (karma_step_info): two main streams, tail on the exchange stream
    int64_t n_two = 0, n_xs = 0, n_own = 0;  // ... and records jobs on the step's own control block
    int stall_s = 120;             // KARMA_STEP_STALL_S: a deferred status this late is KARMA_ERR_STALL
    // deferred records jobs use this step's own control blocks (tail[par].ctrl),
    // kept zero by the status kernel: no probe / clearing launch at their head,
    // the relabel decided in classify (KARMA_STEP_OWN_CTRL=0: the job's own
    // block and the probe kernel)
    bool own_ctrl = true;
    bool emu_xs = false;  // KARMA_STEP_EMU_XS=1 (A/B; see run_deferred)
    int lag = kLag;      // KARMA_STEP_LAG (A/B): deferred steps in flight before the host waits
    void* ring_mem = nullptr;      // this step's own mapped status ring (two steps on one context never share it)
    uint64_t fault_seq = 0;        // KARMA_STEP_FAULT_SEQ (tests only): this deferred step fails before its status
};

namespace {

// The profile buffer grows only with both streams idle: the side stream may
// still be writing the old one, and the allocator would hand it to a
// main-stream allocation (it was allocated there) at once.
int ensure_prof(karma_step* s, DevArray<double>& prof, size_t n) {
    if (prof.n >= n) return KARMA_OK;
    KARMA_HIP(hipStreamSynchronize(s->side_s));
    KARMA_HIP(hipStreamSynchronize(s->side_alt_s));
    KARMA_HIP(hipStreamSynchronize(s->main_s));
    KARMA_HIP(hipStreamSynchronize(s->alt_s));
    return prof.alloc(s->ctx, n);
}
template <typename T>
int ensure_arr(karma_ctx* ctx, DevArray<T>& a, size_t n) {
    return a.n >= n ? KARMA_OK : a.alloc(ctx, n);
}

// The status words of a grave whose copy has landed: errors are returned.
int check_grave(karma_step* s, int slot) {
    const int64_t* w = s->graves_h + 4 * slot;
    KARMA_CHECK(!w[2], KARMA_ERR_UNSORTED, "karma_pairs_merge_runs: a run is not sorted by key");
    KARMA_CHECK(!(int)w[0], KARMA_ERR_ZERO_DIV, "division by zero: a shared count over a zero total");
    return KARMA_OK;
}

int bury(karma_step* s, bool wait) {
    while (!s->graves.empty()) {
        const int slot = s->graves.front();
        if (wait) {
            KARMA_HIP(hipEventSynchronize(s->grave_ev[slot]));
        } else if (hipEventQuery(s->grave_ev[slot]) != hipSuccess) {
            break;
        }
        s->graves.pop_front();
        KARMA_TRY(check_grave(s, slot));
    }
    return KARMA_OK;
}

int drop_outputs(karma_step* s) {
    if (s->edges && s->E < 0) {
        if (const int64_t* st = edges_take_pending(s->edges)) {
            if ((int)s->graves.size() >= kRing) KARMA_TRY(bury(s, true));
            const int slot = s->grave_next;
            s->grave_next = (slot + 1) % kRing;
            if (!s->grave_ev[slot]) KARMA_HIP(hipEventCreateWithFlags(&s->grave_ev[slot], hipEventDisableTiming));
            KARMA_HIP(hipMemcpyAsync(s->graves_h + 4 * slot, st, 24, hipMemcpyDeviceToHost, s->main_s));
            KARMA_HIP(hipEventRecord(s->grave_ev[slot], s->main_s));
            s->graves.push_back(slot);
        }
    }
    if (s->edges) karma_edges_destroy(s->edges);
    if (s->merged) karma_pairs_destroy(s->merged);
    if (s->local) karma_pairs_destroy(s->local);
    if (s->plan) karma_kmer_plan_destroy(s->plan);
    s->edges = nullptr;
    s->merged = s->local = nullptr;
    s->plan = nullptr;
    s->M = s->E = s->pairs_local = s->entries = -1;
    return bury(s, false);
}

// The column set's exchange (kmer.py:146-179 is a global sorted union): OR of
// every rank's presence bitmap, union of every rank's exception keys.  On the
// side communicator, issued in the same order on every rank.
int exchange_columns(karma_step* s, karma_kmer_plan* plan, karma_comm* c) {
    karma_ctx* ctx = s->ctx;
    const int W = s->world;
    int64_t nw = 0;
    KARMA_TRY(karma_kmer_presence_words(plan, &nw));
    DevArray<uint32_t> words, all;
    KARMA_TRY(words.alloc(ctx, nw));
    KARMA_TRY(all.alloc(ctx, nw * W));
    KARMA_TRY(karma_kmer_presence_get(plan, words.ptr));
    KARMA_TRY(karma_comm_allgather(c, words.ptr, all.ptr, nw * 4));
    KARMA_TRY(karma_kmer_presence_merge(plan, all.ptr, W));
    // exception keys: sizes, then one padded all-gather
    int64_t ne = 0;
    KARMA_TRY(karma_kmer_exceptions_count(plan, &ne));
    std::vector<int64_t> sizes(W, 0);
    sizes[s->rank] = ne;
    KARMA_TRY(karma_comm_allreduce_host(c, sizes.data(), W, KARMA_DT_I64, KARMA_OP_SUM));
    int64_t mx = 1, tot = 0;
    for (int64_t x : sizes) {
        mx = std::max(mx, x);
        tot += x;
    }
    if (tot == 0) return karma_kmer_exceptions_set(plan, nullptr, 0);
    DevArray<uint64_t> send, gath, keys;
    KARMA_TRY(send.alloc(ctx, mx));
    KARMA_TRY(gath.alloc(ctx, mx * W));
    KARMA_TRY(keys.alloc(ctx, tot));
    if (ne) KARMA_TRY(karma_kmer_exceptions_get(plan, send.ptr));
    KARMA_TRY(karma_comm_allgather(c, send.ptr, gath.ptr, mx * 8));
    int64_t off = 0;
    for (int r = 0; r < W; ++r) {
        if (sizes[r])
            KARMA_HIP(hipMemcpyAsync(keys.ptr + off, gath.ptr + r * mx, sizes[r] * 8, hipMemcpyDeviceToDevice,
                                     ctx->stream));
        off += sizes[r];
    }
    return karma_kmer_exceptions_set(plan, keys.ptr, tot);  // sorts and dedups (stream-ordered)
}

// The presence bitmaps alone (a deferred step: every rank's store is ACGT-only,
// so there are no exception keys to exchange).
int exchange_presence(karma_step* s, karma_kmer_plan* plan, karma_comm* c) {
    karma_ctx* ctx = s->ctx;
    int64_t nw = 0;
    KARMA_TRY(karma_kmer_presence_words(plan, &nw));
    DevArray<uint32_t> words, all;
    KARMA_TRY(words.alloc(ctx, nw));
    KARMA_TRY(all.alloc(ctx, nw * s->world));
    KARMA_TRY(karma_kmer_presence_get(plan, words.ptr));
    KARMA_TRY(karma_comm_allgather(c, words.ptr, all.ptr, nw * 4));
    return karma_kmer_presence_merge(plan, all.ptr, s->world);  // stream-ordered: words / all back to the cache
}

// The owners' readset totals, gathered from every owner's slice (in place for
// equal shards; otherwise a padded all-gather and copies back).
int allgather_slices(karma_step* s, int64_t* buf) {
    karma_ctx* ctx = s->ctx;
    const int W = s->world;
    const std::vector<int64_t>& b = s->bounds;
    int64_t mx = 0;
    bool equal = b[0] == 0;
    for (int r = 0; r < W; ++r) {
        mx = std::max(mx, b[r + 1] - b[r]);
        equal = equal && (b[r + 1] - b[r]) == (b[1] - b[0]);
    }
    if (equal && mx > 0) return karma_comm_allgather(s->comm, buf + s->rank * mx, buf, mx * 8);
    mx = std::max<int64_t>(mx, 1);
    DevArray<int64_t> send, all;
    KARMA_TRY(send.alloc(ctx, mx));
    KARMA_TRY(all.alloc(ctx, mx * W));
    const int64_t mine = b[s->rank + 1] - b[s->rank];
    if (mine)
        KARMA_HIP(hipMemcpyAsync(send.ptr, buf + b[s->rank], mine * 8, hipMemcpyDeviceToDevice, ctx->stream));
    KARMA_TRY(karma_comm_allgather(s->comm, send.ptr, all.ptr, mx * 8));
    for (int r = 0; r < W; ++r) {
        const int64_t n = b[r + 1] - b[r];
        if (r != s->rank && n)
            KARMA_HIP(hipMemcpyAsync(buf + b[r], all.ptr + r * mx, n * 8, hipMemcpyDeviceToDevice, ctx->stream));
    }
    return KARMA_OK;
}

// stream `w` waits for everything recorded so far on stream `on` (one event
// per purpose, created on first use)
int stream_after(hipEvent_t* ev, hipStream_t on, hipStream_t w) {
    if (!*ev) KARMA_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    if (counted_call("hipEventRecord")) ++t_hip_calls;
    KARMA_HIP(hipEventRecord(*ev, on));
    if (counted_call("hipStreamWaitEvent")) ++t_hip_calls;
    KARMA_HIP(hipStreamWaitEvent(w, *ev, 0));
    return KARMA_OK;
}

// ---- the synchronous step ------------------------------------------------------
int run_sync(karma_step* s, karma_contigs* store, const uint32_t* rec, int64_t A, bool flg, bool keep,
             bool sequential, bool count) {
    const int rfmt = flg ? KARMA_REC_FLAGGED : KARMA_REC_SORTED;
    karma_ctx* ctx = s->ctx;
    KARMA_TRY(drop_outputs(s));
    ++s->n_sync;
    if (s->tail_last >= 0) {
        // deferred steps' exchanges may still be queued on the exchange stream
        // (a re-run checked 3 steps back): the main stream's collectives and
        // the records job's reuse of their lists come after them
        if (counted_call("hipStreamWaitEvent")) ++t_hip_calls;
        KARMA_HIP(hipStreamWaitEvent(s->main_s, s->ev_tail[s->tail_last], 0));
    }
    if (s->world > 1 && s->one_comm && !sequential) {
        // the column exchange below (side stream, the one communicator) after
        // every collective issued so far: the main stream's (an earlier
        // synchronous step's totals all-gather) and, through the wait above,
        // the exchange stream's
        KARMA_TRY(stream_after(&s->ev_pre, s->main_s, s->side_s));
    }
    if (s->exchange) KARMA_TRY(karma_graph_split_hint(ctx, s->bounds.data(), s->nranks));
    int64_t M = 0;
    if (!sequential) {
        // the graph's kernels first on the main stream; the presence pass, the
        // column set's exchange and the column table beside them on the side
        // stream; the profile behind the graph's kernels on the side stream
        karma_graph_job* job = nullptr;
        ctx->fork_use = s->alt_s;  // the general-read branch on the spare main stream (see karma_ctx::fork_use)
        const int brc = karma_graph_records_begin(ctx, rec, A, s->n_glob, rfmt, 1, &job);
        ctx->fork_use = nullptr;
        KARMA_TRY(brc);
        int rc = KARMA_OK;
        ctx->stream = s->side_s;
        rc = karma_kmer_plan_create(ctx, store, s->kmode, &s->plan);
        if (!rc && s->world > 1 && s->acgt_store != store) {
            // may later steps skip the exception keys' exchange?  (every rank agrees)
            int64_t exc = 0;
            rc = karma_contigs_info(store, nullptr, nullptr, &exc, nullptr);
            if (!rc) rc = karma_comm_allreduce_host(s->scomm ? s->scomm : s->comm, &exc, 1, KARMA_DT_I64, KARMA_OP_SUM);
            if (!rc) s->acgt_store = exc == 0 ? store : nullptr;
        }
        if (!rc && s->world > 1) rc = exchange_columns(s, s->plan, s->scomm ? s->scomm : s->comm);
        if (!rc) rc = karma_kmer_plan_finalize_async(s->plan);
        ctx->stream = s->main_s;
        if (!rc) rc = karma_kmer_plan_finalize_wait(s->plan, &M);
        if (!rc) rc = ensure_prof(s, s->prof, (size_t)std::max<int64_t>(1, s->n_loc * M));
        if (!rc && s->n_loc * M) rc = karma_kmer_profile_side(s->plan, s->prof.ptr, M, s->side_s);
        const int rc2 = karma_graph_records_end(job, &s->local);  // consumes the job on every path
        KARMA_TRY(rc);
        KARMA_TRY(rc2);
    } else {
        // everything on the main stream (every kernel alone on the chip)
        KARMA_TRY(karma_kmer_plan_create(ctx, store, s->kmode, &s->plan));
        if (s->world > 1) KARMA_TRY(exchange_columns(s, s->plan, s->comm));
        KARMA_TRY(karma_kmer_plan_finalize(s->plan, &M));
        KARMA_TRY(ensure_prof(s, s->prof, (size_t)std::max<int64_t>(1, s->n_loc * M)));
        if (s->n_loc * M) KARMA_TRY(karma_kmer_profile(s->plan, s->prof.ptr, M, 1));
        KARMA_TRY(karma_graph_records(ctx, rec, A, s->n_glob, rfmt, 1, &s->local));
    }
    s->M = M;
    s->prof_M = M;
    s->prof_seq = 0;
    if (keep) {
        KARMA_TRY(karma_pairs_count(s->local, &s->pairs_local));
        std::vector<int64_t> c(std::max<int64_t>(1, s->pairs_local));
        KARMA_TRY(karma_pairs_get(s->local, nullptr, c.data(), nullptr, 0));
        int64_t t = 0;
        for (int64_t i = 0; i < s->pairs_local; ++i) t += c[i];
        s->entries = t;
    }
    int64_t E = -1;
    if (s->exchange) {
        std::vector<int64_t> starts(s->nranks + 1);
        KARMA_TRY(karma_pairs_split(s->local, s->bounds.data(), s->nranks, starts.data()));
        const uint64_t* k = nullptr;
        const int64_t* c = nullptr;
        KARMA_TRY(karma_pairs_device(s->local, &k, &c));
        if (s->world > 1) {
            // each owner's slice of the keys and of the counts, one grouped all-to-all-v
            const int W = s->world;
            std::vector<int64_t> sc(W), rcv(W), so(W + 1, 0), ro(W + 1, 0);
            for (int r = 0; r < W; ++r) sc[r] = starts[r + 1] - starts[r];
            KARMA_TRY(karma_comm_exchange_counts(s->comm, sc.data(), rcv.data()));
            {   // the deferred steps' slot size: the largest slice of any rank, + 25 %
                int64_t mx = 0;
                for (int r = 0; r < W; ++r) mx = std::max(mx, sc[r]);
                KARMA_TRY(karma_comm_allreduce_host(s->comm, &mx, 1, KARMA_DT_I64, KARMA_OP_MAX));
                s->kc = std::max(s->kc, mx + mx / 4 + 1024);
            }
            for (int r = 0; r < W; ++r) {
                so[r + 1] = so[r] + 8 * sc[r];
                ro[r + 1] = ro[r] + 8 * rcv[r];
            }
            const int64_t nr = ro[W] / 8;
            DevArray<uint64_t> rk;
            DevArray<int64_t> rc;
            KARMA_TRY(rk.alloc(ctx, nr));
            KARMA_TRY(rc.alloc(ctx, nr));
            KARMA_TRY(karma_comm_alltoallv_kv(s->comm, k, c, so.data(), rk.ptr, rc.ptr, ro.data()));
            std::vector<int64_t> run(W + 1, 0);
            for (int r = 0; r < W; ++r) run[r + 1] = run[r] + rcv[r];
            KARMA_TRY(karma_pairs_merge_runs(ctx, rk.ptr, rc.ptr, run.data(), W, 1, &s->merged));
            // rk / rc return to the main stream's cache: the merge (stream-ordered) has read them
        } else {  // emulation: this rank's own W slices stand in for the W received ones
            KARMA_TRY(karma_pairs_merge_runs(ctx, k, c, starts.data(), s->nranks, 1, &s->merged));
        }
        int64_t* totals = nullptr;
        KARMA_TRY(karma_edges_begin(ctx, s->merged, KARMA_MODE_READS, s->n_glob, &s->edges, &totals));
        if (s->world > 1) KARMA_TRY(allgather_slices(s, totals));
        KARMA_TRY(karma_edges_end(s->edges, count ? &E : nullptr));
    } else {
        KARMA_TRY(karma_edges_from_pairs(ctx, s->local, KARMA_MODE_READS, nullptr, s->n_glob, &s->edges, &E));
    }
    s->E = E;
    if (!sequential) KARMA_TRY(karma_ctx_join(ctx, s->side_s));
    s->sync_set = s->world > 1;  // the next exchange-stream tail waits for this step's collectives
    return KARMA_OK;
}

// ---- the deferred step -----------------------------------------------------------
int check_entry(karma_step* s, const karma_step::Pending& p, bool* slow) {
    const StepStatus& st = const_cast<const StepStatus&>(s->ring_h[p.seq % kRing]);
    *slow = st.slow != 0;
    // a step that runs again: its pair list may be incomplete (an overflowed
    // bucket or exchange slot), so the merge-order and zero-total words are
    // artifacts of the truncation; the re-run checks them on complete lists
    const int64_t err = *slow ? st.err & ~int64_t(8 | 16) : st.err;
    if (err) {
        KARMA_CHECK(!(err & 1), KARMA_ERR_UNSORTED, "records are not grouped by read (read ids decrease)");
        KARMA_CHECK(!(err & 2), KARMA_ERR_ARG, "a record's contig index is >= n_contigs (%lld)",
                    (long long)s->n_glob);
        KARMA_CHECK(!(err & 16), KARMA_ERR_UNSORTED, "karma_pairs_merge_runs: a run is not sorted by key");
        KARMA_CHECK(!(err & 8), KARMA_ERR_ZERO_DIV, "division by zero: a shared count over a zero total");
        KARMA_CHECK(false, KARMA_ERR_STATE, "code partition: block counts disagree with the classify histogram");
    }
    return KARMA_OK;
}

bool entry_done(const karma_step* s, uint64_t seq) {
    return __atomic_load_n(&s->ring_h[seq % kRing].seq, __ATOMIC_ACQUIRE) == seq;
}

// Checks deferred steps: every finished one (wait = false), or all of them
// after waiting (wait = true), or down to kLag - 1 outstanding (lag = true).
// A step whose words call for the general path runs again synchronously;
// the newest deferred step's profile, M and E stay the ones karma_step_sync
// and karma_step_profile report (a re-run of an older step does not replace them).
int drain(karma_step* s, bool wait, bool lag) {
    while (!s->pending.empty()) {
        karma_step::Pending p = s->pending.front();
        const bool must = wait || (lag && (int)s->pending.size() >= s->lag);
        // several processes: a step's entry is read at the same point of the
        // step sequence on every rank (a rerun issues collectives)
        if (s->world > 1 && !must) break;
        if (!entry_done(s, p.seq)) {
            if (!must) break;
            // the main stream reaches the status kernel within a step's time
            const auto w0 = std::chrono::steady_clock::now();
            for (int spin = 0; !entry_done(s, p.seq); ++spin) {
                if (spin > 64) std::this_thread::yield();
                if (spin % 4096 == 4095 && hipStreamQuery(s->main_s) == hipSuccess &&
                    hipStreamQuery(s->alt_s) == hipSuccess && hipStreamQuery(s->side_alt_s) == hipSuccess &&
                    !entry_done(s, p.seq)) {
                    set_error("karma_step: a deferred step's status never arrived");
                    return KARMA_ERR_STATE;
                }
                // a step takes milliseconds: this long means a peer that
                // stopped issuing collectives; an error beats a silent hang
                if (spin % 65536 == 65535 && std::chrono::steady_clock::now() - w0 > std::chrono::seconds(s->stall_s)) {
                    set_error("karma_step: deferred step %llu's status did not arrive within %d s (rank %d of %d; %s)",
                              (unsigned long long)p.seq, s->stall_s, s->rank, s->world,
                              s->world == 1 ? "one process: device stalled?"
                              : s->one_comm ? "collectives of the main communicator on the exchange stream stalled"
                                            : "collectives of the main or side communicator stalled");
                    return KARMA_ERR_STALL;
                }
            }
            s->wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0)
                              .count();
        }
        s->pending.pop_front();
        bool slow = false;
        KARMA_TRY(check_entry(s, p, &slow));
        if (slow) {
            // the general path (relabelled contigs, more pair room, big reads,
            // an overflowed bucket): the step's work again, synchronously
            ++s->n_redone;
            s->sticky_sync = 8;
            const uint64_t newest = s->prof_seq;
            const int newest_par = s->prof_par;
            const int64_t newest_M = s->prof_M;
            KARMA_TRY(run_sync(s, p.store, p.rec, p.A, p.flg, false, false, true));
            if (newest > p.seq) {  // a newer deferred step is pending: its outputs stay the newest
                s->prof_seq = newest;
                s->prof_par = newest_par;
                s->prof_M = newest_M;
                s->M = s->E = -1;
            }
        }
    }
    return KARMA_OK;
}

int run_deferred(karma_step* s, karma_contigs* store, const uint32_t* rec, int64_t A, bool flg, bool sequential) {
    karma_ctx* ctx = s->ctx;
    KARMA_TRY(drop_outputs(s));  // a deferred step has no outputs to read
    ++s->n_deferred;
    const uint64_t seq = ++s->seq;
    // Two batches in flight pay off only while one batch leaves the chip idle
    // between its short kernels: at config 3's size (308M records) two records
    // jobs side by side took 1.89 ms per batch against 1.23 ms one after the
    // other (they evict each other's partition runs from the caches); the
    // 8-rank strong preview (38.6M records) went 0.237 -> 0.199 ms.
    // several processes: two main streams only with the exchange stream
    // (the main communicator's operations then all go to side_alt_s)
    const bool two = (s->world == 1 || (s->xstream && !sequential)) &&
                     (s->streams ? s->streams == 2 : A < kAltMaxRecords);
    // the exchange stream carries the tail: with two main streams, and with
    // one communicator also behind one main stream (it then holds every
    // collective of the step, the presence all-gather included)
    // (emulated ranks, KARMA_STEP_EMU_XS=1: the same stream layout as several
    // processes, the tail on the exchange stream; its 8 more event calls per
    // step cost more than the overlap gains: 8-rank strong preview 0.200 /
    // 0.204 against 0.193 / 0.186 ms with the tail on the main stream, same box)
    const bool xs_on = !sequential && s->xstream &&
                       ((s->world > 1 && (two || s->one_comm)) || (s->world == 1 && s->emulate && s->emu_xs && two));
    if (two) ++s->n_two;
    if (xs_on) ++s->n_xs;
    const int par = sequential || !two ? 0 : (int)(seq & 1);
    hipStream_t const ms = par ? s->alt_s : s->main_s;
    hipStream_t const xs = s->side_alt_s;
    if (s->tail_set[par]) {
        // the records job's lists (this main stream's cache) and tail[par]
        // were last used on the exchange stream
        if (counted_call("hipStreamWaitEvent")) ++t_hip_calls;
        KARMA_HIP(hipStreamWaitEvent(ms, s->ev_tail[par], 0));
    }
    // One main stream (large batches): the records job does not wait for the
    // previous batch's profile.  With KARMA_STEP_JOIN=1 it does (classify then
    // never shares HBM with a profile): config 3 1.29-1.31 against 1.16-1.21 ms
    // per step without the join (profiles/r04/measurements.md (ab_join)).
    if (!two && !sequential && s->ev_set && s->join) {
        if (counted_call("hipStreamWaitEvent")) ++t_hip_calls;
        KARMA_HIP(hipStreamWaitEvent(ms, s->ev, 0));
        s->ev_set = false;
    }
    karma_step::Tail& tl = s->tail[par];
    // A failure between here and the status kernel's launch leaves this job's
    // flags, counters and block items in the tail's own control block (only
    // the status kernel clears it), and the next job on this tail would take
    // the block as zeroed (no probe, no memset): clear it once every stream is
    // idle (a kernel of this step may still use it), and leave no newest
    // deferred step without a status behind.
    struct FailGuard {
        karma_step* s;
        karma_step::Tail& tl;
        uint64_t seq;
        bool armed = true;
        ~FailGuard() {
            if (!armed) return;
            for (hipStream_t q : {s->side_s, s->side_alt_s, s->main_s, s->alt_s}) (void)hipStreamSynchronize(q);
            if (s->own_ctrl && tl.ctrl.ptr) {
                (void)hipMemsetAsync(tl.ctrl.ptr, 0, tl.ctrl.n * 8, s->main_s);
                (void)hipStreamSynchronize(s->main_s);
            }
            if (s->prof_seq == seq) {
                s->prof_seq = 0;
                s->prof_M = -1;
            }
        }
    } fail{s, tl, seq};
    ctx->stream = ms;
    s->prof_seq = seq;
    s->prof_par = par;
    s->prof_M = -1;
    if (s->exchange) KARMA_TRY(karma_graph_split_hint(ctx, s->bounds.data(), s->nranks));
    // records job (main stream) up to its final kernel; no readback
    SetsJob* job = nullptr;
    SetsDeferred v;
    // the general-read branch: on the idle spare main stream with one main
    // stream; kept on the main stream with two (see side_alt_s)
    ctx->no_fork = two && s->sides == 2;
    ctx->fork_use = two ? nullptr : s->alt_s;
    // where the side stream's profile may start (SetsJob::launch): with one main
    // stream, after the code partition -- the profile's writes then share HBM
    // with the LDS-bound code reduce and final kernel instead of the next
    // batch's classify (config 3: 1.15 against 1.20-1.22 ms per step,
    // profiles/r04/measurements.md (ab_mark3)); with two, after the final kernel
    ctx->mark_pos = two ? kMarkTwo : flg ? kMarkOneFlagged : kMarkOne;
    ctx->job_ctrl = s->own_ctrl ? tl.ctrl.ptr : nullptr;  // zero: the last status kernel of this tail cleared it
    ctx->job_ctrl_words = s->own_ctrl ? (int64_t)tl.ctrl.n : 0;
    RecIn rin;
    if (flg) rin.fw = rec;
    else rin.pr = reinterpret_cast<const uint2*>(rec);
    KARMA_CHECK(!(reinterpret_cast<uintptr_t>(rec) & 15), KARMA_ERR_ARG, "karma_step_run: records must be 16-byte aligned");
    const int jrc = sets_begin_deferred(ctx, rin, A, s->n_glob, &job, &v);
    ctx->job_ctrl = nullptr;
    ctx->job_ctrl_words = 0;
    ctx->mark_pos = -1;
    ctx->no_fork = false;
    ctx->fork_use = nullptr;
    KARMA_TRY(jrc);
    std::unique_ptr<SetsJob, void (*)(SetsJob*)> jg(job, sets_release);
    if (v.ctrl) ++s->n_own;
    if (s->own_ctrl && !v.ctrl) {
        // the job needed a larger block than this tail's: grow it for the next
        // job on this tail (with every stream idle: the old block may still
        // be cleared by a status kernel), zeroed in stream order
        KARMA_HIP(hipStreamSynchronize(s->side_s));
        KARMA_HIP(hipStreamSynchronize(s->side_alt_s));
        KARMA_HIP(hipStreamSynchronize(s->main_s));
        KARMA_HIP(hipStreamSynchronize(s->alt_s));
        KARMA_TRY(tl.ctrl.alloc(ctx, (size_t)(v.ctrl_need + v.ctrl_need / 4 + 64)));
        KARMA_HIP(hipMemsetAsync(tl.ctrl.ptr, 0, tl.ctrl.n * 8, ms));
    }
    // side stream: presence, column table (M stays on the device), then the
    // profile behind the graph's final kernel (sequential: all on the main
    // stream, every kernel alone on the chip -- the per-kernel timing pass)
    hipStream_t const side = sequential ? ms : (par && s->sides == 2 && !xs_on ? s->side_alt_s : s->side_s);
    ctx->stream = side;
    DevArray<uint32_t>& pz = s->plan_zero[side == s->side_alt_s ? 1 : 0];
    if (!sequential) {
        // 2,048 + 2 words: the bitmap of every k <= 8 and the exception counter
        if (!pz.ptr) {
            KARMA_TRY(pz.alloc(ctx, 2048 + 2));
            KARMA_HIP(hipMemsetAsync(pz.ptr, 0, pz.n * 4, side));
        }
        ctx->plan_zeroed = pz.ptr;
        ctx->plan_zeroed_words = (int64_t)pz.n;
    }
    karma_kmer_plan* plan = nullptr;
    int rc = karma_kmer_plan_create(ctx, store, s->kmode, &plan);
    ctx->plan_zeroed = nullptr;
    ctx->plan_zeroed_words = 0;
    if (!rc && s->world > 1) {
        if (xs_on && s->one_comm) {
            // the presence all-gather on the exchange stream (behind the previous
            // batch's tail and a synchronous step's collectives), the column
            // table back on the side stream behind it
            rc = stream_after(&s->ev_pres, side, xs);
            if (!rc && s->sync_set) {
                rc = stream_after(&s->ev_sync, s->main_s, xs);
                s->sync_set = false;
            }
            ctx->stream = xs;
            if (!rc) rc = exchange_presence(s, plan, s->comm);
            if (!rc) rc = stream_after(&s->ev_pres2, xs, side);
            ctx->stream = side;
        } else {
            // sequential (one stream), or the side communicator on the side stream
            rc = exchange_presence(s, plan, s->scomm ? s->scomm : s->comm);
        }
    }
    // M: into the device ring (the profile reads it) and the mapped ring (the
    // host reads it once the step is done); nothing on the main streams waits for it
    int64_t* const m_dev = s->m_ring.ptr + seq % kRing;
    if (!rc) rc = kmer_finalize_device(plan, m_dev, s->mring_d + seq % kRing);
    if (rc && !sequential && pz.ptr) (void)hipMemsetAsync(pz.ptr, 0, pz.n * 4, side);  // not cleared by a column table
    if (!rc) rc = ensure_prof(s, tl.prof, (size_t)std::max<int64_t>(1, s->n_loc * kmer_m_cap(plan)));
    if (!rc && ctx->mark_set && !sequential) {
        if (counted_call("hipStreamWaitEvent")) ++t_hip_calls;
        rc = hipStreamWaitEvent(side, ctx->mark_ev, 0) == hipSuccess ? KARMA_OK : KARMA_ERR_HIP;
    }
    if (!rc && s->n_loc) {
        // KARMA_STEP_HEADROOM (A/B): profile blocks per CU left free for the
        // main stream's kernels (one main stream only)
        static const int headroom = getenv("KARMA_STEP_HEADROOM") ? atoi(getenv("KARMA_STEP_HEADROOM")) : 0;
        ctx->grid_headroom = two || sequential ? 0 : headroom;
        rc = kmer_profile_device_m(plan, tl.prof.ptr, m_dev);
        ctx->grid_headroom = 0;
    }
    if (!rc && !two && !sequential && s->join) {
        if (!s->ev && hipEventCreateWithFlags(&s->ev, hipEventDisableTiming) != hipSuccess) rc = KARMA_ERR_HIP;
        if (counted_call("hipEventRecord")) ++t_hip_calls;
        if (!rc) rc = hipEventRecord(s->ev, side) == hipSuccess ? KARMA_OK : KARMA_ERR_HIP;
        s->ev_set = !rc;
    }
    if (plan) karma_kmer_plan_destroy(plan);  // its buffers return to the side stream's cache
    ctx->stream = ms;
    KARMA_TRY(rc);
    if (xs_on) {  // the tail on the exchange stream, behind this records job (and a synchronous step's collectives)
        KARMA_TRY(stream_after(&s->ev_rec, ms, xs));
        // (one communicator: the presence all-gather above already waited for them)
        if (s->sync_set) {
            KARMA_TRY(stream_after(&s->ev_sync, s->main_s, xs));
            s->sync_set = false;
        }
        ctx->stream = xs;
    }
    // main stream: the tail, sized on the device
    const uint64_t* lk = v.keys;
    const int64_t* lc = v.counts;
    const int64_t* n_dev = v.dst + v.B;
    int64_t* mbad = nullptr;
    const int cu = ctx->cu_count;
    int64_t cap = v.cap;  // entries of the list the edge stage reads, at most
    if (s->exchange) {
        if (!tl.mbad.ptr) {  // the merge sets it, the status kernel reads and clears it
            KARMA_TRY(tl.mbad.alloc(ctx, 1));
            KARMA_HIP(hipMemsetAsync(tl.mbad.ptr, 0, 8, ctx->stream));
        }
        RunSrc rs{};
        rs.nr = s->nranks;
        rs.B = v.B;
        rs.bw = v.bw;
        for (int r = 0; r <= s->nranks; ++r) rs.b[r] = s->bounds[r];
        KARMA_CHECK((int)v.split_b.size() == s->nranks + 1, KARMA_ERR_STATE, "karma_step: the split hint was lost");
        const uint64_t* mkeys = v.keys;
        const int64_t* mcounts = v.counts;
        if (s->world > 1) {
            // each owner's slice into a fixed slot of a padded all-to-all (its
            // length on the device), so nothing waits for the slice sizes
            const int W = s->world;
            const int64_t slot = s->kc + 1;
            KARMA_TRY(ensure_arr(ctx, tl.sk, W * slot));
            KARMA_TRY(ensure_arr(ctx, tl.sc, W * slot));
            KARMA_TRY(ensure_arr(ctx, tl.rk, W * slot));
            KARMA_TRY(ensure_arr(ctx, tl.rc, W * slot));
            KARMA_TRY(ensure_arr(ctx, tl.nm, 1));
            KARMA_LAUNCH(ctx, "exchange_pack", step_pack_kernel,
                         (int)std::max<int64_t>(1, std::min<int64_t>((v.cap + 255) / 256, 4 * cu)), 256, 0, v.keys,
                         v.counts, v.dst, v.split_loc, rs, slot, tl.sk.ptr, tl.sc.ptr, v.flags, v.counters, v.ovf);
            std::vector<int64_t> off(W + 1);
            for (int r = 0; r <= W; ++r) off[r] = (int64_t)r * slot * 8;
            KARMA_TRY(karma_comm_alltoallv_kv(s->comm, tl.sk.ptr, tl.sc.ptr, off.data(), tl.rk.ptr, tl.rc.ptr,
                                              off.data()));
            rs.slot = slot;
            rs.n_out = tl.nm.ptr;
            mkeys = tl.rk.ptr;
            mcounts = tl.rc.ptr;
            cap = W * (slot - 1);
            n_dev = tl.nm.ptr;
        }
        KARMA_TRY(ensure_arr(ctx, tl.mk, cap));
        KARMA_TRY(ensure_arr(ctx, tl.mc, cap));
        const int64_t tiles_cap = (cap + kMT - 1) / kMT + s->nranks;
        // a tile per block up to 8 blocks per CU (the tiles' searches are
        // dependent loads: more tiles in flight, not more tiles per block)
        KARMA_LAUNCH(ctx, "merge_rank", step_merge_kernel, (int)std::min<int64_t>(tiles_cap, 8 * cu), 256, 0, mkeys,
                     mcounts, v.dst, v.split_loc, rs, tl.mk.ptr, tl.mc.ptr, tl.mbad.ptr);
        lk = tl.mk.ptr;
        lc = tl.mc.ptr;
        mbad = tl.mbad.ptr;
    }
    KARMA_TRY(ensure_arr(ctx, tl.tot, s->n_glob));
    KARMA_TRY(ensure_arr(ctx, tl.tile_cnt, (cap + kET - 1) / kET + 1));
    KARMA_TRY(ensure_arr(ctx, tl.est, 3));
    KARMA_TRY(ensure_arr(ctx, tl.ea, cap));
    KARMA_TRY(ensure_arr(ctx, tl.eb, cap));
    KARMA_TRY(ensure_arr(ctx, tl.es, cap));
    KARMA_TRY(ensure_arr(ctx, tl.ew, cap));
    // the edge stage's tiles are chains of dependent loads (keys, totals): up
    // to 4 blocks per CU take a tile each (one block per CU striding over 12
    // tiles at the 8-rank weak preview's 3.2M keys took 29 + 46 us)
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((cap + kET - 1) / kET, 4 * cu));
    KARMA_LAUNCH(ctx, "edge_count", step_edge_count_kernel, grid, kET, 0, lk, lc, n_dev, s->n_glob, tl.tot.ptr,
                 tl.tile_cnt.ptr, tl.est.ptr);
    // the owners' readset totals from every owner (fixed sizes: no host wait)
    if (s->world > 1) KARMA_TRY(allgather_slices(s, tl.tot.ptr));
    KARMA_LAUNCH(ctx, "edge_weights", step_edge_write_kernel, grid, kET, 0, lk, lc, n_dev, tl.tot.ptr,
                 tl.tile_cnt.ptr, tl.ea.ptr, tl.eb.ptr, tl.es.ptr, tl.ew.ptr, tl.est.ptr, s->n_glob);
    // test hook (tests/test_gpu_step.py): fail deferred step `fault_seq` after
    // its tail's kernels, before the status kernel (the control-block error path)
    KARMA_CHECK(seq != s->fault_seq, KARMA_ERR_STATE, "karma_step: injected fault in deferred step %llu",
                (unsigned long long)seq);
    KARMA_LAUNCH(ctx, "step_status", step_status_kernel, 1, 256, 0, v.flags, v.counters, v.ovf, v.B, v.dst, mbad,
                 tl.est.ptr, s->ring_d + seq % kRing, seq, v.ctrl, v.ctrl ? v.ctrl_need : (int64_t)0);
    if (xs_on) {
        if (!s->ev_tail[par]) KARMA_HIP(hipEventCreateWithFlags(&s->ev_tail[par], hipEventDisableTiming));
        if (counted_call("hipEventRecord")) ++t_hip_calls;
        KARMA_HIP(hipEventRecord(s->ev_tail[par], xs));
        s->tail_set[par] = true;
        s->tail_last = par;
        ctx->stream = ms;
    }
    fail.armed = false;
    s->pending.push_back({seq, store, rec, A, flg});
    return KARMA_OK;
}

}  // namespace

extern "C" {

int karma_step_create(karma_ctx* ctx, karma_comm* comm, karma_comm* side_comm, int kmode, int64_t n_glob,
                      const int64_t* bounds, int nranks, int rank, karma_step** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && bounds && nranks >= 1 && nranks <= kMaxRuns && rank >= 0 && rank < nranks && n_glob >= 1,
                KARMA_ERR_ARG, "karma_step_create: bad arguments (nranks %d, rank %d)", nranks, rank);
    int world = 1, crank = 0;
    if (comm) KARMA_TRY(karma_comm_info(comm, &world, &crank));
    KARMA_CHECK(world == 1 || (world == nranks && crank == rank), KARMA_ERR_ARG,
                "karma_step_create: communicator of %d ranks (rank %d) for %d owners (rank %d)", world, crank,
                nranks, rank);
    // several owners: their bounds tile [0, n_glob); one: [bounds[0], bounds[1]) is
    // this process's contig rows (a shard of n_glob ids, no exchange)
    KARMA_CHECK(nranks == 1 || (bounds[0] == 0 && bounds[nranks] == n_glob), KARMA_ERR_ARG,
                "owner bounds must span [0, n_glob)");
    KARMA_CHECK(bounds[0] >= 0 && bounds[nranks] <= n_glob, KARMA_ERR_ARG, "owner bounds outside [0, n_glob)");
    for (int r = 0; r < nranks; ++r)
        KARMA_CHECK(bounds[r] <= bounds[r + 1], KARMA_ERR_ARG, "owner bounds must not decrease");
    std::unique_ptr<karma_step> s(new karma_step());
    s->ctx = ctx;
    s->comm = world > 1 ? comm : nullptr;
    // a side communicator equal to the main one is none (its operations would
    // otherwise go on two streams at once)
    s->scomm = world > 1 && side_comm != comm ? side_comm : nullptr;
    s->one_comm = s->scomm == nullptr;
    s->kmode = kmode;
    s->world = world;
    s->rank = rank;
    s->nranks = nranks;
    s->emulate = world == 1 && nranks > 1 ? nranks : 0;
    if (const char* e = getenv("KARMA_STEP_STREAMS")) s->streams = atoi(e) == 1 ? 1 : atoi(e) == 2 ? 2 : 0;
    if (const char* e = getenv("KARMA_STEP_JOIN")) s->join = atoi(e) != 0;  // A/B only
    if (const char* e = getenv("KARMA_STEP_SIDES")) s->sides = atoi(e) == 1 ? 1 : 2;
    if (const char* e = getenv("KARMA_STEP_DEFER_RANKS")) s->defer_ranks = atoi(e) != 0;
    if (const char* e = getenv("KARMA_STEP_XSTREAM")) s->xstream = atoi(e) != 0;
    if (const char* e = getenv("KARMA_STEP_STALL_S")) s->stall_s = std::max(1, atoi(e));
    if (const char* e = getenv("KARMA_STEP_OWN_CTRL")) s->own_ctrl = atoi(e) != 0;
    if (const char* e = getenv("KARMA_STEP_EMU_XS")) s->emu_xs = atoi(e) != 0;
    if (const char* e = getenv("KARMA_STEP_LAG")) s->lag = std::max(1, std::min(kRing / 2, atoi(e)));
    if (const char* e = getenv("KARMA_STEP_FAULT_SEQ")) s->fault_seq = strtoull(e, nullptr, 10);
    s->n_glob = n_glob;
    s->bounds.assign(bounds, bounds + nranks + 1);
    s->c_lo = bounds[rank];
    s->n_loc = bounds[rank + 1] - bounds[rank];
    s->exchange = nranks > 1;
    int lo = 0, hi = 0;
    KARMA_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // the main stream (the graph and the exchange) at high priority: its
    // blocks dispatch first when CUs free up beside the side-stream profile
    KARMA_HIP(hipStreamCreateWithPriority(&s->main_s, hipStreamNonBlocking, hi));
    KARMA_HIP(hipStreamCreateWithPriority(&s->alt_s, hipStreamNonBlocking, hi));
    // KARMA_STEP_SIDE_PRIO=1 (A/B): the side streams at the main streams' priority
    const int side_prio = getenv("KARMA_STEP_SIDE_PRIO") && atoi(getenv("KARMA_STEP_SIDE_PRIO")) ? hi : 0;
    KARMA_HIP(hipStreamCreateWithPriority(&s->side_s, hipStreamNonBlocking, side_prio));
    KARMA_HIP(hipStreamCreateWithPriority(&s->side_alt_s, hipStreamNonBlocking, side_prio));
    // the status ring in mapped coherent host memory of this step's own: a
    // second live step on the context numbers its steps from 1 too, and a
    // shared ring would hand it this step's verdicts
    void *hm = nullptr, *dm = nullptr;
    KARMA_HIP(hipHostMalloc(&s->ring_mem, kRing * sizeof(StepStatus) + kRing * 8,
                            hipHostMallocMapped | hipHostMallocCoherent));
    hm = s->ring_mem;
    KARMA_HIP(hipHostGetDevicePointer(&dm, hm, 0));
    s->mring_h = reinterpret_cast<int64_t*>(static_cast<uint8_t*>(hm) + kRing * sizeof(StepStatus));
    s->mring_d = reinterpret_cast<int64_t*>(static_cast<uint8_t*>(dm) + kRing * sizeof(StepStatus));
    KARMA_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->graves_h), kRing * 4 * 8, hipHostMallocDefault));
    {
        hipStream_t prev = ctx->stream;
        ctx->stream = s->main_s;
        const int rc = s->m_ring.alloc(ctx, kRing);
        ctx->stream = prev;
        KARMA_TRY(rc);
    }
    s->ring_h = static_cast<StepStatus*>(hm);
    s->ring_d = static_cast<StepStatus*>(dm);
    std::memset(hm, 0, kRing * sizeof(StepStatus) + kRing * 8);
    *out = s.release();
    return KARMA_OK;
}

int karma_step_run(karma_step* s, karma_contigs* store, const uint32_t* records, int64_t n_records, int flags,
                   int64_t* info) {
    KARMA_CHECK(s && store && (records || n_records == 0) && n_records >= 0, KARMA_ERR_ARG,
                "karma_step_run: bad arguments");
    KARMA_CHECK((flags & ~(KARMA_STEP_KEEP | KARMA_STEP_SEQUENTIAL | KARMA_STEP_DEFER | KARMA_STEP_FLAGGED)) == 0,
                KARMA_ERR_ARG,
                "karma_step_run: unknown flags %d", flags);
    karma_ctx* ctx = s->ctx;
    KARMA_TRY(ctx_begin(ctx));
    int64_t n_store = 0;
    KARMA_TRY(karma_contigs_info(store, &n_store, nullptr, nullptr, nullptr));
    KARMA_CHECK(n_store == s->n_loc, KARMA_ERR_ARG, "karma_step_run: the store holds %lld contigs, the shard %lld",
                (long long)n_store, (long long)s->n_loc);
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t prev = ctx->stream;
    ctx->stream = s->main_s;
    const bool keep = flags & KARMA_STEP_KEEP, seq = flags & KARMA_STEP_SEQUENTIAL;
    const bool flg = flags & KARMA_STEP_FLAGGED;
    // deferred: one process (no collective needs a host count), nothing read back
    // several processes: once a synchronous step has sized the exchange's
    // slots and every rank's store is known to be ACGT-only
    // (one communicator: with the exchange stream, which then carries every
    // collective; a side communicator: the main one's operations stay on one stream)
    const bool ranks_ok = s->world == 1 || (s->defer_ranks && (s->one_comm ? s->xstream : s->scomm != nullptr) &&
                                            s->kc > 0 && s->acgt_store == store);
    const bool defer = (flags & KARMA_STEP_DEFER) && !keep && ranks_ok && s->n_glob <= sets_max_contigs();
    int rc = KARMA_OK;
    if (defer && s->sticky_sync > 0) {
        --s->sticky_sync;
        rc = drain(s, false, true);
        if (!rc) rc = run_sync(s, store, records, n_records, flg, false, seq, false);
    } else if (defer) {
        rc = drain(s, false, true);
        if (!rc) rc = run_deferred(s, store, records, n_records, flg, seq);
    } else {
        rc = drain(s, true, false);  // earlier deferred steps complete and checked first
        if (!rc) rc = run_sync(s, store, records, n_records, flg, keep, seq, !(flags & KARMA_STEP_DEFER));
    }
    ctx->stream = prev;
    s->run_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    if (rc) return rc;
    if (info) {
        info[0] = s->M;
        info[1] = s->E;
        info[2] = s->pairs_local;
        info[3] = s->entries;
    }
    return KARMA_OK;
}

int karma_step_sync(karma_step* s) {
    KARMA_CHECK(s, KARMA_ERR_ARG, "null step");
    karma_ctx* ctx = s->ctx;
    KARMA_TRY(ctx_begin(ctx));
    hipStream_t prev = ctx->stream;
    ctx->stream = s->main_s;
    int rc = drain(s, true, false);
    ctx->stream = prev;
    KARMA_TRY(rc);
    KARMA_HIP(hipStreamSynchronize(s->side_s));
    KARMA_HIP(hipStreamSynchronize(s->side_alt_s));
    KARMA_HIP(hipStreamSynchronize(s->alt_s));
    KARMA_HIP(hipStreamSynchronize(s->main_s));
    KARMA_TRY(bury(s, true));
    if (s->prof_seq) {  // every stream is idle: the newest deferred step's column count has landed
        s->prof_M = __atomic_load_n(&s->mring_h[s->prof_seq % kRing], __ATOMIC_ACQUIRE);
        // ... and its status: M and the local edge count read as of a synchronous step
        s->M = s->prof_M;
        s->E = const_cast<const StepStatus&>(s->ring_h[s->prof_seq % kRing]).E;
    }
    if (s->edges && s->E < 0) KARMA_TRY(karma_edges_count(s->edges, &s->E));
    return KARMA_OK;
}

int karma_step_info(karma_step* s, int64_t* info, int n) {
    KARMA_CHECK(s && info && n >= 0, KARMA_ERR_ARG, "karma_step_info: bad arguments");
    const int64_t mode = (s->one_comm ? 1 : 0) | (s->xstream ? 2 : 0) | (s->defer_ranks ? 4 : 0);
    const int64_t v[] = {s->M,          s->E,        s->pairs_local, s->entries,
                         s->n_sync,     s->n_deferred, s->n_redone,  (int64_t)s->pending.size(),
                         s->run_ns,     s->wait_ns,  s->n_two,       s->n_xs,
                         mode,          s->world,    s->n_own};
    for (int i = 0; i < n && i < (int)(sizeof v / sizeof v[0]); ++i) info[i] = v[i];
    return KARMA_OK;
}

// The profile of the newest step (a deferred one's once karma_step_sync has read its column count).
int karma_step_profile(karma_step* s, double** dev, int64_t* rows, int64_t* M) {
    KARMA_CHECK(s && dev && s->prof_M >= 0, KARMA_ERR_STATE, "karma_step_profile: no finished step");
    // a deferred step's profile is in its main stream's buffer
    *dev = s->prof_seq ? s->tail[s->prof_par].prof.ptr : s->prof.ptr;
    if (rows) *rows = s->n_loc;
    if (M) *M = s->prof_M;
    return KARMA_OK;
}

int karma_step_columns(karma_step* s, uint64_t* keys_host) {
    KARMA_CHECK(s && s->plan, KARMA_ERR_STATE, "karma_step_columns: no kept step");
    KARMA_TRY(ctx_begin(s->ctx));
    hipStream_t prev = s->ctx->stream;
    s->ctx->stream = s->main_s;
    const int rc = karma_kmer_columns(s->plan, keys_host);
    s->ctx->stream = prev;
    return rc;
}

int karma_step_edges(karma_step* s, karma_edges** e) {
    KARMA_CHECK(s && e && s->edges, KARMA_ERR_STATE, "karma_step_edges: no kept step");
    *e = s->edges;
    return KARMA_OK;
}

// The newest step's edges as this rank owns them, after karma_step_sync: a
// deferred step's straight from its tail (the arrays step_edge_write_kernel
// wrote, the code path a stream of deferred batches times), a synchronous
// one's (a re-run included) from its karma_edges.
int karma_step_newest_edges(karma_step* s, uint32_t* a, uint32_t* b, int64_t* shared, double* weight,
                            int64_t* totals, int64_t cap, int is_device, int64_t* n_edges, int* deferred) {
    KARMA_CHECK(s && n_edges && cap >= 0, KARMA_ERR_ARG, "karma_step_newest_edges: bad arguments");
    KARMA_CHECK(s->pending.empty() && s->prof_M >= 0, KARMA_ERR_STATE,
                "karma_step_newest_edges: no finished step (karma_step_sync first)");
    KARMA_TRY(ctx_begin(s->ctx));
    const hipMemcpyKind kind = is_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (!s->prof_seq) {  // a synchronous step is the newest
        KARMA_CHECK(s->edges, KARMA_ERR_STATE, "karma_step_newest_edges: the newest step kept no edges");
        int64_t E = 0;
        KARMA_TRY(karma_edges_count(s->edges, &E));
        *n_edges = E;
        if (deferred) *deferred = 0;
        if (a || b || shared || weight) {
            KARMA_CHECK(E <= cap, KARMA_ERR_ARG, "karma_step_newest_edges: %lld edges, room for %lld",
                        (long long)E, (long long)cap);
            KARMA_TRY(karma_edges_get(s->edges, a, b, shared, weight, nullptr, is_device));
        }
        if (totals) KARMA_TRY(karma_edges_totals(s->edges, totals, is_device));
        if (is_device) KARMA_TRY(karma_ctx_sync(s->ctx));
        return KARMA_OK;
    }
    const karma_step::Tail& tl = s->tail[s->prof_par];
    const int64_t E = const_cast<const StepStatus&>(s->ring_h[s->prof_seq % kRing]).E;
    KARMA_CHECK(E >= 0 && E <= (int64_t)tl.ea.n, KARMA_ERR_STATE, "karma_step_newest_edges: bad edge count %lld",
                (long long)E);
    *n_edges = E;
    if (deferred) *deferred = 1;
    if ((a || b || shared || weight) && E > cap) {
        set_error("karma_step_newest_edges: %lld edges, room for %lld", (long long)E, (long long)cap);
        return KARMA_ERR_ARG;
    }
    hipStream_t q = s->main_s;
    if (E) {
        if (a) KARMA_HIP(hipMemcpyAsync(a, tl.ea.ptr, E * 4, kind, q));
        if (b) KARMA_HIP(hipMemcpyAsync(b, tl.eb.ptr, E * 4, kind, q));
        if (shared) KARMA_HIP(hipMemcpyAsync(shared, tl.es.ptr, E * 8, kind, q));
        if (weight) KARMA_HIP(hipMemcpyAsync(weight, tl.ew.ptr, E * 8, kind, q));
    }
    if (totals) KARMA_HIP(hipMemcpyAsync(totals, tl.tot.ptr, s->n_glob * 8, kind, q));
    KARMA_HIP(hipStreamSynchronize(q));
    return KARMA_OK;
}

int karma_step_destroy(karma_step* s) {
    if (!s) return KARMA_OK;
    hipSetDevice(s->ctx->device);
    if (s->main_s) hipStreamSynchronize(s->main_s);
    if (s->alt_s) hipStreamSynchronize(s->alt_s);
    if (s->side_s) hipStreamSynchronize(s->side_s);
    if (s->side_alt_s) hipStreamSynchronize(s->side_alt_s);
    s->pending.clear();
    s->E = 0;  // outputs dropped unread
    drop_outputs(s);
    bury(s, true);
    for (auto& ev : s->grave_ev)
        if (ev) hipEventDestroy(ev);
    for (hipEvent_t ev : {s->ev, s->ev_rec, s->ev_sync, s->ev_tail[0], s->ev_tail[1], s->ev_pres, s->ev_pres2,
                          s->ev_pre})
        if (ev) hipEventDestroy(ev);
    if (s->graves_h) hipHostFree(s->graves_h);
    if (s->ring_mem) hipHostFree(s->ring_mem);
    // the step's buffers return to the context's cache under streams about to
    // be destroyed: release them first, then hand cached blocks to the context
    s->prof.release();
    s->m_ring.release();
    s->plan_zero[0].release();  // allocated on side_s / side_alt_s
    s->plan_zero[1].release();
    for (auto& tl : s->tail) tl.release();
    karma_ctx* ctx = s->ctx;
    hipStream_t prev = ctx->stream;
    if (prev == s->main_s || prev == s->side_s || prev == s->alt_s || prev == s->side_alt_s)
        ctx->stream = ctx->own_stream;
    if (s->side_alt_s) karma_stream_destroy(ctx, s->side_alt_s);
    if (s->side_s) karma_stream_destroy(ctx, s->side_s);
    if (s->alt_s) karma_stream_destroy(ctx, s->alt_s);
    if (s->main_s) karma_stream_destroy(ctx, s->main_s);
    delete s;
    return KARMA_OK;
}

}  // extern "C"
