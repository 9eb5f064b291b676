// graph_sets.hip — shared-read graph from (read, contig) records (gfx950).
//
// Replaces the pair counting of ReadGraph.from_contigs (karma/read_graph.py:31-49)
// on (read, contig) records (contig.py:24 readsets), DESIGN.md §4.  Output: the
// sorted unique (a << 32 | b, count) list over pairs a <= b of contigs sharing
// reads; the diagonal (a, a) counts |readset(a)|, the weight normaliser.
//
// A read's distinct contigs are "compact" when they lie in [m0, m0 + 3]: contigs that share reads are isoforms of one gene, which
// assemblers list next to each other (Trinity: TRINITY_DNx_cy_gz_i1, _i2, ...),
// so nearly every read is compact.  Such a read is one 15-bit code (m0, M),
// bit i of (1 | M << 1) marking contig m0 + i; dedup and order come for free.
// Other reads (wider spans) take the general path: sort network, dedup, every
// pair (p <= q).
//
//   partition   one pass over the records.  A block stages super-tiles of 8192
//               records in LDS.  Codes accumulate in a 64 KB LDS buffer across
//               super-tiles and are flushed bucket-major (code buckets of
//               2^bwc contigs) when full, so a code bucket's run in one flush is
//               ~300 codes.  General reads' pairs are written per super-tile,
//               bucket-major (pair buckets of 2^bw contigs).
//   code reduce per (code bucket, group of flushes): direct-mapped LDS
//               histogram over (m0, M) — one no-return LDS add per read.
//   pair reduce per (pair bucket, group of super-tiles): band counters for
//               b - a < 8 and an LDS hash table for the rest.
//   final       per pair bucket: sums the partials, expands the code histogram
//               into band pairs, merges the hash lists, writes the sorted list.
//   big reads   (> 8 records): separate generic path, merged at the end.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "karma_internal.h"

using namespace karma;

namespace {

#include "graph_device.h"

constexpr int kPT = 1024;                           // partition threads per block (16 waves)
constexpr int kSuperTile = 8192;                    // records per LDS-resident super-tile
constexpr int kPerWave = kSuperTile / (kPT / 64);   // 512 records per wave
constexpr int kCBuf = 16384;                        // codes buffered in LDS (64 KB)
constexpr int kMaxPartBlocks = 256;
constexpr int kMaxB = 512;                          // pair buckets
constexpr int kMaxBc = 128;                         // code buckets
constexpr int kMaxBwCompact = 10;                   // compact reads need 2^(bw+3) band counters <= kBand

struct Geo {
    int bw, bbits, B;  // pair buckets of 2^bw contigs; pair keys a_local << bbits | b
    int bwc, Bc;       // code buckets of 2^bwc contigs (bwc = 0: no compact path)
    int dbits;         // band width 2^dbits (-1: no band)
};

int make_geo(int64_t N, Geo* g) {
    KARMA_CHECK(N >= 1 && N <= (int64_t(1) << 24), KARMA_ERR_ARG, "n_contigs %lld out of range [1, 2^24]",
                (long long)N);
    int bbits = 1;
    while ((int64_t(1) << bbits) < N) ++bbits;
    auto nb = [&](int w) { return (N + (int64_t(1) << w) - 1) >> w; };
    int bw = 4;
    while (nb(bw) > 256 && bw < kMaxBwCompact) ++bw;
    while (nb(bw) > kMaxB) ++bw;
    KARMA_CHECK(bw + bbits <= 31, KARMA_ERR_ARG, "n_contigs too large for 32-bit pair keys");
    g->bw = bw;
    g->bbits = bbits;
    g->B = (int)nb(bw);
    g->dbits = bw + 3 <= 13 ? 3 : (bw <= 13 ? 13 - bw : -1);
    if (bw <= kMaxBwCompact) {
        g->bwc = bw + 2;  // 2^(bwc+3) histogram counters = 128 KB of LDS at most
        g->Bc = (int)nb(g->bwc);
    } else {
        g->bwc = 0;
        g->Bc = 0;
    }
    return KARMA_OK;
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr uint16_t kPadCode = 0xFFFF;               // code-run padding (codes are < 2^15)
constexpr uint32_t kFlushSlack = 4096;              // flush at a tile's end above kCBuf - this

struct PartArgs {
    const uint2* rec;
    int64_t A, chunk;
    int nst;
    Geo g;
    uint32_t N;
    // pair stream: per super-tile slot, bucket-major; st_base = -1 for a slot without pairs
    uint32_t* ent;
    int64_t region_cap;
    int64_t n_slots;
    int64_t* st_base;
    uint32_t* st_off;  // [B + 1][n_slots]
    // code stream: per flush, bucket-major; a block's codes go to [blk * code_region, ...)
    uint16_t* cent;
    int64_t code_region;
    int64_t* cf_base;
    uint32_t* cf_off;  // [max_flush][Bc + 1]
    unsigned* n_flush;
    int64_t max_flush;
    int* flags;  // 0 order, 1 contig range, 2 pair region full, 3 flush directory full
    int64_t* big_list;
    unsigned* big_n;
    unsigned long long* n_pairs;  // pair entries written (all blocks)
};

__global__ void __launch_bounds__(kPT) partition_kernel(PartArgs P) {
    __shared__ uint2 srec[kSuperTile + kMaxFast];
    __shared__ uint16_t wstart[kPT / 64][kPerWave];
    __shared__ uint32_t cbuf[kCBuf];
    __shared__ uint32_t hist[kMaxB + 1];
    __shared__ uint32_t toff[kMaxB + 1];
    __shared__ uint32_t cur[kMaxB];
    __shared__ uint32_t chist[kMaxBc + 1];
    __shared__ uint32_t ctoff[kMaxBc + 1];
    __shared__ uint32_t ccur[kMaxBc];
    __shared__ uint32_t tile_reads[2], cbuf_n;
    __shared__ int cap_fail;
    __shared__ int64_t base_s, fbase_s;
    __shared__ unsigned fidx_s;

    const Geo g = P.g;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t blk = blockIdx.x;
    const int64_t lo = blk * P.chunk, hi = min(P.A, lo + P.chunk);
    const uint32_t wmask = (1u << g.bw) - 1u, cmask = (1u << g.bwc) - 1u;
    const bool compact_ok = g.bwc > 0;
    for (int b = threadIdx.x; b <= g.B; b += kPT) hist[b] = 0;
    for (int b = threadIdx.x; b <= g.Bc; b += kPT) chist[b] = 0;
    for (int b = threadIdx.x; b < g.Bc; b += kPT) ccur[b] = 0;
    for (int b = threadIdx.x; b < g.B; b += kPT) cur[b] = 0;
    if (threadIdx.x == 0) {
        cbuf_n = 0;
        tile_reads[0] = tile_reads[1] = 0;
    }
    __syncthreads();
    int bad_order = 0, bad_contig = 0;
    int64_t used = 0, cused = 0;  // pair / code entries this block has written (uniform)

    // codes in cbuf -> the code stream (all threads call this): one flush is
    // the runs of the code buckets, each padded with kPadCode to a multiple of
    // 8 codes (16-byte aligned).  `staged`: counting-sort into the free srec
    // area, then 16-byte stores; otherwise scattered 2-byte stores.
    auto flush = [&](bool staged) {
        __syncthreads();
        const uint32_t n = cbuf_n;
        if (n == 0) return;
        if (wave == 0) {
            uint32_t c2 = 0;
            for (int base = 0; base < g.Bc; base += 64) {
                const uint32_t val = base + lane < g.Bc ? (chist[base + lane] + 7u) & ~7u : 0u;
                uint32_t x = val;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = __shfl_up(x, d);
                    if (lane >= d) x += y;
                }
                if (base + lane < g.Bc) ctoff[base + lane] = c2 + x - val;
                c2 += __shfl(x, 63);
            }
            if (lane == 0) {
                ctoff[g.Bc] = c2;
                const unsigned f = atomicAdd(P.n_flush, 1u);
                fidx_s = f;
                fbase_s = blk * P.code_region + cused;
                if ((int64_t)f < P.max_flush) P.cf_base[f] = fbase_s;
                else P.flags[3] = 1;
            }
        }
        __syncthreads();
        const unsigned f = fidx_s;
        const int64_t fb = fbase_s;
        const uint32_t total = ctoff[g.Bc];
        if ((int64_t)f < P.max_flush) {
            uint16_t* sorted = reinterpret_cast<uint16_t*>(srec);
            uint16_t* out = staged ? sorted : P.cent + fb;
            for (int b = threadIdx.x; b <= g.Bc; b += kPT) P.cf_off[(int64_t)f * (g.Bc + 1) + b] = ctoff[b];
            for (int b = threadIdx.x; b < g.Bc; b += kPT)
                for (uint32_t i = ctoff[b] + chist[b]; i < ctoff[b + 1]; ++i) out[i] = kPadCode;
            for (uint32_t i = threadIdx.x; i < n; i += kPT) {
                const uint32_t c = cbuf[i], m0 = c & 0xFFFFFFu, b = m0 >> g.bwc;
                const uint32_t pos = ctoff[b] + atomicAdd(&ccur[b], 1u);
                out[pos] = (uint16_t)(((m0 & cmask) << 3) | (c >> 24));
            }
            if (staged) {
                __syncthreads();
                u32x4* dst = reinterpret_cast<u32x4*>(P.cent + fb);
                const u32x4* src = reinterpret_cast<const u32x4*>(sorted);
                for (uint32_t i = threadIdx.x; i < total / 8; i += kPT) dst[i] = src[i];
            }
        }
        cused += total;
        __syncthreads();
        for (int b = threadIdx.x; b < g.Bc; b += kPT) {
            chist[b] = 0;
            ccur[b] = 0;
        }
        if (threadIdx.x == 0) cbuf_n = 0;
        __syncthreads();
    };

    // Register prefetch of a super-tile.  Wave w owns records [w0, w0 + 512)
    // of the tile: unit u, lane l holds records 128u + 2l and 128u + 2l + 1
    // (16 B), plus the record before the slice (its read-boundary carry); wave
    // 15 also fetches the 8 records after the tile (the halo).
    constexpr int PER = kPerWave / 128;
    const int w0 = wave * kPerWave;
    u32x4 nxt[PER];
    uint2 nxc = make_uint2(kEmpty, kEmpty), nxh = make_uint2(kEmpty, kEmpty);
    auto prefetch = [&](int64_t t0) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int64_t gi = t0 + w0 + 128 * u + 2 * lane;
            u32x4 v = {kEmpty, kEmpty, kEmpty, kEmpty};
            if (t0 < hi) {
                if (gi + 1 < P.A) {
                    v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(P.rec + gi));
                } else if (gi < P.A) {
                    const uint2 r = P.rec[gi];
                    v = u32x4{r.x, r.y, kEmpty, kEmpty};
                }
            }
            nxt[u] = v;
        }
        const int64_t gc = t0 + w0 - 1;
        nxc = t0 < hi && gc >= 0 && gc < P.A ? P.rec[gc] : make_uint2(kEmpty, kEmpty);
        if (wave == kPT / 64 - 1 && lane < kMaxFast) {
            const int64_t gh = t0 + kSuperTile + lane;
            nxh = t0 < hi && gh < P.A ? P.rec[gh] : make_uint2(kEmpty, kEmpty);
        }
    };
    prefetch(lo);
    int st = 0;
    for (int64_t ts = lo; ts < hi; ts += kSuperTile, ++st) {
        const int tn = (int)min<int64_t>(kSuperTile, hi - ts);
        // ---- read starts of this wave's slice, from registers (DPP wave_shr) ----
        // (records past tn are the following ones: they close the last read)
        uint32_t carry = nxc.x;
        const bool carry_valid = ts + w0 > 0;
        int ns = 0;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = 128 * u + 2 * lane;  // slice index of the lane's first record
            const uint32_t x0 = nxt[u].x, x1 = nxt[u].z;
            uint32_t p = (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)x1, 0x138, 0xF, 0xF, false);
            if (lane == 0) p = carry;  // lane 0 takes the previous unit's last record
            bool s0 = false, s1 = false;
            if (w0 + j < tn) {
                const bool hp = j > 0 || carry_valid;
                if (hp && p > x0) bad_order = 1;
                if (nxt[u].y >= P.N) bad_contig = 1;
                s0 = !hp || p != x0;
            }
            if (w0 + j + 1 < tn) {
                if (x0 > x1) bad_order = 1;
                if (nxt[u].w >= P.N) bad_contig = 1;
                s1 = x0 != x1;
            }
            const unsigned long long b0 = __ballot(s0), b1 = __ballot(s1), lower = (1ull << lane) - 1ull;
            const int pos = ns + __popcll(b0 & lower) + __popcll(b1 & lower);
            if (s0) wstart[wave][pos] = (uint16_t)j;
            if (s1) wstart[wave][pos + (s0 ? 1 : 0)] = (uint16_t)(j + 1);
            ns += __popcll(b0) + __popcll(b1);
            carry = (uint32_t)__builtin_amdgcn_readlane((int)x1, 63);
        }
        if (lane == 0 && ns) atomicAdd(&tile_reads[st & 1], (uint32_t)ns);
        if (threadIdx.x == 0) tile_reads[(st + 1) & 1] = 0;  // read at tile st - 1, next written at st + 1
        // ---- stage the slice in LDS (every wave is past the previous tile) ----
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = w0 + 128 * u + 2 * lane;
            srec[j] = make_uint2(nxt[u].x, nxt[u].y);
            srec[j + 1] = make_uint2(nxt[u].z, nxt[u].w);
        }
        if (wave == kPT / 64 - 1 && lane < kMaxFast) srec[kSuperTile + lane] = nxh;
        prefetch(ts + kSuperTile);
        __syncthreads();  // tile staged, read starts counted
        if (cbuf_n + tile_reads[st & 1] > (uint32_t)kCBuf) flush(false);  // rare: a tile of many short reads

        // ---- pass A: one lane per read: a code, or dedup + cache + count pairs ----
        int ng = 0;  // general reads of this wave, compacted to the front of wstart
        for (int kb = 0; kb < ns; kb += 64) {
            const int k = kb + lane;
            uint32_t code = kEmpty;
            bool gen = false;
            int j0 = 0;
            if (k < ns) {
                j0 = w0 + wstart[wave][k];
                uint2 r[kMaxFast + 1];
#pragma unroll
                for (int t = 0; t <= kMaxFast; ++t) r[t] = srec[j0 + t];
                const uint32_t rid = r[0].x;
                ReadSet rs;
                bool v = true;
                bool valid[kMaxFast];
                uint32_t mn = kEmpty, mx = 0;
#pragma unroll
                for (int t = 0; t < kMaxFast; ++t) {
                    v = v && (t == 0 || r[t].x == rid);
                    valid[t] = v;
                    rs.m[t] = v ? r[t].y : kEmpty;
                    if (v) {
                        mn = min(mn, r[t].y);
                        mx = max(mx, r[t].y);
                    }
                }
                if (v && r[kMaxFast].x == rid) {  // > 8 records: generic path
                    P.big_list[atomicAdd(P.big_n, 1u)] = ts + j0;
                } else if (compact_ok && mx - mn < 4u && mx < P.N) {
                    uint32_t M = 0;
#pragma unroll
                    for (int t = 0; t < kMaxFast; ++t)
                        if (valid[t]) M |= 1u << (rs.m[t] - mn);
                    code = (M >> 1) << 24 | mn;
                    atomicAdd(&chist[mn >> g.bwc], 1u);
                } else {
                    gen = true;
                    sort_dedup(rs);
                    // the read's slots now hold its sorted distinct contigs, then
                    // kEmpty (.x keeps the read id for the read boundary)
#pragma unroll
                    for (int p = 0; p < kMaxFast; ++p)
                        if (rs.keep[p]) srec[j0 + rs.rank[p]].y = rs.m[p];
#pragma unroll
                    for (int q = 1; q < kMaxFast; ++q)
                        if (valid[q] && (uint32_t)q >= rs.u) srec[j0 + q].y = kEmpty;
                    uint32_t run_b = kEmpty, run_n = 0;
#pragma unroll
                    for (int p = 0; p < kMaxFast; ++p) {
                        if (rs.keep[p]) {
                            const uint32_t b = rs.m[p] >> g.bw;
                            if (b != run_b) {
                                if (run_n && run_b < (uint32_t)g.B) atomicAdd(&hist[run_b], run_n);
                                run_b = b;
                                run_n = 0;
                            }
                            run_n += rs.u - rs.rank[p];
                        }
                    }
                    if (run_n && run_b < (uint32_t)g.B) atomicAdd(&hist[run_b], run_n);
                }
            }
            // wave-aggregated append of the codes; general reads compacted in place
            // (index ng + rank <= k: every lane has read its slot before these writes)
            const unsigned long long cb = __ballot(code != kEmpty);
            if (cb) {
                uint32_t at = 0;
                if (lane == 0) at = atomicAdd(&cbuf_n, (uint32_t)__popcll(cb));
                at = (uint32_t)__builtin_amdgcn_readfirstlane((int)at);
                if (code != kEmpty) cbuf[at + __popcll(cb & ((1ull << lane) - 1ull))] = code;
            }
            const unsigned long long gb = __ballot(gen);
            if (gen) wstart[wave][ng + __popcll(gb & ((1ull << lane) - 1ull))] = (uint16_t)(j0 - w0);
            ng += __popcll(gb);
        }
        const int64_t slot = blk * P.nst + st;
        if (!__syncthreads_or(ng > 0)) {  // no general read in this super-tile: no pairs
            if (threadIdx.x == 0) P.st_base[slot] = -1;
        } else {
            // ---- pairs of general reads: scan, region slice, directory ----
            if (wave == 0) {
                uint32_t c2 = 0;
                for (int base = 0; base < g.B; base += 64) {
                    const uint32_t val = base + lane < g.B ? hist[base + lane] : 0u;
                    uint32_t x = val;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t y = __shfl_up(x, d);
                        if (lane >= d) x += y;
                    }
                    if (base + lane < g.B) toff[base + lane] = c2 + x - val;
                    c2 += __shfl(x, 63);
                }
                if (lane == 0) {
                    toff[g.B] = c2;
                    cap_fail = used + (int64_t)c2 > P.region_cap;
                    if (cap_fail) P.flags[2] = 1;  // the host reruns with room for every entry
                    base_s = blk * P.region_cap + used;
                }
            }
            __syncthreads();
            const uint32_t total = toff[g.B];
            if (total == 0 || cap_fail) {
                if (threadIdx.x == 0) P.st_base[slot] = -1;
            } else {
                if (threadIdx.x == 0) P.st_base[slot] = base_s;
                for (int b = threadIdx.x; b <= g.B; b += kPT) P.st_off[(int64_t)b * P.n_slots + slot] = toff[b];
                // ---- pass B: write the pairs (m[p], m[q]), q >= p, of every general read ----
                uint32_t* dst = P.ent + base_s;
                for (int k = lane; k < ng; k += 64) {
                    const int j0 = w0 + wstart[wave][k];
                    uint2 r[kMaxFast];
#pragma unroll
                    for (int t = 0; t < kMaxFast; ++t) r[t] = srec[j0 + t];
                    const uint32_t rid = r[0].x;
                    uint32_t m[kMaxFast];
                    bool v = true;
                    uint32_t u = 0;
#pragma unroll
                    for (int t = 0; t < kMaxFast; ++t) {
                        v = v && (t == 0 || r[t].x == rid) && r[t].y != kEmpty;
                        m[t] = r[t].y;
                        u += v ? 1u : 0u;
                    }
                    // runs of one bucket: reserve, then write
                    uint32_t rb = kEmpty, rn = 0;
                    int rp0 = 0;
                    uint32_t base[kMaxFast];
#pragma unroll
                    for (int p = 0; p <= kMaxFast; ++p) {
                        const bool in = p < kMaxFast && (uint32_t)p < u;
                        const uint32_t b = in ? (m[p] >> g.bw) : kEmpty;
                        if (p == kMaxFast || (in && b != rb)) {
                            if (rn && rb < (uint32_t)g.B) {
                                uint32_t pos = toff[rb] + atomicAdd(&cur[rb], rn);
#pragma unroll
                                for (int q = 0; q < kMaxFast; ++q) {
                                    if (q >= rp0 && q < p && (uint32_t)q < u) {
                                        base[q] = pos;
                                        pos += u - q;
                                    }
                                }
                            }
                            if (in) {
                                rb = b;
                                rn = 0;
                                rp0 = p;
                            }
                        }
                        if (in) rn += u - p;
                    }
#pragma unroll
                    for (int p = 0; p < kMaxFast; ++p) {
                        if ((uint32_t)p >= u || (m[p] >> g.bw) >= (uint32_t)g.B) continue;
                        const uint32_t hk = (m[p] & wmask) << g.bbits;
#pragma unroll
                        for (int q = p; q < kMaxFast; ++q)
                            if ((uint32_t)q < u) dst[base[p] + (q - p)] = hk | m[q];
                    }
                }
            }
            if (total) used += total;
            __syncthreads();  // pass B done with srec, toff and cur
            for (int b = threadIdx.x; b < g.B; b += kPT) {
                hist[b] = 0;
                cur[b] = 0;
            }
        }
        if (cbuf_n > (uint32_t)kCBuf - kFlushSlack) flush(true);  // srec is free until the next tile
    }
    flush(true);
    if (threadIdx.x == 0 && used) atomicAdd(P.n_pairs, (unsigned long long)used);
    // slots of this block past its last super-tile (chunk shorter than nst)
    for (int s2 = st + threadIdx.x; s2 < P.nst; s2 += kPT) P.st_base[blk * P.nst + s2] = -1;
    if (bad_order) P.flags[0] = 1;
    if (bad_contig) P.flags[1] = 1;
}

// ---- run streams ------------------------------------------------------------------
// A reduce block reads the runs of one bucket from a range of slots (super-tiles
// or flushes).  Each wave takes batches of 64 runs (lane i holds run i) and
// reads them as one stream of T entries, 64 consecutive entries per load; the
// runs a window of 64 overlaps are found with wave-uniform (scalar) loops over
// the lanes' run table, and kWin windows are in flight before they are counted.
constexpr int kWin = 16;

template <typename T, typename Bounds, typename Count>
__device__ __forceinline__ void stream_runs(const T* __restrict__ data, int64_t r_lo, int64_t r_hi, int threads,
                                            Bounds bounds, Count count, bool* stop) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t r0 = r_lo + (int64_t)wave * 64; r0 - (int64_t)wave * 64 < r_hi; r0 += (int64_t)threads) {
        const int64_t r = r0 + lane;
        int64_t beg = 0;
        uint32_t len = 0;
        if (r < r_hi) bounds(r, &beg, &len);
        uint32_t incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if (lane >= d) incl += y;
        }
        const uint32_t excl = incl - len;
        const int64_t roff = beg - (int64_t)excl;  // element j of run r: data[roff + j]
        const uint32_t Tn = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        int rlo = 0;
        for (uint32_t j0 = 0; j0 < Tn; j0 += 64u * kWin) {
            T e[kWin];
#pragma unroll
            for (int u = 0; u < kWin; ++u) {
                const uint32_t w0 = j0 + 64u * u, j = w0 + lane;
                if (w0 >= Tn) continue;  // uniform
                while (rlo < 63 && (uint32_t)__builtin_amdgcn_readlane((int)incl, rlo) <= w0) ++rlo;
                int64_t off = 0;
                for (int rr = rlo; rr < 64; ++rr) {
                    const uint32_t ex = (uint32_t)__builtin_amdgcn_readlane((int)excl, rr);
                    if (ex >= w0 + 64u) break;
                    const int64_t o = readlane64(roff, rr);
                    if (j >= ex) off = o;
                }
                if (j < Tn) e[u] = data[off + j];
            }
#pragma unroll
            for (int u = 0; u < kWin; ++u)
                if (j0 + 64u * u + lane < Tn) count(e[u]);
        }
        if (__syncthreads_or(*stop)) return;
    }
}

// ---- code reduce --------------------------------------------------------------------
constexpr int kCRT = 1024;
constexpr int kHistMax = 1 << (kMaxBwCompact + 2 + 3);  // 32768 counters (128 KB)

// One block per (code bucket, group of flushes): histogram of (m0_local, M).
__global__ void __launch_bounds__(kCRT) code_reduce_kernel(const uint16_t* __restrict__ cent,
                                                           const int64_t* __restrict__ cf_base,
                                                           const uint32_t* __restrict__ cf_off, int64_t n_flush,
                                                           int Bc, int bwc, int n_cg, int64_t per_group,
                                                           uint32_t* __restrict__ part_ch) {
    __shared__ uint32_t h[kHistMax];
    const int bucket = blockIdx.x / n_cg, grp = blockIdx.x % n_cg;
    const int hn = 1 << (bwc + 3);
    for (int i = threadIdx.x; i < hn; i += kCRT) h[i] = 0;
    __syncthreads();
    const int64_t f_lo = (int64_t)grp * per_group, f_hi = min(n_flush, f_lo + per_group);
    bool stop = false;
    // runs are 16-byte aligned and padded: stream them as vectors of 8 codes
    auto add = [&](uint32_t c) {
        if (c != kPadCode) __hip_atomic_fetch_add(&h[c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    stream_runs(
        reinterpret_cast<const u32x4*>(cent), f_lo, f_hi, kCRT,
        [&](int64_t f, int64_t* beg, uint32_t* len) {
            const uint32_t* o = cf_off + f * (Bc + 1) + bucket;
            *beg = (cf_base[f] + o[0]) >> 3;
            *len = (o[1] - o[0]) >> 3;
        },
        [&](const u32x4 v) {
            add(v.x & 0xFFFFu), add(v.x >> 16), add(v.y & 0xFFFFu), add(v.y >> 16);
            add(v.z & 0xFFFFu), add(v.z >> 16), add(v.w & 0xFFFFu), add(v.w >> 16);
        },
        &stop);
    __syncthreads();
    uint32_t* out = part_ch + (int64_t)blockIdx.x * hn;
    for (int i = threadIdx.x; i < hn; i += kCRT) out[i] = h[i];
}

// ---- pair reduce --------------------------------------------------------------------
// A pair (a, b), b >= a, of a bucket is counted in one of two LDS structures:
//   band   dense counters band[a_local * D + (b - a)] for b - a < D = 2^dbits
//   hash   open addressing (key = a_local << bbits | b) for the other pairs.
constexpr int kRT = 1024;               // pair-reduce threads (16 waves)
constexpr int kGroup = 4096;            // super-tile slots per pair-reduce block
constexpr int kBand = 8192;             // band counters per bucket (32 KB)
constexpr int kHashR = 4096;            // hash slots per pair-reduce block
constexpr int kHashF = 8192;            // hash slots per final (per-bucket) block
constexpr int kFT = 1024;               // final-kernel threads
constexpr int kSlotCap = kBand + kHashF;  // output pairs per bucket, at most

template <int CAP, int THREADS>
struct HTab {
    uint32_t* keys;
    uint32_t* vals;
    int* nuniq;
    __device__ void init() {
        for (int t = threadIdx.x; t < CAP; t += THREADS) {
            keys[t] = kEmpty;
            vals[t] = 0;
        }
        if (threadIdx.x == 0) *nuniq = 0;
    }
    // false when CAP slots were probed without room (callers flag overflow)
    __device__ __forceinline__ bool insert(uint32_t key, uint32_t c) {
        uint32_t h = hash32(key) & (CAP - 1);
        for (int probe = 0; probe < CAP; ++probe) {
            const uint32_t k = __hip_atomic_load(&keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (k == key) {
                atomicAdd(&vals[h], c);
                return true;
            }
            if (k == kEmpty) {
                const uint32_t old = atomicCAS(&keys[h], kEmpty, key);
                if (old == kEmpty || old == key) {
                    if (old == kEmpty) atomicAdd(nuniq, 1);
                    atomicAdd(&vals[h], c);
                    return true;
                }
            }
            h = (h + 1) & (CAP - 1);
        }
        return false;
    }
    // occupied slots to the front; returns their number (all threads)
    __device__ int compact(int* cnt) {
        if (threadIdx.x == 0) *cnt = 0;
        __syncthreads();
        uint32_t my_k[CAP / THREADS], my_v[CAP / THREADS];
#pragma unroll
        for (int u = 0; u < CAP / THREADS; ++u) {
            my_k[u] = keys[u * THREADS + threadIdx.x];
            my_v[u] = vals[u * THREADS + threadIdx.x];
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < CAP / THREADS; ++u) {
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

// One block per (pair bucket, group of kGroup super-tile slots).  Output: the
// group's dense band counters and its compacted hash list.
__global__ void __launch_bounds__(kRT) pair_reduce_kernel(
    const uint32_t* __restrict__ ent, const int64_t* __restrict__ st_base, const uint32_t* __restrict__ st_off,
    int64_t n_slots, int n_groups, int bw, int bbits, int dbits, uint32_t* __restrict__ part_band,
    uint32_t* __restrict__ part_keys, uint32_t* __restrict__ part_cnt, int* __restrict__ part_n,
    uint8_t* __restrict__ overflow) {
    __shared__ uint32_t band[kBand];
    __shared__ uint32_t hkeys[kHashR];
    __shared__ uint32_t hvals[kHashR];
    __shared__ int nuniq, cnt, ovf;
    HTab<kHashR, kRT> t{hkeys, hvals, &nuniq};
    const int bucket = blockIdx.x / n_groups, grp = blockIdx.x % n_groups;
    const int band_n = dbits >= 0 ? (1 << (bw + dbits)) : 0;
    const uint32_t D = dbits >= 0 ? (1u << dbits) : 0u;
    t.init();
    for (int i = threadIdx.x; i < band_n; i += kRT) band[i] = 0;
    if (threadIdx.x == 0) ovf = 0;
    __syncthreads();
    const int64_t s_lo = (int64_t)grp * kGroup, s_hi = min(n_slots, s_lo + kGroup);
    const uint32_t bmask = (1u << bbits) - 1u, abase = (uint32_t)bucket << bw;
    bool full = false;
    stream_runs(
        ent, s_lo, s_hi, kRT,
        [&](int64_t r, int64_t* beg, uint32_t* len) {
            const int64_t sb = st_base[r];
            if (sb < 0) return;
            const uint32_t o0 = st_off[(int64_t)bucket * n_slots + r], o1 = st_off[(int64_t)(bucket + 1) * n_slots + r];
            *beg = sb + o0;
            *len = o1 - o0;
        },
        [&](const uint32_t e) {
            const uint32_t al = e >> bbits, d = (e & bmask) - (abase + al);
            if (d < D)
                __hip_atomic_fetch_add(&band[(al << dbits) | d], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else
                full |= !t.insert(e, 1u);
            if (nuniq > kHashR - kHashR / 8) full = true;  // early out: the bucket goes generic
        },
        &full);
    if (full) ovf = 1;
    __syncthreads();
    if (ovf) {
        if (threadIdx.x == 0) overflow[bucket] = 1;
        return;
    }
    const int64_t sl = blockIdx.x;
    uint32_t* pb = part_band + sl * (int64_t)kBand;
    for (int i = threadIdx.x; i < band_n; i += kRT) pb[i] = band[i];
    const int n = t.compact(&cnt);
    uint32_t* pk = part_keys + sl * (int64_t)kHashR;
    uint32_t* pc = part_cnt + sl * (int64_t)kHashR;
    for (int i = threadIdx.x; i < n; i += kRT) {
        pk[i] = hkeys[i];
        pc[i] = hvals[i];
    }
    if (threadIdx.x == 0) part_n[sl] = n;
}

// Summed code histogram entry gi = (m0 << 3 | M), m0 a global contig index.
__device__ __forceinline__ uint32_t code_count(const uint32_t* __restrict__ part_ch, int n_cg, int bw, int bwc,
                                               int gi) {
    const int bc = gi >> (bwc + 3), i = gi & ((8 << bwc) - 1);
    const int hn = 8 << bwc;
    uint32_t k = 0;
    for (int g = 0; g < n_cg; ++g) k += part_ch[((int64_t)bc * n_cg + g) * hn + i];
    return k;
}

// One block per pair bucket: sum the groups' bands, add the compact reads'
// pairs, merge the hash lists, and write the bucket's pairs sorted by (a, b).
// Band pairs and hash pairs are disjoint (b - a < D vs >= D); a pair's output
// position is its rank in its own sorted list plus the number of smaller keys
// in the other one.
__global__ void __launch_bounds__(kFT) final_kernel(
    int n_groups, int n_cg, int bw, int bbits, int dbits, int bwc, const uint32_t* __restrict__ part_band,
    const uint32_t* __restrict__ part_ch, const uint32_t* __restrict__ part_keys,
    const uint32_t* __restrict__ part_cnt, const int* __restrict__ part_n, uint64_t* __restrict__ out_keys,
    int64_t* __restrict__ out_counts, int64_t* __restrict__ out_n, uint8_t* __restrict__ overflow) {
    __shared__ uint32_t bsum[kBand];
    __shared__ uint32_t bpos[kBand + 1];
    __shared__ uint32_t hkeys[kHashF];
    __shared__ uint32_t hvals[kHashF];
    __shared__ uint32_t wsum[kFT / 64];
    __shared__ int nuniq, cnt;
    const int bucket = blockIdx.x;
    if (overflow[bucket]) return;  // generic path
    HTab<kHashF, kFT> t{hkeys, hvals, &nuniq};
    const int band_n = dbits >= 0 ? (1 << (bw + dbits)) : 0;
    t.init();
    for (int i = threadIdx.x; i < band_n; i += kFT) {
        uint32_t v = 0;
        for (int gi = 0; gi < n_groups; ++gi) v += part_band[((int64_t)bucket * n_groups + gi) * kBand + i];
        bsum[i] = v;
    }
    __syncthreads();
    // compact reads: a code (m0, M) with count k adds k to every pair
    // (m0 + i, m0 + j), i <= j, of its contigs; this bucket takes the pairs
    // with m0 + i inside it, from codes with m0 in [start - 3, end)
    if (n_cg > 0) {
        const int first = bucket > 0 ? -24 : 0;  // 3 contigs x 8 codes before the bucket
        for (int i = first + (int)threadIdx.x; i < (8 << bw); i += kFT) {
            const uint32_t k = code_count(part_ch, n_cg, bw, bwc, (bucket << (bw + 3)) + i);
            if (!k) continue;
            const int m0l = i >> 3;  // may be -3..-1
            const uint32_t bits = 1u | ((uint32_t)i & 7u) << 1;
#pragma unroll
            for (int i1 = 0; i1 < 4; ++i1) {
                if (!(bits >> i1 & 1u) || m0l + i1 < 0 || m0l + i1 >= (1 << bw)) continue;
#pragma unroll
                for (int j1 = i1; j1 < 4; ++j1)
                    if (bits >> j1 & 1u) atomicAdd(&bsum[(m0l + i1) << dbits | (j1 - i1)], k);
            }
        }
        __syncthreads();
    }
    for (int gi = 0; gi < n_groups; ++gi) {
        const int64_t sl = (int64_t)bucket * n_groups + gi;
        const int n = part_n[sl];
        bool full = false;
        for (int i = threadIdx.x; i < n; i += kFT)
            full |= !t.insert(part_keys[sl * kHashR + i], part_cnt[sl * kHashR + i]);
        if (__syncthreads_or(full)) {
            if (threadIdx.x == 0) overflow[bucket] = 1;
            return;
        }
    }
    const int nh = t.compact(&cnt);
    int p2 = 1;
    while (p2 < nh) p2 <<= 1;
    for (int i = nh + threadIdx.x; i < p2; i += kFT) {
        hkeys[i] = kEmpty;
        hvals[i] = 0;
    }
    __syncthreads();
    if (nh > 1) lds_bitonic(hkeys, hvals, p2);
    // exclusive scan of the band's nonzero flags (consecutive slots per thread)
    const int per = (band_n + kFT - 1) / kFT;
    const int i0 = threadIdx.x * per;
    uint32_t mine = 0;
    for (int i = i0; i < min(band_n, i0 + per); ++i) mine += bsum[i] != 0;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t x = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    uint32_t wb = 0;
    for (int w = 0; w < wave; ++w) wb += wsum[w];
    uint32_t run = wb + x - mine;
    for (int i = i0; i < min(band_n, i0 + per); ++i) {
        bpos[i] = run;
        run += bsum[i] != 0;
    }
    if (threadIdx.x == kFT - 1) bpos[band_n] = run;
    __syncthreads();
    const uint32_t nb = bpos[band_n];
    const uint32_t bmask = (1u << bbits) - 1u;
    const uint64_t abase = (uint64_t)bucket << bw;
    uint64_t* ok = out_keys + (int64_t)bucket * kSlotCap;
    int64_t* oc = out_counts + (int64_t)bucket * kSlotCap;
    for (int i = threadIdx.x; i < band_n; i += kFT) {
        if (!bsum[i]) continue;
        const uint32_t al = (uint32_t)i >> dbits, b = (uint32_t)abase + al + ((uint32_t)i & ((1u << dbits) - 1u));
        const uint32_t key = (al << bbits) | b;
        int lo = 0, hi = nh;  // hash keys below key
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (hkeys[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        const uint32_t pos = bpos[i] + lo;
        ok[pos] = ((abase + al) << 32) | b;
        oc[pos] = bsum[i];
    }
    for (int j = threadIdx.x; j < nh; j += kFT) {
        const uint32_t k = hkeys[j], al = k >> bbits;
        const uint32_t below = band_n ? bpos[min((int)((al + 1) << dbits), band_n)] : 0u;
        const uint32_t pos = j + below;
        ok[pos] = ((abase + al) << 32) | (k & bmask);
        oc[pos] = hvals[j];
    }
    if (threadIdx.x == 0) out_n[bucket] = nb + nh;
}

// ---- overflow fallback: every pair of one bucket as (key, count), generic sort ----
__global__ void bucket_widen_kernel(const uint32_t* __restrict__ ent, const int64_t* __restrict__ st_base,
                                    const uint32_t* __restrict__ st_off, int64_t n_slots, int bucket, int bw,
                                    int bbits, const uint32_t* __restrict__ part_ch, int n_cg, int bwc,
                                    uint64_t* __restrict__ out_k, int64_t* __restrict__ out_c,
                                    unsigned long long* __restrict__ n_out, int count_only) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t abase = (uint64_t)bucket << bw;
    unsigned long long n = 0, at = 0;
    for (int pass = count_only ? 1 : 0; pass < 2; ++pass) {
        // pass 0 counts this thread's pairs, pass 1 emits (or only counts)
        auto emit = [&](uint64_t key, int64_t c) {
            if (pass == 0 || count_only) {
                ++n;
            } else {
                out_k[at] = key;
                out_c[at] = c;
                ++at;
            }
        };
        if (pass == 1 && !count_only) {
            if (!n) return;
            at = atomicAdd(n_out, n);
        }
        if (t < n_slots && st_base[t] >= 0) {  // pair entries of slot t
            const int64_t beg = st_base[t] + st_off[(int64_t)bucket * n_slots + t];
            const uint32_t len = st_off[(int64_t)(bucket + 1) * n_slots + t] - st_off[(int64_t)bucket * n_slots + t];
            for (uint32_t i = 0; i < len; ++i) {
                const uint32_t k = ent[beg + i];
                emit(((abase + (k >> bbits)) << 32) | (k & ((1u << bbits) - 1u)), 1);
            }
        }
        const int64_t ci = t - (bucket > 0 ? 24 : 0);  // code index relative to the bucket start
        if (n_cg > 0 && t < (8 << bw) + (bucket > 0 ? 24 : 0)) {  // compact reads with m0 = start + (ci >> 3)
            const uint32_t k = code_count(part_ch, n_cg, bw, bwc, (int)((int64_t)(bucket << (bw + 3)) + ci));
            if (k) {
                const int64_t m0 = (int64_t)abase + (ci >> 3);
                const uint32_t bits = 1u | ((uint32_t)ci & 7u) << 1;
                for (int i1 = 0; i1 < 4; ++i1)
                    for (int j1 = i1; j1 < 4; ++j1)
                        if ((bits >> i1 & 1u) && (bits >> j1 & 1u) && m0 + i1 >= (int64_t)abase &&
                            m0 + i1 < (int64_t)abase + (1 << bw))
                            emit(((uint64_t)(m0 + i1) << 32) | (uint64_t)(m0 + j1), k);
            }
        }
    }
    if (count_only && n) atomicAdd(n_out, n);
}

// big reads (> 8 records): pair keys, one thread per read, O(m^3) dedup
__global__ void big_pairs_kernel(const uint2* __restrict__ rec, int64_t A, const int64_t* __restrict__ big_list,
                                 int64_t n_big, uint32_t N, uint64_t* __restrict__ out,
                                 unsigned long long* __restrict__ n_out, int count_only) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_big) return;
    unsigned long long c = 0;
    read_pairs_slow(rec, A, big_list[k], [&](uint32_t a, uint32_t b) {
        if (b >= N) return;
        if (count_only) ++c;
        else out[atomicAdd(n_out, 1ull)] = ((uint64_t)a << 32) | b;
    });
    if (count_only && c) atomicAdd(n_out, c);
}

__global__ void fill_ones_i64_kernel(int64_t* __restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = 1;
}

__global__ void assemble2_kernel(const uint64_t* const* __restrict__ src_k, const int64_t* const* __restrict__ src_c,
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

__global__ void fill_ptrs2_kernel(const uint64_t* base_k, const int64_t* base_c, int64_t n, int64_t stride,
                                  const uint64_t** pk, const int64_t** pc) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b < n) {
        pk[b] = base_k + b * stride;
        pc[b] = base_c + b * stride;
    }
}

int grid_n(int64_t n, int block = 256) { return (int)std::max<int64_t>(1, ceil_div(n, block)); }

int scan_excl_i64(karma_ctx* ctx, const int64_t* in, int64_t* out, int64_t n) {
    size_t tb = 0;
    KARMA_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, n, ctx->stream));
    DevArray<uint8_t> tmp;
    KARMA_TRY(tmp.alloc(ctx, tb));
    KARMA_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.ptr, tb, in, out, n, ctx->stream));
    return KARMA_OK;
}

}  // namespace

namespace karma {

// Records (grouped by read, 16-byte aligned) -> sorted unique (a<<32|b, count).
int records_to_pairs_sets(karma_ctx* ctx, const uint2* rec, int64_t A, int64_t N, karma_pairs* out) {
    Geo g;
    KARMA_TRY(make_geo(N, &g));
    const int B = g.B;
    const int64_t nblk = std::max<int64_t>(1, std::min<int64_t>(kMaxPartBlocks, ceil_div(A, kSuperTile)));
    const int64_t chunk = ceil_div(ceil_div(std::max<int64_t>(A, 1), nblk), kSuperTile) * kSuperTile;
    const int64_t nb = std::max<int64_t>(1, ceil_div(A, chunk));
    const int nst = (int)(chunk / kSuperTile);
    const int64_t n_slots = nb * nst;
    // <= 2 flushes per super-tile (before pass A when a tile of short reads would
    // not fit, and at its end) + the last; codes <= reads <= records, plus < 8
    // codes of padding per run of a flush
    const int64_t max_flush = nb * (2 * nst + 1);
    const int64_t code_region = chunk + (int64_t)(2 * nst + 1) * 8 * g.Bc;
    DevArray<int64_t> st_base, big_list, cf_base;
    DevArray<uint32_t> st_off, ent, cf_off;
    DevArray<uint16_t> cent;
    DevArray<int> flags;
    DevArray<unsigned> counters;  // 0 big reads, 1 flushes
    DevArray<unsigned long long> n_pairs;
    KARMA_TRY(st_base.alloc(ctx, n_slots));
    KARMA_TRY(st_off.alloc(ctx, (int64_t)(B + 1) * n_slots));
    KARMA_TRY(flags.alloc(ctx, 4));
    KARMA_TRY(counters.alloc(ctx, 2));
    KARMA_TRY(n_pairs.alloc(ctx, 1));
    KARMA_TRY(big_list.alloc(ctx, A / (kMaxFast + 1) + 1));
    if (g.Bc > 0) {
        KARMA_TRY(cent.alloc(ctx, nb * code_region));
        KARMA_TRY(cf_base.alloc(ctx, max_flush));
        KARMA_TRY(cf_off.alloc(ctx, max_flush * (g.Bc + 1)));
    }
    // Each block owns a region of the pair array.  Pairs (incl. the diagonal)
    // of general reads with <= 8 records are <= 4.5 per record; start at 1.5
    // per record and rerun once with the bound.
    int64_t region = chunk * 3 / 2 + 4;
    unsigned hc[2] = {0, 0};
    unsigned long long h_pairs = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        KARMA_TRY(ent.alloc(ctx, nb * region + 8));
        KARMA_HIP(hipMemsetAsync(flags.ptr, 0, 16, ctx->stream));
        KARMA_HIP(hipMemsetAsync(counters.ptr, 0, 8, ctx->stream));
        KARMA_HIP(hipMemsetAsync(n_pairs.ptr, 0, 8, ctx->stream));
        if (A > 0) {
            PartArgs P{rec, A, chunk, nst, g, (uint32_t)N, ent.ptr, region, n_slots, st_base.ptr, st_off.ptr,
                       cent.ptr, code_region, cf_base.ptr, cf_off.ptr, counters.ptr + 1, max_flush, flags.ptr, big_list.ptr,
                       counters.ptr, n_pairs.ptr};
            KARMA_LAUNCH(ctx, "graph_partition", partition_kernel, nb, kPT, 0, P);
        } else {
            KARMA_HIP(hipMemsetAsync(st_base.ptr, 0xFF, n_slots * 8, ctx->stream));
        }
        int hf[4];
        KARMA_HIP(hipMemcpyAsync(hf, flags.ptr, 16, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(hc, counters.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(&h_pairs, n_pairs.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        KARMA_CHECK(!hf[0], KARMA_ERR_UNSORTED, "records are not grouped by read (read ids decrease)");
        KARMA_CHECK(!hf[1], KARMA_ERR_ARG, "a record's contig index is >= n_contigs (%lld)", (long long)N);
        KARMA_CHECK(!hf[3], KARMA_ERR_STATE, "code flush directory full");
        if (!hf[2]) break;
        KARMA_CHECK(attempt == 0, KARMA_ERR_STATE, "entry region capacity exceeded twice");
        region = chunk * 9 / 2 + 4;
    }
    const unsigned n_big = hc[0];
    const int64_t n_flush = hc[1];
    // code reduce: per (code bucket, group of flushes)
    int n_cg = 0;
    int64_t per_group = 1;
    DevArray<uint32_t> part_ch;
    if (g.Bc > 0 && n_flush > 0) {
        n_cg = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(512, g.Bc), ceil_div(n_flush, 32)));
        per_group = ceil_div(n_flush, n_cg);
        n_cg = (int)ceil_div(n_flush, per_group);
        KARMA_TRY(part_ch.alloc(ctx, (int64_t)g.Bc * n_cg * (int64_t(8) << g.bwc)));
        KARMA_LAUNCH(ctx, "graph_code_reduce", code_reduce_kernel, (int64_t)g.Bc * n_cg, kCRT, 0, cent.ptr,
                     cf_base.ptr, cf_off.ptr, n_flush, g.Bc, g.bwc, n_cg, per_group, part_ch.ptr);
    }
    // pair reduce: per (pair bucket, group of super-tile slots), then per bucket
    const int n_groups = h_pairs ? (int)std::max<int64_t>(1, ceil_div(n_slots, kGroup)) : 0;
    const int64_t nsl = (int64_t)B * n_groups;
    DevArray<uint64_t> slot_k;
    DevArray<int64_t> slot_c, n_per;
    DevArray<uint8_t> ovf;
    DevArray<uint32_t> part_b, part_k, part_c;
    DevArray<int> part_n;
    KARMA_TRY(slot_k.alloc(ctx, (int64_t)B * kSlotCap));
    KARMA_TRY(slot_c.alloc(ctx, (int64_t)B * kSlotCap));
    KARMA_TRY(n_per.alloc(ctx, B + 1));
    KARMA_TRY(ovf.alloc(ctx, B));
    KARMA_TRY(part_b.alloc(ctx, std::max<int64_t>(nsl, 1) * (int64_t)kBand));
    KARMA_TRY(part_k.alloc(ctx, nsl * (int64_t)kHashR));
    KARMA_TRY(part_c.alloc(ctx, nsl * (int64_t)kHashR));
    KARMA_TRY(part_n.alloc(ctx, nsl));
    KARMA_HIP(hipMemsetAsync(ovf.ptr, 0, B, ctx->stream));
    KARMA_HIP(hipMemsetAsync(n_per.ptr, 0, (B + 1) * 8, ctx->stream));
    if (nsl) KARMA_LAUNCH(ctx, "graph_pair_reduce", pair_reduce_kernel, nsl, kRT, 0, ent.ptr, st_base.ptr, st_off.ptr,
                 n_slots, n_groups, g.bw, g.bbits, g.dbits, part_b.ptr, part_k.ptr, part_c.ptr, part_n.ptr, ovf.ptr);
    KARMA_LAUNCH(ctx, "graph_bucket_final", final_kernel, B, kFT, 0, n_groups, n_cg, g.bw, g.bbits, g.dbits, g.bwc,
                 part_b.ptr, part_ch.ptr, part_k.ptr, part_c.ptr, part_n.ptr, slot_k.ptr, slot_c.ptr, n_per.ptr,
                 ovf.ptr);
    std::vector<uint8_t> hovf(B);
    KARMA_HIP(hipMemcpyAsync(hovf.data(), ovf.ptr, B, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    DevArray<const uint64_t*> pk;
    DevArray<const int64_t*> pc;
    KARMA_TRY(pk.alloc(ctx, B));
    KARMA_TRY(pc.alloc(ctx, B));
    KARMA_LAUNCH(ctx, "bucket_ptrs", fill_ptrs2_kernel, grid_n(B), 256, 0, slot_k.ptr, slot_c.ptr, (int64_t)B,
                 (int64_t)kSlotCap, pk.ptr, pc.ptr);
    std::vector<std::unique_ptr<DevArray<uint64_t>>> keep_k;
    std::vector<std::unique_ptr<DevArray<int64_t>>> keep_c;
    const int64_t widen_threads = std::max<int64_t>(n_slots, (int64_t(8) << g.bw) + 24);
    for (int b = 0; b < B; ++b) {
        if (!hovf[b]) continue;
        // generic path for a bucket whose distinct pairs exceed the LDS tables
        DevArray<unsigned long long> np;
        KARMA_TRY(np.alloc(ctx, 1));
        KARMA_HIP(hipMemsetAsync(np.ptr, 0, 8, ctx->stream));
        KARMA_LAUNCH(ctx, "bucket_widen", bucket_widen_kernel, grid_n(widen_threads, 64), 64, 0, ent.ptr,
                     st_base.ptr, st_off.ptr, n_slots, b, g.bw, g.bbits, part_ch.ptr, n_cg, g.bwc,
                     (uint64_t*)nullptr, (int64_t*)nullptr, np.ptr, 1);
        unsigned long long hp = 0;
        KARMA_HIP(hipMemcpyAsync(&hp, np.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        DevArray<uint64_t> wide;
        DevArray<int64_t> wc;
        KARMA_TRY(wide.alloc(ctx, hp));
        KARMA_TRY(wc.alloc(ctx, hp));
        KARMA_HIP(hipMemsetAsync(np.ptr, 0, 8, ctx->stream));
        KARMA_LAUNCH(ctx, "bucket_widen", bucket_widen_kernel, grid_n(widen_threads, 64), 64, 0, ent.ptr,
                     st_base.ptr, st_off.ptr, n_slots, b, g.bw, g.bbits, part_ch.ptr, n_cg, g.bwc, wide.ptr, wc.ptr,
                     np.ptr, 0);
        keep_k.emplace_back(new DevArray<uint64_t>());
        keep_c.emplace_back(new DevArray<int64_t>());
        int64_t nu = 0;
        KARMA_TRY(sort_reduce_pairs(ctx, wide.ptr, wc.ptr, nullptr, (int64_t)hp, 64, *keep_k.back(),
                                    *keep_c.back(), nullptr, &nu));
        const uint64_t* kp = keep_k.back()->ptr;
        const int64_t* cp = keep_c.back()->ptr;
        KARMA_HIP(hipMemcpyAsync(pk.ptr + b, &kp, sizeof kp, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(pc.ptr + b, &cp, sizeof cp, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(n_per.ptr + b, &nu, 8, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
    }
    DevArray<int64_t> dst;
    KARMA_TRY(dst.alloc(ctx, B + 1));
    KARMA_TRY(scan_excl_i64(ctx, n_per.ptr, dst.ptr, B + 1));
    int64_t U = 0;
    KARMA_HIP(hipMemcpyAsync(&U, dst.ptr + B, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    DevArray<uint64_t> mk;
    DevArray<int64_t> mc;
    const bool merge_big = n_big > 0;
    KARMA_TRY((merge_big ? mk : out->keys).alloc(ctx, U));
    KARMA_TRY((merge_big ? mc : out->counts).alloc(ctx, U));
    KARMA_LAUNCH(ctx, "bucket_assemble", assemble2_kernel, B, 256, 0, pk.ptr, pc.ptr, n_per.ptr, dst.ptr,
                 (merge_big ? mk : out->keys).ptr, (merge_big ? mc : out->counts).ptr);
    out->n = U;
    out->n_contigs = N;
    if (merge_big) {
        // pairs of reads with > 8 records, merged with the main list
        DevArray<unsigned long long> np;
        KARMA_TRY(np.alloc(ctx, 1));
        KARMA_HIP(hipMemsetAsync(np.ptr, 0, 8, ctx->stream));
        KARMA_LAUNCH(ctx, "graph_big_count", big_pairs_kernel, grid_n(n_big, 64), 64, 0, rec, A, big_list.ptr,
                     (int64_t)n_big, (uint32_t)N, (uint64_t*)nullptr, np.ptr, 1);
        unsigned long long hp = 0;
        KARMA_HIP(hipMemcpyAsync(&hp, np.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        DevArray<uint64_t> allk;
        DevArray<int64_t> allc;
        KARMA_TRY(allk.alloc(ctx, U + hp));
        KARMA_TRY(allc.alloc(ctx, U + hp));
        if (U) {
            KARMA_HIP(hipMemcpyAsync(allk.ptr, mk.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
            KARMA_HIP(hipMemcpyAsync(allc.ptr, mc.ptr, U * 8, hipMemcpyDeviceToDevice, ctx->stream));
        }
        KARMA_HIP(hipMemsetAsync(np.ptr, 0, 8, ctx->stream));
        KARMA_LAUNCH(ctx, "graph_big_pairs", big_pairs_kernel, grid_n(n_big, 64), 64, 0, rec, A, big_list.ptr,
                     (int64_t)n_big, (uint32_t)N, allk.ptr + U, np.ptr, 0);
        KARMA_LAUNCH(ctx, "fill_ones", fill_ones_i64_kernel, grid_n(hp), 256, 0, allc.ptr + U, (int64_t)hp);
        KARMA_TRY(sort_reduce_pairs(ctx, allk.ptr, allc.ptr, nullptr, U + (int64_t)hp, 64, out->keys, out->counts,
                                    nullptr, &out->n));
    }
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

}  // namespace karma
