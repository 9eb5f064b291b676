// consumers.hip — the read graph's consumers on the device.
//
// Reference (lmfaber/karma, networkx + Python) being replaced:
//   ReadGraph.get_unconnected_nodes / get_connected_nodes  karma/read_graph.py:150-172
//   ReadGraph.__calculate_node_weights                     karma/read_graph.py:174-190
//   ReadGraph.calculate_representative_sequences (weights) karma/read_graph.py:315-344
//   ReadGraph.edge_list (MCL stdin text)                   karma/read_graph.py:350-357
// as karma.py:255-395 uses them on ReadGraph(full_graph.subgraph(cluster)).
//
// A karma_adj holds a graph the way networkx iterates it: nodes in iteration
// order (position 0..n-1, each with an id into the caller's name table) and,
// per node, its neighbours (positions) and weights in adjacency-dict order.
// Every consumer is a function of that layout:
//   degree(u)        = len(G.adj[u])                     (all_neighbors, self-loop once)
//   node_weight(u)   = 0 + w_1 + w_2 + ... in G.adj[u] order   (f64, left to right)
//   edge_list        = for u in order: for v in G.adj[u] with pos(v) >= pos(u):
//                      "name(u) name(v) repr(w)", joined by '\n'
// The layouts networkx produces are rebuilt here:
//   karma_adj_from_edges  add_edge calls in a known order on pre-added nodes
//                         (adj[u] = incident edges in call order);
//   karma_adj_view        nx.Graph(G.subgraph(nodes)) — from_dict_of_dicts over the
//                         view: nodes in view order (the caller's: networkx walks
//                         the smaller of the filter set and G's nodes); each u's
//                         view neighbours L(u) in G.adj[u] order (FilterAdjacency
//                         filters a node's dict in place); the copy's adj[u] =
//                         neighbours before u by position, then the L(u) entries
//                         at or after u in L order;
//   karma_adj_keep        G.remove_nodes_from (orders kept).
// and the --rearrange aggregation (karma.py:103-118):
//   karma_adj_cross_sums  per subcluster pair (A, B), A < B, the edge weights
//                         between them summed in product(nodes_A, nodes_B) order.

#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "karma_internal.h"
#include "repr.h"

using namespace karma;

struct karma_adj {
    karma_ctx* ctx = nullptr;
    int64_t n = 0;               // nodes
    int64_t m = -1;              // adjacency entries (off[n]); -1 until read back
    int64_t m_cap = 0;           // entry capacity of nbr / w (an upper bound of m)
    DevArray<uint32_t> ids;      // n: name id per position
    DevArray<int64_t> off;       // n + 1
    DevArray<uint32_t> nbr;      // m: neighbour positions
    DevArray<double> w;          // m
    DevArray<uint8_t> text;      // edge_list bytes between the length query and the copy
    int64_t text_len = -1;
    const void* text_names = nullptr;
};

namespace {

__global__ void iota_u32_kernel(uint32_t* p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

int grid_of(int64_t n, int b = 256) { return (int)std::max<int64_t>(1, ceil_div(n, b)); }

// ---- from edges: entries (u, edge) sorted by u then edge --------------------
__global__ void edge_entries_kernel(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, int64_t E,
                                    const int64_t* __restrict__ slot, uint64_t* __restrict__ key,
                                    uint32_t* __restrict__ val, int* __restrict__ bad, uint32_t n) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const uint32_t x = a[e], y = b[e];
    if (x >= n || y >= n) {
        *bad = 1;
        return;
    }
    const int64_t s = slot[e];  // 2 entries, or 1 for a self-loop
    key[s] = (uint64_t)x << 32 | (uint64_t)e;
    val[s] = (uint32_t)e;
    if (x != y) {
        key[s + 1] = (uint64_t)y << 32 | (uint64_t)e;
        val[s + 1] = (uint32_t)e;
    }
}

__global__ void edge_slots_kernel(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, int64_t E,
                                  int64_t* __restrict__ width) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e <= E) width[e] = e < E ? (a[e] != b[e] ? 2 : 1) : 0;
}

__global__ void entries_fill_kernel(const uint64_t* __restrict__ key, const uint32_t* __restrict__ eidx, int64_t m,
                                    const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                    const double* __restrict__ w, uint32_t* __restrict__ nbr,
                                    double* __restrict__ wo, int64_t* __restrict__ cnt) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint32_t u = (uint32_t)(key[j] >> 32), e = eidx[j];
    nbr[j] = a[e] == u ? b[e] : a[e];
    wo[j] = w[e];
    atomicAdd(reinterpret_cast<unsigned long long*>(cnt + u), 1ull);
}

// ---- view -----------------------------------------------------------------
__global__ void posmap_kernel(const int64_t* __restrict__ order, int64_t k, int64_t n_src,
                              int32_t* __restrict__ pos, int* __restrict__ bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const int64_t u = order[i];
    if (u < 0 || u >= n_src) {
        *bad = 1;
        return;
    }
    if (atomicExch(pos + u, (int32_t)i) != -1) *bad = 2;  // a node twice
}

__global__ void view_count_kernel(const int64_t* __restrict__ order, int64_t k, const int64_t* __restrict__ off,
                                  const uint32_t* __restrict__ nbr, const int32_t* __restrict__ pos,
                                  int64_t* __restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > k) return;
    int64_t c = 0;
    if (i < k) {
        const int64_t u = order[i];
        for (int64_t j = off[u]; j < off[u + 1]; ++j) c += pos[nbr[j]] >= 0;
    }
    cnt[i] = c;
}

// key (node << 32 | rank) orders the copy's adjacency: neighbours before the
// node by position, then the rest in list order
__global__ void view_fill_kernel(const int64_t* __restrict__ order, int64_t k, const int64_t* __restrict__ off,
                                 const uint32_t* __restrict__ nbr, const double* __restrict__ w,
                                 const int32_t* __restrict__ pos, const int64_t* __restrict__ noff,
                                 uint64_t* __restrict__ key, uint32_t* __restrict__ x_out,
                                 double* __restrict__ w_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= k) return;
    const int64_t u = order[i];
    int64_t d = noff[i];
    uint32_t r = 0;
    for (int64_t j = off[u]; j < off[u + 1]; ++j) {
        const int32_t x = pos[nbr[j]];
        if (x < 0) continue;
        const uint32_t rank = (int64_t)x < i ? (uint32_t)x : (uint32_t)(k + r);
        key[d] = (uint64_t)i << 32 | rank;
        x_out[d] = (uint32_t)x;
        w_out[d] = w[j];
        ++d;
        ++r;
    }
}

// Within each node's segment the rank keys are distinct: an entry's place is
// the number of smaller keys in its segment (one thread per entry, grid-stride
// over the device-side entry count; O(d^2) per node of degree d).
__global__ void rank_scatter_kernel(const uint64_t* __restrict__ key, const int64_t* __restrict__ off, int64_t k,
                                    const uint32_t* __restrict__ x_in, const double* __restrict__ w_in,
                                    uint32_t* __restrict__ x_out, double* __restrict__ w_out) {
    const int64_t m = off[k];
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t kj = key[j];
        const int64_t i = (int64_t)(kj >> 32);
        int64_t r = 0;
        for (int64_t t = off[i]; t < off[i + 1]; ++t) r += key[t] < kj;
        x_out[off[i] + r] = x_in[j];
        w_out[off[i] + r] = w_in[j];
    }
}

__global__ void gather_ids_kernel(const int64_t* __restrict__ order, int64_t k, const uint32_t* __restrict__ ids_src,
                                  uint32_t* __restrict__ ids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) ids[i] = ids_src[order[i]];
}

// ---- keep -------------------------------------------------------------------
__global__ void keep_count_kernel(const uint8_t* __restrict__ keep, int64_t n, const int64_t* __restrict__ off,
                                  const uint32_t* __restrict__ nbr, int64_t* __restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    int64_t c = 0;
    if (i < n && keep[i])
        for (int64_t j = off[i]; j < off[i + 1]; ++j) c += keep[nbr[j]] != 0;
    cnt[i] = c;
}

__global__ void keep_fill_kernel(const uint8_t* __restrict__ keep, int64_t n, const int64_t* __restrict__ off,
                                 const uint32_t* __restrict__ nbr, const double* __restrict__ w,
                                 const int64_t* __restrict__ npos, const int64_t* __restrict__ ooff,
                                 const uint32_t* __restrict__ ids, uint32_t* __restrict__ nbr_out,
                                 double* __restrict__ w_out, uint32_t* __restrict__ ids_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !keep[i]) return;
    ids_out[npos[i]] = ids[i];
    int64_t d = ooff[i];  // entries of dropped nodes count 0, so the old-index scan is the new start
    for (int64_t j = off[i]; j < off[i + 1]; ++j) {
        const uint32_t v = nbr[j];
        if (!keep[v]) continue;
        nbr_out[d] = (uint32_t)npos[v];
        w_out[d] = w[j];
        ++d;
    }
}

__global__ void keep_off_kernel(const uint8_t* __restrict__ keep, int64_t n, const int64_t* __restrict__ npos,
                                const int64_t* __restrict__ ooff, int64_t* __restrict__ off) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) off[npos[n]] = ooff[n];
    else if (keep[i]) off[npos[i]] = ooff[i];
}

__global__ void u8_to_i64_kernel(const uint8_t* __restrict__ in, int64_t n, int64_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) out[i] = i < n ? (in[i] != 0) : 0;
}

// ---- consumers ----------------------------------------------------------------
__global__ void node_stats_kernel(const int64_t* __restrict__ off, const double* __restrict__ w, int64_t n,
                                  int64_t* __restrict__ deg, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s = 0.0;  // read_graph.py:183-187: 0 + w_1 + w_2 + ..., left to right
    for (int64_t j = off[i]; j < off[i + 1]; ++j) s = __dadd_rn(s, w[j]);
    out[i] = s;
    deg[i] = off[i + 1] - off[i];
}

// bytes of node i's lines, each with its '\n'
__global__ void edge_list_len_kernel(const int64_t* __restrict__ off, const uint32_t* __restrict__ nbr,
                                     const double* __restrict__ w, const uint32_t* __restrict__ ids, int64_t n,
                                     const int64_t* __restrict__ name_off, int64_t* __restrict__ len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    int64_t s = 0;
    if (i < n) {
        const uint32_t a = ids[i];
        const int64_t la = name_off[a + 1] - name_off[a];
        for (int64_t j = off[i]; j < off[i + 1]; ++j) {
            const uint32_t v = nbr[j];
            if ((int64_t)v < i) continue;  // G.edges(): each edge from its earlier end
            const uint32_t b = ids[v];
            s += la + 1 + (name_off[b + 1] - name_off[b]) + 1 + karma_repr::repr_f64(w[j], nullptr) + 1;
        }
    }
    len[i] = s;
}

__global__ void edge_list_write_kernel(const int64_t* __restrict__ off, const uint32_t* __restrict__ nbr,
                                       const double* __restrict__ w, const uint32_t* __restrict__ ids, int64_t n,
                                       const uint8_t* __restrict__ names, const int64_t* __restrict__ name_off,
                                       const int64_t* __restrict__ start, uint8_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint8_t* p = out + start[i];
    const uint32_t a = ids[i];
    for (int64_t j = off[i]; j < off[i + 1]; ++j) {
        const uint32_t v = nbr[j];
        if ((int64_t)v < i) continue;
        const uint32_t b = ids[v];
        for (int64_t t = name_off[a]; t < name_off[a + 1]; ++t) *p++ = names[t];
        *p++ = ' ';
        for (int64_t t = name_off[b]; t < name_off[b + 1]; ++t) *p++ = names[t];
        *p++ = ' ';
        char buf[karma_repr::kMaxRepr];
        const int r = karma_repr::repr_f64(w[j], buf);
        for (int t = 0; t < r; ++t) *p++ = (uint8_t)buf[t];
        *p++ = '\n';
    }
}

// ---- --rearrange: cross-subcluster weight sums (karma.py:103-118) ------------
// Entries u -> v with sub[u] < sub[v] (each undirected edge once, from the side
// in the earlier subcluster).  Keys: (A, B) and, inside a pair, (rank of u in
// A's list, rank of v in B's list) = itertools.product(nodes_A, nodes_B) order.
__global__ void cross_count_kernel(const int64_t* __restrict__ off, const uint32_t* __restrict__ nbr, int64_t n,
                                   const int32_t* __restrict__ sub, int64_t* __restrict__ cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    int64_t c = 0;
    if (i < n && sub[i] >= 0)
        for (int64_t j = off[i]; j < off[i + 1]; ++j) {
            const int32_t sv = sub[nbr[j]];
            c += sv > sub[i];
        }
    cnt[i] = c;
}

__global__ void cross_fill_kernel(const int64_t* __restrict__ off, const uint32_t* __restrict__ nbr,
                                  const double* __restrict__ w, int64_t n, const int32_t* __restrict__ sub,
                                  const int32_t* __restrict__ rank, const int64_t* __restrict__ start,
                                  uint64_t* __restrict__ pair_key, uint64_t* __restrict__ in_key,
                                  double* __restrict__ ew) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || sub[i] < 0) return;
    int64_t d = start[i];
    for (int64_t j = off[i]; j < off[i + 1]; ++j) {
        const uint32_t v = nbr[j];
        if (sub[v] <= sub[i]) continue;
        pair_key[d] = (uint64_t)(uint32_t)sub[i] << 32 | (uint32_t)sub[v];
        in_key[d] = (uint64_t)(uint32_t)rank[i] << 32 | (uint32_t)rank[v];
        ew[d] = w[j];
        ++d;
    }
}

__global__ void gather_u64_kernel(const uint32_t* __restrict__ idx, int64_t m, const uint64_t* __restrict__ in,
                                  uint64_t* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < m) out[j] = in[idx[j]];
}

__global__ void segment_heads_kernel(const uint64_t* __restrict__ key, int64_t m, int64_t* __restrict__ head) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j <= m) head[j] = j < m ? (j == 0 || key[j] != key[j - 1]) : 0;
}

// one thread per (A, B): 0 + w_1 + w_2 + ... in product order (karma.py:111-117)
// (and how many of those partial sums exceed the cutoff: the reference appends
// [A, B] once for each)
__global__ void cross_sum_kernel(const uint64_t* __restrict__ key, const uint32_t* __restrict__ idx,
                                 const double* __restrict__ ew, int64_t m, const int64_t* __restrict__ head,
                                 const int64_t* __restrict__ seg, double cutoff, uint64_t* __restrict__ out_key,
                                 double* __restrict__ out_sum, int64_t* __restrict__ out_n,
                                 int64_t* __restrict__ out_over) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m || !head[j]) return;
    double s = 0.0;
    int64_t t = j, over = 0;
    for (; t < m && key[t] == key[j]; ++t) {
        s = __dadd_rn(s, ew[idx[t]]);
        over += s > cutoff;
    }
    const int64_t o = seg[j];
    out_key[o] = key[j];
    out_sum[o] = s;
    out_n[o] = t - j;
    out_over[o] = over;
}

// ---- small views in one launch ------------------------------------------------
// karma.py's cluster loop (:255-282) copies a few dozen nodes per k-mer cluster;
// there the separate view / stats / text launches and their host round trips
// cost more than the reference's whole Python walk.  One block does the view,
// degrees, node weights and edge_list text of nx.Graph(G.subgraph(order)) and
// writes them straight into mapped pinned host memory: one launch, one sync.
constexpr int kSumT = 1024;     // threads: one per view node
constexpr int kSumHash = 2048;  // LDS hash slots (src position -> view index)
constexpr int kSumEnt = 4096;   // view adjacency entries held in LDS
constexpr int kSumNames = 16384;  // name bytes of the view's nodes in LDS
constexpr int kSumText = 24576;   // edge_list bytes composed in LDS

struct SumHeader {
    int32_t status;  // 0 done, 1 exceeds the one-block limits, 2 bad order
    int32_t pad;
    int64_t text_len;
};

// exclusive block scan (kSumT threads); *total for everyone
__device__ int64_t block_exscan(int64_t v, int64_t* wtot, int64_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    int64_t base = 0, all = 0;
    for (int w = 0; w < kSumT / 64; ++w) {
        const int64_t t = wtot[w];
        base += w < wave ? t : 0;
        all += t;
    }
    *total = all;
    __syncthreads();
    return base + x - v;
}

// The block's last act: every thread's results are out, then the status (the
// host polls it in mapped memory instead of waiting for the stream).
__device__ __forceinline__ void publish(SumHeader* hdr, int status) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(&hdr->status, status, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void __launch_bounds__(kSumT) view_summary_kernel(
    const int64_t* __restrict__ order, int k, int64_t n_src, const int64_t* __restrict__ off,
    const uint32_t* __restrict__ nbr, const double* __restrict__ w, const uint32_t* __restrict__ ids,
    const uint8_t* __restrict__ names, const int64_t* __restrict__ name_off, int with_text, int64_t text_cap,
    SumHeader* hdr, int32_t* __restrict__ deg_out, double* __restrict__ w_out, uint32_t* __restrict__ text_out) {
    __shared__ uint32_t hk[kSumHash];  // source position -> view index
    __shared__ uint16_t hv[kSumHash];
    __shared__ uint32_t ek[kSumEnt];   // copy-order key: x < i ? x : k + (rank in G.adj[u])
    __shared__ double ew[kSumEnt];     // weight
    __shared__ uint16_t ex[kSumEnt];   // neighbour's view index
    __shared__ int32_t se0[kSumT];     // node: first entry, degree, first text line, name in sname
    __shared__ int32_t sd[kSumT];
    __shared__ int32_t sl[kSumT + 1];
    __shared__ int32_t sn0[kSumT + 1];
    __shared__ int64_t snb[kSumT];     // node's name in the device name table
    __shared__ __attribute__((aligned(16))) uint8_t sname[kSumNames];
    __shared__ __attribute__((aligned(16))) uint8_t stext[kSumText];
    __shared__ int64_t wtot[kSumT / 64];
    __shared__ int bad;
    const int i = threadIdx.x;
    for (int t = i; t < kSumHash; t += kSumT) hk[t] = 0xFFFFFFFFu;
    if (i == 0) bad = 0;
    __syncthreads();
    auto lookup = [&](uint32_t key) -> int {
        uint32_t h = (key * 2654435761u) >> 21;  // 11 bits
        while (true) {
            const uint32_t c = hk[h];
            if (c == key) return hv[h];
            if (c == 0xFFFFFFFFu) return -1;
            h = (h + 1) & (kSumHash - 1);
        }
    };
    uint32_t u = 0;
    if (i < k) {
        const int64_t o = order[i];
        if (o < 0 || o >= n_src) {
            bad = 2;
        } else {
            u = (uint32_t)o;
            uint32_t h = (u * 2654435761u) >> 21;
            while (true) {
                const uint32_t c = atomicCAS(&hk[h], 0xFFFFFFFFu, u);
                if (c == 0xFFFFFFFFu) {
                    hv[h] = (uint16_t)i;
                    break;
                }
                if (c == u) {
                    bad = 2;  // a node twice
                    break;
                }
                h = (h + 1) & (kSumHash - 1);
            }
        }
    }
    __syncthreads();
    if (bad) {
        publish(hdr, bad);
        return;
    }
    const int64_t j0 = i < k ? off[u] : 0, j1 = i < k ? off[u + 1] : 0;
    int64_t nb0 = 0, nl = 0;
    if (with_text && i < k) {
        const uint32_t a = ids[u];
        nb0 = name_off[a];
        nl = name_off[a + 1] - nb0;
    }
    int64_t d = 0;
    for (int64_t j = j0; j < j1; ++j) d += lookup(nbr[j]) >= 0;
    int64_t m, NB;
    const int64_t e0 = block_exscan(d, wtot, &m);
    const int64_t n0 = block_exscan(nl, wtot, &NB);
    if (m > kSumEnt || NB > kSumNames) {
        publish(hdr, 1);
        return;
    }
    // this node's entries in copy order: neighbours before it by position, then
    // the rest in G.adj[u] order (from_dict_of_dicts over the view; karma_adj_view)
    {
        uint32_t r = 0;
        int64_t e = e0;
        for (int64_t j = j0; j < j1; ++j) {
            const int x = lookup(nbr[j]);
            if (x < 0) continue;
            const uint32_t key = x < i ? (uint32_t)x : (uint32_t)k + r;
            const double wj = w[j];
            int64_t p = e;  // insertion sort of the segment as it fills
            while (p > e0 && ek[p - 1] > key) {
                ek[p] = ek[p - 1];
                ew[p] = ew[p - 1];
                ex[p] = ex[p - 1];
                --p;
            }
            ek[p] = key;
            ew[p] = wj;
            ex[p] = (uint16_t)x;
            ++e;
            ++r;
        }
    }
    if (i < k) {
        double s = 0.0;  // read_graph.py:183-187: 0 + w_1 + w_2 + ..., left to right
        for (int64_t e = e0; e < e0 + d; ++e) s = __dadd_rn(s, ew[e]);
        deg_out[i] = (int32_t)d;
        w_out[i] = s;
        se0[i] = (int32_t)e0;
        sd[i] = (int32_t)d;
        sn0[i] = (int32_t)n0;
        snb[i] = nb0;
    }
    if (!with_text) {
        if (i == 0) hdr->text_len = -1;
        publish(hdr, 0);
        return;
    }
    if (i == 0) sn0[k] = (int32_t)NB;
    // G.edges(): each edge from its earlier end, i.e. the entries x >= i (keys
    // >= k: the tail of the node's segment), in order; one text line each
    int64_t nt = 0;
    for (int64_t e = e0; e < e0 + d; ++e) nt += ek[e] >= (uint32_t)k;
    int64_t NL;
    const int64_t l0 = block_exscan(nt, wtot, &NL);  // (its barriers order the stores above)
    if (i < k) sl[i] = (int32_t)l0;
    if (i == 0) sl[k] = (int32_t)NL;
    // the view's names into LDS: byte b of the concatenation, node by search
    for (int64_t b = i; b < NB; b += kSumT) {
        int lo = 0, hi = k;  // last node whose name starts at or before b
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (sn0[mid] <= b) lo = mid;
            else hi = mid;
        }
        sname[b] = names[snb[lo] + (b - sn0[lo])];
    }
    __syncthreads();
    // lines [q0, q1) of this thread, contiguous so one scan places them
    const int64_t per = (NL + kSumT - 1) / kSumT;
    const int64_t q0 = min(NL, per * i), q1 = min(NL, q0 + per);
    auto line_at = [&](int64_t q, int* node, int* ent) {
        int lo = 0, hi = k;  // last node whose lines start at or before q
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (sl[mid] <= q) lo = mid;
            else hi = mid;
        }
        // skip nodes without lines that share the start
        while (lo + 1 < k && sl[lo + 1] <= q) ++lo;
        const int nl_node = sl[lo + 1] - sl[lo];
        *node = lo;
        *ent = se0[lo] + sd[lo] - nl_node + (int)(q - sl[lo]);
    };
    int64_t len = 0;
    for (int64_t q = q0; q < q1; ++q) {
        int nd, e;
        line_at(q, &nd, &e);
        const int x = ex[e];
        len += (sn0[nd + 1] - sn0[nd]) + 1 + (sn0[x + 1] - sn0[x]) + 1 +
               karma_repr::parts_len(karma_repr::parts(ew[e])) + 1;
    }
    int64_t T;
    const int64_t t0 = block_exscan(len, wtot, &T);
    if (T > min<int64_t>(text_cap, kSumText)) {
        publish(hdr, 1);
        return;
    }
    {
        int64_t p = t0;
        for (int64_t q = q0; q < q1; ++q) {
            int nd, e;
            line_at(q, &nd, &e);
            const int x = ex[e];
            for (int t = sn0[nd]; t < sn0[nd + 1]; ++t) stext[p++] = sname[t];
            stext[p++] = ' ';
            for (int t = sn0[x]; t < sn0[x + 1]; ++t) stext[p++] = sname[t];
            stext[p++] = ' ';
            const karma_repr::Parts pr = karma_repr::parts(ew[e]);
            karma_repr::parts_write(pr, stext + p);
            p += karma_repr::parts_len(pr);
            stext[p++] = '\n';
        }
    }
    __syncthreads();
    const uint32_t* src = reinterpret_cast<const uint32_t*>(stext);
    for (int64_t t = i; t < (T + 3) / 4; t += kSumT) text_out[t] = src[t];
    if (i == 0) hdr->text_len = T ? T - 1 : 0;  // "\n".join: no newline after the last line
    publish(hdr, 0);
}

int scan_i64(karma_ctx* ctx, const int64_t* in, int64_t* out, int64_t n) {
    return scan_excl_i64(ctx, in, out, n);  // one look-back launch (sort.hip)
}

int read_i64(karma_ctx* ctx, const int64_t* dev, int64_t* host) {
    KARMA_HIP(hipMemcpyAsync(host, dev, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

int check_flag(karma_ctx* ctx, const int* dev, const char* what) {
    int h = 0;
    KARMA_HIP(hipMemcpyAsync(&h, dev, 4, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    KARMA_CHECK(h == 0, KARMA_ERR_ARG, "%s (code %d)", what, h);
    return KARMA_OK;
}

// copy n elements from host or device into a new device array
template <typename T>
int upload(karma_ctx* ctx, const T* src, int64_t n, int is_device, DevArray<T>& dst) {
    KARMA_TRY(dst.alloc(ctx, n ? n : 1));
    if (n)
        KARMA_HIP(hipMemcpyAsync(dst.ptr, src, n * sizeof(T), is_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                 ctx->stream));
    return KARMA_OK;
}

int ids_or_iota(karma_ctx* ctx, const uint32_t* ids, int64_t n, int is_device, DevArray<uint32_t>& dst) {
    if (ids) return upload(ctx, ids, n, is_device, dst);
    KARMA_TRY(dst.alloc(ctx, n ? n : 1));
    KARMA_LAUNCH(ctx, "adj_iota", iota_u32_kernel, grid_of(n), 256, 0, dst.ptr, n);
    return KARMA_OK;
}

}  // namespace

extern "C" {

int karma_adj_from_edges(karma_ctx* ctx, int64_t n, const uint32_t* ids, const uint32_t* a, const uint32_t* b,
                         const double* w, int64_t n_edges, int is_device, karma_adj** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && n >= 0 && n < (int64_t(1) << 32) && n_edges >= 0 && n_edges < (int64_t(1) << 32) &&
                    (n_edges == 0 || (a && b && w)),
                KARMA_ERR_ARG, "karma_adj_from_edges: bad arguments");
    auto g = std::make_unique<karma_adj>();
    g->ctx = ctx;
    g->n = n;
    KARMA_TRY(ids_or_iota(ctx, ids, n, is_device, g->ids));
    DevArray<uint32_t> da, db;
    DevArray<double> dw;
    KARMA_TRY(upload(ctx, a, n_edges, is_device, da));
    KARMA_TRY(upload(ctx, b, n_edges, is_device, db));
    KARMA_TRY(upload(ctx, w, n_edges, is_device, dw));
    DevArray<int64_t> width, slot, cnt;
    KARMA_TRY(width.alloc(ctx, n_edges + 1));
    KARMA_TRY(slot.alloc(ctx, n_edges + 1));
    KARMA_LAUNCH(ctx, "adj_edge_slots", edge_slots_kernel, grid_of(n_edges + 1), 256, 0, da.ptr, db.ptr, n_edges,
                 width.ptr);
    KARMA_TRY(scan_i64(ctx, width.ptr, slot.ptr, n_edges + 1));
    KARMA_TRY(read_i64(ctx, slot.ptr + n_edges, &g->m));
    const int64_t m = g->m;
    g->m_cap = m;
    DevArray<uint64_t> key, key2;
    DevArray<uint32_t> val, val2;
    DevArray<int> bad;
    KARMA_TRY(key.alloc(ctx, m ? m : 1));
    KARMA_TRY(key2.alloc(ctx, m ? m : 1));
    KARMA_TRY(val.alloc(ctx, m ? m : 1));
    KARMA_TRY(val2.alloc(ctx, m ? m : 1));
    KARMA_TRY(bad.alloc(ctx, 1));
    KARMA_HIP(hipMemsetAsync(bad.ptr, 0, 4, ctx->stream));
    if (n_edges)
        KARMA_LAUNCH(ctx, "adj_edge_entries", edge_entries_kernel, grid_of(n_edges), 256, 0, da.ptr, db.ptr, n_edges,
                     slot.ptr, key.ptr, val.ptr, bad.ptr, (uint32_t)n);
    KARMA_TRY(check_flag(ctx, bad.ptr, "edge endpoint >= n"));
    if (m) KARMA_TRY(radix_sort_u64(ctx, key.ptr, val.ptr, m, 64, key2.ptr, val2.ptr));  // stable (sort.hip)
    KARMA_TRY(cnt.alloc(ctx, n + 1));
    KARMA_HIP(hipMemsetAsync(cnt.ptr, 0, (n + 1) * 8, ctx->stream));
    KARMA_TRY(g->nbr.alloc(ctx, m ? m : 1));
    KARMA_TRY(g->w.alloc(ctx, m ? m : 1));
    if (m)
        KARMA_LAUNCH(ctx, "adj_fill", entries_fill_kernel, grid_of(m), 256, 0, key2.ptr, val2.ptr, m, da.ptr, db.ptr,
                     dw.ptr, g->nbr.ptr, g->w.ptr, cnt.ptr);
    KARMA_TRY(g->off.alloc(ctx, n + 1));
    KARMA_TRY(scan_i64(ctx, cnt.ptr, g->off.ptr, n + 1));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    *out = g.release();
    return KARMA_OK;
}

int karma_adj_from_lists(karma_ctx* ctx, int64_t n, const uint32_t* ids, const int64_t* off, const uint32_t* nbr,
                         const double* w, int is_device, karma_adj** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && off && n >= 0 && n < (int64_t(1) << 32), KARMA_ERR_ARG, "karma_adj_from_lists: bad arguments");
    auto g = std::make_unique<karma_adj>();
    g->ctx = ctx;
    g->n = n;
    KARMA_TRY(upload(ctx, off, n + 1, is_device, g->off));
    KARMA_TRY(read_i64(ctx, g->off.ptr + n, &g->m));
    KARMA_CHECK(g->m >= 0, KARMA_ERR_ARG, "bad offsets");
    g->m_cap = g->m;
    KARMA_TRY(ids_or_iota(ctx, ids, n, is_device, g->ids));
    KARMA_TRY(upload(ctx, nbr, g->m, is_device, g->nbr));
    KARMA_TRY(upload(ctx, w, g->m, is_device, g->w));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    *out = g.release();
    return KARMA_OK;
}

int karma_adj_view(karma_adj* src, const int64_t* order, int64_t k, karma_adj** out) {
    // order: distinct positions of src (checked by the caller); no host sync
    KARMA_CHECK(src && out && k >= 0 && k <= src->n && (k == 0 || order), KARMA_ERR_ARG, "karma_adj_view: bad arguments");
    karma_ctx* ctx = src->ctx;
    KARMA_TRY(ctx_begin(ctx));
    auto g = std::make_unique<karma_adj>();
    g->ctx = ctx;
    g->n = k;
    g->m_cap = src->m_cap;  // a view has at most its source's entries
    const int64_t cap = std::max<int64_t>(1, g->m_cap);
    DevArray<int64_t> dorder, cnt;
    DevArray<int32_t> pos;
    DevArray<int> bad;
    KARMA_TRY(upload(ctx, order, k, 0, dorder));
    KARMA_TRY(pos.alloc(ctx, src->n ? src->n : 1));
    KARMA_HIP(hipMemsetAsync(pos.ptr, 0xFF, src->n * 4, ctx->stream));
    KARMA_TRY(bad.alloc(ctx, 1));
    if (k) KARMA_LAUNCH(ctx, "adj_posmap", posmap_kernel, grid_of(k), 256, 0, dorder.ptr, k, src->n, pos.ptr, bad.ptr);
    KARMA_TRY(cnt.alloc(ctx, k + 1));
    KARMA_LAUNCH(ctx, "adj_view_count", view_count_kernel, grid_of(k + 1), 256, 0, dorder.ptr, k, src->off.ptr,
                 src->nbr.ptr, pos.ptr, cnt.ptr);
    KARMA_TRY(g->off.alloc(ctx, k + 1));
    KARMA_TRY(scan_i64(ctx, cnt.ptr, g->off.ptr, k + 1));
    DevArray<uint64_t> key;
    DevArray<uint32_t> x;
    DevArray<double> wv;
    KARMA_TRY(key.alloc(ctx, cap));
    KARMA_TRY(x.alloc(ctx, cap));
    KARMA_TRY(wv.alloc(ctx, cap));
    KARMA_TRY(g->nbr.alloc(ctx, cap));
    KARMA_TRY(g->w.alloc(ctx, cap));
    if (k) {
        KARMA_LAUNCH(ctx, "adj_view_fill", view_fill_kernel, grid_of(k), 256, 0, dorder.ptr, k, src->off.ptr,
                     src->nbr.ptr, src->w.ptr, pos.ptr, g->off.ptr, key.ptr, x.ptr, wv.ptr);
        KARMA_LAUNCH(ctx, "adj_view_sort", rank_scatter_kernel, (int)std::min<int64_t>(grid_of(cap), 2048), 256, 0,
                     key.ptr, g->off.ptr, k, x.ptr, wv.ptr, g->nbr.ptr, g->w.ptr);
    }
    KARMA_TRY(g->ids.alloc(ctx, k ? k : 1));
    if (k) KARMA_LAUNCH(ctx, "adj_ids", gather_ids_kernel, grid_of(k), 256, 0, dorder.ptr, k, src->ids.ptr, g->ids.ptr);
    *out = g.release();
    return KARMA_OK;
}

int karma_adj_view_summary(karma_adj* src, const int64_t* order, int64_t k, const uint8_t* names,
                           const int64_t* name_off, int with_text, int64_t* deg, double* w, uint8_t* text,
                           int64_t text_cap, int64_t* text_len, int* done) {
    KARMA_CHECK(src && done && (k == 0 || (order && deg && w)) && k >= 0 && (!with_text || (names && name_off && text_len)),
                KARMA_ERR_ARG, "karma_adj_view_summary: bad arguments");
    *done = 0;
    if (k > kSumT) return KARMA_OK;  // more than one block: the caller takes the general path
    karma_ctx* ctx = src->ctx;
    KARMA_TRY(ctx_begin(ctx));
    if (k == 0) {
        if (with_text) *text_len = 0;
        *done = 1;
        return KARMA_OK;
    }
    auto al = [](int64_t x) { return (x + 15) & ~int64_t(15); };
    const int64_t o_hdr = al(8 * k), o_deg = o_hdr + 16, o_w = al(o_deg + 4 * k), o_text = al(o_w + 8 * k);
    constexpr int64_t kMapped = 1 << 20;
    const int64_t cap = with_text ? std::max<int64_t>(0, std::min<int64_t>(text_cap, kMapped - o_text - 16)) : 0;
    void *hbuf = nullptr, *dbuf = nullptr;
    KARMA_TRY(ctx_mapped(ctx, kMapConsumers, kMapped, &hbuf, &dbuf));
    uint8_t* hb = static_cast<uint8_t*>(hbuf);
    uint8_t* db = static_cast<uint8_t*>(dbuf);
    std::memcpy(hb, order, 8 * k);
    auto* hdr = reinterpret_cast<SumHeader*>(hb + o_hdr);
    hdr->status = -1;
    KARMA_LAUNCH(ctx, "adj_view_summary", view_summary_kernel, 1, kSumT, 0, reinterpret_cast<const int64_t*>(db),
                 (int)k, src->n, src->off.ptr, src->nbr.ptr, src->w.ptr, src->ids.ptr, names, name_off, with_text,
                 cap, reinterpret_cast<SumHeader*>(db + o_hdr), reinterpret_cast<int32_t*>(db + o_deg),
                 reinterpret_cast<double*>(db + o_w), reinterpret_cast<uint32_t*>(db + o_text));
    // poll the status the kernel publishes (a stream synchronisation costs more
    // than the kernel); the stream's own state ends the wait on any failure
    int st = -1;
    for (uint64_t spin = 1;; ++spin) {
        st = __atomic_load_n(&hdr->status, __ATOMIC_ACQUIRE);
        if (st != -1) break;
        if ((spin & 1023) == 0) {
            const hipError_t q = hipStreamQuery(ctx->stream);
            if (q == hipErrorNotReady) continue;
            KARMA_HIP(q);
            st = __atomic_load_n(&hdr->status, __ATOMIC_ACQUIRE);
            break;
        }
    }
    KARMA_CHECK(st != 2, KARMA_ERR_ARG, "view order: positions must be distinct and in range");
    KARMA_CHECK(st == 0 || st == 1, KARMA_ERR_HIP, "view summary kernel did not finish (status %d)", st);
    if (st == 1) return KARMA_OK;  // over the one-block limits
    const int32_t* d32 = reinterpret_cast<const int32_t*>(hb + o_deg);
    for (int64_t i = 0; i < k; ++i) deg[i] = d32[i];
    std::memcpy(w, hb + o_w, 8 * k);
    if (with_text) {
        *text_len = hdr->text_len;
        if (hdr->text_len && text) std::memcpy(text, hb + o_text, hdr->text_len);
    }
    *done = 1;
    return KARMA_OK;
}

int karma_adj_keep(karma_adj* src, const uint8_t* keep, int64_t n_keep, karma_adj** out) {
    // n_keep = number of ones in keep (checked by the caller); no host sync
    KARMA_CHECK(src && out && (src->n == 0 || keep) && n_keep >= 0 && n_keep <= src->n, KARMA_ERR_ARG,
                "karma_adj_keep: bad arguments");
    karma_ctx* ctx = src->ctx;
    KARMA_TRY(ctx_begin(ctx));
    const int64_t n = src->n;
    DevArray<uint8_t> dkeep;
    DevArray<int64_t> flag, npos, cnt, ooff;
    KARMA_TRY(upload(ctx, keep, n, 0, dkeep));
    KARMA_TRY(flag.alloc(ctx, n + 1));
    KARMA_TRY(npos.alloc(ctx, n + 1));
    KARMA_LAUNCH(ctx, "adj_keep_flags", u8_to_i64_kernel, grid_of(n + 1), 256, 0, dkeep.ptr, n, flag.ptr);
    KARMA_TRY(scan_i64(ctx, flag.ptr, npos.ptr, n + 1));
    auto g = std::make_unique<karma_adj>();
    g->ctx = ctx;
    g->n = n_keep;
    g->m_cap = src->m_cap;
    const int64_t cap = std::max<int64_t>(1, g->m_cap);
    KARMA_TRY(cnt.alloc(ctx, n + 1));
    KARMA_LAUNCH(ctx, "adj_keep_count", keep_count_kernel, grid_of(n + 1), 256, 0, dkeep.ptr, n, src->off.ptr,
                 src->nbr.ptr, cnt.ptr);
    // counts of dropped nodes are 0, so the scan over old positions is each
    // kept node's new start
    KARMA_TRY(ooff.alloc(ctx, n + 1));
    KARMA_TRY(scan_i64(ctx, cnt.ptr, ooff.ptr, n + 1));
    KARMA_TRY(g->off.alloc(ctx, n_keep + 1));
    KARMA_TRY(g->nbr.alloc(ctx, cap));
    KARMA_TRY(g->w.alloc(ctx, cap));
    KARMA_TRY(g->ids.alloc(ctx, n_keep ? n_keep : 1));
    KARMA_LAUNCH(ctx, "adj_keep_off", keep_off_kernel, grid_of(n + 1), 256, 0, dkeep.ptr, n, npos.ptr, ooff.ptr,
                 g->off.ptr);
    if (n)
        KARMA_LAUNCH(ctx, "adj_keep_fill", keep_fill_kernel, grid_of(n), 256, 0, dkeep.ptr, n, src->off.ptr,
                     src->nbr.ptr, src->w.ptr, npos.ptr, ooff.ptr, src->ids.ptr, g->nbr.ptr, g->w.ptr, g->ids.ptr);
    *out = g.release();
    return KARMA_OK;
}

int karma_adj_node_stats(karma_adj* g, int64_t* deg, double* w) {
    KARMA_CHECK(g, KARMA_ERR_ARG, "null graph");
    karma_ctx* ctx = g->ctx;
    KARMA_TRY(ctx_begin(ctx));
    if (!g->n) return KARMA_OK;
    DevArray<int64_t> dd;
    DevArray<double> dw;
    KARMA_TRY(dd.alloc(ctx, g->n));
    KARMA_TRY(dw.alloc(ctx, g->n));
    KARMA_LAUNCH(ctx, "adj_node_stats", node_stats_kernel, grid_of(g->n), 256, 0, g->off.ptr, g->w.ptr, g->n,
                 dd.ptr, dw.ptr);
    if (deg) KARMA_HIP(hipMemcpyAsync(deg, dd.ptr, g->n * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (w) KARMA_HIP(hipMemcpyAsync(w, dw.ptr, g->n * 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

int karma_adj_info(karma_adj* g, int64_t* n, int64_t* n_entries) {
    KARMA_CHECK(g, KARMA_ERR_ARG, "null graph");
    if (n) *n = g->n;
    if (n_entries) {
        if (g->m < 0) {
            KARMA_TRY(ctx_begin(g->ctx));
            KARMA_TRY(read_i64(g->ctx, g->off.ptr + g->n, &g->m));
        }
        *n_entries = g->m;
    }
    return KARMA_OK;
}

int karma_adj_get(karma_adj* g, uint32_t* ids, int64_t* off, uint32_t* nbr, double* w) {
    KARMA_CHECK(g, KARMA_ERR_ARG, "null graph");
    karma_ctx* ctx = g->ctx;
    KARMA_TRY(karma_adj_info(g, nullptr, &g->m));
    if (ids && g->n) KARMA_HIP(hipMemcpyAsync(ids, g->ids.ptr, g->n * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (off) KARMA_HIP(hipMemcpyAsync(off, g->off.ptr, (g->n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (nbr && g->m) KARMA_HIP(hipMemcpyAsync(nbr, g->nbr.ptr, g->m * 4, hipMemcpyDeviceToHost, ctx->stream));
    if (w && g->m) KARMA_HIP(hipMemcpyAsync(w, g->w.ptr, g->m * 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

int karma_adj_degrees(karma_adj* g, int64_t* deg) {
    KARMA_CHECK(g && (g->n == 0 || deg), KARMA_ERR_ARG, "karma_adj_degrees: bad arguments");
    return karma_adj_node_stats(g, deg, nullptr);
}

int karma_adj_node_weights(karma_adj* g, double* out) {
    KARMA_CHECK(g && (g->n == 0 || out), KARMA_ERR_ARG, "karma_adj_node_weights: bad arguments");
    return karma_adj_node_stats(g, nullptr, out);
}

int karma_adj_edge_list(karma_adj* g, const uint8_t* names, const int64_t* name_off, int64_t n_names,
                        int names_on_device, uint8_t* out, int64_t cap, int64_t* len) {
    KARMA_CHECK(g && names && name_off && len, KARMA_ERR_ARG, "karma_adj_edge_list: bad arguments");
    karma_ctx* ctx = g->ctx;
    KARMA_TRY(ctx_begin(ctx));
    if (g->text_len < 0 || g->text_names != names) {
        DevArray<uint8_t> hnames;
        DevArray<int64_t> hoff;
        const uint8_t* dnames = names;
        const int64_t* doff = name_off;
        if (!names_on_device) {
            const int64_t nb = name_off[n_names];
            KARMA_TRY(upload(ctx, names, nb, 0, hnames));
            KARMA_TRY(upload(ctx, name_off, n_names + 1, 0, hoff));
            dnames = hnames.ptr;
            doff = hoff.ptr;
        }
        const int64_t n = g->n;
        DevArray<int64_t> lens, start;
        KARMA_TRY(lens.alloc(ctx, n + 1));
        KARMA_TRY(start.alloc(ctx, n + 1));
        KARMA_LAUNCH(ctx, "adj_edge_list_len", edge_list_len_kernel, grid_of(n + 1), 256, 0, g->off.ptr, g->nbr.ptr,
                     g->w.ptr, g->ids.ptr, n, doff, lens.ptr);
        KARMA_TRY(scan_i64(ctx, lens.ptr, start.ptr, n + 1));
        int64_t total = 0;
        KARMA_TRY(read_i64(ctx, start.ptr + n, &total));
        KARMA_TRY(g->text.alloc(ctx, total ? total : 1));
        if (n)
            KARMA_LAUNCH(ctx, "adj_edge_list_write", edge_list_write_kernel, grid_of(n), 256, 0, g->off.ptr,
                         g->nbr.ptr, g->w.ptr, g->ids.ptr, n, dnames, doff, start.ptr, g->text.ptr);
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        g->text_len = total ? total - 1 : 0;  // "\n".join: no newline after the last line
        g->text_names = names;
    }
    *len = g->text_len;
    if (out) {
        KARMA_CHECK(cap >= g->text_len, KARMA_ERR_ARG, "edge list buffer too small (%lld < %lld)", (long long)cap,
                    (long long)g->text_len);
        if (g->text_len)
            KARMA_HIP(hipMemcpyAsync(out, g->text.ptr, g->text_len, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        g->text.release();  // kept only between the length query and the copy
        g->text_len = -1;
        g->text_names = nullptr;
    }
    return KARMA_OK;
}

int karma_adj_cross_sums(karma_adj* g, const int32_t* sub, const int32_t* rank, double cutoff, uint64_t* pair,
                         double* sum, int64_t* n_edges, int64_t* n_over, int64_t cap, int64_t* n_pairs) {
    KARMA_CHECK(g && sub && rank && n_pairs, KARMA_ERR_ARG, "karma_adj_cross_sums: bad arguments");
    karma_ctx* ctx = g->ctx;
    KARMA_TRY(ctx_begin(ctx));
    const int64_t n = g->n;
    DevArray<int32_t> dsub, drank;
    DevArray<int64_t> cnt, start;
    KARMA_TRY(upload(ctx, sub, n, 0, dsub));
    KARMA_TRY(upload(ctx, rank, n, 0, drank));
    KARMA_TRY(cnt.alloc(ctx, n + 1));
    KARMA_TRY(start.alloc(ctx, n + 1));
    KARMA_LAUNCH(ctx, "adj_cross_count", cross_count_kernel, grid_of(n + 1), 256, 0, g->off.ptr, g->nbr.ptr, n,
                 dsub.ptr, cnt.ptr);
    KARMA_TRY(scan_i64(ctx, cnt.ptr, start.ptr, n + 1));
    int64_t m = 0;
    KARMA_TRY(read_i64(ctx, start.ptr + n, &m));
    if (m == 0) {
        *n_pairs = 0;
        return KARMA_OK;
    }
    KARMA_CHECK(m < (int64_t(1) << 31), KARMA_ERR_ARG, "too many cross-subcluster edges");
    DevArray<uint64_t> pk, ik, k1, k2;
    DevArray<double> ew;
    DevArray<uint32_t> idx, idx2, idx3;
    KARMA_TRY(pk.alloc(ctx, m));
    KARMA_TRY(ik.alloc(ctx, m));
    KARMA_TRY(k1.alloc(ctx, m));
    KARMA_TRY(k2.alloc(ctx, m));
    KARMA_TRY(ew.alloc(ctx, m));
    KARMA_TRY(idx.alloc(ctx, m));
    KARMA_TRY(idx2.alloc(ctx, m));
    KARMA_TRY(idx3.alloc(ctx, m));
    KARMA_LAUNCH(ctx, "adj_cross_fill", cross_fill_kernel, grid_of(n), 256, 0, g->off.ptr, g->nbr.ptr, g->w.ptr, n,
                 dsub.ptr, drank.ptr, start.ptr, pk.ptr, ik.ptr, ew.ptr);
    KARMA_LAUNCH(ctx, "adj_iota", iota_u32_kernel, grid_of(m), 256, 0, idx.ptr, m);
    // LSD: by the in-pair key, then stably by (A, B) (the library's radix sort, sort.hip)
    KARMA_TRY(radix_sort_u64(ctx, ik.ptr, idx.ptr, m, 64, k1.ptr, idx2.ptr));
    KARMA_LAUNCH(ctx, "adj_cross_gather", gather_u64_kernel, grid_of(m), 256, 0, idx2.ptr, m, pk.ptr, k2.ptr);
    KARMA_TRY(radix_sort_u64(ctx, k2.ptr, idx2.ptr, m, 64, k1.ptr, idx3.ptr));
    DevArray<int64_t> head, seg;
    KARMA_TRY(head.alloc(ctx, m + 1));
    KARMA_TRY(seg.alloc(ctx, m + 1));
    KARMA_LAUNCH(ctx, "adj_cross_heads", segment_heads_kernel, grid_of(m + 1), 256, 0, k1.ptr, m, head.ptr);
    KARMA_TRY(scan_i64(ctx, head.ptr, seg.ptr, m + 1));
    int64_t P = 0;
    KARMA_TRY(read_i64(ctx, seg.ptr + m, &P));
    *n_pairs = P;
    if (!pair && !sum && !n_edges && !n_over) return KARMA_OK;
    KARMA_CHECK(cap >= P, KARMA_ERR_ARG, "cross-sum buffers too small (%lld < %lld)", (long long)cap, (long long)P);
    DevArray<uint64_t> okey;
    DevArray<double> osum;
    DevArray<int64_t> on, oo;
    KARMA_TRY(okey.alloc(ctx, P));
    KARMA_TRY(osum.alloc(ctx, P));
    KARMA_TRY(on.alloc(ctx, P));
    KARMA_TRY(oo.alloc(ctx, P));
    KARMA_LAUNCH(ctx, "adj_cross_sum", cross_sum_kernel, grid_of(m), 256, 0, k1.ptr, idx3.ptr, ew.ptr, m, head.ptr,
                 seg.ptr, cutoff, okey.ptr, osum.ptr, on.ptr, oo.ptr);
    if (pair) KARMA_HIP(hipMemcpyAsync(pair, okey.ptr, P * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (sum) KARMA_HIP(hipMemcpyAsync(sum, osum.ptr, P * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (n_edges) KARMA_HIP(hipMemcpyAsync(n_edges, on.ptr, P * 8, hipMemcpyDeviceToHost, ctx->stream));
    if (n_over) KARMA_HIP(hipMemcpyAsync(n_over, oo.ptr, P * 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    return KARMA_OK;
}

int karma_adj_destroy(karma_adj* g) {
    if (!g) return KARMA_OK;
    if (g->ctx) (void)ctx_begin(g->ctx);
    delete g;
    return KARMA_OK;
}

int karma_repr_f64_host(const double* x, int64_t n, char* out, int64_t cap, int64_t* len) {
    KARMA_CHECK(len && (n == 0 || x), KARMA_ERR_ARG, "karma_repr_f64_host: bad arguments");
    int64_t p = 0;
    char buf[karma_repr::kMaxRepr];
    for (int64_t i = 0; i < n; ++i) {
        const int r = karma_repr::repr_f64(x[i], buf);
        if (out && p + r + 1 <= cap) {
            std::memcpy(out + p, buf, r);
            out[p + r] = '\n';
        }
        p += r + 1;
    }
    *len = p;
    return KARMA_OK;
}

}  // extern "C"
