/*
 * oracle.c — CPU restatement of lmfaber/karma's hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this (as liboracle.so through oracle/oracle.py).  The product library
 * (karma_amd/libkarma_hip.so) never links or calls it.
 *
 * Parity pinning: every function here is checked against golden vectors
 * captured by running the reference itself (tests/golden/make_golden.py ->
 * tests/golden/golden.json) and against the reference's own unit test
 * (tests/test_kmer.py:7-8, is_palindrome).
 *
 * Restated reference code (file:line in /root/reference):
 *   k-mer enumeration      karma/kmer.py:181-197  (__kmers_of_seq)
 *   palindrome predicate   karma/kmer.py:46-54    (is_palindrome: s == s[::-1])
 *   column set + order     karma/kmer.py:146-179  (__extract_kmers, sorted())
 *   per-contig counts      karma/kmer.py:56-92    (__count_kmer_occurence)
 *   normalised profile     karma/kmer.py:108-122, :199-233 (count / len(header key))
 *   eq-class graph         karma/read_graph.py:61-148
 *   readset graph          karma/read_graph.py:19-50  (from_contigs)
 *   bipartite update       karma/read_graph.py:192-221 (update_graph)
 *
 * K-mers are compared exactly like Python str objects whose code points are all
 * < 256 (the wrapper encodes sequences as latin-1): lexicographic on bytes,
 * a proper prefix sorts first.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OK_MAXK 15

typedef struct {
    uint8_t len;
    uint8_t b[OK_MAXK];
} okey_t;

static int okey_cmp(const void* pa, const void* pb) {
    const okey_t* a = (const okey_t*)pa;
    const okey_t* b = (const okey_t*)pb;
    int m = a->len < b->len ? a->len : b->len;
    int c = memcmp(a->b, b->b, (size_t)m);
    if (c) return c;
    return (int)a->len - (int)b->len;
}

/* kmer.py:54 — sequence == sequence[::-1] */
int oracle_is_palindrome(const uint8_t* s, int64_t n) {
    for (int64_t i = 0; i < n / 2; ++i)
        if (s[i] != s[n - 1 - i]) return 0;
    return 1;
}

/* Enumerate the k-mers of one contig the way kmer.py:66-86 / :155-170 do.
 * kmode > 0: all k-mers of length kmode; kmode == -1: "5p6" = all 5-mers then
 * palindromic 6-mers.  Calls emit(key) for every occurrence.  Returns count. */
typedef void (*emit_fn)(void* ctx, const okey_t* k);

static int64_t enum_kmers(const uint8_t* s, int64_t L, int kmode, emit_fn emit, void* ctx) {
    int64_t n = 0;
    okey_t k;
    memset(&k, 0, sizeof k); /* bytes past len stay zero in the emitted keys */
    if (kmode == -1) {
        for (int64_t i = 0; i + 5 <= L; ++i) { /* kmer.py:72-73 */
            k.len = 5;
            memcpy(k.b, s + i, 5);
            emit(ctx, &k);
            ++n;
        }
        for (int64_t i = 0; i + 6 <= L; ++i) { /* kmer.py:76-80 */
            if (!oracle_is_palindrome(s + i, 6)) continue;
            k.len = 6;
            memcpy(k.b, s + i, 6);
            emit(ctx, &k);
            ++n;
        }
    } else {
        for (int64_t i = 0; i + kmode <= L; ++i) { /* kmer.py:84-85 */
            k.len = (uint8_t)kmode;
            memcpy(k.b, s + i, (size_t)kmode);
            emit(ctx, &k);
            ++n;
        }
    }
    return n;
}

typedef struct {
    okey_t* v;
    int64_t n, cap;
} kvec_t;

static void kvec_push(void* ctx, const okey_t* k) {
    kvec_t* kv = (kvec_t*)ctx;
    if (kv->n == kv->cap) {
        kv->cap = kv->cap ? kv->cap * 2 : 1024;
        kv->v = (okey_t*)realloc(kv->v, (size_t)kv->cap * sizeof(okey_t));
    }
    memset(&kv->v[kv->n], 0, sizeof(okey_t));
    kv->v[kv->n] = *k;
    kv->n++;
}

static int64_t sort_unique(okey_t* v, int64_t n) {
    if (n == 0) return 0;
    qsort(v, (size_t)n, sizeof(okey_t), okey_cmp);
    int64_t m = 1;
    for (int64_t i = 1; i < n; ++i)
        if (okey_cmp(&v[i], &v[m - 1]) != 0) v[m++] = v[i];
    return m;
}

/* __extract_kmers (kmer.py:146-179): union over all contigs, sorted().
 * keys_out: capacity cap records of 16 bytes ({len, bytes[15]}).
 * Returns M (number of columns), or -M if cap < M (nothing written). */
int64_t oracle_kmer_columns(const uint8_t* seq, const int64_t* offsets, int64_t n, int kmode,
                            uint8_t* keys_out, int64_t cap) {
    if (kmode == 0 || kmode > OK_MAXK || kmode < -1) return INT64_MIN;
    kvec_t kv = {0, 0, 0};
    for (int64_t c = 0; c < n; ++c) {
        /* collect per contig then unique to bound memory */
        kvec_t one = {0, 0, 0};
        enum_kmers(seq + offsets[c], offsets[c + 1] - offsets[c], kmode, kvec_push, &one);
        int64_t m = sort_unique(one.v, one.n);
        for (int64_t i = 0; i < m; ++i) kvec_push(&kv, &one.v[i]);
        free(one.v);
        if (kv.n > (1 << 20)) kv.n = sort_unique(kv.v, kv.n);
    }
    int64_t M = sort_unique(kv.v, kv.n);
    if (M > cap) {
        free(kv.v);
        return -M;
    }
    memcpy(keys_out, kv.v, (size_t)M * sizeof(okey_t));
    free(kv.v);
    return M;
}

typedef struct {
    const okey_t* cols;
    int64_t M;
    int64_t* counts;
    int64_t miss;
} count_ctx_t;

static void count_emit(void* vctx, const okey_t* k) {
    count_ctx_t* c = (count_ctx_t*)vctx;
    okey_t key;
    memset(&key, 0, sizeof key);
    key = *k;
    const okey_t* hit = (const okey_t*)bsearch(&key, c->cols, (size_t)c->M, sizeof(okey_t), okey_cmp);
    if (!hit) {
        c->miss++;
        return;
    }
    c->counts[hit - c->cols]++; /* Counter[kmer] += 1, kmer.py:73/80/85 */
}

/* __calc_kmer_profile body (kmer.py:199-233): profile[row][col] = count / length
 * with length = len(header key) (kmer.py:213 iterates the dict's KEYS).
 * out: N*M float64 C-order, fully written (zeros included).
 * counts_out (optional): N*M int64 raw Counter values.
 * Returns 0, or 1 if some k-mer was missing from the column set,
 * or 2 if a key length is 0 and a count is non-zero (ZeroDivisionError). */
int oracle_kmer_profile(const uint8_t* seq, const int64_t* offsets, const int64_t* key_len, int64_t n,
                        int kmode, const uint8_t* keys, int64_t M, double* out, int64_t* counts_out) {
    int64_t* counts = (int64_t*)calloc((size_t)(M ? M : 1), sizeof(int64_t));
    count_ctx_t ctx = {(const okey_t*)keys, M, counts, 0};
    int rc = 0;
    for (int64_t r = 0; r < n; ++r) {
        memset(counts, 0, (size_t)M * sizeof(int64_t));
        enum_kmers(seq + offsets[r], offsets[r + 1] - offsets[r], kmode, count_emit, &ctx);
        for (int64_t j = 0; j < M; ++j) {
            double v = 0.0;
            if (counts[j]) {
                if (key_len[r] == 0) rc = 2;
                else v = (double)counts[j] / (double)key_len[r]; /* kmer.py:120 */
            }
            out[r * M + j] = v;
            if (counts_out) counts_out[r * M + j] = counts[j];
        }
    }
    free(counts);
    if (ctx.miss) rc = 1;
    return rc;
}

/* ------------------------------------------------------------------------- */
/* Shared-read graph                                                          */
/* ------------------------------------------------------------------------- */

typedef struct {
    uint64_t key; /* (a << 32) | b, a <= b */
    int64_t cnt;
    uint64_t pos; /* global index of the pair in emission order */
} opair_t;

static int opair_cmp(const void* pa, const void* pb) {
    const opair_t* a = (const opair_t*)pa;
    const opair_t* b = (const opair_t*)pb;
    if (a->key != b->key) return a->key < b->key ? -1 : 1;
    if (a->pos != b->pos) return a->pos < b->pos ? -1 : 1;
    return 0;
}

static int u32_cmp(const void* pa, const void* pb) {
    uint32_t a = *(const uint32_t*)pa, b = *(const uint32_t*)pb;
    return a < b ? -1 : (a > b);
}

typedef struct {
    opair_t* v;
    int64_t n, cap;
} pvec_t;

static void pvec_push(pvec_t* p, uint32_t a, uint32_t b, int64_t cnt, uint64_t pos) {
    if (p->n == p->cap) {
        p->cap = p->cap ? p->cap * 2 : 4096;
        p->v = (opair_t*)realloc(p->v, (size_t)p->cap * sizeof(opair_t));
    }
    uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    p->v[p->n].key = ((uint64_t)lo << 32) | hi;
    p->v[p->n].cnt = cnt;
    p->v[p->n].pos = pos;
    p->n++;
}

/* Group-based shared-read counting.  A "group" is either
 *   - a salmon equivalence class (dedup = 0): members as listed, mult = count;
 *     totals += count for EVERY listed member (read_graph.py:86-92); pairs from
 *     itertools.combinations(ids, 2) unless pair_skip[g] (eq_size token "1",
 *     read_graph.py:102-105); a duplicated id yields a self-loop pair (x, x);
 *   - a read / fragment (dedup = 1, mult = 1): members are the contigs its
 *     records map to, deduplicated (contig.py:11 keeps QNAMEs in a set), so
 *     totals[c] = |readset(c)| and pairs count |R_a ∩ R_b| (read_graph.py:34).
 * Output: E unique pairs sorted by (a, b) with summed count, first emission
 * position and weight (s/ta + s/tb)/2 (read_graph.py:128-130 / :39-42); pairs
 * whose summed count is 0 are dropped (read_graph.py:123-124, :46-49).
 * Returns E; if cap < E returns -E (nothing but totals written).
 * *zero_div set to 1 when a nonzero pair meets a zero total (ZeroDivisionError
 * in read_graph.py:128-130).  Counts are exact int64 (Python ints are exact). */
int64_t oracle_graph_groups(const int64_t* grp_off, const uint32_t* members, const int64_t* mult,
                            const uint8_t* pair_skip, int64_t G, int64_t N, int dedup, int64_t* totals,
                            uint32_t* ea, uint32_t* eb, int64_t* es, uint64_t* efirst, double* ew, int64_t cap,
                            int* zero_div) {
    memset(totals, 0, (size_t)N * sizeof(int64_t));
    pvec_t pv = {0, 0, 0};
    uint64_t pos = 0;
    uint32_t* buf = NULL;
    int64_t bufcap = 0;
    for (int64_t g = 0; g < G; ++g) {
        int64_t lo = grp_off[g], hi = grp_off[g + 1], m = hi - lo;
        int64_t c = mult ? mult[g] : 1;
        if (m > bufcap) {
            bufcap = m * 2;
            buf = (uint32_t*)realloc(buf, (size_t)bufcap * sizeof(uint32_t));
        }
        memcpy(buf, members + lo, (size_t)m * sizeof(uint32_t));
        if (dedup) {
            qsort(buf, (size_t)m, sizeof(uint32_t), u32_cmp);
            int64_t u = m ? 1 : 0;
            for (int64_t i = 1; i < m; ++i)
                if (buf[i] != buf[u - 1]) buf[u++] = buf[i];
            m = u;
        }
        for (int64_t i = 0; i < m; ++i) totals[buf[i]] += c;
        if (pair_skip && pair_skip[g]) continue;
        for (int64_t i = 0; i < m; ++i)
            for (int64_t j = i + 1; j < m; ++j) pvec_push(&pv, buf[i], buf[j], c, pos++);
    }
    free(buf);
    if (pv.n) qsort(pv.v, (size_t)pv.n, sizeof(opair_t), opair_cmp);
    int64_t E = 0;
    *zero_div = 0;
    for (int64_t i = 0; i < pv.n;) {
        int64_t j = i;
        int64_t s = 0;
        while (j < pv.n && pv.v[j].key == pv.v[i].key) s += pv.v[j++].cnt;
        if (s != 0) {
            if (E < cap) {
                uint32_t a = (uint32_t)(pv.v[i].key >> 32), b = (uint32_t)pv.v[i].key;
                ea[E] = a;
                eb[E] = b;
                es[E] = s;
                efirst[E] = pv.v[i].pos;
                if (totals[a] == 0 || totals[b] == 0) {
                    *zero_div = 1;
                    ew[E] = 0.0;
                } else {
                    ew[E] = ((double)s / (double)totals[a] + (double)s / (double)totals[b]) / 2.0;
                }
            }
            E++;
        }
        i = j;
    }
    free(pv.v);
    return E <= cap ? E : -E;
}

/* Direct restatement of ReadGraph.from_contigs (read_graph.py:31-49) for small
 * N: every pair (i, j), i < j, of readsets given as sorted unique u32 read ids
 * (CSR rs_off/rs_ids).  Emits pairs with weight > 0 in combinations order.
 * ZeroDivisionError -> weight 0 (read_graph.py:43-44).  Returns E or -E. */
static int64_t isect(const uint32_t* a, int64_t na, const uint32_t* b, int64_t nb) {
    int64_t i = 0, j = 0, s = 0;
    while (i < na && j < nb) {
        if (a[i] < b[j]) ++i;
        else if (a[i] > b[j]) ++j;
        else { ++s; ++i; ++j; }
    }
    return s;
}

static double pair_weight(int64_t s, int64_t na, int64_t nb) {
    if (na == 0 || nb == 0) return 0.0; /* ZeroDivisionError -> 0 */
    return ((double)s / (double)na + (double)s / (double)nb) / 2.0;
}

int64_t oracle_readset_pairs(const int64_t* rs_off, const uint32_t* rs_ids, int64_t N, uint32_t* ea, uint32_t* eb,
                             int64_t* es, double* ew, int64_t cap) {
    int64_t E = 0;
    for (int64_t i = 0; i < N; ++i)
        for (int64_t j = i + 1; j < N; ++j) {
            int64_t na = rs_off[i + 1] - rs_off[i], nb = rs_off[j + 1] - rs_off[j];
            int64_t s = isect(rs_ids + rs_off[i], na, rs_ids + rs_off[j], nb);
            double w = pair_weight(s, na, nb);
            if (w > 0) {
                if (E < cap) { ea[E] = (uint32_t)i; eb[E] = (uint32_t)j; es[E] = s; ew[E] = w; }
                E++;
            }
        }
    return E <= cap ? E : -E;
}

/* ReadGraph.update_graph (read_graph.py:201-221): product(original, new). */
int64_t oracle_update_pairs(const int64_t* o_off, const uint32_t* o_ids, int64_t NO, const int64_t* n_off,
                            const uint32_t* n_ids, int64_t NN, uint32_t* ea, uint32_t* eb, int64_t* es, double* ew,
                            int64_t cap) {
    int64_t E = 0;
    for (int64_t i = 0; i < NO; ++i)
        for (int64_t j = 0; j < NN; ++j) {
            int64_t na = o_off[i + 1] - o_off[i], nb = n_off[j + 1] - n_off[j];
            int64_t s = isect(o_ids + o_off[i], na, n_ids + n_off[j], nb);
            double w = pair_weight(s, na, nb);
            if (w > 0) {
                if (E < cap) { ea[E] = (uint32_t)i; eb[E] = (uint32_t)j; es[E] = s; ew[E] = w; }
                E++;
            }
        }
    return E <= cap ? E : -E;
}

/* ------------------------------------------------------------------------- */
/* OpenMP twins (the on-node CPU baseline; bench.py        */
/* cpu_baseline).  Same arithmetic as the scalar functions above, checked      */
/* against them by tests/test_oracle_golden.py; only the work is split over    */
/* threads.                                                                    */
/* ------------------------------------------------------------------------- */

int oracle_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* oracle_kmer_columns over contigs in parallel: every thread keeps the sorted
 * union of its contigs' k-mers, then the thread unions are merged (the CPU
 * baseline's column table; same result as the scalar restatement). */
/* Per-thread exact set of k-mer keys (open addressing over the 16-byte keys;
 * bytes past len are zero in every emitted key, so whole-key equality is
 * str equality).  The OpenMP twin collects the union with it instead of
 * sorting each contig's k-mers: the set stays a few thousand keys, so an
 * insert is a probe of an L1-resident table. */
typedef struct {
    okey_t* slot;
    uint8_t* used;
    int64_t cap, n;
} kset_t;

static uint64_t okey_hash(const okey_t* k) {
    uint64_t a, b;
    memcpy(&a, k, 8);
    memcpy(&b, (const uint8_t*)k + 8, 8);
    uint64_t h = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xC2B2AE3D27D4EB4Full;
    return h ^ (h >> 31);
}

static void kset_insert(kset_t* s, const okey_t* k) {
    uint64_t i = okey_hash(k) & (uint64_t)(s->cap - 1);
    while (s->used[i]) {
        if (!memcmp(&s->slot[i], k, sizeof *k)) return;
        i = (i + 1) & (uint64_t)(s->cap - 1);
    }
    s->used[i] = 1;
    s->slot[i] = *k;
    s->n++;
}

static void kset_add(void* ctx, const okey_t* k) {
    kset_t* s = (kset_t*)ctx;
    if (2 * (s->n + 1) > s->cap) { /* grow: rehash into twice the slots */
        kset_t t = {0, 0, s->cap ? 2 * s->cap : 4096, 0};
        t.slot = (okey_t*)malloc((size_t)t.cap * sizeof(okey_t));
        t.used = (uint8_t*)calloc((size_t)t.cap, 1);
        for (int64_t i = 0; i < s->cap; ++i)
            if (s->used[i]) kset_insert(&t, &s->slot[i]);
        free(s->slot);
        free(s->used);
        *s = t;
    }
    kset_insert(s, k);
}

int64_t oracle_omp_kmer_columns(const uint8_t* seq, const int64_t* offsets, int64_t n, int kmode, uint8_t* keys_out,
                                int64_t cap) {
    if (kmode == 0 || kmode > OK_MAXK || kmode < -1) return INT64_MIN;
    int T = oracle_threads();
    kset_t* part = (kset_t*)calloc((size_t)T, sizeof(kset_t));
#pragma omp parallel num_threads(T)
    {
        kset_t* ks = &part[omp_get_thread_num()];
#pragma omp for schedule(dynamic, 256)
        for (int64_t c = 0; c < n; ++c) enum_kmers(seq + offsets[c], offsets[c + 1] - offsets[c], kmode, kset_add, ks);
    }
    kvec_t all = {0, 0, 0};
    for (int t = 0; t < T; ++t) {
        for (int64_t i = 0; i < part[t].cap; ++i)
            if (part[t].used[i]) kvec_push(&all, &part[t].slot[i]);
        free(part[t].slot);
        free(part[t].used);
    }
    free(part);
    int64_t M = sort_unique(all.v, all.n); /* sorted() of the union, kmer.py:172 */
    if (M > cap) {
        free(all.v);
        return -M;
    }
    memcpy(keys_out, all.v, (size_t)M * sizeof(okey_t));
    free(all.v);
    return M;
}

/* oracle_kmer_profile over rows in parallel (no counts_out). */
int oracle_omp_kmer_profile(const uint8_t* seq, const int64_t* offsets, const int64_t* key_len, int64_t n,
                            int kmode, const uint8_t* keys, int64_t M, double* out) {
    int rc = 0;
#pragma omp parallel
    {
        int64_t* counts = (int64_t*)calloc((size_t)(M ? M : 1), sizeof(int64_t));
        count_ctx_t ctx = {(const okey_t*)keys, M, counts, 0};
        int my = 0;
#pragma omp for schedule(dynamic, 256)
        for (int64_t r = 0; r < n; ++r) {
            memset(counts, 0, (size_t)M * sizeof(int64_t));
            enum_kmers(seq + offsets[r], offsets[r + 1] - offsets[r], kmode, count_emit, &ctx);
            for (int64_t j = 0; j < M; ++j) {
                double v = 0.0;
                if (counts[j]) {
                    if (key_len[r] == 0) my = 2;
                    else v = (double)counts[j] / (double)key_len[r]; /* kmer.py:120 */
                }
                out[r * M + j] = v;
            }
        }
        if (ctx.miss) my = 1;
#pragma omp critical
        if (my > rc) rc = my;
        free(counts);
    }
    return rc;
}

static int u64_cmp(const void* pa, const void* pb) {
    uint64_t a = *(const uint64_t*)pa, b = *(const uint64_t*)pb;
    return a < b ? -1 : (a > b);
}

/* oracle_graph_groups for reads (dedup = 1, mult = 1, no pair_skip, no first
 * position): pairs emitted per thread, scattered into NB buckets by a, each
 * bucket sorted and run-length counted on its own.  Buckets are ranges of a, so
 * concatenating them gives the (a, b) order.  Returns E, or -E if cap < E. */
int64_t oracle_omp_graph_reads(const int64_t* grp_off, const uint32_t* members, int64_t G, int64_t N,
                               int64_t* totals, uint32_t* ea, uint32_t* eb, int64_t* es, double* ew, int64_t cap,
                               int* zero_div) {
    const int T = oracle_threads();
    const int NB = 1024;
    uint64_t** tv = (uint64_t**)calloc((size_t)T, sizeof(uint64_t*));
    int64_t* tn = (int64_t*)calloc((size_t)T, sizeof(int64_t));
    int64_t* tb = (int64_t*)calloc((size_t)T * NB, sizeof(int64_t)); /* per thread per bucket counts */
    int64_t* ttot = (int64_t*)calloc((size_t)T * (size_t)(N ? N : 1), sizeof(int64_t));
    const uint64_t nn = (uint64_t)(N ? N : 1);
#pragma omp parallel num_threads(T)
    {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        int64_t g0 = G * t / T, g1 = G * (t + 1) / T;
        int64_t cap_t = 1024, n_t = 0;
        uint64_t* v = (uint64_t*)malloc((size_t)cap_t * 8);
        int64_t* tot = ttot + (size_t)t * nn;
        uint32_t buf[4096];
        for (int64_t g = g0; g < g1; ++g) {
            int64_t lo = grp_off[g], m = grp_off[g + 1] - lo;
            uint32_t* b = m <= 4096 ? buf : (uint32_t*)malloc((size_t)m * 4);
            memcpy(b, members + lo, (size_t)m * 4);
            qsort(b, (size_t)m, 4, u32_cmp);
            int64_t u = m ? 1 : 0;
            for (int64_t i = 1; i < m; ++i)
                if (b[i] != b[u - 1]) b[u++] = b[i];
            for (int64_t i = 0; i < u; ++i) tot[b[i]] += 1;
            for (int64_t i = 0; i < u; ++i)
                for (int64_t j = i + 1; j < u; ++j) {
                    if (n_t == cap_t) {
                        cap_t *= 2;
                        v = (uint64_t*)realloc(v, (size_t)cap_t * 8);
                    }
                    v[n_t++] = ((uint64_t)b[i] << 32) | b[j];
                    tb[(size_t)t * NB + (int64_t)((uint64_t)b[i] * NB / nn)]++;
                }
            if (b != buf) free(b);
        }
        tv[t] = v;
        tn[t] = n_t;
    }
    /* bucket offsets: bucket-major, thread-minor */
    int64_t* boff = (int64_t*)calloc((size_t)NB + 1, sizeof(int64_t));
    int64_t* woff = (int64_t*)calloc((size_t)T * NB, sizeof(int64_t));
    int64_t P = 0;
    for (int k = 0; k < NB; ++k) {
        boff[k] = P;
        for (int t = 0; t < T; ++t) {
            woff[(size_t)t * NB + k] = P;
            P += tb[(size_t)t * NB + k];
        }
    }
    boff[NB] = P;
    uint64_t* all = (uint64_t*)malloc((size_t)(P ? P : 1) * 8);
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; ++t) {
        int64_t* w = woff + (size_t)t * NB;
        for (int64_t i = 0; i < tn[t]; ++i) {
            uint64_t k = tv[t][i];
            all[w[(int64_t)((k >> 32) * NB / nn)]++] = k;
        }
        free(tv[t]);
    }
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t c = 0; c < N; ++c) {
        int64_t s = 0;
        for (int t = 0; t < T; ++t) s += ttot[(size_t)t * nn + c];
        totals[c] = s;
    }
    /* per bucket: sort, count unique keys */
    int64_t* bu = (int64_t*)calloc((size_t)NB + 1, sizeof(int64_t));
#pragma omp parallel for num_threads(T) schedule(dynamic, 1)
    for (int k = 0; k < NB; ++k) {
        uint64_t* a = all + boff[k];
        int64_t n = boff[k + 1] - boff[k];
        if (n > 1) qsort(a, (size_t)n, 8, u64_cmp);
        int64_t u = 0;
        for (int64_t i = 0; i < n; ++i)
            if (i == 0 || a[i] != a[i - 1]) ++u;
        bu[k + 1] = u;
    }
    for (int k = 0; k < NB; ++k) bu[k + 1] += bu[k];
    const int64_t E = bu[NB];
    int zd = 0;
    if (E <= cap) {
#pragma omp parallel for num_threads(T) schedule(dynamic, 1) reduction(| : zd)
        for (int k = 0; k < NB; ++k) {
            uint64_t* a = all + boff[k];
            int64_t n = boff[k + 1] - boff[k], e = bu[k];
            for (int64_t i = 0; i < n;) {
                int64_t j = i;
                while (j < n && a[j] == a[i]) ++j;
                uint32_t x = (uint32_t)(a[i] >> 32), y = (uint32_t)a[i];
                int64_t s = j - i;
                ea[e] = x;
                eb[e] = y;
                es[e] = s;
                if (totals[x] == 0 || totals[y] == 0) {
                    zd = 1;
                    ew[e] = 0.0;
                } else {
                    ew[e] = ((double)s / (double)totals[x] + (double)s / (double)totals[y]) / 2.0;
                }
                ++e;
                i = j;
            }
        }
    }
    *zero_div = zd;
    free(all);
    free(bu);
    free(boff);
    free(woff);
    free(tb);
    free(tn);
    free(tv);
    free(ttot);
    return E <= cap ? E : -E;
}
