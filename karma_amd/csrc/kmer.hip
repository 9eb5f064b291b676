// kmer.hip — contig store + k-mer profile kernels for gfx950.
//
// Reference (lmfaber/karma, pure Python) being replaced:
//   KmerClustering.__calc_kmer_profile   karma/kmer.py:199-264
//   __extract_kmers (sorted column set)  karma/kmer.py:146-179
//   __kmers_of_seq / is_palindrome       karma/kmer.py:181-197, :46-54
//   __count_kmer_occurence               karma/kmer.py:56-92
//   fill_array_for_contig (count/len)    karma/kmer.py:108-122 (len = len(FASTA key), :213)
//
// Device data layout:
//   packed[w]  u32, 16 bases per word, FIRST base in bits 31:30 (so a 64-bit
//              window of two words yields the k-mer's lexicographic 2-bit code);
//              every contig starts on a word boundary (woff[c]); one pad word.
//   mask[w]    u16, bit 15-j set when base j of word w is not one of A,C,G,T
//              (an "exception" base: N, IUPAC, lowercase, '\r', ...).
//   raw        original bytes, read only for k-mers that touch an exception.
// Ordinals: k-mer code for integer k (4^k values); for "5p6" the 5-mer q has
// ordinal 5q and the 6-mer (q, x) ordinal 5q + 1 + x, so ordinal order equals
// Python str order (a proper prefix sorts first).

#include <algorithm>
#include <cstring>

#include "karma_internal.h"

using namespace karma;

struct karma_contigs {
    karma_ctx* ctx = nullptr;
    int64_t n = 0, total = 0, words = 0, exc_bases = 0;
    int64_t zero_key_maxlen = -1;  // longest contig with an empty FASTA key (-1: none)
    int64_t max_len = 0;           // longest contig (bases)
    DevArray<uint8_t> raw_own;
    DevArray<int64_t> off_own;
    DevArray<int32_t> keylen_own;
    const uint8_t* raw = nullptr;
    const int64_t* off = nullptr;
    const int32_t* keylen = nullptr;
    DevArray<int64_t> woff;
    DevArray<uint32_t> packed;
    DevArray<uint16_t> mask;
    DevArray<uint8_t> has_exc;
    DevArray<uint32_t> exc_list;  // contigs with exception bases (any order), count in exc_n
    DevArray<unsigned> exc_n;
};

struct karma_kmer_plan {
    karma_ctx* ctx = nullptr;
    karma_contigs* store = nullptr;
    int kmode = 0;
    int kmin = 0, kmax = 0;
    uint32_t S = 0;  // ordinal space
    int64_t nwords = 0;
    DevArray<uint32_t> presence;
    // the bitmap (nwords, padded to even) then the exception k-mer counter (2
    // words): inside `presence`, or the caller's zeroed block (bits_ext:
    // ctx->plan_zeroed, karma_step's; the column table kernel clears it again)
    uint32_t* bits = nullptr;
    bool bits_ext = false;
    DevArray<uint64_t> exc_keys;  // sorted unique
    int64_t n_exc = 0;
    DevArray<int32_t> col_of_ord;
    DevArray<int32_t> col_of_exc;
    DevArray<uint64_t> col_keys;
    int64_t* row_tot = nullptr;  // per row: k-mer occurrences (inside `presence`'s allocation)
    DevArray<int> err;  // zero-length-key guard flag of the profile kernels (the host checks first)
    DevArray<int64_t> m_dev;
    hipEvent_t fin_ev = nullptr;  // after the column table and M's readback
    bool fin_pending = false;
    int64_t M = -1;
    ~karma_kmer_plan() {
        if (fin_ev) hipEventDestroy(fin_ev);
    }
};

namespace karma {
// The most columns a plan can have: every reachable ACGT ordinal (4^k, or for
// 5p6 the 1024 5-mers and the 64 palindromic 6-mers) plus its exception keys.
int64_t kmer_m_cap(const karma_kmer_plan* p) {
    return (p->kmode == KARMA_KMER_5P6 ? 1088 : (int64_t)p->S) + p->n_exc;
}
}  // namespace karma

namespace {

// Sorted unique copy of n u64 keys (the exception k-mers; low volume): the
// library's radix sort and reduce-by-key (sort.hip), one wait for the count.
int sort_unique_keys(karma_ctx* ctx, const uint64_t* src, int64_t n, DevArray<uint64_t>& out, int64_t* n_out) {
    DevArray<uint64_t> sorted, uniq;
    DevArray<int64_t> nsel;
    int rc;
    if ((rc = sorted.alloc(ctx, n)) || (rc = uniq.alloc(ctx, n)) || (rc = nsel.alloc(ctx, 1))) return rc;
    KARMA_TRY(radix_sort_u64(ctx, src, nullptr, n, 64, sorted.ptr, nullptr));
    KARMA_TRY(reduce_sorted(ctx, sorted.ptr, nullptr, nullptr, nullptr, n, uniq.ptr, nullptr, nullptr, nsel.ptr));
    int64_t nu = 0;
    KARMA_HIP(hipMemcpyAsync(&nu, nsel.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    if ((rc = out.alloc(ctx, nu))) return rc;
    KARMA_HIP(hipMemcpyAsync(out.ptr, uniq.ptr, nu * 8, hipMemcpyDeviceToDevice, ctx->stream));
    *n_out = nu;
    return KARMA_OK;
}

constexpr int kBlock = 256;
constexpr int kPBlock = 512;  // profile: 8 waves share one LDS column table
constexpr int kPadWords = 80;    // zero words after the store (stages may read past the last contig)

// ---------------------------------------------------------------- pack -------
typedef unsigned int u32x4a __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-byte load

// One wave per contig (grid-stride over contigs), lane l packs word w = l + 64t:
// bases 16w .. 16w + 15 come from five aligned dword loads (a dword that starts
// inside the contig cannot cross a page, so nothing past the buffer is touched)
// and alignbyte.  Four bases at a time (SWAR): code = ((b >> 1) ^ (b >> 2)) & 3
// maps A C G T to 0 1 2 3; a byte is an exception when "ACGT"[code] (v_perm)
// differs from it, and then packs as 0 with its mask bit set.
__device__ __forceinline__ uint32_t pack4(uint32_t x, uint32_t nvalid, uint32_t* m4, uint32_t* nexc) {
    // nvalid (0..4): bytes of x inside the contig; the others pack as 0, no mask
    const uint32_t keep = nvalid >= 4 ? 0xFFFFFFFFu : (1u << (8 * nvalid)) - 1u;
    uint32_t t = ((x >> 1) ^ (x >> 2)) & 0x03030303u;
    const uint32_t expect = __builtin_amdgcn_perm(0u, 0x54474341u, t);  // 'A' 'C' 'G' 'T' by code
    const uint32_t d = expect ^ x;
    const uint32_t nz = (((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u & keep;  // exception bytes
    t &= ~((nz >> 7) * 3u) & keep;
    *nexc += (uint32_t)__builtin_popcount(nz);
    *m4 = (nz >> 4 & 8u) | (nz >> 13 & 4u) | (nz >> 22 & 2u) | (nz >> 31);
    return (t << 6 & 0xC0u) | (t >> 4 & 0x30u) | (t >> 14 & 0x0Cu) | (t >> 24 & 0x03u);
}

__global__ void __launch_bounds__(kBlock) pack_kernel(const uint8_t* __restrict__ raw, const int64_t* __restrict__ off,
                                                      const int64_t* __restrict__ woff, int64_t n,
                                                      uint32_t* __restrict__ packed, uint16_t* __restrict__ mask,
                                                      uint8_t* __restrict__ has_exc,
                                                      unsigned long long* __restrict__ exc_count,
                                                      uint32_t* __restrict__ exc_list, unsigned* __restrict__ exc_n) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * (kBlock / 64);
    int64_t c = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    // the next contig's offsets are loaded while this one's bytes are in flight
    int64_t s = 0, e = 0, w0 = 0, w1 = 0;
    if (c < n) s = off[c], e = off[c + 1], w0 = woff[c], w1 = woff[c + 1];
    while (c < n) {
        const int64_t cn = c + waves;
        int64_t sn = 0, en = 0, w0n = 0, w1n = 0;
        if (cn < n) sn = off[cn], en = off[cn + 1], w0n = woff[cn], w1n = woff[cn + 1];
        const int64_t nw = w1 - w0;
        const uint64_t end = (uint64_t)(raw + e);  // first byte past the contig
        uint32_t nexc = 0;
        for (int64_t w = lane; w < nw; w += 64) {
            const uint64_t p = (uint64_t)(raw + s + 16 * w);  // absolute byte address
            const uint64_t abyte = p & ~uint64_t(3);
            const uint32_t* a = reinterpret_cast<const uint32_t*>(abyte);
            const uint32_t sh = (uint32_t)(p & 3);
            uint32_t d[5];
            if (abyte + 20 <= end) {  // whole window inside the contig
                const u32x4a v = *reinterpret_cast<const u32x4a*>(a);
                d[0] = v.x, d[1] = v.y, d[2] = v.z, d[3] = v.w;
                d[4] = a[4];
            } else {  // the contig's last word: dwords that start inside it only
#pragma unroll
                for (int t = 0; t < 5; ++t) d[t] = abyte + 4 * t < end ? a[t] : 0u;
            }
            const int64_t rem = (int64_t)(end - p);  // bases of this word inside the contig (>= 1)
            uint32_t word = 0, m = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t x = __builtin_amdgcn_alignbyte(d[q + 1], d[q], sh);
                const int64_t nv = rem - 4 * q;
                uint32_t m4;
                const uint32_t v = pack4(x, nv <= 0 ? 0u : nv >= 4 ? 4u : (uint32_t)nv, &m4, &nexc);
                word |= v << (24 - 8 * q);
                m |= m4 << (12 - 4 * q);
            }
            packed[w0 + w] = word;
            mask[w0 + w] = (uint16_t)m;
        }
        if (nexc) atomicAdd(exc_count, (unsigned long long)nexc);
        const bool any = __ballot(nexc != 0) != 0;
        if (lane == 0) {
            has_exc[c] = any ? 1 : 0;
            if (any) exc_list[atomicAdd(exc_n, 1u)] = (uint32_t)c;
        }
        c = cn, s = sn, e = en, w0 = w0n, w1 = w1n;
    }
}

__global__ void word_count_kernel(const int64_t* __restrict__ off, int64_t n, int64_t* __restrict__ wc) {
    int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n) wc[c] = (off[c + 1] - off[c] + 15) / 16;
    if (c == n) wc[c] = 0;
}

// ------------------------------------------------------------- k-mer keys ----
// Byte key of a k-mer: bytes big-endian from bit 63; the low byte holds the
// length unless the mode is k = 8 (all keys one length, 8 bytes).
__device__ __forceinline__ uint64_t key_from_bytes(const uint8_t* p, int len, bool with_len) {
    uint64_t k = 0;
    for (int j = 0; j < len; ++j) k |= (uint64_t)p[j] << (56 - 8 * j);
    return with_len ? (k | (uint64_t)len) : k;
}

__device__ __forceinline__ uint64_t key_from_code(uint32_t code, int len, bool with_len) {
    const uint64_t ACGT = 0x54474341ull;  // 'A','C','G','T' little-endian bytes
    uint64_t k = 0;
    for (int j = 0; j < len; ++j) {
        uint32_t b = (code >> (2 * (len - 1 - j))) & 3u;
        k |= ((ACGT >> (8 * b)) & 0xFF) << (56 - 8 * j);
    }
    return with_len ? (k | (uint64_t)len) : k;
}

__device__ __forceinline__ uint64_t ord_key(uint32_t o, bool p56, int k, bool with_len) {
    if (!p56) return key_from_code(o, k, with_len);
    uint32_t q = o / 5, r = o % 5;
    return r == 0 ? key_from_code(q, 5, with_len) : key_from_code((q << 2) | (r - 1), 6, with_len);
}

__device__ __forceinline__ bool pal6_code(uint32_t c) {
    return ((c >> 10) & 3) == (c & 3) && ((c >> 8) & 3) == ((c >> 2) & 3) && ((c >> 6) & 3) == ((c >> 4) & 3);
}

__device__ __forceinline__ bool pal_bytes(const uint8_t* p, int len) {
    for (int j = 0; j < len / 2; ++j)
        if (p[j] != p[len - 1 - j]) return false;
    return true;
}

// lower_bound over a sorted device array (count of elements < key)
__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t* a, int64_t n, uint64_t key) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Window view of one contig position: 2-bit code of up to 8 bases + exception bits.
struct Window {
    uint64_t x;  // two packed words
    uint32_t m;  // two mask halves
    int o;       // base offset inside the first word
    __device__ __forceinline__ uint32_t code(int k) const {
        return (uint32_t)(x >> (64 - 2 * o - 2 * k)) & ((1u << (2 * k)) - 1u);
    }
    __device__ __forceinline__ bool clean(int k) const { return ((m >> (32 - o - k)) & ((1u << k) - 1u)) == 0; }
};

__device__ __forceinline__ Window load_window(const uint32_t* packed, const uint16_t* mask, int64_t w0, int64_t i,
                                              bool need_mask) {
    const int64_t w = w0 + (i >> 4);
    Window v;
    v.o = (int)(i & 15);
    v.x = ((uint64_t)packed[w] << 32) | packed[w + 1];
    v.m = need_mask ? (((uint32_t)mask[w] << 16) | mask[w + 1]) : 0u;
    return v;
}

// ------------------------------------------------------------- staging -------
// A wave walks its contig in stages of 1024 positions: the 65 packed words
// (and, for contigs with exception bases, the 65 mask half-words) of a stage
// are loaded once, coalesced, into the wave's LDS slice; every k-mer window is
// then read from LDS.
template <typename Body>
__device__ __forceinline__ void window_round(int64_t base, int64_t npos, bool excp, const uint32_t* wbuf,
                                             const uint16_t* mbuf, int lane, Body& body) {
    const int64_t lim = min(npos, base + 1024);
    for (int64_t i = base + lane; i < lim; i += 64) {
        const int l = (int)(i - base), w = l >> 4;
        Window v;
        v.o = l & 15;
        v.x = ((uint64_t)wbuf[w] << 32) | wbuf[w + 1];
        v.m = excp ? (((uint32_t)mbuf[w] << 16) | mbuf[w + 1]) : 0u;
        body(i, v);
    }
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The 65 packed words (and mask half-words) of one 1024-position stage, held
// in registers: lane l has word l, lane 0 also word 64.
struct Stage {
    uint32_t w = 0, w64 = 0;
    uint16_t m = 0, m64 = 0;
    __device__ __forceinline__ void load(const uint32_t* __restrict__ packed, const uint16_t* __restrict__ mask,
                                         bool excp, int64_t wb, int lane) {
        w = packed[wb + lane];
        if (lane == 0) w64 = packed[wb + 64];
        if (excp) {
            m = mask[wb + lane];
            if (lane == 0) m64 = mask[wb + 64];
        }
    }
    __device__ __forceinline__ void put(uint32_t* wbuf, uint16_t* mbuf, bool excp, int lane) const {
        wbuf[lane] = w;
        if (lane == 0) wbuf[64] = w64;
        if (excp) {
            mbuf[lane] = m;
            if (lane == 0) mbuf[64] = m64;
        }
    }
};

// A wave walks its contig in stages of 1024 positions: the 65 packed words
// (and, for contigs with exception bases, the 65 mask half-words) of a stage
// are loaded once, coalesced, into the wave's LDS slice; every k-mer window is
// then read from LDS.  `first`, when given, is stage 0 already in registers.
template <typename Body>
__device__ __forceinline__ void for_each_window(const uint32_t* __restrict__ packed,
                                                const uint16_t* __restrict__ mask, bool excp, int64_t w0,
                                                int64_t npos, uint32_t* wbuf, uint16_t* mbuf, int lane, Body body,
                                                const Stage* first = nullptr) {
    for (int64_t base = 0; base < npos; base += 1024) {
        Stage st;
        if (first && base == 0) st = *first;
        else st.load(packed, mask, excp, w0 + (base >> 4), lane);
        st.put(wbuf, mbuf, excp, lane);
        wave_lds_sync();
        window_round(base, npos, excp, wbuf, mbuf, lane, body);
        wave_lds_sync();
    }
}

// ------------------------------------------------------------- presence ------
// One wave per contig.  Sets the ACGT-ordinal presence bitmap (LDS-private per
// block, test-before-set so the hot bits stop costing atomics, OR-flushed once
// per block) and appends the byte keys of k-mers touching an exception base.
__device__ __forceinline__ void set_bit(uint32_t* bits, uint32_t o) {
    const uint32_t m = 1u << (o & 31);
    if (!(bits[o >> 5] & m)) atomicOr(&bits[o >> 5], m);
}

template <bool P56>
__global__ void __launch_bounds__(kBlock) presence_kernel(const uint32_t* __restrict__ packed,
                                                          const uint16_t* __restrict__ mask,
                                                          const uint8_t* __restrict__ has_exc,
                                                          const int64_t* __restrict__ woff,
                                                          const int64_t* __restrict__ off,
                                                          const uint8_t* __restrict__ raw, int64_t n, int k,
                                                          int nwords, bool with_len, uint32_t* __restrict__ presence,
                                                          uint64_t* __restrict__ exc_buf, int64_t exc_cap,
                                                          unsigned long long* __restrict__ exc_cnt,
                                                          int64_t c_begin, uint32_t n_can,
                                                          const uint32_t* __restrict__ exc_list,
                                                          const unsigned* __restrict__ exc_n) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_bits[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
    uint32_t* wbuf = lds_bits + nwords + wave * 80;
    uint16_t* mbuf = reinterpret_cast<uint16_t*>(lds_bits + nwords + wpb * 80) + wave * 80;
    // the second pass (n_can = the ACGT ordinals that can occur: 4^k, or
    // 1,024 + 64 for 5p6): once all are present, only contigs with exception
    // bases can still add columns.  Each block counts the bitmap's bits itself
    // (no saturation launch between the passes)
    __shared__ unsigned present;
    if (threadIdx.x == 0) present = 0;
    __syncthreads();
    if (n_can) {
        unsigned c = 0;
        for (int w = threadIdx.x; w < nwords; w += blockDim.x) c += __popc(presence[w]);
        if (c) atomicAdd(&present, c);
    }
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) lds_bits[w] = 0;
    __syncthreads();
    const bool saturated = n_can != 0 && present >= n_can;
    const int kmin = P56 ? 5 : k;
    auto push_exc = [&](uint64_t key) {
        const unsigned long long slot = atomicAdd(exc_cnt, 1ull);
        if ((int64_t)slot < exc_cap) exc_buf[slot] = key;
    };
    auto scan = [&](int64_t c) {
        const int64_t L = off[c + 1] - off[c];
        const uint8_t* craw = raw + off[c];
        for_each_window(packed, mask, has_exc[c] != 0, woff[c], L - kmin + 1, wbuf, mbuf, lane,
                        [&](int64_t i, const Window& v) {
            if (P56) {
                if (v.clean(5)) set_bit(lds_bits, v.code(5) * 5u);  // kmer.py:72-73
                else push_exc(key_from_bytes(craw + i, 5, true));
                if (i + 6 <= L) {  // palindromic 6-mers, kmer.py:76-80
                    if (v.clean(6)) {
                        const uint32_t c6 = v.code(6);
                        if (pal6_code(c6)) set_bit(lds_bits, (c6 >> 2) * 5u + 1u + (c6 & 3u));
                    } else if (pal_bytes(craw + i, 6)) {
                        push_exc(key_from_bytes(craw + i, 6, true));
                    }
                }
            } else {
                if (v.clean(k)) set_bit(lds_bits, v.code(k));
                else push_exc(key_from_bytes(craw + i, k, with_len));
            }
        });
    };
    const int64_t w0 = (int64_t)blockIdx.x * wpb + wave, ws = (int64_t)gridDim.x * wpb;
    if (!n_can) {  // the first pass: every contig of the prefix
        for (int64_t c = c_begin + w0; c < n; c += ws) scan(c);
    } else {
        // Blocks may see different verdicts (a late block can find the set
        // completed by other blocks' flushes), so the contigs with exception
        // bases are listed out independently of it (slots of the store's
        // list) and an unsaturated block adds the ACGT-only contigs of its
        // contig slots: a saturated set gains nothing from those
        const int64_t ne = *exc_n;
        for (int64_t i = w0; i < ne; i += ws) {
            const int64_t c = exc_list[i];
            if (c >= c_begin && c < n) scan(c);
        }
        if (!saturated)
            for (int64_t c = c_begin + w0; c < n; c += ws)
                if (!has_exc[c]) scan(c);
    }
    __syncthreads();
    // OR-flush only the bits the global bitmap lacks: every block of the
    // prefix sets nearly every bit, and one atomic per block and word queued
    // ~1,000 deep on the same 160 words
    for (int w = threadIdx.x; w < nwords; w += blockDim.x) {
        const uint32_t b = lds_bits[w];
        if (b & ~__hip_atomic_load(&presence[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicOr(&presence[w], b);
    }
}

// ----------------------------------------------------------- column table ---
// One block: merges present ACGT ordinals with the sorted exception keys in
// byte-key order (= Python sorted() over str, kmer.py:172).
constexpr int kColBlock = 1024;

__global__ void __launch_bounds__(kColBlock) columns_kernel(const uint32_t* presence, int nwords,
                                                            uint32_t S, bool p56, int k, bool with_len,
                                                            const uint64_t* __restrict__ exc, int64_t X,
                                                            int32_t* __restrict__ col_of_ord,
                                                            int32_t* __restrict__ col_of_exc,
                                                            uint64_t* __restrict__ col_keys, int64_t* __restrict__ M_out,
                                                            int64_t* __restrict__ M_host, uint32_t* clear,
                                                            int clear_words) {
    extern __shared__ __attribute__((aligned(16))) uint32_t prefix[];  // nwords + 1
    // exclusive popcount prefix over the bitmap (nwords <= 2048)
    __shared__ uint32_t chunk_sum[kColBlock];
    const int per = (nwords + kColBlock - 1) / kColBlock;
    const int lo = threadIdx.x * per, hi = min(nwords, lo + per);
    uint32_t s = 0;
    for (int w = lo; w < hi; ++w) s += __popc(presence[w]);
    // exclusive scan of the chunk sums over the block: wave scans, then the
    // wave totals (a serial loop in one thread took ~15 us)
    {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        uint32_t x = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        __shared__ uint32_t wtot[kColBlock / 64];
        if (lane == 63) wtot[wave] = x;
        __syncthreads();
        uint32_t base = 0, all = 0;
        for (int w = 0; w < kColBlock / 64; ++w) {
            base += w < wave ? wtot[w] : 0u;
            all += wtot[w];
        }
        chunk_sum[threadIdx.x] = base + x - s;
        if (threadIdx.x == 0) prefix[nwords] = all;
    }
    __syncthreads();
    uint32_t run = chunk_sum[threadIdx.x];
    for (int w = lo; w < hi; ++w) {
        prefix[w] = run;
        run += __popc(presence[w]);
    }
    __syncthreads();
    const uint32_t n_present = prefix[nwords];
    for (uint32_t o = threadIdx.x; o < S; o += blockDim.x) {
        uint32_t word = presence[o >> 5];
        if ((word >> (o & 31)) & 1u) {
            uint32_t rank = prefix[o >> 5] + __popc(word & ((1u << (o & 31)) - 1u));
            uint64_t key = ord_key(o, p56, k, with_len);
            int64_t col = (int64_t)rank + lower_bound_u64(exc, X, key);
            col_of_ord[o] = (int32_t)col;
            col_keys[col] = key;
        } else {
            col_of_ord[o] = -1;
        }
    }
    for (int64_t x = threadIdx.x; x < X; x += blockDim.x) {
        const uint64_t key = exc[x];
        // number of ordinals whose key < exc key (ord_key is monotone in o)
        uint32_t lo2 = 0, hi2 = S;
        while (lo2 < hi2) {
            uint32_t mid = (lo2 + hi2) >> 1;
            if (ord_key(mid, p56, k, with_len) < key) lo2 = mid + 1;
            else hi2 = mid;
        }
        uint32_t below = prefix[lo2 >> 5] + (lo2 < S ? __popc(presence[lo2 >> 5] & ((1u << (lo2 & 31)) - 1u)) : 0u);
        if (lo2 >= S) below = n_present;
        const int64_t col = x + below;
        col_of_exc[x] = (int32_t)col;
        col_keys[col] = key;
    }
    if (threadIdx.x == 0) {
        *M_out = (int64_t)n_present + X;
        // karma_step: also into mapped host memory, read there once the step is done
        if (M_host) __hip_atomic_store(M_host, (int64_t)n_present + X, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // a caller's bitmap block (karma_step): cleared for the next plan on this
    // stream once every read above is done
    if (clear) {
        __syncthreads();
        for (int w = threadIdx.x; w < clear_words; w += blockDim.x) clear[w] = 0;
    }
}

// -------------------------------------------------------------- profile ------
// profile_wave_kernel: one wave per contig (M <= kWaveMaxM); profile_kernel:
// one block per contig (large M).
constexpr int kWaveMaxM = 4096;
#ifndef KARMA_PROF_C16
#define KARMA_PROF_C16 1
#endif
typedef double d2 __attribute__((ext_vector_type(2)));
#ifndef KARMA_ROW_AUX
// cache policy of the profile's 16-byte row stores, as buffer stores (-1: global
// stores, non-temporal per KARMA_PROF_NT).  18 = sc1 | nt: profile 0.361 -> 0.348 ms;
// measured alongside: 2 (nt) 0.358, 3 (sc0 | nt) 0.357, 19 0.353, 16 (sc1) 0.355
// with a slower step (1.30 vs 1.25 ms), 17 (sc0 | sc1) 0.354 with 1.28 ms
#define KARMA_ROW_AUX 18
#endif
#ifndef KARMA_PROF_NT
#define KARMA_PROF_NT 1  // profile rows written with non-temporal stores
#endif
template <typename T>
__device__ __forceinline__ void row_store(T v, T* p) {
    if (KARMA_PROF_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool P56, typename Add>
__device__ __forceinline__ void count_contig(const uint32_t* __restrict__ packed, const uint16_t* __restrict__ mask,
                                             bool excp, int64_t w0, const uint8_t* __restrict__ craw, int64_t L,
                                             int k, bool with_len, const int32_t* __restrict__ col_of_ord,
                                             const uint64_t* __restrict__ exc, int64_t X,
                                             const int32_t* __restrict__ col_of_exc, int64_t i0, int64_t step,
                                             Add add) {
    const int kmin = P56 ? 5 : k;
    for (int64_t i = i0; i + kmin <= L; i += step) {
        const Window v = load_window(packed, mask, w0, i, excp);
        if (P56) {
            if (v.clean(5)) add(col_of_ord[v.code(5) * 5u]);
            else add(col_of_exc[lower_bound_u64(exc, X, key_from_bytes(craw + i, 5, true))]);
            if (i + 6 <= L) {
                if (v.clean(6)) {
                    const uint32_t c6 = v.code(6);
                    if (pal6_code(c6)) add(col_of_ord[(c6 >> 2) * 5u + 1u + (c6 & 3u)]);
                } else if (pal_bytes(craw + i, 6)) {
                    add(col_of_exc[lower_bound_u64(exc, X, key_from_bytes(craw + i, 6, true))]);
                }
            }
        } else {
            if (v.clean(k)) add(col_of_ord[v.code(k)]);
            else add(col_of_exc[lower_bound_u64(exc, X, key_from_bytes(craw + i, k, with_len))]);
        }
    }
}

__device__ __forceinline__ void write_row(double* __restrict__ row, const uint32_t* __restrict__ counts, int64_t M,
                                          int32_t klen, int* __restrict__ err, int t0, int step) {
    const double len = (double)klen;
    if ((reinterpret_cast<uintptr_t>(row) & 15) == 0) {
        const int64_t M2 = M >> 1;
        for (int64_t j = t0; j < M2; j += step) {
            const uint32_t a = counts[2 * j], b = counts[2 * j + 1];
            if ((a | b) && klen == 0) *err = 1;
            d2 v;
            v.x = a ? (double)a / len : 0.0;  // IEEE correctly rounded (kmer.py:120)
            v.y = b ? (double)b / len : 0.0;
            __builtin_nontemporal_store(v, reinterpret_cast<d2*>(row) + j);
        }
        if ((M & 1) && t0 == 0) {
            const uint32_t a = counts[M - 1];
            if (a && klen == 0) *err = 1;
            __builtin_nontemporal_store(a ? (double)a / len : 0.0, row + M - 1);
        }
    } else {
        for (int64_t j = t0; j < M; j += step) {
            const uint32_t a = counts[j];
            if (a && klen == 0) *err = 1;
            __builtin_nontemporal_store(a ? (double)a / len : 0.0, row + j);
        }
    }
}

// ---- wave-per-contig profile (M <= kWaveMaxM) -------------------------------
// One wave per contig, its own LDS histogram, no block barriers after the
// table fill.  Blocks of 8 waves share one LDS column table:
//   5p6: 1024 entries by 5-mer code, then 64 by the first three bases of a
//        palindromic 6-mer (they determine it);  k: 4^k entries by code.
// C16: counters are u16, two per u32 (used when every contig is shorter than
// 2^16 bases, so no count can carry into its neighbour); this halves the
// histogram and lets 4 blocks share a CU.
// Per wave LDS: [counts][window region 128 u32] -- the window region holds the
// staged words (+ mask) while counting and the count/len table while writing.
constexpr int kProfWin = 128;  // u32 per wave past the counts

__device__ __forceinline__ uint32_t rev3(uint32_t l3) { return ((l3 & 3u) << 4) | (l3 & 12u) | (l3 >> 4); }

template <bool C16>
__device__ __forceinline__ void hist_add(uint32_t* counts, uint32_t col) {
    if (C16) atomicAdd(&counts[col >> 1], 1u << ((col & 1u) << 4));
    else atomicAdd(&counts[col], 1u);
}

// Counting for a contig without exception bases (every base A/C/G/T): lane l
// takes positions 64t + l of each 1024-position stage, so its offset inside a
// word (l mod 16) is fixed and its 16-base window is one alignbit of the word
// pair staged in LDS as a u64 (one 8-byte read per position).  The k-mer code
// is the window's top 2k bits; for 5p6 the 5-mer is the 6-mer's top 10 bits.
template <bool P56, bool C16>
__device__ __forceinline__ void count_clean(const Stage& first, const uint32_t* __restrict__ packed, int64_t w0,
                                            int64_t L, int kmin, int k, const uint16_t* __restrict__ tab,
                                            uint32_t* __restrict__ counts, uint32_t* __restrict__ win, int lane,
                                            unsigned& my) {
    uint64_t* pairs = reinterpret_cast<uint64_t*>(win);
    const int64_t npos = L - kmin + 1;
    const int o = lane & 15;
    const uint32_t sh = 32u - 2u * (uint32_t)o;
    for (int64_t b0 = 0; b0 < npos; b0 += 1024) {
        Stage st;
        if (b0 == 0) st = first;
        else st.load(packed, nullptr, false, w0 + (b0 >> 4), lane);
        // lane l: words l and l + 1 of the stage (DPP wave_shl:1; lane 63 takes word 64)
        const uint32_t w64s = (uint32_t)__builtin_amdgcn_readlane((int)st.w64, 0);
        const uint32_t wn = (uint32_t)__builtin_amdgcn_update_dpp((int)w64s, (int)st.w, 0x130, 0xF, 0xF, false);
        pairs[lane] = ((uint64_t)st.w << 32) | wn;
        wave_lds_sync();
        const uint64_t* pw = pairs + (lane >> 4);
        const int64_t lim = npos - b0 - lane;  // position 64t + lane is valid iff 64t < lim
        const int nt = (int)min<int64_t>(16, (npos - b0 + 63) >> 6);
#pragma unroll 2
        for (int t = 0; t < nt; ++t) {
            if (64 * t < lim) {
                const uint64_t x = pw[4 * t];
                const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
                const uint32_t W = o ? __builtin_amdgcn_alignbit(hi, lo, sh) : hi;
                if (P56) {
                    hist_add<C16>(counts, tab[W >> 22]);  // kmer.py:72-73
                    ++my;
                    const uint32_t c6 = W >> 20;
                    // palindromic 6-mers that fit in the contig, kmer.py:76-80
                    if ((c6 >> 6) == rev3(c6 & 63u) && 64 * t + 1 < lim) {
                        hist_add<C16>(counts, tab[1024u + (c6 >> 6)]);
                        ++my;
                    }
                } else {
                    hist_add<C16>(counts, tab[W >> (32 - 2 * k)]);
                    ++my;
                }
            }
        }
        wave_lds_sync();
    }
}

// The dense row count / len(key) (kmer.py:120, :231-233).  Counts below 64
// come from a per-row table the wave fills with the same IEEE division (lane c
// holds c / len), so a value costs one LDS read instead of one f64 division;
// larger counts still divide.  The histogram is cleared as it is read, so the
// next contig starts from zero.  16-byte non-temporal stores when the row
// start is 16-byte aligned.
template <bool C16>
__device__ __forceinline__ void write_row_wave(double* __restrict__ row, uint32_t* __restrict__ counts, int64_t M,
                                               int32_t klen, int* __restrict__ err, double* __restrict__ lut,
                                               int lane) {
    const double len = (double)klen;
    lut[lane] = lane ? (double)lane / len : 0.0;  // IEEE correctly rounded (kmer.py:120)
    wave_lds_sync();
    auto val = [&](uint32_t a) {
        double v = lut[min(a, 63u)];
        if (a >= 64u) v = (double)a / len;
        return v;
    };
    if ((reinterpret_cast<uintptr_t>(row) & 15) == 0) {
        const int64_t M2 = M >> 1;
        for (int64_t j = lane; j < M2; j += 64) {
            uint32_t a, b;
            if (C16) {
                const uint32_t ab = counts[j];
                counts[j] = 0;
                a = ab & 0xFFFFu;
                b = ab >> 16;
            } else {
                const uint2 ab = reinterpret_cast<uint2*>(counts)[j];
                reinterpret_cast<uint2*>(counts)[j] = make_uint2(0u, 0u);
                a = ab.x;
                b = ab.y;
            }
            if ((a | b) && klen == 0) *err = 1;
            d2 v;
            v.x = val(a);
            v.y = val(b);
#if KARMA_ROW_AUX >= 0  // the row's 16-byte stores as buffer stores with this cache policy
            {
                typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
                const uint64_t u = (uint64_t)row;
                const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
                    reinterpret_cast<void*>(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                                            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u)),
                    0, (int)(M * 8), 0x00020000);
                const u32x4_t w = {(uint32_t)__double2loint(v.x), (uint32_t)__double2hiint(v.x),
                                   (uint32_t)__double2loint(v.y), (uint32_t)__double2hiint(v.y)};
                __builtin_amdgcn_raw_buffer_store_b128(w, rr, (int)(j * 16), 0, KARMA_ROW_AUX);
            }
#else
            row_store(v, reinterpret_cast<d2*>(row) + j);
#endif
        }
        if ((M & 1) && lane == 0) {
            const uint32_t a = C16 ? counts[M >> 1] & 0xFFFFu : counts[M - 1];
            counts[C16 ? M >> 1 : M - 1] = 0;
            if (a && klen == 0) *err = 1;
            row_store(val(a), row + M - 1);
        }
    } else {
        uint16_t* c16 = reinterpret_cast<uint16_t*>(counts);
        for (int64_t j = lane; j < M; j += 64) {
            const uint32_t a = C16 ? c16[j] : counts[j];
            if (C16) c16[j] = 0;
            else counts[j] = 0;
            if (a && klen == 0) *err = 1;
            row_store(val(a), row + j);
        }
    }
}

// Sum over the wave's 64 lanes, in every lane: DPP row shifts and row
// broadcasts (no ds_bpermute address registers, which stayed live across the
// contig loop and spilled), then lane 63's value read as a scalar.
__device__ __forceinline__ unsigned wave_total(unsigned x) {
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (unsigned)__builtin_amdgcn_readlane((int)x, 63);
}

// u32 slots of a wave's histogram
__host__ __device__ constexpr int64_t hist_words(int64_t M, bool c16) {
    return c16 ? (((M + 1) >> 1) + 3) & ~int64_t(3) : (M + 3) & ~int64_t(3);
}
// column-table entries (u16) in LDS
__host__ __device__ constexpr int64_t tab_entries(bool p56, uint32_t S) { return p56 ? 1088 : (int64_t)S; }
// KARMA_PROF_TABREP=1 (measurement variant): the column
// table twice in LDS, lanes 32-63 reading the second copy, when it is small
// (5p6's 1,088 entries), to test whether the lookup's bank collisions bound
// the counting
#ifndef KARMA_PROF_TABREP
#define KARMA_PROF_TABREP 0
#endif
__host__ __device__ constexpr int tab_copies(int64_t t_pad) { return KARMA_PROF_TABREP && t_pad <= 4096 ? 2 : 1; }

template <bool P56, bool C16>
// 6 waves per SIMD (3 blocks per CU): fewer rows written at once write faster
// than 8 waves (4 blocks) do, and the counting still hides under the writes:
// profile 0.345-0.355 -> 0.335-0.337 ms at config 3 (round 3,
// profiles/r03/measurements.md (ab_profwaves); 7 waves: 0.407, 5: 0.497, 4: 0.499 ms)
#ifndef KARMA_PROF_WAVES
#define KARMA_PROF_WAVES 6
#endif
__global__ void __launch_bounds__(kPBlock) __attribute__((amdgpu_waves_per_eu(KARMA_PROF_WAVES, KARMA_PROF_WAVES)))
profile_wave_kernel(
    const uint32_t* __restrict__ packed, const uint16_t* __restrict__ mask, const uint8_t* __restrict__ has_exc,
    const int64_t* __restrict__ woff, const int64_t* __restrict__ off, const uint8_t* __restrict__ raw,
    const int32_t* __restrict__ keylen, int64_t n, int k, bool with_len, const int32_t* __restrict__ col_of_ord,
    const uint64_t* __restrict__ exc, int64_t X, const int32_t* __restrict__ col_of_exc, int64_t M,
    double* __restrict__ out, int64_t ld, int* __restrict__ err, int S, int64_t* __restrict__ row_tot,
    int64_t exc0, const int64_t* __restrict__ m_dev) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    // wave index in an SGPR: contig offsets and lengths load with scalar loads
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, wpb = blockDim.x >> 6;
    uint16_t* tab = reinterpret_cast<uint16_t*>(lds);
    const int t_pad = (int)((tab_entries(P56, S) + 7) & ~7);
    const int t_rep = tab_copies(t_pad);
    // LDS is laid out for M; with m_dev (the column table's count, not read
    // back to the host first) M is its capacity and the rows are dense
    const int h_words = (int)hist_words(M, C16);
    if (m_dev) {
        M = *m_dev;
        ld = M;
    }
    uint32_t* counts = lds + t_rep * t_pad / 2 + wave * (h_words + kProfWin);
    uint32_t* win = counts + h_words;
    uint16_t* mbuf = reinterpret_cast<uint16_t*>(win + 80);
    double* lut = reinterpret_cast<double*>(win);
    if (P56) {
        for (int o = threadIdx.x; o < 1088; o += blockDim.x) {
            uint32_t ord;
            if (o < 1024) {
                ord = 5u * o;
            } else {
                const uint32_t h3 = o - 1024, c6 = h3 << 6 | rev3(h3);
                ord = (c6 >> 2) * 5u + 1u + (c6 & 3u);
            }
            tab[o] = (uint16_t)col_of_ord[ord];
            if (t_rep == 2) tab[t_pad + o] = (uint16_t)col_of_ord[ord];
        }
    } else {
        for (int o = threadIdx.x; o < S; o += blockDim.x) {
            tab[o] = (uint16_t)col_of_ord[o];
            if (t_rep == 2) tab[t_pad + o] = (uint16_t)col_of_ord[o];
        }
    }
    if (t_rep == 2 && lane >= 32) tab += t_pad;  // this lane's copy
    for (int j = lane; j < h_words; j += 64) counts[j] = 0;  // write_row_wave clears it after each row
    __syncthreads();
    const int kmin = P56 ? 5 : k;
    // software pipeline over this wave's contigs: the next contig's offsets
    // load at the top of the current one, and its first stage of packed
    // words before the current row is written
    struct Meta {
        int64_t s = 0, L = 0, w0 = 0;
        int32_t klen = 0;
        bool exc = false;
    };
    auto meta = [&](int64_t cc, Meta& m) {
        if (cc < n) {
            m.s = off[cc];
            m.L = off[cc + 1] - m.s;
            m.w0 = woff[cc];
            m.klen = keylen[cc];
            // the flag byte from its dword by a scalar load (a byte load is a
            // vector load, whose wait also drains the previous row's stores)
            // (has_exc is the store's whole array, dword-aligned: contig cc of
            // these rows is entry exc0 + cc)
            const int64_t ce = exc0 + cc;
            const uint32_t hw = reinterpret_cast<const uint32_t*>(has_exc)[ce >> 2];
            m.exc = ((hw >> (8 * (ce & 3))) & 0xFFu) != 0;
        }
    };
    const int64_t stride = (int64_t)gridDim.x * wpb;
    int64_t c = (int64_t)blockIdx.x * wpb + wave;
    Meta cur, nxt;
    Stage st0;
    meta(c, cur);
    if (c < n) st0.load(packed, mask, cur.exc, cur.w0, lane);
    for (; c < n; c += stride) {
        meta(c + stride, nxt);
        const int64_t L = cur.L;
        unsigned my = 0;
        if (!cur.exc) {
            count_clean<P56, C16>(st0, packed, cur.w0, L, kmin, k, tab, counts, win, lane, my);
        } else {
            // a contig with exception bases: windows that touch one are keyed by
            // their bytes and looked up among the sorted exception keys
            const uint8_t* craw = raw + cur.s;
            auto add = [&](uint32_t cl) {
                hist_add<C16>(counts, cl);
                ++my;
            };
            for_each_window(packed, mask, true, cur.w0, L - kmin + 1, win, mbuf, lane,
                            [&](int64_t i, const Window& v) {
                if (P56) {
                    if (v.clean(5)) add(tab[v.code(5)]);
                    else add(col_of_exc[lower_bound_u64(exc, X, key_from_bytes(craw + i, 5, true))]);
                    if (i + 6 <= L) {
                        if (v.clean(6)) {
                            const uint32_t c6 = v.code(6);
                            if (pal6_code(c6)) add(tab[1024u + (c6 >> 6)]);
                        } else if (pal_bytes(craw + i, 6)) {
                            add(col_of_exc[lower_bound_u64(exc, X, key_from_bytes(craw + i, 6, true))]);
                        }
                    }
                } else {
                    if (v.clean(k)) add(tab[v.code(k)]);
                    else add(col_of_exc[lower_bound_u64(exc, X, key_from_bytes(craw + i, k, with_len))]);
                }
            }, &st0);
        }
        if (c + stride < n) st0.load(packed, mask, nxt.exc, nxt.w0, lane);
        // k-mer occurrences of the contig (0 = the all-zero row of kmer.py:250-258)
        my = wave_total(my);
        if (lane == 0) row_tot[c] = (int64_t)my;
        write_row_wave<C16>(out + c * ld, counts, M, cur.klen, err, lut, lane);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        cur = nxt;
    }
}

// ---- block-per-contig profile (large M) --------------------------------------
// One block per contig: histogram in LDS or, past the LDS budget, in a global
// scratch row.
template <bool P56, bool LDS_COUNTS>
__global__ void __launch_bounds__(kPBlock) profile_kernel(
    const uint32_t* __restrict__ packed, const uint16_t* __restrict__ mask, const uint8_t* __restrict__ has_exc,
    const int64_t* __restrict__ woff, const int64_t* __restrict__ off, const uint8_t* __restrict__ raw,
    const int32_t* __restrict__ keylen, int64_t n, int k, bool with_len, const int32_t* __restrict__ col_of_ord,
    const uint64_t* __restrict__ exc, int64_t X, const int32_t* __restrict__ col_of_exc, int64_t M,
    double* __restrict__ out, int64_t ld, uint32_t* __restrict__ scratch, int* __restrict__ err, int S,
    int64_t* __restrict__ row_tot, const int64_t* __restrict__ m_dev) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_counts[];
    {
        // scratch rows are M apart (the capacity when m_dev gives the count)
        uint32_t* counts = LDS_COUNTS ? lds_counts : scratch + (int64_t)blockIdx.x * M;
        if (m_dev) {
            M = *m_dev;
            ld = M;
        }
        for (int64_t c = blockIdx.x; c < n; c += gridDim.x) {
            for (int64_t j = threadIdx.x; j < M; j += blockDim.x) counts[j] = 0;
            __syncthreads();
            const int64_t s = off[c];
            count_contig<P56>(packed, mask, has_exc[c] != 0, woff[c], raw + s, off[c + 1] - s, k, with_len,
                              col_of_ord, exc, X, col_of_exc, threadIdx.x, blockDim.x, [&](int32_t col) {
                                  atomicAdd(&counts[col], 1u);
                                  atomicAdd(reinterpret_cast<unsigned long long*>(row_tot + c), 1ull);
                              });
            __syncthreads();
            write_row(out + c * ld, counts, M, keylen[c], err, threadIdx.x, blockDim.x);
            __syncthreads();
        }
    }
}

int grid_for(int64_t n, int64_t cap) { return (int)std::max<int64_t>(1, std::min<int64_t>(n, cap)); }

// longest contig whose key is empty: it divides by zero iff it has k-mers
// (kmer.py:213), so karma_kmer_profile can refuse before launching
// (also the longest contig overall, which sizes the profile's counters)
__global__ void zero_key_kernel(const int64_t* __restrict__ off, const int32_t* __restrict__ keylen, int64_t n,
                                unsigned long long* __restrict__ maxlen_plus1, unsigned long long* __restrict__ maxlen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long L = (unsigned long long)(off[i + 1] - off[i]);
    if (keylen[i] == 0) atomicMax(maxlen_plus1, L + 1);
    // wave maximum first: one atomic per wave
    unsigned long long m = L;
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
        const unsigned long long y = __shfl_xor(m, d);
        m = y > m ? y : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(maxlen, m);
}

int kmer_shape(int kmode, int* kmin, int* kmax, uint32_t* S, bool* with_len) {
    if (kmode == KARMA_KMER_5P6) {
        *kmin = 5;
        *kmax = 6;
        *S = 1024u * 5u;
        *with_len = true;
        return KARMA_OK;
    }
    KARMA_CHECK(kmode >= 1 && kmode <= 8, KARMA_ERR_KMER, "unsupported k-mer size %d (supported: 1..8, 5p6)", kmode);
    *kmin = *kmax = kmode;
    *S = 1u << (2 * kmode);
    *with_len = kmode < 8;
    return KARMA_OK;
}

}  // namespace

// OR of n_sets presence bitmaps laid out one after another (the ranks' bitmaps
// after an all-gather): the global column set is the union (kmer.py:146-179).
static __global__ void presence_or_kernel(const uint32_t* __restrict__ all, int n_sets, int64_t nw, uint32_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nw) return;
    uint32_t v = 0;
    for (int r = 0; r < n_sets; ++r) v |= all[(int64_t)r * nw + i];
    out[i] = v;
}

extern "C" {

int karma_contigs_create(karma_ctx* ctx, const uint8_t* seq, const int64_t* offsets, const int32_t* key_len, int64_t n,
                         int is_device, karma_contigs** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(out && offsets && key_len && n >= 0, KARMA_ERR_ARG, "karma_contigs_create: bad arguments");
    auto* c = new karma_contigs();
    c->ctx = ctx;
    c->n = n;
    int64_t total = 0;
    int rc = KARMA_OK;
    if (is_device) {
        KARMA_HIP(hipMemcpyAsync(&total, offsets + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
        c->raw = seq;
        c->off = offsets;
        c->keylen = key_len;
    } else {
        total = offsets[n];
        if ((rc = c->raw_own.alloc(ctx, (size_t)total + 16)) || (rc = c->off_own.alloc(ctx, n + 1)) ||
            (rc = c->keylen_own.alloc(ctx, n ? n : 1))) {
            delete c;
            return rc;
        }
        if (total) KARMA_HIP(hipMemcpyAsync(c->raw_own.ptr, seq, total, hipMemcpyHostToDevice, ctx->stream));
        KARMA_HIP(hipMemcpyAsync(c->off_own.ptr, offsets, (n + 1) * sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
        if (n) KARMA_HIP(hipMemcpyAsync(c->keylen_own.ptr, key_len, n * sizeof(int32_t), hipMemcpyHostToDevice, ctx->stream));
        c->raw = c->raw_own.ptr;
        c->off = c->off_own.ptr;
        c->keylen = c->keylen_own.ptr;
    }
    c->total = total;
    // word offsets: exclusive scan of ceil(L/16)
    DevArray<int64_t> wc;
    if ((rc = wc.alloc(ctx, n + 1)) || (rc = c->woff.alloc(ctx, n + 1)) || (rc = c->has_exc.alloc(ctx, (n + 4) & ~int64_t(3))) ||
        (rc = c->exc_list.alloc(ctx, n ? n : 1)) || (rc = c->exc_n.alloc(ctx, 1))) {
        delete c;
        return rc;
    }
    KARMA_LAUNCH(ctx, "word_count", word_count_kernel, ceil_div(n + 1, 256), 256, 0, c->off, n, wc.ptr);
    if ((rc = scan_excl_i64(ctx, wc.ptr, c->woff.ptr, n + 1))) {  // one look-back launch (sort.hip)
        delete c;
        return rc;
    }
    KARMA_HIP(hipMemcpyAsync(&c->words, c->woff.ptr + n, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    if ((rc = c->packed.alloc(ctx, c->words + kPadWords)) || (rc = c->mask.alloc(ctx, c->words + kPadWords))) {
        delete c;
        return rc;
    }
    KARMA_HIP(hipMemsetAsync(c->packed.ptr + c->words, 0, kPadWords * sizeof(uint32_t), ctx->stream));
    KARMA_HIP(hipMemsetAsync(c->mask.ptr + c->words, 0, kPadWords * sizeof(uint16_t), ctx->stream));
    DevArray<unsigned long long> stat;  // 0 exception bases, 1 zero-key max length + 1, 2 max length
    if ((rc = stat.alloc(ctx, 3))) {
        delete c;
        return rc;
    }
    KARMA_HIP(hipMemsetAsync(stat.ptr, 0, 3 * sizeof(unsigned long long), ctx->stream));
    KARMA_HIP(hipMemsetAsync(c->exc_n.ptr, 0, sizeof(unsigned), ctx->stream));
    if (n) {
        KARMA_LAUNCH(ctx, "pack_2bit", pack_kernel, grid_for(ceil_div(n, kBlock / 64), 8192), kBlock, 0, c->raw,
                     c->off, c->woff.ptr, n,
                     c->packed.ptr, c->mask.ptr, c->has_exc.ptr, stat.ptr, c->exc_list.ptr, c->exc_n.ptr);
        KARMA_LAUNCH(ctx, "zero_key", zero_key_kernel, ceil_div(n, 256), 256, 0, c->off, c->keylen, n, stat.ptr + 1,
                     stat.ptr + 2);
    }
    unsigned long long hs[3] = {0, 0, 0};
    KARMA_HIP(hipMemcpyAsync(hs, stat.ptr, sizeof hs, hipMemcpyDeviceToHost, ctx->stream));
    KARMA_HIP(hipStreamSynchronize(ctx->stream));
    c->exc_bases = (int64_t)hs[0];
    c->zero_key_maxlen = (int64_t)hs[1] - 1;
    c->max_len = (int64_t)hs[2];
    *out = c;
    return KARMA_OK;
}

int karma_contigs_destroy(karma_contigs* c) {
    if (!c) return KARMA_OK;
    hipSetDevice(c->ctx->device);
    delete c;
    return KARMA_OK;
}

int karma_contigs_info(karma_contigs* c, int64_t* n, int64_t* total, int64_t* exc, int64_t* packed_bytes) {
    KARMA_CHECK(c, KARMA_ERR_ARG, "null contigs");
    if (n) *n = c->n;
    if (total) *total = c->total;
    if (exc) *exc = c->exc_bases;
    if (packed_bytes) *packed_bytes = c->words * 4 + c->words * 2;
    return KARMA_OK;
}

int karma_kmer_plan_create(karma_ctx* ctx, karma_contigs* c, int kmode, karma_kmer_plan** out) {
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(c && out, KARMA_ERR_ARG, "karma_kmer_plan_create: bad arguments");
    int kmin, kmax;
    uint32_t S;
    bool with_len;
    KARMA_TRY(kmer_shape(kmode, &kmin, &kmax, &S, &with_len));
    auto* p = new karma_kmer_plan();
    p->ctx = ctx;
    p->store = c;
    p->kmode = kmode;
    p->kmin = kmin;
    p->kmax = kmax;
    p->S = S;
    p->nwords = (S + 31) / 32;
    int rc;
    const int64_t exc_cap = c->exc_bases * (kmode == KARMA_KMER_5P6 ? 11 : kmax) + 1;
    DevArray<uint64_t> exc_buf;
    // one zeroed allocation (one memset): the presence bitmap, the exception
    // k-mer counter, the row totals (8-byte aligned behind the bitmap)
    const int64_t pw = (p->nwords + 1) & ~int64_t(1);
    const int64_t nrow = c->n ? c->n : 1;
    // a caller's zeroed bitmap block (karma_step): no clearing memset; the
    // row totals need none (every profile launch writes or clears its rows)
    p->bits_ext = ctx->plan_zeroed && ctx->plan_zeroed_words >= pw + 2;
    if ((rc = p->presence.alloc(ctx, (p->bits_ext ? 0 : pw + 2) + 2 * nrow)) || (rc = p->err.alloc(ctx, 1)) ||
        (rc = exc_buf.alloc(ctx, exc_cap))) {
        delete p;
        return rc;
    }
    p->bits = p->bits_ext ? ctx->plan_zeroed : p->presence.ptr;
    if (!p->bits_ext) KARMA_HIP(hipMemsetAsync(p->presence.ptr, 0, (pw + 2 + 2 * nrow) * 4, ctx->stream));
    struct {
        unsigned long long* ptr;
    } exc_cnt{reinterpret_cast<unsigned long long*>(p->bits + pw)};
    p->row_tot = reinterpret_cast<int64_t*>(p->presence.ptr + (p->bits_ext ? 0 : pw + 2));
    if (c->n) {
        // phase A over a prefix, saturation test, phase B over the rest (only
        // contigs with exception bases once the ACGT ordinals are saturated)
        const int64_t nA = std::min<int64_t>(c->n, 4096);
        const size_t lds = p->nwords * 4 + (kBlock / 64) * 80 * (4 + 2);
        const bool p56 = kmode == KARMA_KMER_5P6;
        auto launch = [&](int64_t lo, int64_t hi, uint32_t n_can) -> int {
            if (hi <= lo) return KARMA_OK;
            const int grid = grid_for(ceil_div(hi - lo, kBlock / 64), 2048);
            if (p56)
                KARMA_LAUNCH(ctx, "kmer_presence", presence_kernel<true>, grid, kBlock, lds, c->packed.ptr,
                             c->mask.ptr, c->has_exc.ptr, c->woff.ptr, c->off, c->raw, hi, kmode, (int)p->nwords,
                             with_len, p->bits, exc_buf.ptr, exc_cap, exc_cnt.ptr, lo, n_can, c->exc_list.ptr,
                             c->exc_n.ptr);
            else
                KARMA_LAUNCH(ctx, "kmer_presence", presence_kernel<false>, grid, kBlock, lds, c->packed.ptr,
                             c->mask.ptr, c->has_exc.ptr, c->woff.ptr, c->off, c->raw, hi, kmode, (int)p->nwords,
                             with_len, p->bits, exc_buf.ptr, exc_cap, exc_cnt.ptr, lo, n_can, c->exc_list.ptr,
                             c->exc_n.ptr);
            return KARMA_OK;
        };
        KARMA_TRY(launch(0, nA, 0u));
        if (nA < c->n) KARMA_TRY(launch(nA, c->n, p56 ? 1088u : S));
    }
    unsigned long long ninst = 0;
    if (c->exc_bases) {  // exception k-mers exist only in contigs with non-ACGT bases
        KARMA_HIP(hipMemcpyAsync(&ninst, exc_cnt.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
    }
    KARMA_CHECK((int64_t)ninst <= exc_cap, KARMA_ERR_STATE, "exception k-mer buffer overflow (%llu > %lld)", ninst,
                (long long)exc_cap);
    if (ninst && (rc = sort_unique_keys(ctx, exc_buf.ptr, (int64_t)ninst, p->exc_keys, &p->n_exc))) {
        delete p;
        return rc;
    }
    *out = p;
    return KARMA_OK;
}

int karma_kmer_plan_destroy(karma_kmer_plan* p) {
    if (!p) return KARMA_OK;
    hipSetDevice(p->ctx->device);
    delete p;
    return KARMA_OK;
}

int karma_kmer_presence_words(karma_kmer_plan* p, int64_t* nwords) {
    KARMA_CHECK(p && nwords, KARMA_ERR_ARG, "null argument");
    *nwords = p->nwords;
    return KARMA_OK;
}

int karma_kmer_presence_get(karma_kmer_plan* p, uint32_t* dst) {
    KARMA_CHECK(p && dst, KARMA_ERR_ARG, "null argument");
    KARMA_TRY(ctx_begin(p->ctx));
    KARMA_HIP(hipMemcpyAsync(dst, p->bits, p->nwords * 4, hipMemcpyDeviceToDevice, p->ctx->stream));
    return KARMA_OK;
}

int karma_kmer_presence_set(karma_kmer_plan* p, const uint32_t* src) {
    KARMA_CHECK(p && src, KARMA_ERR_ARG, "null argument");
    KARMA_TRY(ctx_begin(p->ctx));
    KARMA_HIP(hipMemcpyAsync(p->bits, src, p->nwords * 4, hipMemcpyDeviceToDevice, p->ctx->stream));
    p->M = -1;
    return KARMA_OK;
}

int karma_kmer_presence_merge(karma_kmer_plan* p, const uint32_t* all, int n_sets) {
    KARMA_CHECK(p && all && n_sets >= 1, KARMA_ERR_ARG, "bad argument");
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    const int64_t nw = p->nwords;
    KARMA_LAUNCH(ctx, "kmer_presence_merge", presence_or_kernel, (int)ceil_div(nw, 256), 256, 0, all, n_sets, nw,
                 p->bits);
    p->M = -1;
    return KARMA_OK;
}

int karma_kmer_exceptions_count(karma_kmer_plan* p, int64_t* n) {
    KARMA_CHECK(p && n, KARMA_ERR_ARG, "null argument");
    *n = p->n_exc;
    return KARMA_OK;
}

int karma_kmer_exceptions_get(karma_kmer_plan* p, uint64_t* dst) {
    KARMA_CHECK(p && (dst || !p->n_exc), KARMA_ERR_ARG, "null argument");
    KARMA_TRY(ctx_begin(p->ctx));
    if (p->n_exc)
        KARMA_HIP(hipMemcpyAsync(dst, p->exc_keys.ptr, p->n_exc * 8, hipMemcpyDeviceToDevice, p->ctx->stream));
    return KARMA_OK;
}

int karma_kmer_exceptions_set(karma_kmer_plan* p, const uint64_t* src, int64_t n) {
    KARMA_CHECK(p && (src || n == 0) && n >= 0, KARMA_ERR_ARG, "bad argument");
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    p->M = -1;
    if (n == 0) {
        p->n_exc = 0;
        return KARMA_OK;
    }
    return sort_unique_keys(ctx, src, n, p->exc_keys, &p->n_exc);
}

int karma_kmer_plan_finalize_async(karma_kmer_plan* p) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null argument");
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(!p->fin_pending, KARMA_ERR_STATE, "finalize already in flight");
    int kmin, kmax;
    uint32_t S;
    bool with_len;
    KARMA_TRY(kmer_shape(p->kmode, &kmin, &kmax, &S, &with_len));
    int rc;
    if ((rc = p->col_of_ord.alloc(ctx, S)) || (rc = p->col_of_exc.alloc(ctx, p->n_exc ? p->n_exc : 1)) ||
        (rc = p->col_keys.alloc(ctx, S + p->n_exc)) || (rc = p->m_dev.alloc(ctx, 1)))
        return rc;
    const size_t lds = (p->nwords + 1) * 4;
    KARMA_LAUNCH(ctx, "kmer_columns", columns_kernel, 1, kColBlock, lds, p->bits, (int)p->nwords, S,
                 p->kmode == KARMA_KMER_5P6, p->kmode == KARMA_KMER_5P6 ? 5 : p->kmode, with_len, p->exc_keys.ptr,
                 p->n_exc, p->col_of_ord.ptr, p->col_of_exc.ptr, p->col_keys.ptr, p->m_dev.ptr, (int64_t*)nullptr,
                 p->bits_ext ? p->bits : nullptr, (int)(((p->nwords + 1) & ~int64_t(1)) + 2));
    if (!ctx->fin_pinned) KARMA_HIP(hipHostMalloc(reinterpret_cast<void**>(&ctx->fin_pinned), 64, hipHostMallocDefault));
    KARMA_HIP(hipMemcpyAsync(ctx->fin_pinned, p->m_dev.ptr, 8, hipMemcpyDeviceToHost, ctx->stream));
    if (!p->fin_ev) KARMA_HIP(hipEventCreateWithFlags(&p->fin_ev, hipEventDisableTiming));
    KARMA_HIP(hipEventRecord(p->fin_ev, ctx->stream));
    p->fin_pending = true;
    return KARMA_OK;
}

}  // extern "C"

static int profile_rows(karma_kmer_plan* p, int64_t lo, int64_t hi, double* out, int64_t ld, int out_is_device,
                        const int64_t* m_dev);

namespace karma {
// The column table without M's readback (karma_step's deferred steps): M is
// written to m_out on the device (the caller's word) for the profile kernels;
// the host learns it later.
int kmer_finalize_device(karma_kmer_plan* p, int64_t* m_out, int64_t* m_host) {
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    int kmin, kmax;
    uint32_t S;
    bool with_len;
    KARMA_TRY(kmer_shape(p->kmode, &kmin, &kmax, &S, &with_len));
    int rc;
    if ((rc = p->col_of_ord.alloc(ctx, S)) || (rc = p->col_of_exc.alloc(ctx, p->n_exc ? p->n_exc : 1)) ||
        (rc = p->col_keys.alloc(ctx, S + p->n_exc)))
        return rc;
    const size_t lds = (p->nwords + 1) * 4;
    KARMA_LAUNCH(ctx, "kmer_columns", columns_kernel, 1, kColBlock, lds, p->bits, (int)p->nwords, S,
                 p->kmode == KARMA_KMER_5P6, p->kmode == KARMA_KMER_5P6 ? 5 : p->kmode, with_len, p->exc_keys.ptr,
                 p->n_exc, p->col_of_ord.ptr, p->col_of_exc.ptr, p->col_keys.ptr, m_out, m_host,
                 p->bits_ext ? p->bits : nullptr, (int)(((p->nwords + 1) & ~int64_t(1)) + 2));
    return KARMA_OK;
}

int kmer_profile_device_m(karma_kmer_plan* p, double* out_dev, const int64_t* m_dev) {
    return profile_rows(p, 0, p->store->n, out_dev, 0, 1, m_dev);
}

// the column keys of a plan finalized on the device, once M is known
int kmer_set_m(karma_kmer_plan* p, int64_t M) {
    KARMA_CHECK(M >= 0 && M <= kmer_m_cap(p), KARMA_ERR_STATE, "column count %lld outside [0, %lld]", (long long)M,
                (long long)kmer_m_cap(p));
    p->M = M;
    return KARMA_OK;
}
}  // namespace karma

extern "C" {

int karma_kmer_plan_finalize_wait(karma_kmer_plan* p, int64_t* M) {
    KARMA_CHECK(p && M, KARMA_ERR_ARG, "null argument");
    KARMA_CHECK(p->fin_pending, KARMA_ERR_STATE, "no finalize in flight");
    KARMA_TRY(ctx_begin(p->ctx));
    KARMA_HIP(hipEventSynchronize(p->fin_ev));  // the column table only, not later work on the stream
    p->fin_pending = false;
    p->M = *p->ctx->fin_pinned;
    *M = p->M;
    return KARMA_OK;
}

int karma_kmer_plan_finalize(karma_kmer_plan* p, int64_t* M) {
    KARMA_TRY(karma_kmer_plan_finalize_async(p));
    return karma_kmer_plan_finalize_wait(p, M);
}

int karma_kmer_columns(karma_kmer_plan* p, uint64_t* keys_host) {
    KARMA_CHECK(p && p->M >= 0, KARMA_ERR_STATE, "karma_kmer_columns before finalize");
    KARMA_TRY(ctx_begin(p->ctx));
    if (p->M) {
        KARMA_CHECK(keys_host, KARMA_ERR_ARG, "null keys");
        KARMA_HIP(hipMemcpyAsync(keys_host, p->col_keys.ptr, p->M * 8, hipMemcpyDeviceToHost, p->ctx->stream));
        KARMA_HIP(hipStreamSynchronize(p->ctx->stream));
    }
    return KARMA_OK;
}

int karma_kmer_row_totals(karma_kmer_plan* p, int64_t* dst) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null plan");
    KARMA_TRY(ctx_begin(p->ctx));
    if (p->store->n) {
        KARMA_CHECK(dst, KARMA_ERR_ARG, "null dst");
        KARMA_HIP(hipMemcpyAsync(dst, p->row_tot, p->store->n * 8, hipMemcpyDeviceToHost, p->ctx->stream));
        KARMA_HIP(hipStreamSynchronize(p->ctx->stream));
    }
    return KARMA_OK;
}

// Rows [lo, hi) of the profile: the per-contig arrays are passed shifted by lo
// (packed words and raw bytes are addressed through them), so row r of `out`
// is contig lo + r.
// m_dev: M is read by the kernels from the column table's count on the device
// (karma_step's path: no host wait for it); the launch is sized for
// kmer_m_cap(p) >= M and rows are written dense (ld = M).
static int profile_rows(karma_kmer_plan* p, int64_t lo, int64_t hi, double* out, int64_t ld, int out_is_device,
                        const int64_t* m_dev) {
    KARMA_CHECK(p && (p->M >= 0 || m_dev), KARMA_ERR_STATE, "karma_kmer_profile before finalize");
    karma_ctx* ctx = p->ctx;
    karma_contigs* c = p->store;
    KARMA_TRY(ctx_begin(ctx));
    KARMA_CHECK(m_dev || ld >= p->M, KARMA_ERR_ARG, "ld (%lld) < M (%lld)", (long long)ld, (long long)p->M);
    KARMA_CHECK(!m_dev || out_is_device, KARMA_ERR_ARG, "device M needs a device output");
    KARMA_CHECK(0 <= lo && lo <= hi && hi <= c->n, KARMA_ERR_ARG, "rows [%lld, %lld) outside [0, %lld)",
                (long long)lo, (long long)hi, (long long)c->n);
    const int64_t n = hi - lo, M = m_dev ? kmer_m_cap(p) : p->M;
    if (n == 0) return KARMA_OK;
    int64_t* const row_tot = p->row_tot + lo;
    const uint8_t* const has_exc = c->has_exc.ptr + lo;
    const int64_t* const woff = c->woff.ptr + lo;
    const int64_t* const off = c->off + lo;
    const int32_t* const keylen = c->keylen + lo;
    const bool wave = M <= kWaveMaxM && p->S <= 8192;
    // row totals: with M == 0 every row is all-zero (kmer.py:250-258); the
    // block kernel adds to them; the wave kernel writes every row's total
    if (M == 0 || !wave) KARMA_HIP(hipMemsetAsync(row_tot, 0, n * 8, ctx->stream));
    if (M == 0) return KARMA_OK;
    KARMA_CHECK(out, KARMA_ERR_ARG, "null out");
    KARMA_CHECK(c->zero_key_maxlen < p->kmin, KARMA_ERR_ZERO_DIV,
                "division by zero: a contig with a zero-length key has k-mers");
    int rc;
    DevArray<double> dev_out;
    double* dst = out;
    if (!out_is_device) {
        if ((rc = dev_out.alloc(ctx, (size_t)n * ld))) return rc;
        dst = dev_out.ptr;
    }
    // a kernel-side flag for a zero-length key's row with k-mers; the host
    // check above (zero_key_maxlen) is the error path, so the flag is never
    // read and not cleared per launch
    int* const err = p->err.ptr;  // no temporaries: the launch may run on a side stream
    bool with_len = p->kmode != 8;
    const int k = p->kmode == KARMA_KMER_5P6 ? 5 : p->kmode;
    if (wave) {
        // one round of resident blocks, each wave striding over contigs; u16
        // counters when no contig reaches 2^16 bases (a count is <= L)
        const bool p56 = p->kmode == KARMA_KMER_5P6;
        const bool c16 = KARMA_PROF_C16 && c->max_len < 65536;
        const int64_t t_pad = (tab_entries(p56, p->S) + 7) & ~7;
        size_t lds = (size_t)(t_pad * tab_copies(t_pad)) * 2 +
                     (kPBlock / 64) * (size_t)(hist_words(M, c16) + kProfWin) * 4;
        // KARMA_PROF_LDS_MIN (A/B): LDS per block at least this many bytes
        static const size_t lds_min = [] {
            const char* e = std::getenv("KARMA_PROF_LDS_MIN");
            return e ? (size_t)std::atoll(e) : (size_t)0;
        }();
        lds = std::max(lds, lds_min);
#define KARMA_WAVE_LAUNCH(P56, C16)                                                                              \
    do {                                                                                                         \
        const int g_ = resident_grid(ctx, reinterpret_cast<const void*>(&profile_wave_kernel<P56, C16>), kPBlock, \
                                     lds, ceil_div(n, kPBlock / 64));                                            \
        KARMA_LAUNCH(ctx, "kmer_profile", (profile_wave_kernel<P56, C16>), g_, kPBlock, lds, c->packed.ptr,      \
                     c->mask.ptr, c->has_exc.ptr, woff, off, c->raw, keylen, n, k, with_len,                     \
                     p->col_of_ord.ptr, p->exc_keys.ptr, p->n_exc, p->col_of_exc.ptr, M, dst, ld, err,       \
                     (int)p->S, row_tot, lo, m_dev);                                                             \
    } while (0)
        if (p56) {
            if (c16) KARMA_WAVE_LAUNCH(true, true);
            else KARMA_WAVE_LAUNCH(true, false);
        } else {
            if (c16) KARMA_WAVE_LAUNCH(false, true);
            else KARMA_WAVE_LAUNCH(false, false);
        }
#undef KARMA_WAVE_LAUNCH
    } else {
        const bool lds_ok = M * 4 <= 144 * 1024;
        const int grid = grid_for(n, lds_ok ? 4096 : 1024);
        DevArray<uint32_t> scratch;
        if (!lds_ok && (rc = scratch.alloc(ctx, (size_t)grid * M))) return rc;
        const size_t lds = lds_ok ? M * 4 : 0;
#define KARMA_PROFILE_LAUNCH(P56, LDS)                                                                           \
    KARMA_LAUNCH(ctx, "kmer_profile", (profile_kernel<P56, LDS>), grid, kPBlock, lds, c->packed.ptr, c->mask.ptr, \
                 has_exc, woff, off, c->raw, keylen, n, k, with_len, p->col_of_ord.ptr,                          \
                 p->exc_keys.ptr, p->n_exc, p->col_of_exc.ptr, M, dst, ld, scratch.ptr, err, (int)p->S,      \
                 row_tot, m_dev)
        if (p->kmode == KARMA_KMER_5P6) {
            if (lds_ok) KARMA_PROFILE_LAUNCH(true, true);
            else KARMA_PROFILE_LAUNCH(true, false);
        } else {
            if (lds_ok) KARMA_PROFILE_LAUNCH(false, true);
            else KARMA_PROFILE_LAUNCH(false, false);
        }
#undef KARMA_PROFILE_LAUNCH
    }
    if (!out_is_device) {
        KARMA_HIP(hipMemcpyAsync(out, dst, (size_t)n * ld * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
        KARMA_HIP(hipStreamSynchronize(ctx->stream));
    }
    return KARMA_OK;
}

int karma_kmer_profile(karma_kmer_plan* p, double* out, int64_t ld, int out_is_device) {
    KARMA_CHECK(p && p->store, KARMA_ERR_STATE, "karma_kmer_profile: null plan");
    return profile_rows(p, 0, p->store->n, out, ld, out_is_device, nullptr);
}

int karma_kmer_profile_rows(karma_kmer_plan* p, int64_t row_lo, int64_t row_hi, double* out, int64_t ld,
                            int out_is_device) {
    return profile_rows(p, row_lo, row_hi, out, ld, out_is_device, nullptr);
}

int karma_kmer_profile_side(karma_kmer_plan* p, double* out_dev, int64_t ld, void* side) {
    KARMA_CHECK(p, KARMA_ERR_ARG, "null plan");
    karma_ctx* ctx = p->ctx;
    KARMA_TRY(ctx_begin(ctx));
    // the general kernel past 36,864 columns allocates scratch: main stream
    if (!side || (p->M > kWaveMaxM && p->M * 4 > 144 * 1024)) return karma_kmer_profile(p, out_dev, ld, 1);
    hipStream_t s = static_cast<hipStream_t>(side);
    KARMA_CHECK(p->fin_ev && p->M >= 0, KARMA_ERR_STATE, "karma_kmer_profile_side before finalize");
    if (ctx->mark_set) {
        // an open graph job: start once its classify kernel and this plan's
        // column table are done (the job's later kernels overlap the profile)
        KARMA_HIP(hipStreamWaitEvent(s, ctx->mark_ev, 0));
        KARMA_HIP(hipStreamWaitEvent(s, p->fin_ev, 0));
    } else {
        if (!ctx->side_ev) KARMA_HIP(hipEventCreateWithFlags(&ctx->side_ev, hipEventDisableTiming));
        KARMA_HIP(hipEventRecord(ctx->side_ev, ctx->stream));  // after everything enqueued on the main stream
        KARMA_HIP(hipStreamWaitEvent(s, ctx->side_ev, 0));
    }
    hipStream_t main_stream = ctx->stream;
    ctx->stream = s;  // launches and timing events go to the side stream
    // its one-round grid leaves a block slot per CU, so the main stream's
    // short kernels find room beside it instead of queueing behind it
    ctx->grid_headroom = ctx->side_headroom;
    const int rc = karma_kmer_profile(p, out_dev, ld, 1);
    ctx->grid_headroom = 0;
    ctx->stream = main_stream;
    return rc;
}

int karma_ctx_set_side_headroom(karma_ctx* ctx, int blocks_per_cu) {
    KARMA_CHECK(ctx && blocks_per_cu >= 0, KARMA_ERR_ARG, "karma_ctx_set_side_headroom: bad arguments");
    ctx->side_headroom = blocks_per_cu;
    return KARMA_OK;
}

int karma_ctx_join(karma_ctx* ctx, void* side) {
    KARMA_CHECK(ctx, KARMA_ERR_ARG, "null ctx");
    if (!side) return KARMA_OK;
    KARMA_TRY(ctx_begin(ctx));
    if (!ctx->side_ev) KARMA_HIP(hipEventCreateWithFlags(&ctx->side_ev, hipEventDisableTiming));
    KARMA_HIP(hipEventRecord(ctx->side_ev, static_cast<hipStream_t>(side)));
    KARMA_HIP(hipStreamWaitEvent(ctx->stream, ctx->side_ev, 0));
    return KARMA_OK;
}

}  // extern "C"
