// ingest.cpp — host-side parsers of the path's input formats (SURVEY.md §8(b),
// §8(f) row 1), multi-threaded C++ over an in-memory buffer.
//
//   karma_fasta_*  read_fasta_file              karma/karma.py:40-61
//   karma_eq_*     the eq_classes.txt parse of  karma/read_graph.py:75-92
//   karma_sam_*    Contig readsets from SAM     karma/contig.py:24,34 + hisat2.py:49-53
//
// Text semantics follow Python's text-mode open(): UTF-8 (strict) and
// universal newlines ("\r\n", "\r" and "\n" each end a line and are not part
// of it).  A parser accepts only input whose reference result it reproduces
// exactly; everything else returns KARMA_ERR_PARSE with the offending line, and
// the Python front end re-runs the reference-semantics reader to raise the
// reference's own exception (karma_amd/fasta.py, read_graph.py, contig.py).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/karma.h"

namespace karma {
void set_error(const char* fmt, ...);
}

namespace {

using karma::set_error;

// Minimum work per thread is divided by this; the sanitizer fuzz build
// (Makefile `asan`) raises it so that small random texts still split into
// many thread chunks and the chunk-merge code runs under the sanitizers.
#ifndef KARMA_INGEST_SPLIT_DIV
#define KARMA_INGEST_SPLIT_DIV 1
#endif

int clamp_threads(int threads, size_t work, size_t per_thread) {
    per_thread = std::max<size_t>(1, per_thread / KARMA_INGEST_SPLIT_DIV);
    int t = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
    t = std::max(1, std::min(t, 64));
    const size_t by_work = std::max<size_t>(1, work / per_thread);
    return (int)std::min<size_t>((size_t)t, by_work);
}

template <typename F>
void parallel_for(int T, F&& f) {
    if (T == 1) {
        f(0);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(T);
    for (int t = 0; t < T; ++t) th.emplace_back([&, t] { f(t); });
    for (auto& x : th) x.join();
}

// Strict UTF-8 as CPython decodes it (no overlongs, no surrogates, <= U+10FFFF).
// Returns the offset of the first invalid byte, or len.
size_t utf8_invalid_at(const uint8_t* s, size_t len) {
    size_t i = 0;
    while (i < len) {
        const uint8_t c = s[i];
        if (c < 0x80) {
            ++i;
            continue;
        }
        int n;
        uint32_t lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) n = 1;
        else if (c == 0xE0) n = 2, lo = 0xA0;
        else if (c >= 0xE1 && c <= 0xEC) n = 2;
        else if (c == 0xED) n = 2, hi = 0x9F;
        else if (c >= 0xEE && c <= 0xEF) n = 2;
        else if (c == 0xF0) n = 3, lo = 0x90;
        else if (c >= 0xF1 && c <= 0xF3) n = 3;
        else if (c == 0xF4) n = 3, hi = 0x8F;
        else return i;
        if (i + (size_t)n >= len) return i;  // truncated sequence
        if (s[i + 1] < lo || s[i + 1] > hi) return i;
        for (int k = 2; k <= n; ++k)
            if (s[i + k] < 0x80 || s[i + k] > 0xBF) return i;
        i += n + 1;
    }
    return len;
}

bool is_ascii(const uint8_t* s, size_t len) {
    uint8_t acc = 0;
    for (size_t i = 0; i < len; ++i) acc |= s[i];
    return acc < 0x80;
}

// code points of a valid UTF-8 range
int64_t code_points(const uint8_t* s, size_t len) {
    int64_t n = 0;
    for (size_t i = 0; i < len; ++i) n += (s[i] & 0xC0) != 0x80;
    return n;
}

inline bool is_nl(uint8_t c) { return c == '\n' || c == '\r'; }

// end of the line starting at p (first '\r' or '\n', or len)
inline size_t line_end(const uint8_t* s, size_t len, size_t p) {
    while (p < len && !is_nl(s[p])) ++p;
    return p;
}

// start of the next line after a line ending at e (skips one terminator)
inline size_t next_line(const uint8_t* s, size_t len, size_t e) {
    if (e >= len) return len;
    if (s[e] == '\r' && e + 1 < len && s[e + 1] == '\n') return e + 2;
    return e + 1;
}

// T + 1 cut points of [lo, len) at line starts (cut[0] = lo, cut[T] = len)
std::vector<size_t> line_cuts(const uint8_t* s, size_t lo, size_t len, int T) {
    std::vector<size_t> cut(T + 1, len);
    cut[0] = lo;
    for (int t = 1; t < T; ++t) {
        size_t c = std::max(cut[t - 1], lo + (len - lo) * t / T);
        const bool at_start = c == lo || c >= len || s[c - 1] == '\n' || (s[c - 1] == '\r' && s[c] != '\n');
        if (!at_start) c = next_line(s, len, line_end(s, len, c));
        cut[t] = c;
    }
    return cut;
}

// Python int(str) restricted to ASCII: surrounding whitespace, optional sign,
// digits with single underscores between them.  false: not decided here (the
// Python front end re-parses).
bool py_int_ascii(const uint8_t* s, size_t n, int64_t* out) {
    auto ws = [](uint8_t c) { return c == ' ' || (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x1F); };
    size_t a = 0, b = n;
    while (a < b && ws(s[a])) ++a;
    while (b > a && ws(s[b - 1])) --b;
    if (a == b) return false;
    bool neg = false;
    if (s[a] == '+' || s[a] == '-') {
        neg = s[a] == '-';
        ++a;
    }
    if (a == b || s[a] == '_' || s[b - 1] == '_') return false;
    uint64_t v = 0;
    for (size_t i = a; i < b; ++i) {
        const uint8_t c = s[i];
        if (c == '_') {
            if (s[i - 1] == '_') return false;
            continue;
        }
        if (c < '0' || c > '9') return false;
        if (v > (UINT64_C(1) << 62)) return false;  // beyond int64: Python path
        v = v * 10 + (c - '0');
    }
    if (v > (uint64_t)INT64_MAX) return false;
    *out = neg ? -(int64_t)v : (int64_t)v;
    return true;
}

// canonical str(i) for 0 <= i < n (no sign, no leading zero, no whitespace)
inline bool canonical_index(const uint8_t* s, size_t len, int64_t n, uint32_t* out) {
    if (len == 0 || len > 19 || (len > 1 && s[0] == '0')) return false;
    uint64_t v = 0;
    for (size_t i = 0; i < len; ++i) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (s[i] - '0');
    }
    if (v >= (uint64_t)n) return false;
    *out = (uint32_t)v;
    return true;
}

struct SVHash {
    size_t operator()(std::string_view v) const noexcept {
        // FNV-1a 64
        uint64_t h = 1469598103934665603ull;
        for (unsigned char c : v) h = (h ^ c) * 1099511628211ull;
        return (size_t)h;
    }
};

uint64_t hash_bytes(const uint8_t* s, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ s[i]) * 1099511628211ull;
    return h ^ (h >> 29);
}

}  // namespace

// ============================================================================
// FASTA — read_fasta_file (karma/karma.py:40-61)
//   name = first line, "\n" stripped, split(" ")[0] (">" kept); any later line
//   starting with ">" opens the next record; sequence = concatenated lines;
//   a repeated name keeps its first position and takes the last sequence
//   (OrderedDict assignment).  Key lengths are in code points (kmer.py:213
//   normalises by len(key)).
// ============================================================================
struct karma_fasta {
    std::unique_ptr<uint8_t[]> seq;  // seq_off[N] bytes + 16 zero bytes of padding (karma_contigs_create)
    std::vector<int64_t> seq_off;    // N + 1
    std::unique_ptr<char[]> keys;
    std::vector<int64_t> key_off;    // N + 1
    std::vector<int32_t> key_len;    // code points
    bool ascii = true;
};

namespace {

// line terminator bytes in [p, p + n), and the OR of all bytes (high bit: not ASCII)
inline int64_t count_nl(const uint8_t* p, size_t n, uint8_t* acc) {
    int64_t c = 0;
    uint8_t o = 0;
    for (size_t i = 0; i < n; ++i) {
        c += (p[i] == '\n') | (p[i] == '\r');
        o |= p[i];
    }
    *acc |= o;
    return c;
}

// open-addressing set of byte strings: first index of each distinct key
struct KeyTable {
    std::vector<int64_t> slot;  // -1 empty, else an item index
    size_t mask;
    explicit KeyTable(size_t n) {
        size_t cap = 16;
        while (cap < 2 * n + 16) cap <<= 1;
        slot.assign(cap, -1);
        mask = cap - 1;
    }
    // returns the index stored for the key (inserting `idx` if new)
    template <typename Eq>
    int64_t find_or_insert(uint64_t h, int64_t idx, Eq eq) {
        for (size_t i = h & mask;; i = (i + 1) & mask) {
            if (slot[i] < 0) {
                slot[i] = idx;
                return idx;
            }
            if (eq(slot[i])) return slot[i];
        }
    }
};

}  // namespace

static int fasta_parse_impl(const char* data_c, size_t len, int threads, karma_fasta** out) {
    if (!out || (!data_c && len)) {
        set_error("karma_fasta_parse: null argument");
        return KARMA_ERR_ARG;
    }
    *out = nullptr;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(data_c);
    const int T = clamp_threads(threads, len, 1 << 20);
    const size_t per = (len + T - 1) / (size_t)T;
    // ---- 1 (one pass): header line starts (a '>' right after a line terminator),
    // terminator counts between them, and the byte OR (ASCII check)
    struct Chunk {
        int64_t head_nl = 0;          // terminators before the chunk's first header
        std::vector<size_t> pos;      // headers found in the chunk
        std::vector<int64_t> nl;      // terminators from each header to the next / the chunk end
        uint8_t acc = 0;
    };
    std::vector<Chunk> ch(T);
    parallel_for(T, [&](int t) {
        Chunk& C = ch[t];
        const size_t lo = std::min(len, (size_t)t * per), hi = std::min(len, lo + per);
        size_t seg = lo;
        int64_t* cur = &C.head_nl;
        for (size_t p = std::max<size_t>(lo, 1); p < hi;) {
            const void* q = memchr(s + p, '>', hi - p);
            if (!q) break;
            const size_t i = (const uint8_t*)q - s;
            p = i + 1;
            if (!is_nl(s[i - 1])) continue;
            *cur += count_nl(s + seg, i - seg, &C.acc);
            C.pos.push_back(i);
            C.nl.push_back(0);
            cur = &C.nl.back();
            seg = i;
        }
        *cur += count_nl(s + seg, hi - seg, &C.acc);
    });
    bool ascii = true;
    for (auto& C : ch) ascii = ascii && C.acc < 0x80;
    if (!ascii) {
        const size_t bad = utf8_invalid_at(s, len);
        if (bad != len) {
            set_error("fasta: invalid UTF-8 at byte %zu", bad);
            return KARMA_ERR_PARSE;
        }
    }
    // record r: header line at h[r], up to h[r + 1]; nl[r] terminators inside
    std::vector<size_t> h(1, 0);
    std::vector<int64_t> nl(1, 0);
    for (auto& C : ch) {
        nl.back() += C.head_nl;
        h.insert(h.end(), C.pos.begin(), C.pos.end());
        nl.insert(nl.end(), C.nl.begin(), C.nl.end());
    }
    const int64_t R = (int64_t)h.size();
    h.push_back(len);
    // ---- 2: per record key range, body start, sequence size, key hash
    std::vector<size_t> kend(R), body(R);
    std::vector<int64_t> slen(R);
    std::vector<uint64_t> kh(R);
    const int TR = clamp_threads(threads, (size_t)R, 1024);
    parallel_for(TR, [&](int t) {
        const int64_t lo = R * t / TR, hi = R * (t + 1) / TR;
        for (int64_t r = lo; r < hi; ++r) {
            const size_t e = line_end(s, len, h[r]);
            const void* sp = memchr(s + h[r], ' ', e - h[r]);
            kend[r] = sp ? (size_t)((const uint8_t*)sp - s) : e;
            body[r] = next_line(s, len, e);
            slen[r] = (int64_t)(h[r + 1] - e) - nl[r];  // the header line holds no terminator
            kh[r] = hash_bytes(s + h[r], kend[r] - h[r]);
        }
    });
    // ---- 3: OrderedDict assignment: first position, last value
    std::vector<int64_t> slot(R);  // output slot of record r
    std::vector<int64_t> src;      // output slot -> record providing the value
    std::vector<int64_t> first_rec;
    src.reserve(R);
    first_rec.reserve(R);
    {
        KeyTable tab((size_t)R);
        for (int64_t r = 0; r < R; ++r) {
            const size_t kl = kend[r] - h[r];
            const int64_t f0 = tab.find_or_insert(kh[r], r, [&](int64_t o) {
                return kh[o] == kh[r] && kend[o] - h[o] == kl && memcmp(s + h[o], s + h[r], kl) == 0;
            });
            if (f0 == r) {
                slot[r] = (int64_t)src.size();
                src.push_back(r);
                first_rec.push_back(r);
            } else {
                slot[r] = slot[f0];
                src[slot[r]] = r;
            }
        }
    }
    const int64_t N = (int64_t)src.size();
    auto* f = new karma_fasta;
    f->ascii = ascii;
    f->seq_off.assign(N + 1, 0);
    f->key_off.assign(N + 1, 0);
    f->key_len.assign(N, 0);
    for (int64_t i = 0; i < N; ++i) {
        const int64_t kr = first_rec[i], vr = src[i];
        f->seq_off[i + 1] = f->seq_off[i] + slen[vr];
        f->key_off[i + 1] = f->key_off[i] + (int64_t)(kend[kr] - h[kr]);
    }
    try {
        f->seq.reset(new uint8_t[(size_t)f->seq_off[N] + 16]);
        f->keys.reset(new char[(size_t)f->key_off[N] + 1]);
    } catch (...) {
        delete f;
        set_error("fasta: out of host memory");
        return KARMA_ERR_OOM;
    }
    memset(f->seq.get() + f->seq_off[N], 0, 16);
    // ---- 4: copy keys and sequences (terminators dropped)
    const int TN = clamp_threads(threads, (size_t)N, 1024);
    parallel_for(TN, [&](int t) {
        const int64_t lo = N * t / TN, hi = N * (t + 1) / TN;
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t kr = first_rec[i], vr = src[i];
            const size_t kl = kend[kr] - h[kr];
            memcpy(f->keys.get() + f->key_off[i], s + h[kr], kl);
            f->key_len[i] = (int32_t)(ascii ? (int64_t)kl : code_points(s + h[kr], kl));
            uint8_t* d = f->seq.get() + f->seq_off[i];
            for (size_t p = body[vr]; p < h[vr + 1];) {
                const void* q = memchr(s + p, '\n', h[vr + 1] - p);
                size_t e = q ? (size_t)((const uint8_t*)q - s) : h[vr + 1];
                const void* r = memchr(s + p, '\r', e - p);  // a '\r' ends the line first
                if (r) e = (size_t)((const uint8_t*)r - s);
                memcpy(d, s + p, e - p);
                d += e - p;
                p = next_line(s, h[vr + 1], e);
            }
        }
    });
    *out = f;
    return KARMA_OK;
}

// Host allocation failures (e.g. a count in the input far beyond its size)
// must not unwind through the C boundary.
extern "C" int karma_fasta_parse(const char* data_c, size_t len, int threads, karma_fasta** out) {
    try {
        return fasta_parse_impl(data_c, len, threads, out);
    } catch (const std::bad_alloc&) {
        set_error("karma_fasta_parse: out of host memory");
        return KARMA_ERR_OOM;
    } catch (const std::exception& e) {
        set_error("karma_fasta_parse: %s", e.what());
        return KARMA_ERR_PARSE;
    }
}

extern "C" int karma_fasta_info(karma_fasta* f, int64_t* n, int64_t* seq_bytes, int64_t* key_bytes, int* ascii) {
    if (!f) {
        set_error("karma_fasta_info: null handle");
        return KARMA_ERR_ARG;
    }
    const int64_t N = (int64_t)f->key_len.size();
    if (n) *n = N;
    if (seq_bytes) *seq_bytes = f->seq_off[N];
    if (key_bytes) *key_bytes = f->key_off[N];
    if (ascii) *ascii = f->ascii ? 1 : 0;
    return KARMA_OK;
}

// Output copies of the get calls: nothing to do for a null destination or an
// empty array (whose data() may be null, which memcpy must not see).
static inline void copy_out(void* dst, const void* src, size_t bytes) {
    if (dst && bytes) memcpy(dst, src, bytes);
}

extern "C" int karma_fasta_get(karma_fasta* f, uint8_t* seq, int64_t* seq_off, char* keys, int64_t* key_off,
                               int32_t* key_len) {
    if (!f) {
        set_error("karma_fasta_get: null handle");
        return KARMA_ERR_ARG;
    }
    const int64_t N = (int64_t)f->key_len.size();
    copy_out(seq, f->seq.get(), (size_t)f->seq_off[N] + 16);
    copy_out(seq_off, f->seq_off.data(), sizeof(int64_t) * (N + 1));
    copy_out(keys, f->keys.get(), (size_t)f->key_off[N]);
    copy_out(key_off, f->key_off.data(), sizeof(int64_t) * (N + 1));
    copy_out(key_len, f->key_len.data(), sizeof(int32_t) * N);
    return KARMA_OK;
}

extern "C" int karma_fasta_view(karma_fasta* f, const uint8_t** seq, const int64_t** seq_off, const char** keys,
                                const int64_t** key_off, const int32_t** key_len) {
    if (!f) {
        set_error("karma_fasta_view: null handle");
        return KARMA_ERR_ARG;
    }
    if (seq) *seq = f->seq.get();
    if (seq_off) *seq_off = f->seq_off.data();
    if (keys) *keys = f->keys.get();
    if (key_off) *key_off = f->key_off.data();
    if (key_len) *key_len = f->key_len.data();
    return KARMA_OK;
}

extern "C" int karma_fasta_destroy(karma_fasta* f) {
    delete f;
    return KARMA_OK;
}

// ============================================================================
// Salmon eq_classes.txt — karma/read_graph.py:75-92
//   line 1: int(n); line 2 ignored; n name lines ("\n" stripped; "" past EOF);
//   every remaining line: split("\t") -> eq_size, *contig_ids, count with
//   count = int(count), each id a key str(i) of the name table, eq_size
//   compared with "1" as a string (:102).  Duplicate names fail the assert at
//   :93 (totals are keyed by name).
// ============================================================================
struct karma_eq {
    std::vector<char> names;
    std::vector<int64_t> name_off;  // n + 1
    std::vector<int64_t> cls_off;   // C + 1
    std::vector<uint32_t> members;
    std::vector<int64_t> counts;
    std::vector<uint8_t> pair_skip;
};

namespace {

struct EqPart {
    std::vector<int64_t> sizes;
    std::vector<uint32_t> members;
    std::vector<int64_t> counts;
    std::vector<uint8_t> skip;
    int64_t bad_line = -1;  // first failing line (local index)
    const char* why = nullptr;
    int64_t lines = 0;
};

void parse_eq_lines(const uint8_t* s, size_t lo, size_t hi, int64_t n, EqPart& P) {
    size_t p = lo;
    while (p < hi) {
        const size_t e = line_end(s, hi, p);
        // tokens: [p, e) split on '\t'
        const void* ft = memchr(s + p, '\t', e - p);
        const size_t first_tab = ft ? (size_t)((const uint8_t*)ft - s) : e;
        if (first_tab == e) {  // one token: "not enough values to unpack"
            P.bad_line = P.lines;
            P.why = "eq line with fewer than 2 fields";
            return;
        }
        const bool size1 = first_tab - p == 1 && s[p] == '1';
        size_t a = first_tab + 1;
        // count = last token
        size_t last_tab = e;
        while (last_tab > first_tab && s[last_tab - 1] != '\t') --last_tab;
        // last_tab is the start of the last token; its preceding '\t' at last_tab - 1
        int64_t cnt;
        if (!py_int_ascii(s + last_tab, e - last_tab, &cnt)) {
            P.bad_line = P.lines;
            P.why = "eq count is not a plain integer";
            return;
        }
        const size_t before = P.members.size();
        while (a < last_tab) {
            size_t b = a;
            while (b < last_tab - 1 && s[b] != '\t') ++b;
            // id token [a, b)
            uint32_t id;
            if (!canonical_index(s + a, b - a, n, &id)) {
                P.bad_line = P.lines;
                P.why = "eq contig id is not a name-table index";
                return;
            }
            P.members.push_back(id);
            a = b + 1;
        }
        P.sizes.push_back((int64_t)(P.members.size() - before));
        P.counts.push_back(cnt);
        P.skip.push_back(size1 ? 1 : 0);
        ++P.lines;
        p = next_line(s, hi, e);
    }
}

}  // namespace

static int eq_parse_impl(const char* data_c, size_t len, int threads, karma_eq** out) {
    if (!out || (!data_c && len)) {
        set_error("karma_eq_parse: null argument");
        return KARMA_ERR_ARG;
    }
    *out = nullptr;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(data_c);
    if (!is_ascii(s, len)) {
        const size_t bad = utf8_invalid_at(s, len);
        if (bad != len) {
            set_error("eq_classes: invalid UTF-8 at byte %zu", bad);
            return KARMA_ERR_PARSE;
        }
    }
    size_t p = 0;
    size_t e = line_end(s, len, p);
    int64_t n;
    if (!py_int_ascii(s, e, &n) || n < 0) {
        set_error("eq_classes: line 1 is not a non-negative plain integer");
        return KARMA_ERR_PARSE;
    }
    if (n >= (int64_t)1 << 32) {
        set_error("eq_classes: more than 2^32 contigs");
        return KARMA_ERR_ARG;
    }
    p = next_line(s, len, e);
    p = next_line(s, len, line_end(s, len, p));  // line 2 ignored
    // Past EOF readline returns "" (read_graph.py:80): a second name read past
    // the end duplicates the first one, which the :93 assert rejects.  Checked
    // before anything is sized by the untrusted count n.
    {
        size_t pp = p;
        int64_t avail = 0;
        while (avail < n && pp < len) {
            pp = next_line(s, len, line_end(s, len, pp));
            ++avail;
        }
        if (n - avail >= 2) {
            set_error("eq_classes: duplicate contig name (read_graph.py:93 assert: names past the end of the file)");
            return KARMA_ERR_PARSE;
        }
    }
    std::unique_ptr<karma_eq> qh(new karma_eq);
    karma_eq* q = qh.get();
    q->name_off.assign(n + 1, 0);
    std::vector<std::pair<size_t, size_t>> nm((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        const size_t ne = line_end(s, len, p);  // past EOF: "" (readline returns "")
        nm[i] = {p, ne};
        q->name_off[i + 1] = q->name_off[i] + (int64_t)(ne - p);
        p = next_line(s, len, ne);
    }
    q->names.resize((size_t)q->name_off[n]);
    {
        std::unordered_set<std::string_view, SVHash> uniq;
        uniq.reserve((size_t)n * 2);
        for (int64_t i = 0; i < n; ++i) {
            std::string_view v(reinterpret_cast<const char*>(s + nm[i].first), nm[i].second - nm[i].first);
            if (!v.empty()) memcpy(q->names.data() + q->name_off[i], v.data(), v.size());
            if (!uniq.insert(v).second) {
                set_error("eq_classes: duplicate contig name (read_graph.py:93 assert)");
                return KARMA_ERR_PARSE;
            }
        }
    }
    // eq lines: split the rest at line starts into T parts
    const size_t body = p;
    const int T = clamp_threads(threads, len - body, 1 << 20);
    const std::vector<size_t> cut = line_cuts(s, body, len, T);
    std::vector<EqPart> parts(T);
    parallel_for(T, [&](int t) { parse_eq_lines(s, cut[t], cut[t + 1], n, parts[t]); });
    int64_t line0 = 0;
    for (int t = 0; t < T; ++t) {
        if (parts[t].bad_line >= 0) {
            set_error("eq_classes: %s (eq line %lld)", parts[t].why, (long long)(line0 + parts[t].bad_line + 1));
            return KARMA_ERR_PARSE;
        }
        line0 += parts[t].lines;
    }
    q->cls_off.assign(line0 + 1, 0);
    size_t nm_total = 0;
    for (auto& P : parts) nm_total += P.members.size();
    q->members.reserve(nm_total);
    int64_t c = 0;
    for (auto& P : parts) {
        for (size_t i = 0; i < P.sizes.size(); ++i, ++c) q->cls_off[c + 1] = q->cls_off[c] + P.sizes[i];
        q->members.insert(q->members.end(), P.members.begin(), P.members.end());
        q->counts.insert(q->counts.end(), P.counts.begin(), P.counts.end());
        q->pair_skip.insert(q->pair_skip.end(), P.skip.begin(), P.skip.end());
    }
    *out = qh.release();
    return KARMA_OK;
}

// Host allocation failures (e.g. a count in the input far beyond its size)
// must not unwind through the C boundary.
extern "C" int karma_eq_parse(const char* data_c, size_t len, int threads, karma_eq** out) {
    try {
        return eq_parse_impl(data_c, len, threads, out);
    } catch (const std::bad_alloc&) {
        set_error("karma_eq_parse: out of host memory");
        return KARMA_ERR_OOM;
    } catch (const std::exception& e) {
        set_error("karma_eq_parse: %s", e.what());
        return KARMA_ERR_PARSE;
    }
}

extern "C" int karma_eq_info(karma_eq* q, int64_t* n_contigs, int64_t* n_classes, int64_t* n_members,
                             int64_t* name_bytes) {
    if (!q) {
        set_error("karma_eq_info: null handle");
        return KARMA_ERR_ARG;
    }
    if (n_contigs) *n_contigs = (int64_t)q->name_off.size() - 1;
    if (n_classes) *n_classes = (int64_t)q->counts.size();
    if (n_members) *n_members = (int64_t)q->members.size();
    if (name_bytes) *name_bytes = (int64_t)q->names.size();
    return KARMA_OK;
}

extern "C" int karma_eq_get(karma_eq* q, char* names, int64_t* name_off, int64_t* cls_off, uint32_t* members,
                            int64_t* counts, uint8_t* pair_skip) {
    if (!q) {
        set_error("karma_eq_get: null handle");
        return KARMA_ERR_ARG;
    }
    copy_out(names, q->names.data(), q->names.size());
    copy_out(name_off, q->name_off.data(), q->name_off.size() * sizeof(int64_t));
    copy_out(cls_off, q->cls_off.data(), q->cls_off.size() * sizeof(int64_t));
    copy_out(members, q->members.data(), q->members.size() * sizeof(uint32_t));
    copy_out(counts, q->counts.data(), q->counts.size() * sizeof(int64_t));
    copy_out(pair_skip, q->pair_skip.data(), q->pair_skip.size());
    return KARMA_OK;
}

extern "C" int karma_eq_get_compact(karma_eq* q, char* names, int64_t* name_off, uint8_t* sizes, uint32_t* members,
                                    uint32_t* counts) {
    if (!q) {
        set_error("karma_eq_get_compact: null handle");
        return KARMA_ERR_ARG;
    }
    const int64_t C = (int64_t)q->counts.size();
    for (int64_t c = 0; c < C; ++c) {  // checked first: nothing is written when a class does not fit
        if (q->cls_off[c + 1] - q->cls_off[c] > 127 || q->counts[c] < 0 || q->counts[c] > (int64_t)UINT32_MAX) {
            set_error("karma_eq_get_compact: class %lld does not fit (%lld members, count %lld)", (long long)c,
                      (long long)(q->cls_off[c + 1] - q->cls_off[c]), (long long)q->counts[c]);
            return KARMA_ERR_ARG;
        }
    }
    copy_out(names, q->names.data(), q->names.size());
    copy_out(name_off, q->name_off.data(), q->name_off.size() * sizeof(int64_t));
    copy_out(members, q->members.data(), q->members.size() * sizeof(uint32_t));
    for (int64_t c = 0; c < C; ++c) {
        sizes[c] = (uint8_t)((q->cls_off[c + 1] - q->cls_off[c]) | (q->pair_skip[c] ? 0x80 : 0));
        counts[c] = (uint32_t)q->counts[c];
    }
    return KARMA_OK;
}

extern "C" int karma_eq_destroy(karma_eq* q) {
    delete q;
    return KARMA_OK;
}

// ============================================================================
// SAM — Contig readsets (karma/contig.py:24,34): per line
//   read, _, name, position, *_ = line.split("\t")   (>= 4 fields)
// and the readset is set(read).  Lines starting with "@" are dropped when
// skip_headers is set (the hisat2 generator filter, hisat2.py:49-53).  One
// record (read id, contig id) per line; contig ids number the RNAMEs (field 3)
// in order of first appearance, read ids are an injective numbering of the
// QNAMEs (the graph depends only on which records share a read).
// ============================================================================
struct karma_sam {
    std::vector<uint32_t> records;    // 2 per line: read id, contig id
    std::vector<char> rnames;
    std::vector<int64_t> rname_off;   // n_contigs + 1
    std::vector<int64_t> q_start;     // per record: QNAME byte range in the caller's buffer
    std::vector<int32_t> q_len;
    int64_t n_reads = 0;
    int64_t id_bound = 0;  // read ids < id_bound
};

namespace {

struct SamPart {
    std::vector<size_t> q0;   // QNAME start
    std::vector<uint32_t> ql;
    std::vector<uint64_t> qh;
    std::vector<size_t> r0;   // RNAME start
    std::vector<uint32_t> rl;
    std::vector<uint64_t> rh;
    int64_t bad_line = -1;
    int64_t lines = 0;        // parsed data lines
    int64_t all_lines = 0;    // including headers
};

void parse_sam_lines(const uint8_t* s, size_t lo, size_t hi, bool skip_headers, SamPart& P) {
    size_t p = lo;
    while (p < hi) {
        const size_t e = line_end(s, hi, p);
        ++P.all_lines;
        if (!(skip_headers && e > p && s[p] == '@')) {
            // fields 0..3 must exist
            size_t f[4] = {p, 0, 0, 0}, fe[3] = {0, 0, 0};
            size_t a = p;
            int k = 0;
            for (; k < 3; ++k) {
                const void* t = memchr(s + a, '\t', e - a);
                if (!t) break;
                fe[k] = (const uint8_t*)t - s;
                a = fe[k] + 1;
                f[k + 1] = a;
            }
            if (k < 3) {
                P.bad_line = P.all_lines - 1;
                return;
            }
            const size_t ql = fe[0] - f[0], rl = fe[2] - f[2];
            if (ql >= (1u << 31) || rl >= (1u << 31)) {
                P.bad_line = P.all_lines - 1;
                return;
            }
            P.q0.push_back(f[0]);
            P.ql.push_back((uint32_t)ql);
            P.qh.push_back(hash_bytes(s + f[0], ql));
            P.r0.push_back(f[2]);
            P.rl.push_back((uint32_t)rl);
            P.rh.push_back(hash_bytes(s + f[2], rl));
            ++P.lines;
        }
        p = next_line(s, hi, e);
    }
}

}  // namespace

static int sam_parse_impl(const char* data_c, size_t len, int skip_headers, int threads, karma_sam** out) {
    if (!out || (!data_c && len)) {
        set_error("karma_sam_parse: null argument");
        return KARMA_ERR_ARG;
    }
    *out = nullptr;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(data_c);
    const int T = clamp_threads(threads, len, 1 << 20);
    const std::vector<size_t> cut = line_cuts(s, 0, len, T);
    std::vector<char> ok(T, 1);
    parallel_for(T, [&](int t) { ok[t] = is_ascii(s + cut[t], cut[t + 1] - cut[t]); });
    if (std::find(ok.begin(), ok.end(), 0) != ok.end() && utf8_invalid_at(s, len) != len) {
        set_error("sam: invalid UTF-8");
        return KARMA_ERR_PARSE;
    }
    std::vector<SamPart> parts(T);
    parallel_for(T, [&](int t) { parse_sam_lines(s, cut[t], cut[t + 1], skip_headers != 0, parts[t]); });
    int64_t base = 0, L = 0;
    for (int t = 0; t < T; ++t) {
        if (parts[t].bad_line >= 0) {
            set_error("sam: line %lld has fewer than 4 tab-separated fields (contig.py:34 unpack)",
                      (long long)(base + parts[t].bad_line + 1));
            return KARMA_ERR_PARSE;
        }
        base += parts[t].all_lines;
        L += parts[t].lines;
    }
    std::vector<int64_t> first(T + 1, 0);
    for (int t = 0; t < T; ++t) first[t + 1] = first[t] + parts[t].lines;
    auto* S = new karma_sam;
    try {
        S->records.resize((size_t)L * 2);
        S->q_start.resize((size_t)L);
        S->q_len.resize((size_t)L);
    } catch (...) {
        delete S;
        set_error("sam: out of host memory");
        return KARMA_ERR_OOM;
    }
    // ---- RNAME ids in order of first appearance: distinct names per part
    // (parallel), numbered part by part, then every line mapped (parallel)
    std::vector<std::vector<int64_t>> local_first(T);  // part-local distinct -> first local line
    std::vector<std::vector<uint32_t>> local_id(T);    // local line -> part-local distinct id
    parallel_for(T, [&](int t) {
        const SamPart& P = parts[t];
        KeyTable tab((size_t)P.lines);
        local_id[t].resize(P.lines);
        std::vector<int64_t>& lf = local_first[t];
        for (int64_t i = 0; i < P.lines; ++i) {
            const int64_t f0 = tab.find_or_insert(P.rh[i], i, [&](int64_t o) {
                return P.rh[o] == P.rh[i] && P.rl[o] == P.rl[i] && memcmp(s + P.r0[o], s + P.r0[i], P.rl[i]) == 0;
            });
            if (f0 == i) {
                local_id[t][i] = (uint32_t)lf.size();
                lf.push_back(i);
            } else {
                local_id[t][i] = local_id[t][f0];
            }
        }
    });
    std::vector<std::vector<uint32_t>> global_of_local(T);
    {
        size_t total = 0;
        for (auto& v : local_first) total += v.size();
        KeyTable tab(total);
        std::vector<std::pair<int, int64_t>> owner;  // global id -> (part, local line)
        S->rname_off.push_back(0);
        for (int t = 0; t < T; ++t) {
            const SamPart& P = parts[t];
            for (int64_t i : local_first[t]) {
                const int64_t idx = (int64_t)owner.size();
                const int64_t g = tab.find_or_insert(P.rh[i], idx, [&](int64_t o) {
                    const SamPart& Q = parts[owner[o].first];
                    const int64_t j = owner[o].second;
                    return Q.rh[j] == P.rh[i] && Q.rl[j] == P.rl[i] && memcmp(s + Q.r0[j], s + P.r0[i], P.rl[i]) == 0;
                });
                if (g == idx) {
                    owner.emplace_back(t, i);
                    S->rnames.insert(S->rnames.end(), s + P.r0[i], s + P.r0[i] + P.rl[i]);
                    S->rname_off.push_back((int64_t)S->rnames.size());
                }
                global_of_local[t].push_back((uint32_t)g);
            }
        }
    }
    parallel_for(T, [&](int t) {
        const SamPart& P = parts[t];
        for (int64_t i = 0; i < P.lines; ++i) {
            const int64_t g = first[t] + i;
            S->records[2 * g + 1] = global_of_local[t][local_id[t][i]];
            S->q_start[g] = (int64_t)P.q0[i];
            S->q_len[g] = (int32_t)P.ql[i];
        }
    });
    // ---- QNAME ids: shard by hash, one thread per shard; id = local * T + shard
    std::vector<uint64_t> n_local(T, 0);
    parallel_for(T, [&](int sh) {
        KeyTable tab((size_t)(L / T + 16) * 2);
        std::vector<std::pair<int, int64_t>> own;  // shard-local id -> (part, line)
        for (int t = 0; t < T; ++t) {
            const SamPart& P = parts[t];
            for (int64_t i = 0; i < P.lines; ++i) {
                if ((int)((P.qh[i] >> 40) % (uint64_t)T) != sh) continue;
                const int64_t idx = (int64_t)own.size();
                if (own.size() * 2 + 16 > tab.slot.size()) {  // grow: rehash the shard
                    KeyTable big(tab.slot.size());
                    for (int64_t o = 0; o < idx; ++o) {
                        const SamPart& Q = parts[own[o].first];
                        big.find_or_insert(Q.qh[own[o].second], o, [](int64_t) { return false; });
                    }
                    tab = std::move(big);
                }
                const int64_t id = tab.find_or_insert(P.qh[i], idx, [&](int64_t o) {
                    const SamPart& Q = parts[own[o].first];
                    const int64_t j = own[o].second;
                    return Q.qh[j] == P.qh[i] && Q.ql[j] == P.ql[i] && memcmp(s + Q.q0[j], s + P.q0[i], P.ql[i]) == 0;
                });
                if (id == idx) own.emplace_back(t, i);
                S->records[2 * (first[t] + i)] = (uint32_t)((uint64_t)id * (uint64_t)T + (uint64_t)sh);
            }
        }
        n_local[sh] = own.size();
    });
    uint64_t nreads = 0, maxid = 0;
    for (int t = 0; t < T; ++t) {
        nreads += n_local[t];
        if (n_local[t]) maxid = std::max(maxid, (n_local[t] - 1) * (uint64_t)T + t);
    }
    if (maxid >= (UINT64_C(1) << 32) - 1) {
        delete S;
        set_error("sam: more than 2^32 distinct reads");
        return KARMA_ERR_ARG;
    }
    S->n_reads = (int64_t)nreads;
    S->id_bound = nreads ? (int64_t)maxid + 1 : 0;
    *out = S;
    return KARMA_OK;
}

// Host allocation failures (e.g. a count in the input far beyond its size)
// must not unwind through the C boundary.
extern "C" int karma_sam_parse(const char* data_c, size_t len, int skip_headers, int threads, karma_sam** out) {
    try {
        return sam_parse_impl(data_c, len, skip_headers, threads, out);
    } catch (const std::bad_alloc&) {
        set_error("karma_sam_parse: out of host memory");
        return KARMA_ERR_OOM;
    } catch (const std::exception& e) {
        set_error("karma_sam_parse: %s", e.what());
        return KARMA_ERR_PARSE;
    }
}

extern "C" int karma_sam_info(karma_sam* S, int64_t* n_records, int64_t* n_reads, int64_t* n_contigs,
                              int64_t* rname_bytes, int64_t* read_id_bound) {
    if (!S) {
        set_error("karma_sam_info: null handle");
        return KARMA_ERR_ARG;
    }
    if (n_records) *n_records = (int64_t)S->q_len.size();
    if (n_reads) *n_reads = S->n_reads;
    if (n_contigs) *n_contigs = (int64_t)S->rname_off.size() - 1;
    if (rname_bytes) *rname_bytes = (int64_t)S->rnames.size();
    if (read_id_bound) *read_id_bound = S->id_bound;
    return KARMA_OK;
}

extern "C" int karma_sam_get(karma_sam* S, uint32_t* records, char* rnames, int64_t* rname_off, int64_t* q_start,
                             int32_t* q_len) {
    if (!S) {
        set_error("karma_sam_get: null handle");
        return KARMA_ERR_ARG;
    }
    const size_t L = S->q_len.size();
    copy_out(records, S->records.data(), L * 2 * sizeof(uint32_t));
    copy_out(rnames, S->rnames.data(), S->rnames.size());
    copy_out(rname_off, S->rname_off.data(), S->rname_off.size() * sizeof(int64_t));
    copy_out(q_start, S->q_start.data(), L * sizeof(int64_t));
    copy_out(q_len, S->q_len.data(), L * sizeof(int32_t));
    return KARMA_OK;
}

extern "C" int karma_sam_destroy(karma_sam* S) {
    delete S;
    return KARMA_OK;
}
