// ingest.cpp — host-side parsers of the path's input formats (SURVEY.md §8(b),
// §8(f) row 1), multi-threaded C++ over an in-memory buffer.
//
//   karma_fasta_*  read_fasta_file              karma/karma.py:40-61
//   karma_eq_*     the eq_classes.txt parse of  karma/read_graph.py:75-92
//   karma_sam_*    Contig readsets from SAM     karma/contig.py:24,34 + hisat2.py:76-81
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

int clamp_threads(int threads, size_t work, size_t per_thread) {
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
    std::vector<uint8_t> seq;
    std::vector<int64_t> seq_off;  // N + 1
    std::vector<char> keys;
    std::vector<int64_t> key_off;  // N + 1
    std::vector<int32_t> key_len;  // code points
    bool ascii = true;
};

extern "C" int karma_fasta_parse(const char* data_c, size_t len, int threads, karma_fasta** out) {
    if (!out || (!data_c && len)) {
        set_error("karma_fasta_parse: null argument");
        return KARMA_ERR_ARG;
    }
    *out = nullptr;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(data_c);
    const int T = clamp_threads(threads, len, 1 << 20);
    const size_t per = (len + T - 1) / (size_t)T;
    // ---- 1: header line starts (a '>' right after a line terminator) + ASCII check
    std::vector<std::vector<size_t>> hs(T);
    std::vector<char> t_ascii(T, 1);
    parallel_for(T, [&](int t) {
        const size_t lo = std::min(len, (size_t)t * per), hi = std::min(len, lo + per);
        t_ascii[t] = is_ascii(s + lo, hi - lo);
        for (size_t p = std::max<size_t>(lo, 1); p < hi;) {
            const void* q = memchr(s + p, '>', hi - p);
            if (!q) break;
            const size_t i = (const uint8_t*)q - s;
            if (is_nl(s[i - 1])) hs[t].push_back(i);
            p = i + 1;
        }
    });
    bool ascii = true;
    for (int t = 0; t < T; ++t) ascii = ascii && t_ascii[t];
    if (!ascii) {
        const size_t bad = utf8_invalid_at(s, len);
        if (bad != len) {
            set_error("fasta: invalid UTF-8 at byte %zu", bad);
            return KARMA_ERR_PARSE;
        }
    }
    std::vector<size_t> h(1, 0);  // record r: header line at h[r], body up to h[r + 1]
    for (auto& v : hs) h.insert(h.end(), v.begin(), v.end());
    const int64_t R = (int64_t)h.size();
    h.push_back(len);
    // ---- 2: per record key range and sequence size (bytes that are not terminators)
    std::vector<size_t> kend(R), body(R);
    std::vector<int64_t> slen(R);
    const int TR = clamp_threads(threads, (size_t)R, 256);
    parallel_for(TR, [&](int t) {
        const int64_t lo = R * t / TR, hi = R * (t + 1) / TR;
        for (int64_t r = lo; r < hi; ++r) {
            const size_t e = line_end(s, len, h[r]);
            const void* sp = memchr(s + h[r], ' ', e - h[r]);
            kend[r] = sp ? (size_t)((const uint8_t*)sp - s) : e;
            body[r] = next_line(s, len, e);
            int64_t n = 0;
            for (size_t p = body[r]; p < h[r + 1]; ++p) n += !is_nl(s[p]);
            slen[r] = n;
        }
    });
    // ---- 3: OrderedDict assignment: first position, last value
    std::vector<int64_t> slot(R);  // output slot of record r
    std::vector<int64_t> src;      // output slot -> record providing the value
    {
        std::unordered_map<std::string_view, int64_t, SVHash> seen;
        seen.reserve((size_t)R * 2);
        for (int64_t r = 0; r < R; ++r) {
            std::string_view k(reinterpret_cast<const char*>(s + h[r]), kend[r] - h[r]);
            auto it = seen.emplace(k, (int64_t)src.size());
            if (it.second) src.push_back(r);
            else src[it.first->second] = r;
            slot[r] = it.first->second;
        }
    }
    const int64_t N = (int64_t)src.size();
    auto* f = new karma_fasta;
    f->ascii = ascii;
    f->seq_off.assign(N + 1, 0);
    f->key_off.assign(N + 1, 0);
    f->key_len.assign(N, 0);
    std::vector<int64_t> first_rec(N, -1);
    for (int64_t r = 0; r < R; ++r)
        if (first_rec[slot[r]] < 0) first_rec[slot[r]] = r;
    for (int64_t i = 0; i < N; ++i) {
        const int64_t kr = first_rec[i], vr = src[i];
        f->seq_off[i + 1] = f->seq_off[i] + slen[vr];
        f->key_off[i + 1] = f->key_off[i] + (int64_t)(kend[kr] - h[kr]);
    }
    try {
        f->seq.resize((size_t)f->seq_off[N] + 16, 0);  // 16 zero bytes of padding (karma_contigs_create)
        f->keys.resize((size_t)f->key_off[N]);
    } catch (...) {
        delete f;
        set_error("fasta: out of host memory");
        return KARMA_ERR_OOM;
    }
    const int TN = clamp_threads(threads, (size_t)N, 256);
    parallel_for(TN, [&](int t) {
        const int64_t lo = N * t / TN, hi = N * (t + 1) / TN;
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t kr = first_rec[i], vr = src[i];
            const size_t kl = kend[kr] - h[kr];
            memcpy(f->keys.data() + f->key_off[i], s + h[kr], kl);
            f->key_len[i] = (int32_t)(ascii ? (int64_t)kl : code_points(s + h[kr], kl));
            uint8_t* d = f->seq.data() + f->seq_off[i];
            for (size_t p = body[vr]; p < h[vr + 1];) {
                const size_t e = line_end(s, h[vr + 1], p);
                memcpy(d, s + p, e - p);
                d += e - p;
                p = next_line(s, h[vr + 1], e);
            }
        }
    });
    *out = f;
    return KARMA_OK;
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

extern "C" int karma_fasta_get(karma_fasta* f, uint8_t* seq, int64_t* seq_off, char* keys, int64_t* key_off,
                               int32_t* key_len) {
    if (!f) {
        set_error("karma_fasta_get: null handle");
        return KARMA_ERR_ARG;
    }
    const int64_t N = (int64_t)f->key_len.size();
    if (seq) memcpy(seq, f->seq.data(), (size_t)f->seq_off[N] + 16);
    if (seq_off) memcpy(seq_off, f->seq_off.data(), sizeof(int64_t) * (N + 1));
    if (keys) memcpy(keys, f->keys.data(), (size_t)f->key_off[N]);
    if (key_off) memcpy(key_off, f->key_off.data(), sizeof(int64_t) * (N + 1));
    if (key_len) memcpy(key_len, f->key_len.data(), sizeof(int32_t) * N);
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

extern "C" int karma_eq_parse(const char* data_c, size_t len, int threads, karma_eq** out) {
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
    auto* q = new karma_eq;
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
            memcpy(q->names.data() + q->name_off[i], v.data(), v.size());
            if (!uniq.insert(v).second) {
                delete q;
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
            delete q;
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
    *out = q;
    return KARMA_OK;
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
    if (names) memcpy(names, q->names.data(), q->names.size());
    if (name_off) memcpy(name_off, q->name_off.data(), q->name_off.size() * sizeof(int64_t));
    if (cls_off) memcpy(cls_off, q->cls_off.data(), q->cls_off.size() * sizeof(int64_t));
    if (members) memcpy(members, q->members.data(), q->members.size() * sizeof(uint32_t));
    if (counts) memcpy(counts, q->counts.data(), q->counts.size() * sizeof(int64_t));
    if (pair_skip) memcpy(pair_skip, q->pair_skip.data(), q->pair_skip.size());
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
// skip_headers is set (the hisat2 generator filter, hisat2.py:76-81).  One
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
};

namespace {

struct SamPart {
    std::vector<size_t> q0;   // QNAME start
    std::vector<uint32_t> ql;
    std::vector<uint64_t> qh;
    std::vector<size_t> r0;   // RNAME start
    std::vector<uint32_t> rl;
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
            ++P.lines;
        }
        p = next_line(s, hi, e);
    }
}

}  // namespace

extern "C" int karma_sam_parse(const char* data_c, size_t len, int skip_headers, int threads, karma_sam** out) {
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
    // ---- RNAME ids in order of first appearance (sequential over few names)
    {
        std::unordered_map<std::string_view, uint32_t, SVHash> rid;
        S->rname_off.push_back(0);
        for (int t = 0; t < T; ++t) {
            const SamPart& P = parts[t];
            for (int64_t i = 0; i < P.lines; ++i) {
                std::string_view v(reinterpret_cast<const char*>(s + P.r0[i]), P.rl[i]);
                auto it = rid.find(v);
                uint32_t id;
                if (it == rid.end()) {
                    id = (uint32_t)rid.size();
                    rid.emplace(v, id);
                    S->rnames.insert(S->rnames.end(), v.begin(), v.end());
                    S->rname_off.push_back((int64_t)S->rnames.size());
                } else {
                    id = it->second;
                }
                const int64_t g = first[t] + i;
                S->records[2 * g + 1] = id;
                S->q_start[g] = (int64_t)P.q0[i];
                S->q_len[g] = (int32_t)P.ql[i];
            }
        }
    }
    // ---- QNAME ids: shard by hash, one thread per shard; id = local * T + shard
    std::vector<uint64_t> n_local(T, 0);
    parallel_for(T, [&](int sh) {
        std::unordered_map<std::string_view, uint64_t, SVHash> qid;
        for (int t = 0; t < T; ++t) {
            const SamPart& P = parts[t];
            for (int64_t i = 0; i < P.lines; ++i) {
                if ((int)(P.qh[i] % (uint64_t)T) != sh) continue;
                std::string_view v(reinterpret_cast<const char*>(s + P.q0[i]), P.ql[i]);
                auto it = qid.emplace(v, (uint64_t)qid.size());
                S->records[2 * (first[t] + i)] = (uint32_t)(it.first->second * (uint64_t)T + (uint64_t)sh);
            }
        }
        n_local[sh] = qid.size();
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
    *out = S;
    return KARMA_OK;
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
    if (read_id_bound) {
        uint64_t m = 0;
        for (size_t i = 0; i < S->q_len.size(); ++i) m = std::max<uint64_t>(m, S->records[2 * i] + 1ull);
        *read_id_bound = (int64_t)m;
    }
    return KARMA_OK;
}

extern "C" int karma_sam_get(karma_sam* S, uint32_t* records, char* rnames, int64_t* rname_off, int64_t* q_start,
                             int32_t* q_len) {
    if (!S) {
        set_error("karma_sam_get: null handle");
        return KARMA_ERR_ARG;
    }
    const size_t L = S->q_len.size();
    if (records) memcpy(records, S->records.data(), L * 2 * sizeof(uint32_t));
    if (rnames) memcpy(rnames, S->rnames.data(), S->rnames.size());
    if (rname_off) memcpy(rname_off, S->rname_off.data(), S->rname_off.size() * sizeof(int64_t));
    if (q_start) memcpy(q_start, S->q_start.data(), L * sizeof(int64_t));
    if (q_len) memcpy(q_len, S->q_len.data(), L * sizeof(int32_t));
    return KARMA_OK;
}

extern "C" int karma_sam_destroy(karma_sam* S) {
    delete S;
    return KARMA_OK;
}
