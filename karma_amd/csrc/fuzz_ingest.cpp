// fuzz_ingest.cpp — sanitizer fuzz driver for the host parsers (SURVEY.md §5:
// ASan/UBSan on the C++ host library).  Built by `make -C karma_amd/csrc asan`
// together with ingest.cpp under -fsanitize=address,undefined (no GPU code:
// set_error is defined here instead of core.hip).  Run by
// tests/test_ingest_asan.py.
//
// Each round builds random texts for the three readers -- karma_fasta_parse
// (karma.py:40-61), karma_eq_parse (read_graph.py:75-92) and karma_sam_parse
// (contig.py:24,34; hisat2.py:49-53) -- from a token alphabet that mixes
// structure (headers, tabs, counts, ids) with CR/LF/CRLF, NUL, valid and
// invalid UTF-8, signs, underscores and huge integers, then parses each at
// 1 and at 2..8 threads and, on success, reads every output back through the
// info/get/view calls; both runs must agree exactly (status and outputs).  Any sanitizer report aborts the process (the build
// uses -fno-sanitize-recover=all), so exit status 0 means a clean run.
//
// usage: fuzz_ingest_asan ROUNDS SEED
#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/karma.h"

namespace karma {
void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
}
}  // namespace karma

namespace {

long g_ok[3];  // successful parses per reader (coverage sanity: the fuzz must reach the get paths)

struct Rng {
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
    bool chance(int pct) { return (int)below(100) < pct; }
};

const char* const kNewlines[] = {"\n", "\r\n", "\r"};
const char* const kNoise[] = {"\0", "\xc3\xa9", "\xe2\x82\xac", "\xf0\x9f\x98\x80", "\x80", "\xff", "\xc3",
                              "\xed\xa0\x80", " ", "\t", "_", "+", "-", "@", ">", "N", "acgt", "\x7f"};

void put(std::string& t, const char* s) { t.append(s, s[0] ? strlen(s) : 1); }

std::string newline(Rng& r) { return kNewlines[r.below(3)]; }

void noise(Rng& r, std::string& t, int pct) {
    while (r.chance(pct)) put(t, kNoise[r.below(sizeof kNoise / sizeof *kNoise)]);
}

std::string integer(Rng& r) {
    switch (r.below(8)) {
        case 0: return "4294967296";
        case 1: return "99999999999999999999999";
        case 2: return "-" + std::to_string(r.below(10));
        case 3: return "+" + std::to_string(r.below(100));
        case 4: return "1_0";
        case 5: return " " + std::to_string(r.below(50)) + " ";
        default: return std::to_string(r.below(r.chance(50) ? 8 : 100000));
    }
}

std::string seq(Rng& r, size_t n) {
    static const char kB[] = "ACGTACGTACGTNacgtRY";
    std::string s;
    for (size_t i = 0; i < n; ++i) s += kB[r.below(sizeof kB - 1)];
    return s;
}

std::string fasta_text(Rng& r) {
    std::string t;
    if (r.chance(10)) t += seq(r, r.below(20)) + newline(r);  // sequence before any header
    const int n = (int)r.below(40);
    for (int i = 0; i < n; ++i) {
        t += ">ctg" + std::to_string(r.below(20));
        if (r.chance(30)) t += " desc" + std::to_string(i);
        noise(r, t, 10);
        t += newline(r);
        const int lines = (int)r.below(4);
        for (int l = 0; l < lines; ++l) {
            t += seq(r, r.below(r.chance(5) ? 5000 : 90));
            noise(r, t, 5);
            if (l + 1 < lines || r.chance(80)) t += newline(r);
        }
    }
    return t;
}

std::string eq_text(Rng& r) {
    std::string t;
    const int64_t n = r.chance(5) ? (int64_t)r.below(1000000) : (int64_t)r.below(12);
    t += r.chance(10) ? integer(r) : std::to_string(n);
    t += newline(r);
    t += integer(r) + newline(r);
    const int64_t names = r.chance(10) ? (int64_t)r.below(15) : n;
    for (int64_t i = 0; i < names && i < 64; ++i) {
        t += r.chance(5) ? std::string() : "c" + std::to_string(r.chance(5) ? 0 : i);
        noise(r, t, 5);
        t += newline(r);
    }
    const int cls = (int)r.below(30);
    for (int c = 0; c < cls; ++c) {
        const int k = (int)r.below(6);
        t += r.chance(10) ? integer(r) : std::to_string(k);
        for (int j = 0; j < k; ++j) t += "\t" + (r.chance(8) ? integer(r) : std::to_string(r.below(n + 2)));
        if (r.chance(90)) t += "\t" + integer(r);
        noise(r, t, 5);
        t += newline(r);
    }
    return t;
}

std::string sam_text(Rng& r) {
    std::string t;
    const int n = (int)r.below(60);
    for (int i = 0; i < n; ++i) {
        if (r.chance(10)) {
            t += "@HD\tVN:1.0" + newline(r);
            continue;
        }
        const int fields = r.chance(10) ? (int)r.below(4) : 4 + (int)r.below(8);
        for (int f = 0; f < fields; ++f) {
            if (f) t += "\t";
            if (f == 0) t += "r" + std::to_string(r.below(30));
            else if (f == 2) t += r.chance(5) ? std::string("*") : "ctg" + std::to_string(r.below(10));
            else t += std::to_string(r.below(300));
            noise(r, t, 3);
        }
        t += newline(r);
    }
    return t;
}

// Each run_* returns the reader's status and a serialisation of its outputs,
// so the same text parsed at 1 and at T threads can be compared.
template <typename T>
void ser(std::string& o, const std::vector<T>& v, size_t n) {
    o.append(reinterpret_cast<const char*>(v.data()), n * sizeof(T));
    o += '|';
}

int run_fasta(const std::string& t, int threads, std::string& o) {
    karma_fasta* f = nullptr;
    const int rc = karma_fasta_parse(t.data(), t.size(), threads, &f);
    if (rc != KARMA_OK) return rc;
    ++g_ok[0];
    int64_t n = 0, sb = 0, kb = 0;
    int ascii = 0;
    karma_fasta_info(f, &n, &sb, &kb, &ascii);
    std::vector<uint8_t> s((size_t)sb + 16);
    std::vector<int64_t> so((size_t)n + 1), ko((size_t)n + 1);
    std::vector<char> k((size_t)kb + 1);
    std::vector<int32_t> kl((size_t)n + 1);
    karma_fasta_get(f, s.data(), so.data(), k.data(), ko.data(), kl.data());
    const uint8_t* vs;
    const int64_t *vso, *vko;
    const char* vk;
    const int32_t* vkl;
    karma_fasta_view(f, &vs, &vso, &vk, &vko, &vkl);
    if (n && (memcmp(vso, so.data(), (size_t)(n + 1) * 8) || memcmp(vs, s.data(), (size_t)sb))) abort();
    karma_fasta_destroy(f);
    ser(o, s, (size_t)sb + 16), ser(o, so, (size_t)n + 1), ser(o, k, (size_t)kb), ser(o, ko, (size_t)n + 1);
    ser(o, kl, (size_t)n);
    return rc;
}

int run_eq(const std::string& t, int threads, std::string& o) {
    karma_eq* q = nullptr;
    const int rc = karma_eq_parse(t.data(), t.size(), threads, &q);
    if (rc != KARMA_OK) return rc;
    ++g_ok[1];
    int64_t n = 0, c = 0, m = 0, nb = 0;
    karma_eq_info(q, &n, &c, &m, &nb);
    std::vector<char> names((size_t)nb + 1);
    std::vector<int64_t> no((size_t)n + 1), co((size_t)c + 1), cnt((size_t)c + 1);
    std::vector<uint32_t> mem((size_t)m + 1);
    std::vector<uint8_t> skip((size_t)c + 1);
    karma_eq_get(q, names.data(), no.data(), co.data(), mem.data(), cnt.data(), skip.data());
    for (int64_t i = 0; i < m; ++i)
        if (mem[i] >= (uint64_t)n) abort();  // every id must index the name table
    karma_eq_destroy(q);
    ser(o, names, (size_t)nb), ser(o, no, (size_t)n + 1), ser(o, co, (size_t)c + 1), ser(o, mem, (size_t)m);
    ser(o, cnt, (size_t)c), ser(o, skip, (size_t)c);
    return rc;
}

// Read ids are an injective numbering that depends on the thread count, so the
// serialisation replaces each by the index of its first line.
int run_sam(const std::string& t, int threads, int skip_headers, std::string& o) {
    karma_sam* s = nullptr;
    const int rc = karma_sam_parse(t.data(), t.size(), skip_headers, threads, &s);
    if (rc != KARMA_OK) return rc;
    ++g_ok[2];
    int64_t L = 0, reads = 0, nc = 0, rb = 0, bound = 0;
    karma_sam_info(s, &L, &reads, &nc, &rb, &bound);
    std::vector<uint32_t> rec((size_t)L * 2 + 2);
    std::vector<char> rn((size_t)rb + 1);
    std::vector<int64_t> ro((size_t)nc + 1), qs((size_t)L + 1);
    std::vector<int32_t> ql((size_t)L + 1);
    karma_sam_get(s, rec.data(), rn.data(), ro.data(), qs.data(), ql.data());
    for (int64_t i = 0; i < L; ++i) {
        if (rec[2 * i + 1] >= (uint64_t)nc || rec[2 * i] >= (uint64_t)bound) abort();
        if (qs[i] < 0 || qs[i] + ql[i] > (int64_t)t.size()) abort();
    }
    karma_sam_destroy(s);
    std::vector<int64_t> first_line((size_t)L);
    {
        std::vector<std::pair<uint32_t, int64_t>> ids;
        for (int64_t i = 0; i < L; ++i) ids.push_back({rec[2 * i], i});
        std::sort(ids.begin(), ids.end());
        for (size_t i = 0; i < ids.size(); ++i)
            first_line[ids[i].second] = (i && ids[i].first == ids[i - 1].first) ? first_line[ids[i - 1].second]
                                                                                  : ids[i].second;
    }
    std::vector<uint32_t> contig((size_t)L);
    for (int64_t i = 0; i < L; ++i) contig[i] = rec[2 * i + 1];
    ser(o, first_line, (size_t)L), ser(o, contig, (size_t)L), ser(o, rn, (size_t)rb), ser(o, ro, (size_t)nc + 1);
    ser(o, qs, (size_t)L), ser(o, ql, (size_t)L);
    return rc;
}

}  // namespace

int main(int argc, char** argv) {
    const long rounds = argc > 1 ? atol(argv[1]) : 1000;
    Rng r{argc > 2 ? strtoull(argv[2], nullptr, 10) : 1};
    for (long i = 0; i < rounds; ++i) {
        const int threads = 2 + (int)r.below(7);
        // the same text at 1 and at `threads` threads: same status, same outputs
        auto same = [&](const char* what, const std::string& t, auto&& run) {
            std::string a, b;
            const int ra = run(t, 1, a), rb = run(t, threads, b);
            if (ra != rb || a != b) {
                fprintf(stderr, "fuzz_ingest: %s differs between 1 and %d threads (round %ld)\n", what, threads, i);
                abort();
            }
        };
        const int skip = (int)r.below(2);
        same("fasta", fasta_text(r), run_fasta);
        same("eq", eq_text(r), run_eq);
        same("sam", sam_text(r), [&](const std::string& t, int th, std::string& o) { return run_sam(t, th, skip, o); });
        // raw byte soup through all three
        std::string soup;
        const size_t len = r.below(r.chance(5) ? 20000 : 300);
        for (size_t j = 0; j < len; ++j) soup += (char)(r.chance(70) ? "ACGT>\t\n\r0123456789@"[r.below(20)] : r.below(256));
        same("fasta soup", soup, run_fasta);
        same("eq soup", soup, run_eq);
        same("sam soup", soup, [&](const std::string& t, int th, std::string& o) { return run_sam(t, th, 1, o); });
    }
    printf("fuzz_ingest: %ld rounds clean; parsed ok: fasta %ld eq %ld sam %ld\n", rounds, g_ok[0], g_ok[1], g_ok[2]);
    return 0;
}
