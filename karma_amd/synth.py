"""Deterministic synthetic contigs + read->contig assignments.

Integer-only, counter-based SplitMix64 so that the pure-Python generator below,
the C++ generator in ``csrc/synth.cpp`` (``karma_synth_*`` in include/karma.h)
and any future device generator produce byte-identical data.  The pure-Python
version is the specification and is used for small fixtures; large inputs come
from the native generator (tests check both agree).

Spec (all arithmetic mod 2**64):
    mix(z)            = SplitMix64 finaliser
    key(seed, s)      = mix(seed ^ (s * 0xD1B54A32D192ED03))
    u(seed, s, i)     = mix(key(seed, s) + (i + 1) * 0x9E3779B97F4A7C15)
Contig i: L_i = len_min + u(LEN, i) % (len_span + 1); header ">ctg<i>".
Base at global position g (contigs concatenated in order): code
    (u(BASE, g >> 5) >> (2 * (g & 31))) & 3 -> "ACGT"; replaced by 'N' when
    n_rate > 0 and u(NINJ, g) % n_rate == 0.
Genes: consecutive runs of contigs, size 1 + u(GENE, j) % gene_max (last one
    truncated at N).
Fragment r: gene j = u(FGENE, r) % n_genes, g = |gene|, mask1 = 1 + u(MASK1, r)
    % (2**g - 1); paired and u(DISC, r) % 16 == 0 -> mask2 = 1 + u(MASK2, r) %
    (2**g - 1), else mask2 = mask1.  Records: mate 1 emits (r, first + bit) for
    every set bit of mask1 (ascending), mate 2 (paired only) likewise for mask2.
    The fragment's deduplicated contig set is mask1 | mask2 (QNAME dedup,
    karma/contig.py:24 keeps reads in a set).
"""

from __future__ import annotations

from collections import OrderedDict

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
STREAM_MUL = 0xD1B54A32D192ED03

S_LEN, S_BASE, S_NINJ, S_GENE, S_FGENE, S_MASK1, S_DISC, S_MASK2 = 1, 2, 3, 4, 5, 6, 7, 8

# Named configurations from BASELINE.json "configs" (index = seed).
CONFIGS = {
    1: dict(n_contigs=1_000, n_frags=100_000, paired=False, kmer="5"),
    2: dict(n_contigs=50_000, n_frags=10_000_000, paired=True, kmer="5p6"),
    3: dict(n_contigs=200_000, n_frags=100_000_000, paired=True, kmer="5p6"),
}


def mix(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def stream_key(seed: int, stream: int) -> int:
    return mix((seed ^ (stream * STREAM_MUL)) & M64)


def u(seed: int, stream: int, i: int) -> int:
    return mix(stream_key(seed, stream) + (i + 1) * GOLDEN)


def contig_lengths(seed, n, len_min=400, len_span=800):
    k = stream_key(seed, S_LEN)
    return [len_min + mix(k + (i + 1) * GOLDEN) % (len_span + 1) for i in range(n)]


def contig_sequences(seed, n, len_min=400, len_span=800, n_rate=0):
    """OrderedDict[">ctg<i>" -> sequence] exactly as karma.py:40-61 would read it."""
    lens = contig_lengths(seed, n, len_min, len_span)
    kb = stream_key(seed, S_BASE)
    kn = stream_key(seed, S_NINJ)
    out = OrderedDict()
    g = 0
    word_idx, word = -1, 0
    for i, L in enumerate(lens):
        chars = []
        for _ in range(L):
            wi = g >> 5
            if wi != word_idx:
                word_idx, word = wi, mix(kb + (wi + 1) * GOLDEN)
            c = "ACGT"[(word >> (2 * (g & 31))) & 3]
            if n_rate > 0 and mix(kn + (g + 1) * GOLDEN) % n_rate == 0:
                c = "N"
            chars.append(c)
            g += 1
        out[f">ctg{i}"] = "".join(chars)
    return out


def genes(seed, n, gene_max=4):
    """List of (first_contig, size) runs covering contigs 0..n-1."""
    k = stream_key(seed, S_GENE)
    out, c, j = [], 0, 0
    while c < n:
        size = min(1 + mix(k + (j + 1) * GOLDEN) % gene_max, n - c)
        out.append((c, size))
        c += size
        j += 1
    return out


def fragment_masks(seed, r, gene_list, paired):
    first, g = gene_list[u(seed, S_FGENE, r) % len(gene_list)]
    full = (1 << g) - 1
    m1 = 1 + u(seed, S_MASK1, r) % full
    m2 = m1
    if paired and u(seed, S_DISC, r) % 16 == 0:
        m2 = 1 + u(seed, S_MASK2, r) % full
    return first, m1, m2


def read_records(seed, n_contigs, n_frags, paired, gene_max=4):
    """(read_id, contig) records grouped by read, as a SAM stream would be."""
    gl = genes(seed, n_contigs, gene_max)
    recs = []
    for r in range(n_frags):
        first, m1, m2 = fragment_masks(seed, r, gl, paired)
        for b in range(m1.bit_length()):
            if m1 >> b & 1:
                recs.append((r, first + b))
        if paired:
            for b in range(m2.bit_length()):
                if m2 >> b & 1:
                    recs.append((r, first + b))
    return recs


def eq_classes(seed, n_contigs, n_frags, paired, gene_max=4):
    """Salmon-style classes: fragment dedup sets aggregated in first-seen order.

    Returns list of (tuple(contig ids ascending), count)."""
    gl = genes(seed, n_contigs, gene_max)
    counts = OrderedDict()
    for r in range(n_frags):
        first, m1, m2 = fragment_masks(seed, r, gl, paired)
        m = m1 | m2
        key = tuple(first + b for b in range(m.bit_length()) if m >> b & 1)
        counts[key] = counts.get(key, 0) + 1
    return list(counts.items())


def eq_file_text(names, classes):
    """salmon `eq_classes.txt` text (format parsed by karma/read_graph.py:75-82)."""
    lines = [str(len(names)), str(len(classes))]
    lines += list(names)
    for ids, cnt in classes:
        lines.append("\t".join([str(len(ids))] + [str(i) for i in ids] + [str(cnt)]))
    return "\n".join(lines) + "\n"


def fasta_text(seqs, width=80):
    out = []
    for h, s in seqs.items():
        out.append(h)
        out += [s[i:i + width] for i in range(0, len(s), width)] or [""]
    return "\n".join(out) + "\n"
