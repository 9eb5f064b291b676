"""FASTA reader with the reference's exact key semantics (karma/karma.py:40-61).

The keys of the returned OrderedDict are what KmerClustering normalises by
(kmer.py:213 takes len() of the KEYS), so they must match byte for byte:
key = first line (or header line) with only "\\n" stripped, split on " " only,
first token, ">" kept; sequence lines are concatenated; duplicate keys keep
their first position and take the last sequence.  Text mode: UTF-8 and
universal newlines ("\\r\\n" and a lone "\\r" end a line too).

The file is parsed by the multi-threaded C++ reader (csrc/ingest.cpp,
karma_fasta_parse).  Input outside what it reproduces exactly (invalid UTF-8,
a non-UTF-8 locale) goes through `_read_fasta_text`, the reference's own
line loop, so the result or the exception is the reference's.  The returned
dict carries the packed (bytes, offsets, key lengths) arrays, so
KmerClustering can skip re-encoding them; any mutation drops them.
"""
from collections import OrderedDict

import numpy as np

from . import ingest
from .logs import logger


class FastaDict(OrderedDict):
    """OrderedDict of FASTA records that also holds the packed arrays the
    contig store is built from (`karma_packed`: blob, offsets, key lengths),
    valid until the dict is mutated."""

    karma_packed = None

    def _drop(self):
        self.karma_packed = None

    def __setitem__(self, k, v):
        self._drop()
        super().__setitem__(k, v)

    def __delitem__(self, k):
        self._drop()
        super().__delitem__(k)

    def pop(self, *a):
        self._drop()
        return super().pop(*a)

    def popitem(self, *a, **kw):
        self._drop()
        return super().popitem(*a, **kw)

    def clear(self):
        self._drop()
        super().clear()

    def setdefault(self, *a):
        self._drop()
        return super().setdefault(*a)

    def update(self, *a, **kw):
        self._drop()
        super().update(*a, **kw)

    def move_to_end(self, *a, **kw):
        self._drop()
        super().move_to_end(*a, **kw)


def _read_fasta_text(fasta_file):
    """karma.py:49-61, line by line (the path for input the C++ reader declines)."""
    sequences = OrderedDict()
    with open(fasta_file, "r") as reader:
        name = reader.readline().rstrip("\n").split(" ")[0]
        parts = []
        for line in reader:
            if line.startswith(">"):
                sequences[name] = "".join(parts)
                name = line.rstrip("\n").split(" ")[0]
                parts = []
            else:
                parts.append(line.rstrip("\n"))
        sequences[name] = "".join(parts)
    return sequences


def read_fasta_file(fasta_file, threads=0):
    logger.info("Reading fasta file.")
    try:
        rec = ingest.parse_fasta(ingest._read(fasta_file), threads)
    except ingest.ParseDeferred:
        sequences = _read_fasta_text(fasta_file)
    else:
        sequences = FastaDict(zip(rec.names(), rec.sequences()))
        if rec.ascii:  # latin-1 bytes == the file's bytes: the contig store's input as is
            sequences.karma_packed = (rec.seq, rec.seq_off, rec.key_len.astype(np.int32))
    logger.debug(f"Read {len(sequences)} sequences in total.")
    return sequences
