"""Contig read sets (drop-in for karma/contig.py:4-35).

A contig keeps the set of QNAMEs (SAM column 1) mapped to it, so the two
mates of a pair count once (contig.py:11).  `contig_records` turns a list of
Contig objects into the (read id, contig index) record stream the HIP graph
kernels consume (karma_amd.engine.graph_from_records).
"""
import io

import numpy as np

from . import ingest
from .logs import logger


class Contig:
    def __init__(self, name):
        self.name = name
        self.readset = set()

    def add_read(self, name, position):
        self.readset.add(name)

    def has_read(self, name):
        # the reference reads a non-existent self.reads here (contig.py:13-14 raises
        # AttributeError); this answers the question the method's name asks.
        return name in self.readset

    def load_contig_info_from_sam(self, sam_file):
        logger.debug("Creating new contig object...")
        with open(sam_file, "r") as sam_reader:
            self.load_from_iterator(sam_reader)

    def load_from_iterator(self, sam_infos):
        for line in sam_infos:
            read, _, name, position, *_ = line.split("\t")
            self.add_read(read, position)


def _sam_bytes(sam):
    """SAM input as bytes: a path, str/bytes text, or an iterable of lines."""
    if isinstance(sam, (bytes, bytearray)):
        return bytes(sam)
    if isinstance(sam, str):
        if "\t" in sam or "\n" in sam:
            return sam.encode("utf-8")
        return ingest._read(sam)
    return "".join(line if line.endswith(("\n", "\r")) else line + "\n" for line in sam).encode("utf-8")


def _check_sam_text(data, skip_headers):
    """The reference's per-line unpack (contig.py:34) over lines the C++ reader
    declined: raises its ValueError / UnicodeDecodeError."""
    for line in io.StringIO(data.decode("utf-8"), newline=None):  # text-mode lines
        if skip_headers and line.startswith("@"):
            continue
        read, _, name, position, *_ = line.split("\t")


def load_sam_records(sam, skip_headers=True, threads=0):
    """SAM lines -> ingest.SamRecords: one (read id, contig id) record per line,
    contig ids numbering RNAMEs (field 3) in order of first appearance
    (csrc/ingest.cpp, karma_sam_parse).  skip_headers drops "@" lines as the
    hisat2 generator does (hisat2.py:49-53).

    Line splitting follows file mode (contig.py:31 iterates an open() file):
    universal newlines.  The hisat2 generator instead splits samtools' stdout
    on "\n" only and drops what follows the last "\n" (hisat2.py:51).  The two
    agree on any text without "\r" and with a final newline, which is what
    samtools writes; generator-style text holding "\r" keeps it inside the
    line there, and must be normalised by the caller before it comes here."""
    data = _sam_bytes(sam)
    try:
        return ingest.parse_sam(data, skip_headers, threads), data
    except ingest.ParseDeferred:
        _check_sam_text(data, skip_headers)
        raise


def contigs_from_sam(sam, skip_headers=True, threads=0):
    """Contig objects grouped by RNAME (first appearance order), each with the
    readset contig.py:24,34 builds from its lines."""
    rec, data = load_sam_records(sam, skip_headers, threads)
    contigs = [Contig(n) for n in rec.rnames]
    qs, ql, cid = rec.q_start.tolist(), rec.q_len.tolist(), rec.records[:, 1].tolist()
    for s0, n, c in zip(qs, ql, cid):
        contigs[c].readset.add(data[s0:s0 + n].decode("utf-8"))
    return contigs


def contig_records(contigs, start_index=0, read_ids=None):
    """Flatten readsets to uint32 (read_id, contig_index) records (contig-major).

    read_ids: shared dict QNAME -> dense id (pass the same dict for several
    calls that must agree)."""
    if read_ids is None:
        read_ids = {}
    rows, cols = [], []
    for k, c in enumerate(contigs):
        ids = [read_ids.setdefault(q, len(read_ids)) for q in c.readset]
        rows.extend(ids)
        cols.extend([start_index + k] * len(ids))
    if len(read_ids) >= 2**32:
        raise ValueError("more than 2^32 distinct reads")
    rec = np.empty((len(rows), 2), dtype=np.uint32)
    if rows:
        rec[:, 0] = rows
        rec[:, 1] = cols
    return rec, read_ids
