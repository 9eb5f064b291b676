"""Contig read sets (drop-in for karma/contig.py:4-35).

A contig keeps the set of QNAMEs (SAM column 1) mapped to it, so the two
mates of a pair count once (contig.py:11).  `contig_records` turns a list of
Contig objects into the (read id, contig index) record stream the HIP graph
kernels consume (karma_amd.engine.graph_from_records).
"""
import numpy as np

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
