"""FASTA reader with the reference's exact key semantics (karma/karma.py:40-61).

The keys of the returned OrderedDict are what KmerClustering normalises by
(kmer.py:213 takes len() of the KEYS), so they must match byte for byte:
key = first line (or header line) with only "\\n" stripped, split on " " only,
first token, ">" kept; sequence lines are concatenated with "\\n" stripped
(a trailing "\\r" stays); duplicate keys overwrite in place.
"""
from collections import OrderedDict

from .logs import logger


def read_fasta_file(fasta_file):
    logger.info("Reading fasta file.")
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
    logger.debug(f"Read {len(sequences)} sequences in total.")
    return sequences
