"""karma_amd — MI355X-native k-mer profile + shared-read graph hot path of lmfaber/karma.

Drop-in modules mirroring the reference API (karma/kmer.py, karma/read_graph.py,
karma/contig.py) live in ``karma_amd.kmer``, ``karma_amd.read_graph`` and
``karma_amd.contig``; all compute goes through the HIP C-ABI library
``libkarma_hip.so`` (include/karma.h) loaded by ``karma_amd._lib``.
"""

__version__ = "0.1.0"
