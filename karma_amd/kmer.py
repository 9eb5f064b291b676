"""K-mer profile clustering — drop-in for karma/kmer.py:14-325.

The profile (the hot path, kmer.py:146-264) runs on the MI355X through
libkarma_hip.so: 2-bit packed contigs, LDS-private presence bitmaps, a
one-block column-table merge, and an LDS histogram per contig streamed out as
the dense float64 row count / len(FASTA key).  Results are bit-identical to the
reference (tests/test_gpu_parity.py).  The clustering tail (UMAP + HDBSCAN,
kmer.py:283-301) is third-party and used only if those packages import.
"""

import os
import sys

import numpy as np

from . import engine
from .logs import logger


class KmerClustering:
    def __init__(self, sequences, output_dir, kmer_size, threads):
        self.sequences = sequences
        self.output_dir = output_dir
        self.output_eval = f"{self.output_dir}/eval.txt"
        self.output_file = f"{self.output_dir}/cluster.txt"
        self.threads = threads
        self.kmer_size = kmer_size
        self.clusters = []
        self.unlabeled_cluster = []
        self.kmers = None
        self.sorted_kmer_set = set()

    @staticmethod
    def is_palindrome(sequence):
        """kmer.py:46-54: string reversal (not reverse complement)."""
        return sequence == sequence[::-1]

    @staticmethod
    def __mask_list(list_to_mask, mask):
        """kmer.py:29-44: contig names (">" stripped) grouped by cluster label."""
        names = [k.lstrip(">") for k in list_to_mask.keys()]
        labeled, unlabeled = [], []
        for label in set(mask):
            members = [names[j] for j, x in enumerate(mask) if x == label]
            (unlabeled if label == -1 else labeled).append(members)
        return labeled, unlabeled

    def __calc_kmer_profile(self, out=None):
        """kmer.py:199-264 on the GPU.  Same return value, side effects
        (self.kmers, self.sorted_kmer_set) and failure modes (ZeroDivisionError
        for a zero-length key, logger.error + exit(1) for an all-zero row).

        out (an addition; the reference has no such argument): a caller
        float64[N, M] C-order array or numpy.memmap that the profile fills one
        row block at a time and that is returned -- config 5's 131 GB profile
        need not exist in host memory as a fresh array.  M is the column count
        (KmerClustering.columns_count)."""
        return self.__profile(lambda seqs, k: engine.kmer_profile(seqs, k, out=out))

    def columns_count(self):
        """M, the column count __calc_kmer_profile will have (to size `out`)."""
        return engine.kmer_columns_count(self.sequences, self.kmer_size)

    def calc_kmer_profile_device(self):
        """The same profile left in HBM for a GPU consumer (SURVEY.md §8(f) row 4,
        the UMAP input of kmer.py:283-290): a device_profile.DeviceProfile
        (DLPack / __cuda_array_interface__, float64 N x M row-major), with the
        same side effects and failure modes as __calc_kmer_profile."""
        return self.__profile(engine.kmer_profile_device)

    def __profile(self, compute):
        logger.info("Extracting kmers from contigs.")
        try:
            profile, columns, row_totals = compute(self.sequences, self.kmer_size)
        except engine._lib.KarmaError as e:
            if e.code == engine._lib.KARMA_ERR_ZERO_DIV:
                raise ZeroDivisionError("division by zero") from e
            raise
        self.sorted_kmer_set = columns
        self.kmers = {kmer: i for i, kmer in enumerate(columns)}
        logger.debug(f"Dict has {len(self.kmers)} entries.")
        # kmer.py:236-248 — every column holds a k-mer that occurs, so no
        # column can be all zero; kmer.py:250-258 — a contig shorter than k has
        # no k-mer, hence an all-zero row.
        zero_rows = np.flatnonzero(row_totals == 0)
        if len(zero_rows):
            logger.error(f"Values of row {int(zero_rows[0])} are all zero, which should not be the case.")
            exit(1)
        self.sorted_kmer_set.clear()
        logger.debug(f"KMER-PROFILE - Size: {sys.getsizeof(profile)}, Shape: {profile.shape}")
        return profile

    def __fix_fasta_headers(self):
        """kmer.py:94-106."""
        logger.debug(f"unlabeled: {self.unlabeled_cluster}")
        self.unlabeled_cluster = [[name.split(" ")[0] for name in self.unlabeled_cluster[0]]]
        self.clusters = [[name.split(" ")[0] for name in cluster] for cluster in self.clusters]

    def __save_groups_to_file(self):
        """kmer.py:124-133: first line unlabeled, then one cluster per line."""
        with open(self.output_file, "w") as fh:
            fh.write("\t".join(self.unlabeled_cluster[0]) + "\n")
            for cluster in self.clusters:
                fh.write("\t".join(cluster) + "\n")

    def __read_clusters(self):
        """kmer.py:135-144 (cache of a previous run)."""
        with open(self.output_file, "r") as fh:
            self.unlabeled_cluster = [fh.readline().rstrip("\n").split("\t")]
            for line in fh:
                self.clusters.append(line.rstrip("\n").split("\t"))

    def __write_eval_information(self, **kwargs):
        """kmer.py:266-272."""
        with open(self.output_eval, "w") as fh:
            fh.write("\t".join(kwargs.keys()) + "\n")
            fh.write("\t".join(str(v) for v in kwargs.values()) + "\n")

    def run(self, neighbors, components, dist, r_state, min_cluster_size):
        """kmer.py:274-325.  The profile is computed on the GPU; UMAP/HDBSCAN
        are the reference's third-party dependencies and must be importable."""
        if os.path.isfile(self.output_file):
            logger.info(f"Read from previous calculation: {self.output_file}")
            self.__read_clusters()
        else:
            logger.info("Calculate kmer profiles.")
            kmer_profile = self.__calc_kmer_profile()
            try:
                import hdbscan
                import umap
            except ImportError as e:
                raise ImportError("KmerClustering.run needs umap-learn and hdbscan (the reference's clustering "
                                  "dependencies); the k-mer profile itself does not") from e
            logger.info("Dimension reduction with UMAP.")
            reduced = umap.UMAP(n_neighbors=neighbors, n_components=components, min_dist=dist,
                                random_state=r_state).fit_transform(kmer_profile)
            logger.info(f"Perform clustering with HDBSCAN. (min_cluster_size: {min_cluster_size})")
            if min_cluster_size == 1:
                clusterer = hdbscan.HDBSCAN(allow_single_cluster=True).fit(reduced)
            else:
                clusterer = hdbscan.HDBSCAN(min_cluster_size=min_cluster_size).fit(reduced)
            self.clusters, self.unlabeled_cluster = self.__mask_list(self.sequences, clusterer.labels_)
            self.__save_groups_to_file()
            labels = list(clusterer.labels_)
            self.__write_eval_information(
                kmer_size=self.kmer_size, n_neighbors=neighbors, n_components=components, min_dist=dist,
                random_state=r_state, min_cluster_size=min_cluster_size, unlabeled=labels.count(-1),
                no_groups=max(labels) + 1, mean_probability=np.mean(clusterer.probabilities_))
        self.__fix_fasta_headers()
