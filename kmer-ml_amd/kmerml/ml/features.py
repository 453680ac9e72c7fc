"""Organisms x k-mers feature matrix -- drop-in for the reference's kmerml/ml/features.py
(KmerFeatureBuilder; row f4), vectorised.

build_from_statistics_files() reads the per-organism feature CSVs exactly as the reference
does (features.py:28-77) and returns the same DataFrame: one row per organism in file order
(organism id = first two '_' tokens of the file stem, features.py:79-85), one column per
label in sorted order, the metric of the LAST row carrying a label when a label repeats
(``dict(zip(...))`` semantics, so a label shared by two k values keeps the later file's
value), 0 where an organism lacks the label (features.py:87-117).  The reference fills the
matrix with a Python list comprehension per organism; here it is one scatter per organism.

from_count_matrix() builds the same count matrix directly from the dense [G, 4^k] counts of
kmerml.kmers.matrix.count_matrix (the GPU path), labelling columns the way the reference's
file round trip would (digits A0 T1 C2 G3, leading zeros lost to integer parsing).
"""
from pathlib import Path
from typing import Dict, Union

import numpy as np
import pandas as pd

from kmerml.utils.path_utils import find_files


class KmerFeatureBuilder:
    """Convert k-mer statistics data into ML-ready feature matrices (features.py:13-26)."""

    def __init__(self, stats_dir: Union[str, Path] = None):
        self.stats_dir = Path(stats_dir) if stats_dir else None
        self.feature_matrix = None
        self.organisms = []
        self.kmers = []

    def build_from_statistics_files(self, metric: str = "count",
                                    file_pattern: str = "*kmer_features.csv") -> pd.DataFrame:
        if not self.stats_dir:
            raise ValueError("Statistics directory not set")
        stats_files = find_files(self.stats_dir, patterns=[file_pattern], recursive=True)
        if not stats_files:
            raise ValueError(f"No statistics files found matching pattern: {file_pattern}")
        organism_data = {}
        for file_path in stats_files:
            organism_id = self._extract_organism_id(file_path)
            try:
                df = pd.read_csv(file_path)
                if 'kmer' not in df.columns or metric not in df.columns:
                    available_cols = ', '.join(df.columns)
                    raise ValueError(f"Required columns not found in {file_path}. Available: {available_cols}")
                organism_data[organism_id] = (df['kmer'].to_numpy(), df[metric].to_numpy())
            except Exception as e:
                print(f"Error processing {file_path}: {e}")
        return self._build_matrix(organism_data)

    def _extract_organism_id(self, file_path: Path) -> str:
        parts = file_path.stem.split('_')
        return f"{parts[0]}_{parts[1]}" if len(parts) >= 2 else file_path.stem

    def _build_matrix(self, organism_data: Dict[str, tuple]) -> pd.DataFrame:
        """organism -> (labels, values); same DataFrame as features.py:87-117."""
        per_org = {}
        for org, (labels, values) in organism_data.items():
            s = pd.Series(values, index=pd.Index(labels, dtype=object))
            per_org[org] = s[~s.index.duplicated(keep='last')]     # dict(zip()): last value wins
        all_labels = set()
        for s in per_org.values():
            all_labels.update(s.index.tolist())
        columns = sorted(all_labels)
        self.organisms = list(per_org)
        kinds = {s.dtype.kind for s in per_org.values()}
        if not kinds <= {'i', 'u', 'f', 'b'} or not columns:
            # general values: the reference's own construction
            rows = [[s.get(c, 0) if c in s.index else 0 for c in columns] for s in per_org.values()]
            self.feature_matrix = pd.DataFrame(rows, index=self.organisms, columns=columns)
        else:
            float_cols = None
            dtype = np.float64 if 'f' in kinds else np.int64
            mat = np.zeros((len(per_org), len(columns)), dtype=dtype)
            col_index = pd.Index(columns, dtype=object)
            for r, s in enumerate(per_org.values()):
                pos = col_index.get_indexer(s.index)
                mat[r, pos] = s.to_numpy()
            if dtype is np.float64 and kinds != {'f'}:
                # a column is float64 in the reference only if some organism with that label
                # holds a float; elsewhere it stays int64
                float_cols = np.zeros(len(columns), dtype=bool)
                for s in per_org.values():
                    if s.dtype.kind == 'f':
                        float_cols[col_index.get_indexer(s.index)] = True
            if float_cols is None:
                self.feature_matrix = pd.DataFrame(mat, index=self.organisms, columns=columns)
            else:
                data = {c: (mat[:, j] if float_cols[j] else mat[:, j].astype(np.int64))
                        for j, c in enumerate(columns)}
                self.feature_matrix = pd.DataFrame(data, index=self.organisms, columns=columns)
        self.kmers = columns
        return self.feature_matrix

    # ------------------------------------------------------------------ GPU path
    @staticmethod
    def _label_levels(k: int):
        """The compat labels level by level.  Codes with m significant letters (leading A's
        stripped; code 0 is "A") are exactly the range [4^(m-1), 4^m) (codes 0..3 for m = 1),
        and a level-m label is a level-(m-1) label plus one letter: L_m = repeat(L_{m-1}, 4)
        beside tile("ACGT").  Returns the [count, m] uint8 letter blocks, m = 1..k."""
        lut = np.frombuffer(b"ACGT", np.uint8)
        levels = [lut.reshape(4, 1).copy()]
        for m in range(2, k + 1):
            prev = levels[-1] if m > 2 else levels[0][1:]         # parents: first letter not A
            cur = np.empty((prev.shape[0] * 4, m), dtype=np.uint8)
            cur[:, :m - 1] = np.repeat(prev, 4, axis=0)
            cur[:, m - 1] = np.tile(lut, prev.shape[0])
            levels.append(cur)
        return levels

    @staticmethod
    def compat_label_arrow(k: int):
        """The labels of compat_labels(k) as a pyarrow string array (one buffer of letters plus
        offsets, no Python objects)."""
        import pyarrow as pa

        if not 1 <= k <= 19:
            raise NotImplementedError("compat labels are defined for 1 <= k <= 19")
        levels = KmerFeatureBuilder._label_levels(k)
        buf = np.concatenate([lv.ravel() for lv in levels])
        lens = np.concatenate([np.full(lv.shape[0], lv.shape[1], dtype=np.int64) for lv in levels])
        offsets = np.zeros(lens.size + 1, dtype=np.int32 if buf.size < 2**31 else np.int64)
        np.cumsum(lens, out=offsets[1:])
        typ = pa.string() if offsets.dtype == np.int32 else pa.large_string()
        return pa.Array.from_buffers(typ, lens.size, [None, pa.py_buffer(offsets), pa.py_buffer(buf)])

    @staticmethod
    def compat_labels(k: int):
        """Column label of every k-mer code (A0 C1 G2 T3, first base most significant) after
        the reference's file round trip: digits A0 T1 C2 G3, parsed as an integer (leading
        zeros lost) and decoded back (statistics.py:157, :248-272).  Exact for k <= 19
        (labels that fit int64).  A pandas Index of Arrow-backed strings, indexable by code."""
        return pd.Index(pd.arrays.ArrowStringArray(KmerFeatureBuilder.compat_label_arrow(k)))

    @staticmethod
    def compat_label_order(k: int) -> np.ndarray:
        """The codes in the order of their compat labels (Python string order, a label before
        every label it prefixes), without sorting: the labels are the nodes of a trie -- "A",
        then complete 4-ary subtrees of k levels under C, G and T -- and string order is its
        pre-order.  With N(d) = (4^d - 1) / 3 nodes in d levels: rank("A") = 0, rank of a
        one-letter label s = 1 + (s - 1) N(k), and appending letter r to a label of m - 1
        letters gives rank + 1 + r N(k - m + 1)."""
        N = [(4 ** d - 1) // 3 for d in range(k + 2)]
        rank = np.array([0] + [1 + (s - 1) * N[k] for s in (1, 2, 3)], dtype=np.int64)
        ranks = [rank]
        prev = rank[1:]
        for m in range(2, k + 1):
            cur = (prev[:, None] + 1 + np.arange(4, dtype=np.int64)[None, :] * N[k - m + 1]).ravel()
            ranks.append(cur)
            prev = cur
        rank = np.concatenate(ranks)
        order = np.empty_like(rank)
        order[rank] = np.arange(rank.size, dtype=np.int64)
        return order

    @staticmethod
    def _from_assembled(mat, order, block=8):
        """from_count_matrix on an AssembledMatrix without widening it whole: rows are widened
        `block` at a time on the device, once for the presence test and once for the values."""
        import torch

        G = mat.shape[0]
        dev = mat.recv.device if mat.recv is not None else mat._dense.device
        dev_order = torch.from_numpy(order).to(dev)
        present = torch.zeros(mat.shape[1], dtype=torch.bool, device=dev)
        for lo in range(0, G, block):
            present |= (mat.rows(lo, min(G, lo + block)) != 0).any(dim=0)
        cols_t = dev_order[present[dev_order]]
        values = np.empty((G, cols_t.numel()), np.int64)
        for lo in range(0, G, block):
            hi = min(G, lo + block)
            values[lo:hi] = (mat.rows(lo, hi)[:, cols_t].to(torch.int64) & 0xFFFFFFFF).cpu().numpy()
        return values, cols_t.cpu().numpy()

    def from_count_matrix(self, counts, k: int, organisms) -> pd.DataFrame:
        """Count matrix DataFrame for organisms with one k-mer file each, from the dense
        [G, 4^k] count rows (numpy or torch, u32 stored as int32 is fine; or a
        kmerml.kmers.matrix.AssembledMatrix).  Equal to build_from_statistics_files(
        metric="count") on the files the extractor writes (statistics.py:95-147 ->
        features.py:85-117): columns = labels present in any organism, in label order."""
        order = self.compat_label_order(k)
        if hasattr(counts, "dense") and hasattr(counts, "rows"):     # AssembledMatrix
            values, cols = self._from_assembled(counts, order)
        elif hasattr(counts, "is_cuda") and counts.is_cuda:
            # device counts: presence test and the column permutation on the GPU, then one copy;
            # an int32 cell holding a u32 is non-zero iff the count is, so only the gathered
            # columns are widened
            import torch

            dev_order = torch.from_numpy(order).to(counts.device)
            keep = (counts != 0).any(dim=0)[dev_order] if counts.shape[0] else torch.zeros(0, dtype=torch.bool)
            cols_t = dev_order[keep]
            values = (counts[:, cols_t].to(torch.int64) & 0xFFFFFFFF).cpu().numpy()
            cols = cols_t.cpu().numpy()
        else:
            rows = counts.cpu().numpy() if hasattr(counts, "cpu") else np.asarray(counts)
            rows = rows.view(np.uint32) if rows.dtype == np.int32 else rows
            cols = order[(rows > 0).any(axis=0)[order]] if rows.shape[0] else order[:0]
            values = rows[:, cols].astype(np.int64)
        labels = self.compat_label_arrow(k).take(cols)
        self.organisms = list(organisms)
        columns = pd.Index(pd.arrays.ArrowStringArray(labels))
        self.kmers = columns
        self.feature_matrix = pd.DataFrame(values, index=self.organisms, columns=columns)
        return self.feature_matrix
