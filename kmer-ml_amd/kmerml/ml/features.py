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
    def compat_labels(k: int) -> np.ndarray:
        """Column label of every k-mer code (A0 C1 G2 T3, first base most significant) after
        the reference's file round trip: digits A0 T1 C2 G3, parsed as an integer (leading
        zeros lost) and decoded back (statistics.py:157, :248-272).  Exact for k <= 19
        (labels that fit int64)."""
        if not 1 <= k <= 19:
            raise NotImplementedError("compat labels are defined for 1 <= k <= 19")
        to_letter = np.frombuffer(b"ACGT", np.uint8)          # device code -> letter
        codes = np.arange(1 << (2 * k), dtype=np.int64)
        letters = np.empty((codes.size, k), dtype=np.uint8)
        for i in range(k):
            letters[:, i] = to_letter[(codes >> (2 * (k - 1 - i))) & 3]
        # strip leading A's (digit 0), keeping one when the k-mer is all A's
        lead = np.argmax(letters != ord('A'), axis=1)
        lead[(letters == ord('A')).all(axis=1)] = k - 1
        flat = letters.tobytes().decode('ascii')
        return np.array([flat[c * k + s:(c + 1) * k] for c, s in enumerate(lead.tolist())], dtype=object)

    def from_count_matrix(self, counts, k: int, organisms) -> pd.DataFrame:
        """Count matrix DataFrame for organisms with one k-mer file each, from the dense
        [G, 4^k] count rows (numpy or torch, u32 stored as int32 is fine).  Equal to
        build_from_statistics_files(metric="count") on the files the extractor writes."""
        rows = counts.cpu().numpy() if hasattr(counts, "cpu") else np.asarray(counts)
        rows = rows.view(np.uint32) if rows.dtype == np.int32 else rows
        labels = self.compat_labels(k)
        present = (rows > 0).any(axis=0)
        order = np.argsort(labels[present].astype(str), kind='stable')
        cols = np.nonzero(present)[0][order]
        self.organisms = list(organisms)
        self.kmers = labels[cols].tolist()
        self.feature_matrix = pd.DataFrame(rows[:, cols].astype(np.int64), index=self.organisms, columns=self.kmers)
        return self.feature_matrix
