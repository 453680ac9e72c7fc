"""Route the reference's k-mer modules to the MI355X implementation.

Importing this module installs a meta-path finder (ahead of every sys.path entry, including
the current directory) that serves

    kmerml.kmers.generate  -> kmer-ml_amd/kmerml/kmers/generate.py  (GPU KmerExtractor)
    kmerml.kmers.matrix    -> kmer-ml_amd/kmerml/kmers/matrix.py    (multi-GPU count matrix)
    kmerml.kmers.statistics-> kmer-ml_amd/kmerml/kmers/statistics.py (vectorised feature CSVs)
    kmerml.ml.features     -> kmer-ml_amd/kmerml/ml/features.py     (vectorised feature matrix)
    kmerml._native         -> kmer-ml_amd/kmerml/_native.py         (ctypes binding)

while the `kmerml` package itself and all its other modules keep coming from the reference
checkout.  So `python -m scripts.extract_kmers ...` run from the reference root counts on the
GPU, and `python -m scripts.generate_kmers_features ...` builds the same feature CSVs with the
vectorised extractor, with no change to the reference (activate/sitecustomize.py imports this
at startup).
"""
import importlib.abc
import importlib.util
import os
import sys

_ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kmerml")
MODULES = {
    "kmerml._native": "_native.py",
    "kmerml.kmers.generate": os.path.join("kmers", "generate.py"),
    "kmerml.kmers.matrix": os.path.join("kmers", "matrix.py"),
    "kmerml.kmers.statistics": os.path.join("kmers", "statistics.py"),
    "kmerml.ml.features": os.path.join("ml", "features.py"),
}


class _Finder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path=None, target=None):
        rel = MODULES.get(name)
        if rel is None:
            return None
        return importlib.util.spec_from_file_location(name, os.path.join(_ROOT, rel))


def activate():
    if not any(isinstance(f, _Finder) for f in sys.meta_path):
        sys.meta_path.insert(0, _Finder())


activate()
