"""MI355X-native drop-in for the hot path of Masthetheus/kmer-ml's ``kmerml`` package.

This package provides ``kmerml.kmers.generate`` (GPU k-mer counting behind the
reference's ``KmerExtractor`` API), ``kmerml.kmers.matrix`` (the genomes x k-mers count
matrix, sharded one block of genomes per GPU and assembled with an RCCL all-gather) and
the ``kmerml.utils.path_utils`` helpers they need.  ``__path__`` is extended over every
``kmerml`` directory on ``sys.path`` (pkgutil.extend_path), so with the reference
checkout later on the path its other modules (statistics, features, metadata, ...) keep
importing as before, while the modules provided here take precedence.
"""
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)
__version__ = "0.2.0"
