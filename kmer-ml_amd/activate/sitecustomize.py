"""Put kmer-ml_amd/activate on PYTHONPATH to run the reference's scripts on the GPU path:

    PYTHONPATH=<repo>/kmer-ml_amd/activate python -m scripts.extract_kmers -i data/raw ...
"""
import os
import sys

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG not in sys.path:
    sys.path.append(_PKG)
import kmerml_gpu  # noqa: E402,F401
