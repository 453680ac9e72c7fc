"""TEST INFRASTRUCTURE ONLY: CPU restatements of the reference's k-mer path.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
The product package (kmer-ml_amd/kmerml) never imports anything from here.
"""
