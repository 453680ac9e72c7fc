"""Row f4 timing: the feature CSV of one organism with one dense k = 12 k-mer file of N lines
(default 4 M; the reference's statistics.py:95-147 path, served by kmerml.kmers.statistics).
Prints the time of the whole _process_organism_kmers call, of the feature block, and of the
CSV text + file write alone (write_feature_csv), and checks the text against pandas' to_csv.

    python profiles/f4_csv_r03.py [lines]
"""
import contextlib
import io
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "kmer-ml_amd"), os.path.join(HERE, "..")]

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

from kmerml import _native  # noqa: E402
from kmerml.kmers import statistics as st  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    k = 12
    rng = np.random.default_rng(12)
    codes = rng.choice(1 << (2 * k), n, replace=False).astype(np.uint64)
    counts = rng.integers(1, 40, n).astype(np.uint64)
    with tempfile.TemporaryDirectory() as tmp:
        kdir = os.path.join(tmp, "kmers", "orgX")
        os.makedirs(kdir)
        kfile = os.path.join(kdir, "k12.txt")
        _native.write_file(kfile, _native.format_lines(k, codes, counts))
        ext = st.KmerFeatureExtractor(input_paths=[kfile], output_dir=os.path.join(tmp, "feat"))
        from pathlib import Path
        st.feature_table(k)                     # the per-k table once (cached), as in a multi-organism run
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            out = ext._process_organism_kmers("orgX", [Path(kfile)], st.DEFAULT_FEATURES)
        t_all = time.perf_counter() - t0
        df = ext._load_kmer_file(kfile)
        t0 = time.perf_counter()
        block = ext.feature_block(df, k, st.DEFAULT_FEATURES)
        t_block = time.perf_counter() - t0
        t0 = time.perf_counter()
        st.write_feature_csv([block], os.path.join(tmp, "again.csv"))
        t_write = time.perf_counter() - t0
        t0 = time.perf_counter()
        want = block.frame().to_csv(index=False)
        t_pandas = time.perf_counter() - t0
        same = open(out).read() == want == open(os.path.join(tmp, "again.csv")).read()
        print({"lines": n, "k": k, "process_organism_s": round(t_all, 3), "feature_block_s": round(t_block, 3),
               "write_feature_csv_s": round(t_write, 3), "pandas_to_csv_s": round(t_pandas, 3),
               "bytes": os.path.getsize(out), "identical_to_pandas": same, "cpus": os.cpu_count()})


if __name__ == "__main__":
    main()
