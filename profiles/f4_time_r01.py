"""Time the feature CSV step (row f4) on one k = 12 file: the reference's KmerFeatureExtractor
(run from /root/reference in a child process) vs the vectorised one here.  Build container
only (needs the reference checkout); CPU, one core each.

    python profiles/f4_time_r01.py [bases]
"""
import contextlib
import io
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "kmer-ml_amd"), REPO]
from oracle import kmers as okmers  # noqa: E402
from oracle import synth as osynth  # noqa: E402

CHILD = r"""
import contextlib, io, sys, time
from kmerml.kmers.statistics import KmerFeatureExtractor
t0 = time.perf_counter()
with contextlib.redirect_stdout(io.StringIO()):
    KmerFeatureExtractor(input_paths=[sys.argv[1]], output_dir=sys.argv[2]).extract_features()
print(time.perf_counter() - t0)
"""


def main():
    bases = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    tmp = tempfile.mkdtemp(prefix="f4_")
    seq = osynth.synth_bases(bases, osynth.genome_seed(0)).tobytes().decode()
    os.makedirs(os.path.join(tmp, "k", "orgX"))
    kfile = os.path.join(tmp, "k", "orgX", "k12.txt")
    t = okmers.count_sequence(seq, 12)
    with open(kfile, "w") as f:
        f.write(okmers.kmer_text(t))
    rows = len(t)
    ref = float(subprocess.run([sys.executable, "-c", CHILD, kfile, os.path.join(tmp, "ref")],
                               env=dict(os.environ, PYTHONPATH="/root/reference", PYTHONDONTWRITEBYTECODE="1"),
                               capture_output=True, text=True, check=True).stdout.strip())
    from kmerml.kmers.statistics import KmerFeatureExtractor
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        KmerFeatureExtractor(input_paths=[kfile], output_dir=os.path.join(tmp, "ours")).extract_features()
    ours = time.perf_counter() - t0
    a = open(os.path.join(tmp, "ref", "orgX_kmer_features.csv")).read()
    b = open(os.path.join(tmp, "ours", "orgX_kmer_features.csv")).read()
    same = sum(x == y for x, y in zip(a.splitlines(), b.splitlines()))
    print(f"k=12, {rows} rows: reference {ref:.2f} s ({ref / rows * 1e6:.1f} us/row), "
          f"vectorised {ours:.2f} s ({ours / rows * 1e6:.2f} us/row), speedup {ref / ours:.1f}x; "
          f"identical lines {same}/{len(a.splitlines())}")


if __name__ == "__main__":
    main()
