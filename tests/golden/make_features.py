"""Regenerate tests/golden/features2/: L3 fixtures produced by
the REFERENCE's own KmerFeatureExtractor (statistics.py) and KmerFeatureBuilder
(features.py) on k-mer files that the reference's generate.py wrote.

Needs /root/reference (build container only).  Run from the repo root:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_features.py

Cases (inputs regenerated from oracle/synth.py; nothing from the reference is stored but
its outputs):
  orgC  6 kbp synthetic genome with N runs and lowercase, k = 3, 12, 20, 21
        (k = 20: labels that fit uint64 and labels that do not -> the whole column stays
        text and keeps its leading zeros; k <= 19: integer labels lose them)
  orgD  low-complexity 3 kbp genome (poly-A run, dinucleotide and CpG repeats), k = 1, 5, 12
Outputs: <org>_kmer_features.csv.gz (the feature CSVs), matrix_count.csv.gz and
matrix_gc_percent.csv.gz (KmerFeatureBuilder with metric "count" / "gc_percent").
"""
import contextlib
import gzip
import io
import os
import shutil
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, run_reference  # noqa: E402  (puts bio_shim + REF on sys.path)
from feature_inputs import CASES  # noqa: E402


def _gz_write(path, data):
    with open(path, "wb") as raw, gzip.GzipFile(fileobj=raw, mode="wb", mtime=0, filename="") as g:
        g.write(data)


def main():
    from kmerml.kmers.statistics import KmerFeatureExtractor
    from kmerml.ml.features import KmerFeatureBuilder
    from kmerml.utils.path_utils import find_files
    import kmerml
    assert os.path.realpath(kmerml.__file__).startswith(REF), kmerml.__file__

    tmp = tempfile.mkdtemp(prefix="kmh_feat_")
    try:
        kroot = os.path.join(tmp, "kmers")
        for org, make, ks in CASES:
            seq = make()
            fa = os.path.join(tmp, org + ".fa")
            with open(fa, "wb") as f:
                f.write(b">" + org.encode() + b" synthetic\n")
                for i in range(0, len(seq), 80):
                    f.write(seq[i:i + 80] + b"\n")
            run_reference(fa, ks, org, kroot)
        fdir = os.path.join(tmp, "features")
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            files = find_files(kroot, patterns=["k*.txt"], recursive=True)
            KmerFeatureExtractor(input_paths=files, output_dir=fdir).extract_features()
            mats = {m: KmerFeatureBuilder(fdir).build_from_statistics_files(metric=m)
                    for m in ("count", "gc_percent")}
        dst = os.path.join(HERE, "features2")
        shutil.rmtree(dst, ignore_errors=True)
        os.makedirs(dst)
        for name in sorted(os.listdir(fdir)):
            with open(os.path.join(fdir, name), "rb") as f:
                _gz_write(os.path.join(dst, name + ".gz"), f.read())
        for m, mat in mats.items():
            _gz_write(os.path.join(dst, f"matrix_{m}.csv.gz"), mat.to_csv().encode())
        print("features2:", sorted(os.listdir(dst)))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
