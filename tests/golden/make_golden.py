"""Regenerate the golden fixtures in tests/golden/ by running the REFERENCE's own code.

Needs /root/reference (present only in the build container, never on the GPU box).
Run from the repo root:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference's generate.py imports ``from Bio import SeqIO`` (generate.py:4) and
biopython 1.85 is absent, so tests/golden/bio_shim (a restatement of Biopython's FASTA
parser, oracle/fasta.py) is put first on sys.path.  Everything else -- the window loop,
ACGT filter, counting, short-record rule, duplicate-k behaviour, A0/T1/C2/G3 text and
first-occurrence line order -- is the reference's own code running unchanged
(generate.py:21-91, statistics.py, features.py).

Outputs (all committed):
  edge_cases.json      exact k{k}.txt text + stdout for every (input, k-list) case
  synthetic.json       SHA-256 of k{k}.txt for seeded synthetic genomes (inputs are
                       regenerated in tests from oracle/synth.py)
  features/            L3: the reference's feature CSVs and matrix for one edge case
"""
import contextlib
import hashlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [os.path.join(HERE, "bio_shim"), REF, REPO]

from kmerml.kmers.generate import KmerExtractor  # noqa: E402  (the reference's module)
import kmerml  # noqa: E402

assert os.path.realpath(kmerml.__file__).startswith(REF), kmerml.__file__

from oracle.synth import genome_seed, synth_bases, write_fasta, yeast_standin_records  # noqa: E402

EDGE_CASES = [
    ("e1_mixed.fa", [1, 2, 3]),
    ("e1_mixed.fa", [4]),
    ("e1_mixed.fa", [5, 5]),
    ("e1_mixed.fa", [2, 7, 4]),
    ("e1_mixed.fa", [12]),
    ("e1_mixed.fa", [21]),
    ("e1_mixed.fa", [40]),
    ("e2_crlf.fa", [3, 8]),
    ("e2_crlf.fa", [33]),
    ("e3_empty.fa", [4]),
    ("e4_short.fa", [3, 8]),
    ("e4_short.fa", [2]),
    ("e5_lonecr.fa", [6]),
    ("e6_lowcomplex.fa", [1, 4, 12]),
    ("e6_lowcomplex.fa", [16, 2, 2]),
    ("e7_headers.fa", [5]),
    # str.upper() of non-ASCII characters (generate.py:41): ß -> SS (the record grows, which
    # moves the short-record rule of :44), U+FB05 / U+FB06 -> ST, U+1E97 -> T + U+0308,
    # U+1E9A -> A + U+02BE: the only code points whose upper() contains A, C, G or T
    ("e8_unicode.fa", [4]),
    ("e8_unicode.fa", [6]),
    ("e8_unicode.fa", [2, 3]),
    # k <= 0, bool and non-integer k (scripts/extract_kmers.py:34 accepts any int): the window
    # loop of generate.py:51-58 still runs -- k = 0 counts the empty k-mer len + 1 times per
    # record, a negative k counts the slices seq[i:i + k] -- and _save_kmers_to_file writes
    # "\t{count}" for the empty k-mer (:90-91); True / False are k = 1 / 0 under the dict key
    # True / False (file kTrue.txt); a float k raises TypeError from range() at the first kept
    # record (after the "Skipping" lines before it) and writes nothing, but an empty file
    # writes an empty k2.5.txt
    ("e1_mixed.fa", [0]),
    ("e1_mixed.fa", [0, 3]),
    ("e1_mixed.fa", [-1]),
    ("e1_mixed.fa", [True]),
    ("e1_mixed.fa", [1, True]),
    ("e4_short.fa", [True, 2, False]),
    ("e4_short.fa", [-2, 2]),
    ("e4_short.fa", [-7]),
    ("e6_lowcomplex.fa", [-3, 0, -3]),
    ("e7_headers.fa", [0, 5]),
    ("e8_unicode.fa", [-2]),
    ("e3_empty.fa", [0, -1]),
    ("e4_short.fa", [6, 2.5]),
    ("e3_empty.fa", [2.5]),
]


def run_reference(fasta, k_values, organism_id, outdir, compress=False, errors=None):
    buf = io.StringIO()
    ret = None
    with contextlib.redirect_stdout(buf):
        ext = KmerExtractor(output_dir=outdir, compress=compress)
        try:
            ret = ext.extract_kmers_from_fasta(fasta, k_values, organism_id=organism_id)
        except Exception as e:   # recorded for the error cases, re-raised for every other call
            if errors is None:
                raise
            errors.append({"type": type(e).__name__, "message": str(e)})
    files = {}
    odir = os.path.join(outdir, organism_id)
    if os.path.isdir(odir):
        for name in sorted(os.listdir(odir)):
            with open(os.path.join(odir, name), "r") as f:
                files[name] = f.read()
    return ret, buf.getvalue().splitlines(), files


def sha(text):
    return hashlib.sha256(text.encode()).hexdigest()


def main():
    out = {"generator": "tests/golden/make_golden.py", "reference": REF, "cases": []}
    tmp = tempfile.mkdtemp(prefix="kmh_golden_")
    try:
        for name, ks in EDGE_CASES:
            odir = os.path.join(tmp, f"edge_{len(out['cases'])}")
            errors = []
            ret, lines, files = run_reference(os.path.join(HERE, "inputs", name), ks,
                                              "org", odir, errors=errors)
            case = {"input": name, "k_values": ks, "returned": ret, "stdout": lines, "files": files}
            if errors:
                case["error"] = errors[0]
            out["cases"].append(case)
            print(name, ks, {k: len(v) for k, v in files.items()})
        with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        if "--edge-only" in sys.argv:
            return

        syn = {"generator": "tests/golden/make_golden.py", "fasta_width": 80, "cases": []}
        # (a) 1 Mbp single-record genome, several k
        g = 1000
        seq = synth_bases(1_000_000, genome_seed(g)).tobytes()
        fa = os.path.join(tmp, "syn1m.fa")
        write_fasta(fa, [(f"SYN_{g:04d}", seq)])
        for k in (4, 8, 12, 21):
            t0 = time.time()
            ret, lines, files = run_reference(fa, [k], "syn1m", os.path.join(tmp, f"s1m_{k}"))
            text = files[f"k{k}.txt"]
            syn["cases"].append({"name": "syn1m", "genomes": [{"id": f"SYN_{g:04d}", "seed": genome_seed(g), "start": 0, "length": 1_000_000}],
                                 "k_values": [k], "stdout": lines,
                                 "sha256": {f"k{k}.txt": sha(text)},
                                 "lines": {f"k{k}.txt": text.count("\n")},
                                 "sorted_sha256": {f"k{k}.txt": sha("".join(sorted(text.splitlines(True))))}})
            print("syn1m", k, round(time.time() - t0, 1), "s")
        # (b) config-1 stand-in: 17 records with yeast chromosome lengths, k=4
        recs = yeast_standin_records()
        fa = os.path.join(tmp, "yeast_standin.fa")
        write_fasta(fa, recs)
        t0 = time.time()
        ret, lines, files = run_reference(fa, [4], "yeast_standin", os.path.join(tmp, "ys"))
        text = files["k4.txt"]
        syn["cases"].append({"name": "yeast_standin", "records": [r[0] for r in recs],
                             "k_values": [4], "stdout": lines,
                             "sha256": {"k4.txt": sha(text)}, "text": {"k4.txt": text}})
        print("yeast standin", round(time.time() - t0, 1), "s")
        # (c) config-2 shaped: two 10 Mbp synthetic genomes, k=8 (exact text hashes)
        for g in (0, 1):
            seq = synth_bases(10_000_000, genome_seed(g)).tobytes()
            fa = os.path.join(tmp, f"SYN_{g:04d}.fa")
            write_fasta(fa, [(f"SYN_{g:04d}", seq)])
            t0 = time.time()
            ret, lines, files = run_reference(fa, [8], f"SYN_{g:04d}", os.path.join(tmp, "c2"))
            text = files["k8.txt"]
            syn["cases"].append({"name": f"c2_SYN_{g:04d}", "genomes": [{"id": f"SYN_{g:04d}", "seed": genome_seed(g), "start": 0, "length": 10_000_000}],
                                 "k_values": [8], "stdout": lines,
                                 "sha256": {"k8.txt": sha(text)},
                                 "lines": {"k8.txt": text.count("\n")}})
            print("c2", g, round(time.time() - t0, 1), "s")
        with open(os.path.join(HERE, "synthetic.json"), "w") as f:
            json.dump(syn, f, indent=1, sort_keys=True)

        make_features(tmp)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def make_features(tmp):
    """L3 fixtures: the reference's per-organism feature CSV and its count matrix."""
    from kmerml.kmers.statistics import KmerFeatureExtractor
    from kmerml.ml.features import KmerFeatureBuilder
    from kmerml.utils.path_utils import find_files
    kroot = os.path.join(tmp, "l3_kmers")
    for org, name, ks in (("orgA", "e1_mixed.fa", [2, 7, 4]), ("orgB", "e6_lowcomplex.fa", [1, 4, 12])):
        run_reference(os.path.join(HERE, "inputs", name), ks, org, kroot)
    fdir = os.path.join(tmp, "l3_features")
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        files = find_files(kroot, patterns=["k*.txt"], recursive=True)
        KmerFeatureExtractor(input_paths=files, output_dir=fdir).extract_features()
        mat = KmerFeatureBuilder(fdir).build_from_statistics_files()
    dst = os.path.join(HERE, "features")
    os.makedirs(dst, exist_ok=True)
    for name in sorted(os.listdir(fdir)):
        shutil.copy(os.path.join(fdir, name), os.path.join(dst, name))
    mat.to_csv(os.path.join(dst, "matrix_count.csv"))
    with open(os.path.join(dst, "README.txt"), "w") as f:
        f.write("Generated by tests/golden/make_golden.py:make_features from the reference's\n"
                "KmerFeatureExtractor (statistics.py) and KmerFeatureBuilder (features.py) on\n"
                "k-mer files of inputs/e1_mixed.fa (k=2,7,4 as orgA) and inputs/e6_lowcomplex.fa\n"
                "(k=1,4,12 as orgB).\n")
    print("features:", sorted(os.listdir(dst)))


if __name__ == "__main__":
    main()
