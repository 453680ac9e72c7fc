"""CPU: row f4 -- the vectorised KmerFeatureExtractor / KmerFeatureBuilder against the
reference's own outputs (tests/golden/features*/, made by tests/golden/make_golden.py and
make_features.py from the reference's statistics.py / features.py).

k-mer files are rebuilt with the oracle (oracle/kmers.py restates generate.py and is pinned
to the reference's k{k}.txt goldens).  Feature CSVs and matrices must match byte for byte,
except the two entropy columns: the reference sums them in set() order, which depends on
the interpreter's string-hash seed, so across processes they may differ in the last bits
(up to 4 ulp allowed here, 2 observed).  Within one process they are checked bit-exact against a scalar
restatement of statistics.py:214-224.
"""
import contextlib
import gzip
import io
import json
import math
import os

import numpy as np
import pandas as pd
import pytest

from kmerml.kmers.statistics import KmerFeatureExtractor, label_features
from kmerml.ml.features import KmerFeatureBuilder
from kmerml.utils.path_utils import find_files
from oracle import kmers as okmers

from conftest import REPO

GOLDEN = os.path.join(REPO, "tests", "golden")
ENTROPY = ("shannon_entropy", "normalized_entropy")


def _write_kfiles(root, org, seq, ks):
    tables = okmers.count_records([(org, seq)], ks)
    os.makedirs(os.path.join(root, org), exist_ok=True)
    for k, t in tables.items():
        with open(os.path.join(root, org, f"k{k}.txt"), "w") as f:
            f.write(okmers.kmer_text(t))


def _run_extractor(kroot, fdir):
    with contextlib.redirect_stdout(io.StringIO()):
        files = find_files(kroot, patterns=["k*.txt"], recursive=True)
        return KmerFeatureExtractor(input_paths=files, output_dir=fdir).extract_features()


def _assert_csv_equal(got_text, want_text):
    g = pd.read_csv(io.StringIO(got_text), dtype=str, keep_default_na=False)
    w = pd.read_csv(io.StringIO(want_text), dtype=str, keep_default_na=False)
    assert list(g.columns) == list(w.columns)
    assert len(g) == len(w)
    for c in g.columns:
        if c in ENTROPY:
            a, b = g[c].astype(float).to_numpy(), w[c].astype(float).to_numpy()
            # a different summation order of <= 5 terms: at most a few ulp (4 allowed)
            assert np.all(np.abs(a - b) <= 4 * np.spacing(np.maximum(np.abs(a), np.abs(b)))), c
        else:
            assert (g[c] == w[c]).all(), c


def _read(path):
    if path.endswith(".gz"):
        with gzip.open(path, "rt") as f:
            return f.read()
    with open(path) as f:
        return f.read()


def test_features_edge_fixtures(tmp_path):
    """features/: e1_mixed.fa k=2,7,4 as orgA and e6_lowcomplex.fa k=1,4,12 as orgB."""
    cases = json.load(open(os.path.join(GOLDEN, "edge_cases.json")))["cases"]
    kroot = tmp_path / "kmers"
    for org, name, ks in (("orgA", "e1_mixed.fa", [2, 7, 4]), ("orgB", "e6_lowcomplex.fa", [1, 4, 12])):
        case = next(c for c in cases if c["input"] == name and c["k_values"] == ks)
        os.makedirs(kroot / org)
        for fname, text in case["files"].items():
            (kroot / org / fname).write_text(text)
    fdir = tmp_path / "features"
    out = _run_extractor(str(kroot), str(fdir))
    assert sorted(out) == ["orgA", "orgB"]
    for org in ("orgA", "orgB"):
        _assert_csv_equal(_read(str(fdir / f"{org}_kmer_features.csv")),
                          _read(os.path.join(GOLDEN, "features", f"{org}_kmer_features.csv")))
    with contextlib.redirect_stdout(io.StringIO()):
        mat = KmerFeatureBuilder(str(fdir)).build_from_statistics_files()
    assert mat.to_csv() == _read(os.path.join(GOLDEN, "features", "matrix_count.csv"))


@pytest.fixture(scope="module")
def features2(tmp_path_factory):
    import sys
    sys.path.insert(0, GOLDEN)
    from feature_inputs import CASES
    root = tmp_path_factory.mktemp("f2")
    for org, make, ks in CASES:
        _write_kfiles(str(root / "kmers"), org, make().decode(), ks)
    fdir = root / "features"
    _run_extractor(str(root / "kmers"), str(fdir))
    return fdir


@pytest.mark.parametrize("org", ["orgC", "orgD"])
def test_features_k12_k20_k21(features2, org):
    """Integer labels lose their leading A's (k <= 19); k = 20/21 text labels keep them."""
    _assert_csv_equal(_read(str(features2 / f"{org}_kmer_features.csv")),
                      _read(os.path.join(GOLDEN, "features2", f"{org}_kmer_features.csv.gz")))


@pytest.mark.parametrize("metric", ["count", "gc_percent"])
def test_matrix_last_k_wins(features2, metric):
    with contextlib.redirect_stdout(io.StringIO()):
        mat = KmerFeatureBuilder(str(features2)).build_from_statistics_files(metric=metric)
    want = _read(os.path.join(GOLDEN, "features2", f"matrix_{metric}.csv.gz"))
    assert mat.to_csv() == want


def _scalar_entropy(kmer):
    """statistics.py:214-224 restated (set() order of this interpreter)."""
    base_counts = {base: kmer.count(base) for base in set(kmer)}
    entropy = 0
    for base, count in base_counts.items():
        prob = count / len(kmer)
        entropy -= prob * math.log2(prob) if prob > 0 else 0
    return entropy


def test_entropy_bit_exact_in_process():
    rng = np.random.default_rng(3)
    labels = ["".join("ACGT"[x] for x in rng.integers(0, 4, rng.integers(1, 22))) for _ in range(3000)]
    labels += ["A", "AC", "CA", "ACGT", "TGCA", "GGGG", "N", "ANA", "CGNT", "NNNN"]
    got = label_features(labels)["shannon_entropy"]
    want = np.array([_scalar_entropy(s) for s in labels])
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_label_features_scalar_restatement():
    rng = np.random.default_rng(4)
    labels = ["".join("ACGTN"[x] for x in rng.integers(0, 5, rng.integers(1, 14))) for _ in range(2000)]
    f = label_features(labels)
    for i, s in enumerate(labels):
        c, g = s.count("C"), s.count("G")
        assert f["gc_percent"][i] == (g + c) / len(s) * 100
        cpg = sum(1 for j in range(len(s) - 1) if s[j:j + 2] == "CG")
        assert f["cpg_count"][i] == cpg
        cf, gf = c / len(s), g / len(s)
        exp = cf * gf * (len(s) - 1) if cf * gf > 0 else 0.001
        assert f["cpg_obs_exp"][i] == cpg / exp
        rep = any(s[j:j + 2] == s[j + 2:j + 4] for j in range(len(s) - 3))
        assert f["has_repeat"][i] == int(rep)
        for b in "ACGT":
            assert f[f"{b}_count"][i] == s.count(b)


def test_compat_labels_match_file_round_trip():
    """from_count_matrix labels = the reference's label after writing + integer parsing."""
    k = 6
    labels = KmerFeatureBuilder.compat_labels(k)
    dec = KmerFeatureExtractor.decode_labels
    for code in (0, 1, 2, 3, 4, 100, 2047, 4095):
        digits = "".join(okmers.DIGIT[b] for b in okmers.code_kmer(code, k))
        assert labels[code] == dec(pd.Series([int(digits)]))[0]


def test_from_count_matrix_equals_file_path(tmp_path):
    from oracle import synth as osynth
    k, orgs = 5, ["GCF_000001_x", "GCF_000002_y"]
    kroot = tmp_path / "kmers"
    rows = []
    for i, org in enumerate(orgs):
        seq = osynth.synth_bases(3000 + 500 * i, osynth.genome_seed(i)).tobytes().decode()
        _write_kfiles(str(kroot), org, seq, [k])
        t = okmers.count_sequence(seq, k)
        row = np.zeros(1 << (2 * k), np.uint32)
        for kmer, n in t.items():
            row[okmers.kmer_code(kmer)] = n
        rows.append(row)
    fdir = tmp_path / "features"
    _run_extractor(str(kroot), str(fdir))
    with contextlib.redirect_stdout(io.StringIO()):
        want = KmerFeatureBuilder(str(fdir)).build_from_statistics_files()
    got = KmerFeatureBuilder().from_count_matrix(np.stack(rows), k, list(want.index))
    assert got.to_csv() == want.to_csv()


def test_fast_csv_equals_pandas(features2):
    """The direct CSV writer produces pandas' to_csv(index=False) text exactly."""
    from kmerml.kmers.statistics import csv_text
    for org in ("orgC", "orgD"):
        df = pd.read_csv(features2 / f"{org}_kmer_features.csv", keep_default_na=False)
        assert csv_text(df) == df.to_csv(index=False)
    rng = np.random.default_rng(9)
    odd = pd.DataFrame({"kmer": ["A", "CG", "T"], "count": [1, 2, 3],
                        "x": [1e-05, 123456789012345.0, 0.1 + 0.2], "y": [1e16, 5e-324, -0.0],
                        "z": rng.random(3) * 10.0 ** rng.integers(-20, 20, 3)})
    assert csv_text(odd) == odd.to_csv(index=False)
    assert csv_text(pd.DataFrame({"kmer": ["a,b"], "count": [1]})) is None   # quoting: pandas path
    assert csv_text(pd.DataFrame({"x": [float("nan")]})) is None


def test_feature_table_matches_label_features():
    """The per-k feature table (statistics.feature_table, computed once per k on the GPU when
    there is one) holds, bit for bit, the features label_features computes for each code's
    compat label -- the function pinned to the reference's CSVs above."""
    from kmerml.kmers.statistics import feature_table, label_features
    for k in range(1, 8):
        t = feature_table(k)
        f = label_features(list(KmerFeatureBuilder.compat_labels(k)))
        for name, want in f.items():
            want = np.asarray(want)
            got = t[name]
            if want.dtype.kind == 'f':
                assert np.array_equal(got.view(np.int64), want.view(np.int64)), (k, name)
            else:
                assert np.array_equal(got, want), (k, name)


def test_feature_frame_table_path_equals_label_path(monkeypatch):
    """feature_frame takes table rows for integer-parsed k-mer labels and the per-label path
    for anything else (a digit outside 0-3, more digits than k); both give the same frame."""
    import kmerml.kmers.statistics as st
    rng = np.random.default_rng(5)
    k = 7
    codes = rng.choice(4 ** k, 3000, replace=False)
    codes[:3] = [0, 1, 4 ** k - 1]
    dig = np.array([0, 2, 3, 1])
    lab = np.zeros(codes.size, np.int64)
    for i in range(k):
        lab = lab * 10 + dig[(codes >> (2 * (k - 1 - i))) & 3]
    df = pd.DataFrame({'kmer': lab, 'count': rng.integers(1, 50, codes.size)})
    assert np.array_equal(st.label_codes(df['kmer'].to_numpy(), k), codes)
    fast = st.KmerFeatureExtractor.feature_frame(df, k, st.DEFAULT_FEATURES)
    monkeypatch.setattr(st, "label_codes", lambda v, kk: None)
    slow = st.KmerFeatureExtractor.feature_frame(df, k, st.DEFAULT_FEATURES)
    assert fast.to_csv() == slow.to_csv()
    monkeypatch.undo()
    assert st.label_codes(np.array([104], np.int64), 3) is None          # digit 4
    assert st.label_codes(np.array([1233], np.int64), 3) is None         # 4 digits at k = 3
    assert st.label_codes(np.array(["12"], dtype=object), 2) is None     # text labels


@pytest.mark.parametrize("k", [15, 16, 19])
def test_feature_frame_sparse_large_k(monkeypatch, k):
    """Integer labels of a sparse k = 15..19 file: features of the distinct codes
    only -- never a 4^k table -- equal to the per-label path, bit for bit."""
    import kmerml.kmers.statistics as st
    rng = np.random.default_rng(k)
    codes = rng.integers(0, 4 ** k, 4000, dtype=np.int64)
    codes[:4] = [0, 1, 4 ** k - 1, codes[5]]           # A...A, leading A's, a repeat
    dig = np.array([0, 2, 3, 1])
    lab = np.zeros(codes.size, np.int64)
    for i in range(k):
        lab = lab * 10 + dig[(codes >> (2 * (k - 1 - i))) & 3]
    df = pd.DataFrame({'kmer': lab, 'count': rng.integers(1, 50, codes.size)})
    monkeypatch.setattr(st, "feature_table", lambda kk: pytest.fail("4^k table built"))
    fast = st.KmerFeatureExtractor.feature_frame(df, k, st.DEFAULT_FEATURES)
    monkeypatch.setattr(st, "label_codes", lambda v, kk: None)
    slow = st.KmerFeatureExtractor.feature_frame(df, k, st.DEFAULT_FEATURES)
    assert fast.to_csv() == slow.to_csv()


def test_native_csv_equals_pandas(features2):
    """kmh_csv_format (the native writer of the feature CSV rows) prints exactly the text of
    pandas' to_csv(index=False): the reference-fixture frames, floats over every exponent, labels
    printed from k-mer codes; NaN / inf and text that needs quotes are refused (pandas path)."""
    from kmerml import _native
    from kmerml.kmers.statistics import FeatureBlock, _native_columns

    def native_text(df, codes=None, k=None):
        cols = {c: df[c].to_numpy() for c in df.columns}
        b = FeatureBlock(cols, len(df), df["kmer"] if "kmer" in df else None, codes, k)
        nc = _native_columns(b)
        t = _native.csv_format(nc, len(df)) if nc is not None else None
        return None if t is None else ",".join(df.columns) + "\n" + t.tobytes().decode()

    for org in ("orgC", "orgD"):
        df = pd.read_csv(features2 / f"{org}_kmer_features.csv", keep_default_na=False)
        assert native_text(df) == df.to_csv(index=False)
    rng = np.random.default_rng(21)
    bits = rng.integers(0, 2**63, 200_000, dtype=np.uint64) | (rng.integers(0, 2, 200_000, dtype=np.uint64) << np.uint64(63))
    x = bits.view(np.float64)
    x = x[np.isfinite(x)]
    extra = np.array([0.0, -0.0, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 0.1 + 0.2, 5e-324, 50.0,
                      1.7976931348623157e308, 123456789012345678.0, 2 / 3, 100.0, 1e22, 1e-300])
    x = np.concatenate([x, extra, rng.random(5000) * 100])
    df = pd.DataFrame({"kmer": ["ACGT"] * x.size, "count": rng.integers(-5, 2**62, x.size), "x": x})
    assert native_text(df) == df.to_csv(index=False)
    # labels from codes = the integer-parsed labels decoded (k = 1, 12, 19; A...A, leading A's)
    for k in (1, 12, 19):
        codes = rng.integers(0, 4 ** k, 3000, dtype=np.int64)
        codes[:2] = [0, 4 ** k - 1]
        dig = np.array([0, 2, 3, 1])
        lab = np.zeros(codes.size, np.int64)
        for i in range(k):
            lab = lab * 10 + dig[(codes >> (2 * (k - 1 - i))) & 3]
        raw = pd.DataFrame({"kmer": lab, "count": np.ones(codes.size, np.int64)})
        want = pd.DataFrame({"kmer": KmerFeatureExtractor.decode_labels(raw["kmer"]), "count": raw["count"]})
        assert native_text(raw, codes=codes, k=k) == want.to_csv(index=False)
    assert native_text(pd.DataFrame({"kmer": ["A"], "x": [float("nan")]})) is None
    assert native_text(pd.DataFrame({"kmer": ["A"], "x": [float("inf")]})) is None
    assert native_text(pd.DataFrame({"kmer": ["a,b"], "count": [1]})) is None
    assert native_text(pd.DataFrame({"kmer": [""], "count": [1]})) is None
