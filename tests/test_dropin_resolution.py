"""CPU: with kmer-ml_amd/activate on PYTHONPATH and the reference root as the working directory
(how the reference's README runs its scripts), the reference's own CLI modules import unchanged,
`kmerml.kmers.generate`, `.statistics` and `kmerml.ml.features` resolve to this package, and the
reference's other modules (utils, scripts) still resolve to the reference.  Skipped where
/root/reference is absent (GPU box)."""
import os
import subprocess
import sys

import pytest

from conftest import PKG, REFERENCE

pytestmark = pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout absent")

PROBE = r"""
import importlib, json, sys
import kmerml.kmers.generate as g
import kmerml.kmers.statistics as st
import kmerml.ml.features as ft
import scripts.extract_kmers as cli
out = {"generate": g.__file__, "statistics": st.__file__, "features": ft.__file__,
       "cli_extractor": cli.KmerExtractor.__module__, "cli_file": cli.__file__}
print(json.dumps(out))
"""


ACTIVATE = os.path.join(PKG, "activate")


def test_reference_cli_imports_this_package():
    env = dict(os.environ, PYTHONPATH=ACTIVATE, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", PROBE], env=env, capture_output=True, text=True,
                       cwd=REFERENCE, timeout=120)
    assert r.returncode == 0, r.stderr
    import json
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["generate"].startswith(PKG)
    assert d["statistics"].startswith(PKG)
    assert d["features"].startswith(PKG)
    assert d["cli_file"].startswith(REFERENCE)
    assert d["cli_extractor"] == "kmerml.kmers.generate"


def test_reference_cli_help_runs():
    env = dict(os.environ, PYTHONPATH=ACTIVATE, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-m", "scripts.extract_kmers", "--help"], env=env,
                       capture_output=True, text=True, cwd=REFERENCE, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "--k-values" in r.stdout


def test_reference_cli_counts_through_the_hip_library(tmp_path):
    """The unchanged CLI reaches libkmerhip: on a machine without a GPU it must fail loudly
    with the library's error (no CPU fallback); on a GPU box it would count."""
    import torch
    fa = os.path.join(os.path.dirname(__file__), "golden", "inputs", "e2_crlf.fa")
    env = dict(os.environ, PYTHONPATH=ACTIVATE, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-m", "scripts.extract_kmers", "-i", fa, "-o", str(tmp_path),
                        "-k", "3,8"], env=env, capture_output=True, text=True, cwd=REFERENCE,
                       timeout=300)
    if torch.cuda.is_available():
        assert r.returncode == 0, r.stderr
    else:
        assert r.returncode != 0
        assert "libkmerhip error" in r.stderr and "no HIP device" in r.stderr


def test_reference_feature_cli_through_the_vectorised_extractor(tmp_path):
    """scripts/generate_kmers_features.py, unchanged, on the k-mer files of the features/
    fixture: the CSVs it writes equal the reference's own (entropy within 4 ulp)."""
    import json
    from test_features import GOLDEN, _assert_csv_equal, _read
    cases = json.load(open(os.path.join(GOLDEN, "edge_cases.json")))["cases"]
    kroot = tmp_path / "kmers"
    for org, name, ks in (("orgA", "e1_mixed.fa", [2, 7, 4]), ("orgB", "e6_lowcomplex.fa", [1, 4, 12])):
        case = next(c for c in cases if c["input"] == name and c["k_values"] == ks)
        os.makedirs(kroot / org)
        for fname, text in case["files"].items():
            (kroot / org / fname).write_text(text)
    out = tmp_path / "features"
    env = dict(os.environ, PYTHONPATH=ACTIVATE, PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-m", "scripts.generate_kmers_features", "-i", str(kroot),
                        "-o", str(out), "-m", ""], env=env, capture_output=True, text=True,
                       cwd=REFERENCE, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Generated 2 feature files" in r.stdout
    for org in ("orgA", "orgB"):
        _assert_csv_equal(_read(str(out / f"{org}_kmer_features.csv")),
                          _read(os.path.join(GOLDEN, "features", f"{org}_kmer_features.csv")))
