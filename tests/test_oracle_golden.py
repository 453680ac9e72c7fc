"""CPU: pin the oracle (Python + C restatements) to the reference's own outputs.

The fixtures in tests/golden/ were produced by running the reference's generate.py
(tests/golden/make_golden.py).  If the oracle reproduces them exactly, it can be trusted
as the checker for the HIP path on inputs the fixtures do not cover.
"""
import hashlib
import os

import numpy as np
import pytest

from oracle import fasta as ofasta
from oracle import kmers as okmers
from oracle import synth as osynth


def _inputs(golden_dir, name):
    return os.path.join(golden_dir, "inputs", name)


def test_python_oracle_reproduces_edge_cases(golden_dir, edge_cases):
    for case in edge_cases:
        recs = [(rid, seq) for rid, _, seq in ofasta.parse_fasta(_inputs(golden_dir, case["input"]))]
        msgs = []
        if "error" in case:   # a non-integer k: the reference raised from range() (generate.py:51)
            with pytest.raises(Exception) as e:
                okmers.count_records(recs, case["k_values"], msgs)
            assert (type(e.value).__name__, str(e.value)) == (case["error"]["type"], case["error"]["message"])
            assert msgs == case["stdout"] and case["files"] == {}
            continue
        if recs:
            res = okmers.count_records(recs, case["k_values"], msgs)
        else:
            res = {k: {} for k in case["k_values"]}
        assert msgs == case["stdout"], case["input"]
        files = {f"k{k}.txt": okmers.kmer_text(v) for k, v in res.items()}
        assert files == case["files"], (case["input"], case["k_values"])


def _plain_k(ks):
    """k lists the C restatement covers: integers 1 <= k <= 32 (no bool, no k <= 0)."""
    return all(type(k) is int and 1 <= k <= 32 for k in ks)


def _text_from_sparse(k, codes, counts, first, mult=1):
    order = np.argsort(first, kind="stable")
    return "".join(
        "".join("0231"[(int(c) >> (2 * (k - 1 - i))) & 3] for i in range(k)) + f"\t{int(n) * mult}\n"
        for c, n in zip(codes[order], counts[order]))


def _pack(golden_dir, name, longest):
    # generate.py:41,44: upper() first (non-ASCII characters can expand), then the length rule;
    # non-ASCII characters left after upper() are non-bases ('?')
    recs = ofasta.parse_fasta(_inputs(golden_dir, name))
    kept = [s.upper() for _, _, s in recs if len(s.upper()) >= longest]
    return "".join(s + "\n" for s in kept).encode("ascii", errors="replace")


def test_c_oracle_reproduces_edge_cases(golden_dir, edge_cases, oracle_lib):
    for case in edge_cases:
        ks = case["k_values"]
        if not _plain_k(ks):
            continue  # the C restatement covers 1 <= k <= 32 (k > 32, k <= 0: Python oracle above)
        packed = _pack(golden_dir, case["input"], max(ks))
        for k in dict.fromkeys(ks):
            codes, counts, first = oracle_lib.count_sparse(packed, k)
            text = _text_from_sparse(k, codes, counts, first, ks.count(k))
            assert text == case["files"][f"k{k}.txt"], (case["input"], k)
            if k <= 12:
                dense, dfirst = oracle_lib.count_dense(packed, k, with_first=True)
                nz = np.nonzero(dense)[0]
                assert np.array_equal(nz.astype(np.uint64), codes)
                assert np.array_equal(dense[nz], counts)
                assert np.array_equal(dfirst[nz].astype(np.uint64), first)


def test_c_oracle_reproduces_synthetic_hashes(synthetic_cases, oracle_lib):
    for case in synthetic_cases:
        if "genomes" not in case:
            continue
        (g,) = case["genomes"]
        seq = osynth.synth_bases(g["length"], g["seed"], g["start"]).tobytes()
        (k,) = case["k_values"]
        codes, counts, first = oracle_lib.count_sparse(seq + b"\n", k)
        text = _text_from_sparse(k, codes, counts, first)
        assert hashlib.sha256(text.encode()).hexdigest() == case["sha256"][f"k{k}.txt"], case["name"]


def test_yeast_standin_text(synthetic_cases, oracle_lib):
    case = next(c for c in synthetic_cases if c["name"] == "yeast_standin")
    recs = osynth.yeast_standin_records()
    assert [r[0] for r in recs] == case["records"]
    packed = b"".join(s + b"\n" for _, s in recs)
    codes, counts, first = oracle_lib.count_sparse(packed, 4)
    assert _text_from_sparse(4, codes, counts, first) == case["text"]["k4.txt"]
    assert case["stdout"] == [f"Processed chromosome/contig: {r[0]}" for r in recs]


def test_synth_python_matches_c(oracle_lib):
    for g, start, n in ((0, 0, 1000), (5, 31, 4097), (63, 99_999_900, 100)):
        seed = osynth.genome_seed(g)
        assert np.array_equal(osynth.synth_bases(n, seed, start), oracle_lib.synth(n, seed, start))


def test_canonical_oracle_is_strand_symmetric(oracle_lib):
    rng = np.random.default_rng(7)
    seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 5000)].tobytes()
    comp = bytes.maketrans(b"ACGT", b"TGCA")
    rc = seq.translate(comp)[::-1]
    for k in (5, 13, 21, 32):
        a = oracle_lib.count_sparse(seq, k, canonical=True)
        b = oracle_lib.count_sparse(rc, k, canonical=True)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("k", [1, 3, 8])
def test_dense_matches_dict_loop(k, oracle_lib):
    rng = np.random.default_rng(k)
    seq = np.frombuffer(b"ACGTNacgt", np.uint8)[rng.integers(0, 9, 20000)].tobytes()
    ref = okmers.count_sequence(seq.decode(), k)
    dense = oracle_lib.count_dense(seq, k)
    got = {okmers.code_kmer(int(c), k): int(dense[c]) for c in np.nonzero(dense)[0]}
    assert got == dict(ref)
