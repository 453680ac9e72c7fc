"""CPU: the drop-in KmerExtractor on the golden cases that need no device -- every k <= 0
(bool False included) and the non-integer k that make the reference raise -- byte-identical
to the files, stdout lines and exceptions the reference produced (tests/golden/make_golden.py;
reference anchor /root/reference/kmerml/kmers/generate.py:36-58, 86-91).  The cases with a
k >= 1 run through the GPU in tests/test_gpu_parity.py::test_dropin_edge_cases_byte_identical."""
import operator
import os

from _dropin import run_extractor


def _host_only(ks):
    try:
        return all(operator.index(k) <= 0 for k in ks)
    except TypeError:
        return True


def test_degenerate_k_cases_byte_identical(tmp_path, golden_dir, edge_cases):
    cases = [c for c in edge_cases if _host_only(c["k_values"]) or "error" in c]
    assert len(cases) >= 7
    for i, case in enumerate(cases):
        ret, out, files = run_extractor(tmp_path / f"c{i}", os.path.join(golden_dir, "inputs", case["input"]),
                                        case["k_values"], expect_error=case.get("error"))
        assert ret == case["returned"]
        assert out == case["stdout"], (case["input"], case["k_values"])
        assert files == case["files"], (case["input"], case["k_values"])
