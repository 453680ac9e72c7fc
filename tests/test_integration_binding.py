"""The reference-side ctypes binding printed in INTEGRATION.md ("The C ABI"), executed as
written against the built libkmerhip.so: the block a maintainer would paste into the reference
in place of generate.py:36-58 (count) and generate.py:86-91 (the k{k}.txt text)."""
import os
import re

import numpy as np
import pytest

from conftest import REPO

LIB = os.path.join(REPO, "kmer-ml_amd", "kmerml", "_lib", "libkmerhip.so")


def _binding_source():
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = text[text.index("## The C ABI"):]
    block = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    assert 'ctypes.CDLL("libkmerhip.so")' in block
    return block.replace('ctypes.CDLL("libkmerhip.so")', f"ctypes.CDLL({LIB!r})")


def _split(src):
    """(lines up to and including the context creation, the rest)."""
    head, sep, tail = src.partition("check(lib.kmh_ctx_create(0, ctypes.byref(ctx)))")
    assert sep, "INTEGRATION.md binding no longer creates its context with check(...)"
    line_end = tail.index("\n")
    return head + sep + tail[:line_end + 1], tail[line_end + 1:]


def _text_vs_oracle(ns, seq, k):
    from oracle import kmers as okmers
    table = okmers.count_sequence(seq.decode(), k)
    codes = np.array([okmers.kmer_code(m) for m in table], np.uint64)
    counts = np.array(list(table.values()), np.uint64)
    return ns["kmer_file_text"](k, codes, counts).decode(), okmers.kmer_text(table)


def test_binding_error_path_carries_library_message():
    """Without a GPU (this container) kmh_ctx_create fails: the binding must raise a
    RuntimeError whose text is the library's message (the restype of kmh_last_error set to
    c_char_p; before round 5 the snippet raised with the pointer value as an int)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present: the error path is covered by test_binding_counts_gpu")
    head, _ = _split(_binding_source())
    ns = {}
    with pytest.raises(RuntimeError) as ei:
        exec(compile(head, "INTEGRATION.md", "exec"), ns)
    msg = str(ei.value)
    assert msg.startswith("no HIP device available"), msg
    assert not msg.isdigit()


def test_binding_writer_without_device(oracle_lib):
    """The writer half of the binding (kmh_format_lines: argtypes / restype as printed) needs
    no device: its text equals the restated generate.py:86-91 writer."""
    head, tail = _split(_binding_source())
    ns = {}
    try:
        exec(compile(head, "INTEGRATION.md", "exec"), ns)
    except RuntimeError:
        pass   # no GPU: the defs below do not need the context
    exec(compile(tail, "INTEGRATION.md", "exec"), ns)
    from oracle import synth as osynth
    seq = osynth.synth_bases(5000, osynth.genome_seed(3)).tobytes()
    for k in (1, 7, 12, 21, 32):
        got, want = _text_vs_oracle(ns, seq, k)
        assert got == want


@pytest.mark.gpu
def test_binding_counts_gpu(oracle_lib):
    """The whole block on a HIP device: count() returns the reference dict's keys and counts in
    first-occurrence order, and kmer_file_text() its k{k}.txt text."""
    from oracle import kmers as okmers
    from oracle import synth as osynth
    ns = {}
    exec(compile(_binding_source(), "INTEGRATION.md", "exec"), ns)
    seq = osynth.synth_bases(20000, osynth.genome_seed(5)).tobytes()
    seq = seq[:9000] + b"NNNN" + seq[9000:15000].lower() + b"\n" + seq[15000:]
    for k in (4, 12, 21):
        codes, counts = ns["count"](seq, k)
        table = okmers.count_sequence(seq.decode().replace("\n", "N"), k)
        assert codes.tolist() == [okmers.kmer_code(m) for m in table]
        assert counts.tolist() == list(table.values())
        assert ns["kmer_file_text"](k, codes, counts).decode() == okmers.kmer_text(table)
    with pytest.raises(RuntimeError) as ei:   # the library's message on a context error
        ns["count"](seq, 0)
    assert not str(ei.value).isdigit() and str(ei.value)
