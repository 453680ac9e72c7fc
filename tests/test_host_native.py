"""CPU: the C-ABI library loads, exports every declared symbol, and its host-side pieces
(FASTA ingest, text formatter, error reporting) match the oracle.  No GPU needed."""
import contextlib
import os
import re

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from kmerml import _native
from oracle import fasta as ofasta
from oracle import kmers as okmers

from conftest import REPO

HEADER = os.path.join(REPO, "include", "kmerhip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kmh_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    names = declared_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(L, name), name
    bound = {n for n, _, _ in _native.SIGNATURES}
    assert bound == set(names), "ctypes signatures and header disagree"


def test_version_string():
    assert _native.lib().kmh_version().decode().startswith("kmerhip")


def test_ctx_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(_native.KmhError):
        _native.Context(0)
    with pytest.raises(_native.KmhError):   # the cached-context path must not deadlock
        _native.context(0)


def _native_records(path):
    f = _native.FastaFile(path)
    out = [(f.ids[i], f.sequence(i), f.char_lens[i]) for i in range(len(f))]
    f.close()
    return out


@contextlib.contextmanager
def _fasta_chunk(nbytes):
    """Parse with pieces of `nbytes` (KMH_FASTA_CHUNK): tiny pieces put piece boundaries at
    nearly every line of a small input, so the threaded parse and the stitching are tested."""
    old = os.environ.get("KMH_FASTA_CHUNK")
    if nbytes is None:
        os.environ.pop("KMH_FASTA_CHUNK", None)
    else:
        os.environ["KMH_FASTA_CHUNK"] = str(nbytes)
    try:
        yield
    finally:
        if old is None:
            os.environ.pop("KMH_FASTA_CHUNK", None)
        else:
            os.environ["KMH_FASTA_CHUNK"] = old


@pytest.mark.parametrize("chunk", [None, 1, 7, 64])
def test_fasta_parser_matches_oracle_on_golden_inputs(golden_dir, chunk):
    inputs = os.path.join(golden_dir, "inputs")
    for name in sorted(os.listdir(inputs)):
        path = os.path.join(inputs, name)
        ref = ofasta.parse_fasta(path)
        with _fasta_chunk(chunk):
            got = _native_records(path)
        assert [r[0] for r in got] == [r[0] for r in ref], name
        assert [r[1].decode() for r in got] == [r[2] for r in ref], name
        assert [r[2] for r in got] == [len(r[2]) for r in ref], name


def test_fasta_missing_file_raises_oserror(tmp_path):
    with pytest.raises(OSError):
        _native.FastaFile(tmp_path / "nope.fa")


_alphabet = st.sampled_from(list("ACGTacgtNnRY \t\r\n>;-*xé") + [" ", " ", "　"])


@settings(max_examples=300, deadline=None)
@given(st.lists(_alphabet, max_size=300).map("".join), st.sampled_from([None, 1, 5, 16]))
def test_fasta_parser_property(tmp_path_factory, text, chunk):
    path = tmp_path_factory.mktemp("fa") / "x.fa"
    path.write_bytes(text.encode("utf-8"))
    ref = ofasta.parse_fasta(path)
    with _fasta_chunk(chunk):
        got = _native_records(path)
    assert [(r[0], r[2]) for r in ref] == [(g[0], g[1].decode("utf-8")) for g in got]
    assert [len(r[2]) for r in ref] == [g[2] for g in got]


def test_pack_applies_short_record_rule(golden_dir):
    path = os.path.join(golden_dir, "inputs", "e1_mixed.fa")
    f = _native.FastaFile(path)
    packed, kept = f.pack(4)
    ref = ofasta.parse_fasta(path)
    assert list(kept) == [len(s) >= 4 for _, _, s in ref]
    assert packed.tobytes() == b"".join(s.encode() + b"\n" for _, _, s in ref if len(s) >= 4)
    f.close()


@pytest.mark.parametrize("k", [1, 2, 5, 12, 21, 32])
def test_format_lines_matches_reference_text(k):
    rng = np.random.default_rng(k)
    codes = rng.integers(0, 1 << min(62, 2 * k), 500, dtype=np.uint64)
    if k == 32:
        codes[0] = np.uint64(0xFFFFFFFFFFFFFFFF)
    counts = rng.integers(1, 1 << 40, 500, dtype=np.uint64)
    got = _native.format_lines(k, codes, counts).decode()
    want = okmers.kmer_text({okmers.code_kmer(int(c), k): int(n) for c, n in zip(codes, counts)}
                            ) if len(set(codes.tolist())) == codes.size else None
    if want is not None:
        assert got == want
    lines = got.splitlines()
    assert len(lines) == 500
    c0 = okmers.code_kmer(int(codes[0]), k)
    assert lines[0] == "".join(okmers.DIGIT[b] for b in c0) + f"\t{int(counts[0])}"


@pytest.mark.parametrize("k", [3, 32, 33, 40, 100])
def test_format_lines_seq_matches_reference_text(k):
    """kmh_format_lines_seq (the k > 32 writer): digits from the sequence at each k-mer's
    first start, equal to the reference's text for the same table (oracle/kmers.py)."""
    rng = np.random.default_rng(k)
    unit = "".join("ACGTacgt"[i] for i in rng.integers(0, 8, 300))
    seq = (unit + "N" + unit[:150] + "\n" + unit).encode()
    table = okmers.count_sequence(seq.decode(), k)
    firsts = {}
    up = seq.decode().upper()
    for i in range(len(up) - k + 1):
        firsts.setdefault(up[i:i + k], i)
    first = np.array([firsts[km] for km in table], np.uint64)
    counts = np.array(list(table.values()), np.uint64)
    got = _native.format_lines_seq(k, np.frombuffer(seq, np.uint8), first, counts)
    assert got.decode() == okmers.kmer_text(table)
    assert counts.max() >= 2
    with pytest.raises(ValueError):
        _native.format_lines_seq(k, np.frombuffer(seq, np.uint8), np.array([len(seq) - k + 1], np.uint64),
                                 np.array([1], np.uint64))


def test_format_lines_empty():
    assert _native.format_lines(8, np.empty(0, np.uint64), np.empty(0, np.uint64)) == b""


def test_write_file_plain_and_parallel_gzip(tmp_path):
    """kmh_write_file: plain bytes, and multi-member gzip that any reader decompresses to the
    same bytes (blocks of 2 MiB deflated on several threads)."""
    import gzip
    rng = np.random.default_rng(0)
    data = ("".join(f"{x}\t{y}\n" for x, y in zip(rng.integers(0, 10**12, 1_300_000),
                                                 rng.integers(1, 99, 1_300_000)))).encode()
    assert len(data) > 2 * (8 << 20)
    p = tmp_path / "k12.txt"
    _native.write_file(p, data)
    assert p.read_bytes() == data
    for level, threads in ((9, 0), (1, 3), (9, 1)):
        g = tmp_path / f"k12_{level}_{threads}.txt.gz"
        _native.write_file(g, data, gzip_level=level, threads=threads)
        assert gzip.decompress(g.read_bytes()) == data
        with gzip.open(g, "rt") as f:
            assert f.read(20) == data[:20].decode()
    e = tmp_path / "empty.txt.gz"
    _native.write_file(e, b"", gzip_level=9)
    assert gzip.decompress(e.read_bytes()) == b""
    with pytest.raises(OSError):
        _native.write_file(tmp_path / "no" / "such" / "dir.txt", b"x")


def test_format_lines_many_blocks_and_partial_buffer():
    """The threaded formatter (blocks of 2^18 lines) equals the reference's text
    (generate.py:86-91, restated by oracle/kmers.py) across block boundaries, and a short
    buffer receives the whole lines that fit."""
    rng = np.random.default_rng(11)
    k, n = 9, 700_000
    codes = rng.integers(0, 1 << (2 * k), n, dtype=np.uint64)
    counts = rng.integers(1, 10**7, n, dtype=np.uint64)
    text = _native.format_lines(k, codes, counts)
    want_head = "".join(okmers.DIGIT[b] for b in okmers.code_kmer(int(codes[0]), k)) + f"\t{counts[0]}\n"
    assert text.startswith(want_head.encode())
    for i in (262_143, 262_144, 524_288, n - 1):
        line = "".join(okmers.DIGIT[b] for b in okmers.code_kmer(int(codes[i]), k)) + f"\t{counts[i]}\n"
        assert line.encode() in text
    lines = text.split(b"\n")[:-1]
    assert len(lines) == n
    assert lines[524_288] == ("".join(okmers.DIGIT[b] for b in okmers.code_kmer(int(codes[524_288]), k))
                              + f"\t{counts[524_288]}").encode()
    L = _native.lib()
    cap = len(text) // 3
    import ctypes
    buf = ctypes.create_string_buffer(cap)
    total = L.kmh_format_lines(k, codes.ctypes.data, counts.ctypes.data, n, buf, cap)
    assert total == len(text)
    cut = text[:cap].rfind(b"\n") + 1
    assert buf.raw[:cut] == text[:cut]


def test_fasta_parser_multi_piece_natural(tmp_path):
    """A 12.16 Mbp, 17-record file (the config-1 stand-in, 80-column lines, CRLF on every other
    record) parsed with the default piece size (4 MiB, so pieces cut records mid-sequence):
    same records, bytes and character counts as the restated parser."""
    from oracle import synth as osynth
    recs = osynth.yeast_standin_records()
    path = tmp_path / "y.fa"
    osynth.write_fasta(path, recs)
    raw = path.read_bytes()
    # CRLF line ends in the odd records: the piece cuts (after a '\n') must never split "\r\n"
    parts = raw.split(b">")
    raw = b">".join(p.replace(b"\n", b"\r\n") if i % 2 else p for i, p in enumerate(parts))
    path.write_bytes(raw)
    ref = ofasta.parse_fasta(path)
    with _fasta_chunk(None):
        got = _native_records(path)
    assert [g[0] for g in got] == [r[0] for r in ref]
    assert all(g[1] == r[2].encode() for g, r in zip(got, ref))
    assert [g[2] for g in got] == [len(r[2]) for r in ref]
    assert len(raw) > 2 * (4 << 20)   # three pieces at the default size
