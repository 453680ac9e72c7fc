"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the golden
fixtures produced by the reference.  Bit-exact for every count, code and position."""
import contextlib
import gzip
import hashlib
import io
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from kmerml import _native  # noqa: E402
from kmerml.kmers.generate import KmerExtractor  # noqa: E402
from kmerml.kmers import matrix as kmatrix  # noqa: E402
from kmerml.utils.path_utils import find_files  # noqa: E402
from oracle import synth as osynth  # noqa: E402
from _dropin import run_extractor  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return _native.context(0)


@pytest.fixture(scope="module")
def dev():
    return torch.device("cuda", 0)


def _rand_seq(rng, n, alphabet=b"ACGTACGTACGTacgtNn-\n"):
    return np.frombuffer(alphabet, np.uint8)[rng.integers(0, len(alphabet), n)]


def _layout(genomes):
    """Concatenate host genomes with 16-byte aligned starts -> (buffer, offsets)."""
    parts, offs, pos = [], [0], 0
    for g in genomes:
        pad = (-g.size) % 16
        parts += [g, np.full(pad, 0x4E, np.uint8)]  # 'N' padding is not a base
        pos += g.size + pad
        offs.append(pos)
    return np.concatenate(parts), np.array(offs, np.uint64)


def _dense_rows(ctx, dev, genomes, k):
    buf, offs = _layout(genomes)
    d_seq = torch.from_numpy(buf.copy()).to(dev)
    out = torch.full((len(genomes), 1 << (2 * k)), -7, dtype=torch.int32, device=dev)
    ctx.count_dense_dev(d_seq.data_ptr(), offs, k, out.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32), buf, offs


# ---------------------------------------------------------------- device generator
def test_synth_matches_oracle(ctx, dev):
    L, stride, G = 100_003, 100_016, 3
    d = torch.zeros(G * stride, dtype=torch.uint8, device=dev)
    ctx.synth_dev(d.data_ptr(), L, stride, G, osynth.SEED_BASE, torch.cuda.current_stream().cuda_stream)
    host = d.cpu().numpy()
    for g in range(G):
        want = osynth.synth_bases(L, osynth.genome_seed(g))
        assert np.array_equal(host[g * stride: g * stride + L], want), g


# ---------------------------------------------------------------- dense, every k
@pytest.mark.parametrize("k", list(range(1, 13)))
def test_dense_all_k_vs_oracle(ctx, dev, oracle_lib, k):
    rng = np.random.default_rng(100 + k)
    genomes = [_rand_seq(rng, 250_000), _rand_seq(rng, k - 1 if k > 1 else 0),
               np.zeros(0, np.uint8), _rand_seq(rng, 70_001), _rand_seq(rng, 16_384 + k)]
    rows, _, _ = _dense_rows(ctx, dev, genomes, k)
    for g, seq in enumerate(genomes):
        want = oracle_lib.count_dense(seq, k)
        assert np.array_equal(rows[g], want), (k, g)


@pytest.mark.parametrize("k", [4, 8, 10, 12])
def test_dense_low_complexity(ctx, dev, oracle_lib, k):
    # every window of a tile in one bucket: A (bucket 0, even: low counter half), T (the last
    # bucket, odd: high half, next to the invalid-window row), C / G (odd / even), AT / TA
    genomes = [np.full(1_000_000, ord("A"), np.uint8),
               np.frombuffer(b"AT" * 300_000 + b"a" * 5000, np.uint8).copy(),
               np.full(700_001, ord("T"), np.uint8),
               np.frombuffer(b"c" * 300_000 + b"N" * 17 + b"G" * 300_000, np.uint8).copy()]
    rows, _, _ = _dense_rows(ctx, dev, genomes, k)
    for g, seq in enumerate(genomes):
        assert np.array_equal(rows[g], oracle_lib.count_dense(seq, k)), (k, g)


def _u4_block(ctx, dev, genomes, k, fused, rows=True):
    """(u32 rows, nibbles, sorted escape pairs, escape count) of count + u4 encode, either fused
    (kmh_count_dense_u4_dev; rows=False: kmh_count_dense_u4only_dev, whose rows are scratch) or as
    two passes (kmh_count_dense_dev + kmh_rows_encode_u4_dev)."""
    buf, offs = _layout(genomes)
    d_seq = torch.from_numpy(buf.copy()).to(dev)
    G, cols = len(genomes), 1 << (2 * k)
    nib = G * cols // 2
    cap = G * cols // 4   # room for every escape (the repeated genome's counts are all >= 15)
    P = nib + 16 + 8 * cap
    out = torch.full((G, cols), -7, dtype=torch.int32, device=dev)
    slot = torch.zeros(P, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    if fused:
        ctx.count_dense_u4_dev(d_seq.data_ptr(), offs, k, out.data_ptr(), slot.data_ptr(),
                               slot[nib + 16:].data_ptr(), cap, slot[nib:].data_ptr(), s, rows=rows)
    else:
        ctx.count_dense_dev(d_seq.data_ptr(), offs, k, out.data_ptr(), s)
        ctx.rows_encode_u4(out.data_ptr(), G, cols, slot.data_ptr(), slot[nib + 16:].data_ptr(), cap,
                           slot[nib:].data_ptr(), s)
    torch.cuda.synchronize()
    h = slot.cpu().numpy()
    n = int(h[nib:nib + 4].view(np.uint32)[0])
    esc = h[nib + 16:nib + 16 + 8 * min(n, cap)].view(np.uint32).reshape(-1, 2)
    esc = esc[np.lexsort((esc[:, 1], esc[:, 0]))]
    return out.cpu().numpy().view(np.uint32), h[:nib], esc, n


@pytest.mark.parametrize("k,rows", [(8, True), (10, True), (12, True), (10, False), (12, False)])
def test_count_dense_u4_fused(ctx, dev, oracle_lib, k, rows):
    """kmh_count_dense_u4_dev writes the same rows, nibbles and escape set as count + encode,
    on ragged random genomes, a low-complexity genome (counts > 255), one whose u16 table
    wraps (counts > 65535: that bucket is re-encoded from the corrected rows) and a 1 Mbp
    segment repeated 16 times (every count >= 15: more escapes per bucket than the kernel
    stages, so those buckets are re-encoded from rows too).  rows=False
    (kmh_count_dense_u4only_dev, the multi-GPU step): the same slot, rows not kept."""
    rng = np.random.default_rng(500 + k)
    rep = _rand_seq(rng, 1_000_000, alphabet=b"ACGT")
    genomes = [_rand_seq(rng, 3_000_000), np.zeros(0, np.uint8), _rand_seq(rng, 70_001),
               np.frombuffer(b"AT" * 300_000 + b"a" * 5000, np.uint8).copy(),
               np.frombuffer(b"A" * 200_000 + b"G" + b"T" * 70_000, np.uint8).copy(),
               np.tile(rep, 16)]
    r1, n1, e1, c1 = _u4_block(ctx, dev, genomes, k, fused=True, rows=rows)
    r2, n2, e2, c2 = _u4_block(ctx, dev, genomes, k, fused=False)
    for g, seq in enumerate(genomes):
        assert np.array_equal(r2[g], oracle_lib.count_dense(seq, k)), g
    if rows:
        assert np.array_equal(r1, r2)
    assert np.array_equal(n1, n2)
    assert c1 == c2 and c1 > 0 and np.array_equal(e1, e2)
    assert e1[:, 1].max() > 65535
    assert e1.shape[0] == c1   # every escape fit the slot
    if k >= 10:   # the repeated genome's buckets hold more escapes than a count workgroup stages
        per_bucket = np.bincount((e1[:, 0] >> 16).astype(np.int64))
        assert per_bucket.max() > 3072


@pytest.mark.parametrize("k", [10, 12])
def test_dense_u16_wraps(ctx, dev, oracle_lib, k):
    """Counts past 65535 in both halves of one packed u16 word of the count table: bins 0
    (A...A) and 1 (A...AC) each exceed 2^16, so their wraps, the carry of the low half into
    the high half and the carry out of the word are all corrected; also a bin > 2^17."""
    genomes = [np.frombuffer(b"A" * 200_000 + b"A" * (k - 1) + b"C" + (b"A" * (k - 1) + b"C") * 70_000, np.uint8).copy(),
               np.frombuffer(b"A" * 140_000 + b"G" + b"T" * 70_000 + b"N" + b"A" * 66_000, np.uint8).copy()]
    rows, _, _ = _dense_rows(ctx, dev, genomes, k)
    for g, seq in enumerate(genomes):
        want = oracle_lib.count_dense(seq, k)
        assert want[0] > 65536 and np.array_equal(rows[g], want), (k, g)
    assert oracle_lib.count_dense(genomes[0], k)[1] > 65536


@pytest.mark.parametrize("k", [10, 11, 12])
def test_dense_partition_many_genomes(ctx, dev, oracle_lib, monkeypatch, k):
    """The partition / count kernels on 120 ragged genomes -- empty ones, one spanning ~120
    tiles, one of exactly one tile of windows -- in one batch; then again with one genome per
    batch (KMH_SUF_BUDGET_MB=1)."""
    rng = np.random.default_rng(7000 + k)
    lens = rng.integers(0, 90_000, 120)
    lens[::29] = 0
    lens[7] = 2_000_003
    lens[8] = 16_384 + k - 1          # exactly one full tile of windows
    genomes = [_rand_seq(rng, int(n)) for n in lens]
    want = [oracle_lib.count_dense(seq, k) for seq in genomes]
    rows, _, _ = _dense_rows(ctx, dev, genomes, k)
    for g in range(len(genomes)):
        assert np.array_equal(rows[g], want[g]), (k, g)
    monkeypatch.setenv("KMH_SUF_BUDGET_MB", "1")
    rows, _, _ = _dense_rows(ctx, dev, genomes[:12], k)
    for g in range(12):
        assert np.array_equal(rows[g], want[g]), (k, g, "batched")


@pytest.mark.parametrize("k", [11, 12])
def test_dense_partition_long_runs_large_offsets(ctx, dev, oracle_lib, k):
    """The genomes lie past byte 2^31 of the buffer (a 2.2 GB genome of 'N' -- tiles but no
    valid window -- comes first): 40 ragged genomes, ~40 Mbp."""
    rng = np.random.default_rng(900 + k)
    lens = rng.integers(0, 2_000_000, 40)
    lens[3] = 0
    lens[10] = 5_000_017
    genomes = [_rand_seq(rng, int(n), b"ACGTACGTACGTacgtN") for n in lens]
    lead = (2**31 + 2**22 + 15) // 16 * 16
    buf, offs = _layout(genomes)
    d_seq = torch.empty(lead + buf.size, dtype=torch.uint8, device=dev)
    d_seq[:lead].fill_(ord("N"))
    d_seq[lead:].copy_(torch.from_numpy(buf))
    offs = np.concatenate([[0], offs + lead]).astype(np.uint64)
    out = torch.full((len(genomes) + 1, 1 << (2 * k)), -7, dtype=torch.int32, device=dev)
    ctx.count_dense_dev(d_seq.data_ptr(), offs, k, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rows = out.cpu().numpy().view(np.uint32)
    assert not rows[0].any()
    for g, seq in enumerate(genomes):
        assert np.array_equal(rows[g + 1], oracle_lib.count_dense(seq, k)), (k, g)


def test_dense_rejects_misaligned_offsets(ctx, dev):
    d_seq = torch.zeros(64, dtype=torch.uint8, device=dev)
    out = torch.zeros((2, 256), dtype=torch.int32, device=dev)
    with pytest.raises(ValueError):
        ctx.count_dense_dev(d_seq.data_ptr(), np.array([0, 7, 64], np.uint64), 4, out.data_ptr())
    with pytest.raises(NotImplementedError):
        ctx.count_dense_dev(d_seq.data_ptr(), np.array([0, 64], np.uint64), 13, out.data_ptr())


# ---------------------------------------------------------------- BASELINE configs
def test_config2_8x10mbp_k8(ctx, dev, oracle_lib, synthetic_cases):
    """Config 2: 8 synthetic 10 Mbp genomes, k=8, bit-exact vs the oracle; genomes 0 and
    1 also match the reference's own k8.txt hashes (first-occurrence order)."""
    G, L, k = 8, 10_000_000, 8
    d = torch.empty(G * L, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ctx.synth_dev(d.data_ptr(), L, L, G, osynth.SEED_BASE, s)
    offs = np.arange(G + 1, dtype=np.uint64) * L
    out = torch.empty((G, 1 << (2 * k)), dtype=torch.int32, device=dev)
    first = torch.empty_like(out)
    ctx.count_dense_dev(d.data_ptr(), offs, k, out.data_ptr(), s)
    ctx.first_dense_dev(d.data_ptr(), offs, k, first.data_ptr(), s)
    torch.cuda.synchronize()
    rows = out.cpu().numpy().view(np.uint32)
    firsts = first.cpu().numpy().view(np.uint32)
    host = d.cpu().numpy()
    for g in range(G):
        want, wfirst = oracle_lib.count_dense(host[g * L:(g + 1) * L], k, with_first=True)
        assert np.array_equal(rows[g], want), g
        assert np.array_equal(firsts[g], wfirst), g
    for case in synthetic_cases:
        if not case["name"].startswith("c2_"):
            continue
        g = int(case["name"][-4:])
        nz = np.nonzero(rows[g])[0]
        order = nz[np.argsort(firsts[g][nz])]
        text = _native.format_lines(k, order.astype(np.uint64), rows[g][order].astype(np.uint64))
        assert hashlib.sha256(text).hexdigest() == case["sha256"]["k8.txt"]


def test_config3_64x100mbp_k12(ctx, dev, oracle_lib):
    """Config 3 at full size: row sums equal the valid-window count for all 64 genomes,
    two runs are identical, and genomes 0, 31 and 63 are bit-exact vs the oracle."""
    G, L, k = 64, 100_000_000, 12
    d = torch.empty(G * L, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ctx.synth_dev(d.data_ptr(), L, L, G, osynth.SEED_BASE, s)
    offs = np.arange(G + 1, dtype=np.uint64) * L
    out = torch.empty((G, 1 << (2 * k)), dtype=torch.int32, device=dev)
    ctx.count_dense_dev(d.data_ptr(), offs, k, out.data_ptr(), s)
    sums = out.sum(1, dtype=torch.int64)
    assert torch.all(sums == L - k + 1).item()
    first_run = out.clone()
    ctx.count_dense_dev(d.data_ptr(), offs, k, out.data_ptr(), s)
    assert torch.equal(first_run, out)
    del first_run
    for g in (0, 31, 63):
        host = d[g * L:(g + 1) * L].cpu().numpy()
        assert np.array_equal(out[g].cpu().numpy().view(np.uint32), oracle_lib.count_dense(host, k)), g


# ---------------------------------------------------------------- sparse, k > 12
@pytest.mark.parametrize("k,canonical", [(13, 0), (16, 0), (21, 0), (21, 1), (31, 0), (32, 0), (32, 1), (5, 1)])
def test_sparse_vs_oracle(ctx, oracle_lib, k, canonical):
    rng = np.random.default_rng(k * 10 + canonical)
    seq = _rand_seq(rng, 300_000)
    codes, counts, first = ctx.count(seq, k, canonical=bool(canonical))
    wc, wn, wf = oracle_lib.count_sparse(seq, k, canonical=bool(canonical))
    order = np.argsort(wf, kind="stable")
    assert np.array_equal(codes, wc[order])
    assert np.array_equal(counts, wn[order])
    assert np.array_equal(first, wf[order])


@pytest.mark.parametrize("k,target,limit", [(21, "37", "12288"), (21, "61", "9"), (27, "100000", "40"),
                                            (17, "5000", "3")])
def test_sparse_host_fallback_first_positions(ctx, oracle_lib, monkeypatch, k, target, limit):
    """The drop-in's 13 <= k <= 32 path is the hash pipeline with window positions carried along:
    capped tables push most passes into the hand-written sort fallback (sort by position, then
    stably by key), which must give the same counts and first positions -- hence the same
    first-occurrence order of k{k}.txt (generate.py:36,58) -- as the oracle.  Repeats make counts
    > 1 and big bins (the count kernel's LDS hash table with its minimum position per slot)."""
    rng = np.random.default_rng(900 + k)
    unit = _rand_seq(rng, 5000, b"ACGTACGTacgt")
    seq = np.concatenate([_rand_seq(rng, 200_000), np.tile(unit, 40), _rand_seq(rng, 90_000),
                          np.tile(np.frombuffer(b"ACGTTGCAT", np.uint8), 4000)])
    monkeypatch.setenv("KMH_SP_TARGET", target)
    monkeypatch.setenv("KMH_SP_LIMIT", limit)
    codes, counts, first = ctx.count(seq, k)
    wc, wn, wf = oracle_lib.count_sparse(seq, k)
    order = np.argsort(wf, kind="stable")
    assert counts.max() >= 40
    assert np.array_equal(first, wf[order])
    assert np.array_equal(codes, wc[order])
    assert np.array_equal(counts, wn[order])


@pytest.mark.parametrize("k", [13, 21, 22, 32])
def test_sparse_host_low_complexity(ctx, oracle_lib, k):
    """poly-A, dinucleotide and short-period repeats through the drop-in path: at k = 32 the
    u64 table slots overflow their count field and the passes go to the fallback."""
    seq = np.concatenate([np.full(300_000, ord("A"), np.uint8), np.frombuffer(b"N", np.uint8),
                          np.frombuffer(b"AC" * 150_000, np.uint8), np.frombuffer(b"acgttgacc" * 20_000, np.uint8)])
    codes, counts, first = ctx.count(seq, k)
    wc, wn, wf = oracle_lib.count_sparse(seq, k)
    order = np.argsort(wf, kind="stable")
    assert np.array_equal(first, wf[order])
    assert np.array_equal(codes, wc[order]) and np.array_equal(counts, wn[order])


def test_count_host_past_2_31_windows(ctx, oracle_lib):
    """An organism of more than 2^31 windows at k = 21 (the reference's dict takes any length,
    generate.py:36,58): a random 1,000,003-base unit repeated 2200 times (2.2 Gbases).  Window p
    holds the k-mer of the circular unit at offset p mod U, so every k-mer's count is R times
    its count over the U circular offsets, less its count over the k - 1 offsets past U - k (they
    fit one copy fewer), and its first start is its first circular offset -- all from the
    oracle's counts of the unit alone."""
    U, R, k = 1_000_003, 2200, 21
    unit = oracle_lib.synth(U, osynth.genome_seed(77))
    seq = np.tile(unit, R)
    assert seq.size - k + 1 > 2**31
    codes, counts, first = ctx.count(seq, k)
    del seq
    circ = np.concatenate([unit, unit[:k - 1]])
    cc, cn, cf = oracle_lib.count_sparse(circ, k)                       # U windows, offsets 0..U-1
    tail = np.concatenate([unit[U - k + 1:], unit[:k - 1]])              # offsets U-k+1 .. U-1
    tc, tn, _ = oracle_lib.count_sparse(tail, k)
    want = cn.astype(np.int64) * R
    want[np.searchsorted(cc, tc)] -= tn
    order = np.argsort(cf, kind="stable")
    assert np.array_equal(codes, cc[order])
    assert np.array_equal(first, cf[order])
    assert np.array_equal(counts.astype(np.int64), want[order])
    assert int(counts.astype(np.int64).sum()) == U * R - k + 1


@pytest.mark.parametrize("k", [33, 40, 63, 64, 65, 100])
def test_long_kmers_vs_python_oracle(ctx, k):
    """k > 32 (the reference's dict takes any k): word-sorted on the GPU, first-occurrence
    order, and the k{k}.txt text written from the sequence, byte-identical to the pure-Python
    restatement of generate.py:49-58 + :86-91 (oracle/kmers.py).  Repeated segments give
    counts > 1; lowercase, N and newlines break or fold windows as in the reference."""
    from oracle import kmers as okmers
    rng = np.random.default_rng(4000 + k)
    seg = _rand_seq(rng, 700, b"ACGTACGTACGTacgt")
    parts = []
    for _ in range(12):
        parts += [_rand_seq(rng, int(rng.integers(50, 5000)), b"ACGTACGTACGTACGTacgtN\n"), seg]
    seq = np.concatenate(parts)
    codes, counts, first = ctx.count(seq, k)
    text = _native.format_lines_seq(k, seq, first, counts.astype(np.uint64))
    want = okmers.count_sequence(seq.tobytes().decode(), k)
    assert text.decode() == okmers.kmer_text(want)
    assert counts.max() >= 12
    prefix = [okmers.kmer_code(km[:32]) for km in want]
    assert np.array_equal(codes, np.array(prefix, np.uint64))


def test_long_kmers_limits(ctx):
    seq = np.frombuffer(b"ACGT" * 300, np.uint8)
    with pytest.raises(NotImplementedError):
        ctx.count(seq, 1025)
    with pytest.raises(NotImplementedError):
        ctx.count(seq, 33, canonical=True)
    codes, counts, first = ctx.count(seq, 1024)   # 177 windows, 4 distinct
    assert codes.size == 4 and counts.sum() == 1200 - 1024 + 1 and list(first) == [0, 1, 2, 3]


@pytest.mark.parametrize("k", [1, 7, 12])
def test_count_host_dense_first_order(ctx, oracle_lib, k):
    rng = np.random.default_rng(k)
    seq = _rand_seq(rng, 200_000)
    codes, counts, first = ctx.count(seq, k)
    wc, wn, wf = oracle_lib.count_sparse(seq, k)
    order = np.argsort(wf, kind="stable")
    assert np.array_equal(codes, wc[order]) and np.array_equal(counts, wn[order])
    assert np.array_equal(first, wf[order])


# ---------------------------------------------------------------- the drop-in API
def test_dropin_edge_cases_byte_identical(tmp_path, golden_dir, edge_cases):
    # every case, k = 33 and k = 40 included (long k-mers: word-sorted on the GPU, lines
    # written from the sequence); k <= 0 / bool / float cases too (tests/test_dropin_degenerate.py
    # runs the ones that need no device on the CPU)
    for i, case in enumerate(edge_cases):
        ret, out, files = run_extractor(tmp_path / f"c{i}", os.path.join(golden_dir, "inputs", case["input"]),
                                         case["k_values"], expect_error=case.get("error"))
        assert ret == case["returned"]
        assert out == case["stdout"], case["input"]
        assert files == case["files"], (case["input"], case["k_values"])


def test_dropin_compressed(tmp_path, golden_dir, edge_cases):
    case = edge_cases[3]
    _, _, files = run_extractor(tmp_path, os.path.join(golden_dir, "inputs", case["input"]),
                                 case["k_values"], compress=True)
    assert files == case["files"]
    assert all(p.name.endswith(".txt.gz") for p in (tmp_path / "org").iterdir())


def test_dropin_synthetic_hashes(tmp_path, synthetic_cases):
    for case in synthetic_cases:
        if case["name"] == "yeast_standin":
            recs = osynth.yeast_standin_records()
            fa = tmp_path / "yeast_standin.fa"
            osynth.write_fasta(fa, recs)
            _, out, files = run_extractor(tmp_path / "ys", fa, [4], org="yeast_standin")
            assert files["k4.txt"] == case["text"]["k4.txt"]
            assert out == case["stdout"]
            continue
        (g,) = case["genomes"]
        fa = tmp_path / f"{case['name']}.fa"
        osynth.write_fasta(fa, [(g["id"], osynth.synth_bases(g["length"], g["seed"], g["start"]).tobytes())])
        (k,) = case["k_values"]
        _, out, files = run_extractor(tmp_path / case["name"], fa, [k])
        assert out == case["stdout"]
        assert hashlib.sha256(files[f"k{k}.txt"].encode()).hexdigest() == case["sha256"][f"k{k}.txt"], case["name"]


def test_cli_call_pattern_and_genome_list(tmp_path, golden_dir, edge_cases):
    """scripts/extract_kmers.py:46-61 and generate.py:93-129 call patterns."""
    src = tmp_path / "raw"
    src.mkdir()
    for name in ("e1_mixed.fa", "e2_crlf.fa", "e4_short.fa"):
        (src / name).write_bytes(open(os.path.join(golden_dir, "inputs", name), "rb").read())
    (src / "notes.txt").write_text("ignored")
    genomes = find_files(src, patterns="*.fa,*.fasta".split(","), recursive=False)
    assert [g.name for g in genomes] == ["e1_mixed.fa", "e2_crlf.fa", "e4_short.fa"]
    ext = KmerExtractor(output_dir=str(tmp_path / "out"), compress=False)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        for genome in genomes:
            ext.extract_kmers_from_fasta(genome, [3, 8], organism_id=genome.stem)
        ids = ext.extract_from_genome_list([str(g) for g in genomes] + [str(src / "missing.fa")], [3, 8])
    assert ids == ["e1_mixed", "e2_crlf", "e4_short"]
    assert "Error processing missing" in buf.getvalue()
    want = next(c for c in edge_cases if c["input"] == "e2_crlf.fa" and c["k_values"] == [3, 8])
    assert (tmp_path / "out" / "e2_crlf" / "k8.txt").read_text() == want["files"]["k8.txt"]
    with pytest.raises(ValueError):
        ext.extract_from_genome_list([str(genomes[0])], [3], organism_ids=["a", "b"])


def test_count_matrix_single_process(tmp_path, oracle_lib):
    rng = np.random.default_rng(3)
    files, seqs = [], []
    for i in range(5):
        s = _rand_seq(rng, 40_000 + 1000 * i, b"ACGTACGTN").tobytes()
        p = tmp_path / f"g{i}.fa"
        osynth.write_fasta(p, [(f"r{i}", s[:20_000]), (f"q{i}", s[20_000:])])
        files.append(p)
        seqs.append(s[:20_000] + b"\n" + s[20_000:] + b"\n")
    m = kmatrix.count_matrix(files, 10).cpu().numpy().view(np.uint32)
    for i, s in enumerate(seqs):
        assert np.array_equal(m[i], oracle_lib.count_dense(s, 10)), i


# ---------------------------------------------------------------- matrix assembly encoding
def _encode(ctx, d_rows, cap):
    rows, cols = d_rows.shape
    s = torch.cuda.current_stream().cuda_stream
    u8 = torch.empty(rows * cols, dtype=torch.uint8, device=d_rows.device)
    esc = torch.full((max(cap, 1) * 3,), 0x7777, dtype=torch.int32, device=d_rows.device)
    n = torch.full((1,), -1, dtype=torch.int32, device=d_rows.device)
    ctx.rows_encode_u8(d_rows.data_ptr(), rows, cols, u8.data_ptr(), esc.data_ptr(), cap, n.data_ptr(), s)
    return u8, esc, n


@pytest.mark.parametrize("ranks", [1, 3])
def test_rows_u8_round_trip_with_escapes(ctx, dev, ranks):
    """Saturating u8 rows + escape list widen back to the exact u32 rows (features.py:85-117
    matrix, multi-rank layout of bench.py / kmerml.kmers.matrix)."""
    rng = np.random.default_rng(5)
    rows_per_rank, cols = 3, 4096
    cap = 2048
    blocks, u8s, escs, ns = [], [], [], []
    for r in range(ranks):
        m = rng.poisson(6, (rows_per_rank, cols)).astype(np.uint32)
        hot = rng.integers(0, m.size, 300 + 50 * r)
        m.reshape(-1)[hot] = rng.choice(np.array([254, 255, 256, 1000, 65535, 65536, 2**32 - 1], np.uint64),
                                        hot.size).astype(np.uint32)
        blocks.append(m)
        u8, esc, n = _encode(ctx, torch.from_numpy(m.view(np.int32)).to(dev), cap)
        torch.cuda.synchronize()
        assert int(n.item()) == int((m >= 255).sum())
        assert np.array_equal(u8.cpu().numpy(), np.minimum(m, 255).astype(np.uint8).reshape(-1))
        u8s.append(u8), escs.append(esc), ns.append(n)
    out = torch.full((ranks * rows_per_rank, cols), -3, dtype=torch.int32, device=dev)
    # keep the concatenations alive until the kernels have run (no allocator reuse)
    all_u8, all_esc, all_n = torch.cat(u8s), torch.cat(escs), torch.cat(ns)
    assert all_esc.numel() == ranks * cap * 3 and all_n.numel() == ranks
    ctx.rows_decode_u8(all_u8.data_ptr(), ranks * rows_per_rank, cols, all_esc.data_ptr(),
                       cap, all_n.data_ptr(), ranks, rows_per_rank, out.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), np.concatenate(blocks))


def _encode_u4(ctx, d_rows, cap):
    rows, cols = d_rows.shape
    s = torch.cuda.current_stream().cuda_stream
    u4 = torch.full((rows * cols // 2,), 0x5A, dtype=torch.uint8, device=d_rows.device)
    esc = torch.full((max(cap, 1) * 2,), 0x7777, dtype=torch.int32, device=d_rows.device)
    n = torch.full((1,), -1, dtype=torch.int32, device=d_rows.device)
    ctx.rows_encode_u4(d_rows.data_ptr(), rows, cols, u4.data_ptr(), esc.data_ptr(), cap, n.data_ptr(), s)
    return u4, esc, n


def test_rows_u4_round_trip_with_escapes(ctx, dev):
    """u4 rows (two counts per byte, >= 15 saturated) + (index, value) escapes widen back to
    the exact u32 rows -- the default wire format of the multi-GPU assembly."""
    rng = np.random.default_rng(15)
    rows, cols, cap = 5, 8192, 8192
    m = rng.poisson(6, (rows, cols)).astype(np.uint32)
    hot = rng.integers(0, m.size, 700)
    m.reshape(-1)[hot] = rng.choice(np.array([14, 15, 16, 255, 256, 65536, 2**32 - 1], np.uint64),
                                    hot.size).astype(np.uint32)
    u4, esc, n = _encode_u4(ctx, torch.from_numpy(m.view(np.int32)).to(dev), cap)
    torch.cuda.synchronize()
    assert int(n.item()) == int((m >= 15).sum()) <= cap
    sat = np.minimum(m, 15).astype(np.uint8).reshape(-1)
    assert np.array_equal(u4.cpu().numpy(), sat[0::2] | (sat[1::2] << 4))
    e = esc.cpu().numpy().view(np.uint32)[:2 * int(n.item())].reshape(-1, 2)
    assert np.array_equal(np.sort(e[:, 0]), np.flatnonzero(m.reshape(-1) >= 15))
    assert np.array_equal(e[:, 1], m.reshape(-1)[e[:, 0]])
    out = torch.full((rows, cols), -3, dtype=torch.int32, device=dev)
    ctx.rows_decode_u4(u4.data_ptr(), rows, cols, esc.data_ptr(), cap, n.data_ptr(), out.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), m)


def test_rows_u4_escape_bounds_and_overflow(ctx, dev):
    """A slot off the wire whose escape index points outside its block writes nothing; more
    escapes than cap are counted, not stored (the caller falls back to another format)."""
    m = torch.full((2, 64), 300, dtype=torch.int32, device=dev)
    _, _, n = _encode_u4(ctx, m, 16)
    torch.cuda.synchronize()
    assert int(n.item()) == 128
    rows, cols = 2, 64
    u4 = torch.zeros(rows * cols // 2, dtype=torch.uint8, device=dev)
    esc = torch.tensor([3, 99, rows * cols, 7, -2**31, 8], dtype=torch.int32, device=dev)  # 2^31 as u32
    n = torch.tensor([3], dtype=torch.int32, device=dev)
    guard = torch.full((3, cols), -1, dtype=torch.int32, device=dev)   # rows 0-1 block, row 2 guard
    ctx.rows_decode_u4(u4.data_ptr(), rows, cols, esc.data_ptr(), 3, n.data_ptr(), guard.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    g = guard.cpu().numpy()
    assert g[0, 3] == 99 and g[0].sum() == 99 and (g[2] == -1).all()
    with pytest.raises(ValueError):
        _encode_u4(ctx, torch.zeros((2, 48), dtype=torch.int32, device=dev), 16)


def test_rows_u8_overflow_is_reported(ctx, dev):
    m = torch.full((2, 64), 300, dtype=torch.int32, device=dev)
    _, _, n = _encode(ctx, m, 16)
    torch.cuda.synchronize()
    assert int(n.item()) == 128     # > cap: the caller must fall back to u32 rows


def test_rows_u8_rejects_ragged_cols(ctx, dev):
    m = torch.zeros((2, 24), dtype=torch.int32, device=dev)
    with pytest.raises(ValueError):
        _encode(ctx, m, 16)


# ---------------------------------------------------------------- sparse, device-resident (config 5)
def _sparse_dev(ctx, dev, genomes, k, canonical):
    """kmh_count_sparse_dev on host genomes -> per-genome (codes, counts) sorted by code."""
    buf, offs = _layout(genomes)
    d_seq = torch.from_numpy(buf.copy()).to(dev)
    out_off = _native.sparse_out_offsets(offs, k)
    cap = max(int(out_off[-1]), 1)
    d_codes = torch.full((cap,), -1, dtype=torch.int64, device=dev)
    d_counts = torch.zeros(cap, dtype=torch.int32, device=dev)
    d_nk = torch.full((len(genomes),), -1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ctx.count_sparse_dev(d_seq.data_ptr(), offs, k, canonical, d_codes.data_ptr(), d_counts.data_ptr(),
                         d_nk.data_ptr(), s)
    torch.cuda.synchronize()
    nk = d_nk.cpu().numpy()
    codes = d_codes.cpu().numpy().view(np.uint64)
    counts = d_counts.cpu().numpy().view(np.uint32)
    res = []
    for g in range(len(genomes)):
        a, n = int(out_off[g]), int(nk[g])
        assert 0 <= n <= int(out_off[g + 1]) - a
        c, m = codes[a:a + n], counts[a:a + n]
        o = np.argsort(c, kind="stable")
        res.append((c[o], m[o]))
    return res


def _ragged_genomes(rng, sizes):
    gs = [_rand_seq(rng, n) for n in sizes]
    gs.append(np.frombuffer(b"ACGTTGCAacgtN" * 3, np.uint8).copy())   # shorter than a tile, mixed
    gs.append(np.zeros(0, np.uint8))                                    # empty genome
    gs.append(np.frombuffer(b"ACGTACGTACGTACGTACGT", np.uint8).copy())  # 20 bases < k = 21
    return gs


@pytest.mark.parametrize("k,canonical", [(13, 0), (13, 1), (17, 1), (20, 0), (21, 0), (21, 1),
                                         (22, 0), (22, 1), (25, 0), (25, 1), (31, 1), (32, 0), (32, 1)])
def test_sparse_dev_vs_oracle(ctx, dev, oracle_lib, k, canonical):
    rng = np.random.default_rng(100 + k * 2 + canonical)
    genomes = _ragged_genomes(rng, [400_000, 32768 + 21, 1_000_003, 17])
    got = _sparse_dev(ctx, dev, genomes, k, canonical)
    for g, seq in enumerate(genomes):
        wc, wn, _ = oracle_lib.count_sparse(seq, k, canonical=bool(canonical))
        assert np.array_equal(got[g][0], wc), g
        assert np.array_equal(got[g][1], wn), g


@pytest.mark.parametrize("k", [21, 27])
def test_sparse_dev_passes_and_fallback(ctx, dev, oracle_lib, monkeypatch, k):
    """Every bucket split into many passes, and tables capped so most passes overflow into
    the sort fallback: the counts must not change (u32 residues at k = 21, u64 at k = 27)."""
    rng = np.random.default_rng(7)
    genomes = _ragged_genomes(rng, [600_000, 70_001])
    want = [oracle_lib.count_sparse(s, k, canonical=True)[:2] for s in genomes]
    for target, limit in (("37", "12288"), ("100000", "40"), ("61", "9")):
        monkeypatch.setenv("KMH_SP_TARGET", target)
        monkeypatch.setenv("KMH_SP_LIMIT", limit)
        got = _sparse_dev(ctx, dev, genomes, k, 1)
        for g in range(len(genomes)):
            assert np.array_equal(got[g][0], want[g][0]), (target, limit, g)
            assert np.array_equal(got[g][1], want[g][1]), (target, limit, g)


def test_sparse_dev_multi_batch(ctx, dev, oracle_lib, monkeypatch):
    """A 1 MB entry budget puts every genome in a batch of its own (each batch plans its items
    on the device), with and without overflowing tables in the later batches."""
    rng = np.random.default_rng(11)
    genomes = _ragged_genomes(rng, [300_000, 70_001, 150_000])
    want = [oracle_lib.count_sparse(s, 21, canonical=True)[:2] for s in genomes]
    monkeypatch.setenv("KMH_SP_BUDGET_MB", "1")
    for limit in ("16384", "50"):
        monkeypatch.setenv("KMH_SP_LIMIT", limit)
        got = _sparse_dev(ctx, dev, genomes, 21, 1)
        for g in range(len(genomes)):
            assert np.array_equal(got[g][0], want[g][0]), (limit, g)
            assert np.array_equal(got[g][1], want[g][1]), (limit, g)


@pytest.mark.parametrize("k", [21, 22, 32])
def test_sparse_dev_low_complexity(ctx, dev, oracle_lib, k):
    """poly-T: at k = 21 the forward code's low 32 bits are all ones (a residue that must not
    be mistaken for an empty slot).  At k = 32 a table slot keeps 10 count bits beside its
    54-bit key: the repeats here count up to ~300 000, so their passes overflow into the exact
    fallback; at k = 22 the count keeps 30 bits."""
    genomes = [np.full(300_000, ord("A"), np.uint8),
               np.full(70_000, ord("T"), np.uint8),
               np.frombuffer(b"A" * 5 + b"T" * 16 + b"G" * 3, np.uint8).copy(),
               np.frombuffer(b"AC" * 150_000, np.uint8).copy(),
               np.frombuffer(b"ACGTTTGACCA" * 30_000, np.uint8).copy()]
    for canonical in (0, 1):
        got = _sparse_dev(ctx, dev, genomes, k, canonical)
        for g, seq in enumerate(genomes):
            wc, wn, _ = oracle_lib.count_sparse(seq, k, canonical=bool(canonical))
            assert np.array_equal(got[g][0], wc)
            assert np.array_equal(got[g][1], wn)


@pytest.mark.parametrize("k,canonical", [(21, 1), (19, 0), (27, 1)])
def test_sparse_dev_repeats(ctx, dev, oracle_lib, k, canonical):
    """Random genomes carrying repeats: 60 copies of a 2 kbp segment and 3000 of a 37 bp unit
    (k-mers counted 60 to ~6000 times).  Their bins hold more keys than a thread compares, so
    they go through the count kernel's LDS hash table beside ordinary keys of the same bins;
    a 9-copy segment stays on the comparison path."""
    rng = np.random.default_rng(500 + k)
    seg = osynth.synth_bases(2000, osynth.genome_seed(71))
    unit = osynth.synth_bases(37, osynth.genome_seed(72))
    small = osynth.synth_bases(900, osynth.genome_seed(73))
    parts = []
    for i in range(60):
        parts.append(osynth.synth_bases(int(rng.integers(500, 20_000)), osynth.genome_seed(1000 + i)))
        parts.append(seg)
        if i % 6 == 0:
            parts.append(small)
    a = np.concatenate(parts + [np.tile(unit, 3000)])
    b = np.concatenate([osynth.synth_bases(700_000, osynth.genome_seed(74)), np.tile(seg, 5), a[:50_000]])
    got = _sparse_dev(ctx, dev, [a, b], k, canonical)
    for g, seq in enumerate((a, b)):
        wc, wn, _ = oracle_lib.count_sparse(seq, k, canonical=bool(canonical))
        assert wn.max() >= (60 if g == 0 else 5)
        assert got[g][0].size == wc.size
        assert np.array_equal(got[g][0], wc) and np.array_equal(got[g][1], wn)


def test_sparse_dev_config5_genome(ctx, dev, oracle_lib):
    """One 25 Mbp synthetic genome (a tenth of a config-5 genome) at k = 21 canonical."""
    seq = osynth.synth_bases(25_000_000, osynth.genome_seed(0))
    got = _sparse_dev(ctx, dev, [seq], 21, 1)[0]
    wc, wn, _ = oracle_lib.count_sparse(seq, 21, canonical=True)
    assert got[0].size == wc.size
    assert np.array_equal(got[0], wc) and np.array_equal(got[1], wn)


@pytest.mark.parametrize("k,canonical", [(25, 1), (32, 0)])
def test_sparse_dev_long_k_genome(ctx, dev, oracle_lib, k, canonical):
    """The u64-residue hash path on a 12 Mbp synthetic genome plus a second one that shares a
    4 Mbp stretch with it (every k-mer of the stretch counted twice per genome pair)."""
    a = osynth.synth_bases(12_000_000, osynth.genome_seed(40 + k))
    b = np.concatenate([a[2_000_000:6_000_000], osynth.synth_bases(3_000_000, osynth.genome_seed(90))])
    got = _sparse_dev(ctx, dev, [a, b], k, canonical)
    for g, seq in enumerate((a, b)):
        wc, wn, _ = oracle_lib.count_sparse(seq, k, canonical=bool(canonical))
        assert got[g][0].size == wc.size
        assert np.array_equal(got[g][0], wc) and np.array_equal(got[g][1], wn)


def test_sparse_dev_multi_batch_long_k(ctx, dev, oracle_lib, monkeypatch):
    """u64 residues with one genome per batch and capped tables."""
    rng = np.random.default_rng(13)
    genomes = _ragged_genomes(rng, [300_000, 70_001, 150_000])
    want = [oracle_lib.count_sparse(s, 30, canonical=False)[:2] for s in genomes]
    monkeypatch.setenv("KMH_SP_BUDGET_MB", "1")
    for limit in ("16384", "50"):
        monkeypatch.setenv("KMH_SP_LIMIT", limit)
        got = _sparse_dev(ctx, dev, genomes, 30, 0)
        for g in range(len(genomes)):
            assert np.array_equal(got[g][0], want[g][0]), (limit, g)
            assert np.array_equal(got[g][1], want[g][1]), (limit, g)


@pytest.mark.parametrize("k", [12, 33])
def test_sparse_dev_rejects_k(ctx, dev, k):
    d = torch.zeros(64, dtype=torch.uint8, device=dev)
    o = torch.zeros(8, dtype=torch.int64, device=dev)
    with pytest.raises(NotImplementedError):
        ctx.count_sparse_dev(d.data_ptr(), np.array([0, 64], np.uint64), k, 0, o.data_ptr(), o.data_ptr(),
                             o.data_ptr())


# ---------------------------------------------------------------- RCCL code paths, one GPU
def _torchrun(args, timeout=600, nproc=1, env=None, gib_per_rank=4):
    import gc
    import socket
    import subprocess
    import sys
    # the ranks share this process's GPU: hand back what earlier tests left in torch's
    # caching allocator (the config-5 batch tests cache ~100 GB), or eight ranks of config 4
    # (~22 GiB each) run out of the 288 GB; the library's contexts cache tens of GB more
    _native.release_all()
    gc.collect()
    torch.cuda.empty_cache()
    # ... and refuse to start ranks that cannot fit (a rank that still runs out reports its own
    # allocation failure and hipMemGetInfo: kmerml.utils.devmem.run_guarded)
    free, total = torch.cuda.mem_get_info()
    need = nproc * gib_per_rank * 2**30
    assert free >= need, (f"{nproc} ranks need ~{nproc * gib_per_rank} GiB of device memory; "
                          f"free {free / 2**30:.1f} of {total / 2**30:.1f} GiB before launch")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env,
                          cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _failure(r):
    """The first rank traceback of a failed torchrun (the launcher's own report follows it and
    would push it out of a plain tail), then the tail."""
    err = r.stderr or ""
    i = err.find("Traceback")
    head = err[i:i + 4000] if i >= 0 else ""
    return head + "\n...\n" + err[-1500:]


def test_count_matrix_rccl_assembly(tmp_path, oracle_lib):
    """count_matrix under an RCCL process group (world size 1 on the test box): encode u4 +
    escapes, all-reduce, all-gather, decode -- bit-identical to counting directly."""
    files = []
    for i in range(3):
        p = tmp_path / f"g{i}.fa"
        seq = osynth.synth_bases(200_000 + 1000 * i, osynth.genome_seed(i)).tobytes()
        if i == 1:   # a k-mer repeated > 255 times: exercises the escape list
            seq = b"ACGTTGCA" * 2000 + seq
        osynth.write_fasta(p, [(f"SYN_{i}", seq)])
        files.append(str(p))
    out = tmp_path / "m.npy"
    here = os.path.dirname(os.path.abspath(__file__))
    r = _torchrun([os.path.join(here, "rccl_probe.py"), str(out), "8"] + files)
    assert r.returncode == 0, _failure(r)
    got = np.load(out).view(np.uint32)
    want = np.stack([kmatrix._hip_count_block([f], 8, 0).cpu().numpy().view(np.uint32)[0] for f in files])
    assert got.shape == want.shape and got.max() > 255
    assert np.array_equal(got, want)


@pytest.mark.parametrize("backend,nproc", [("nccl", 1), ("gloo", 2), ("gloo", 3)])
def test_count_genome_split(tmp_path, oracle_lib, backend, nproc):
    """One genome counted by several ranks (slices + (k - 1)-byte halos on the GPU, all-reduce of
    the rows; RCCL with one rank, gloo with 2-3 ranks sharing cuda:0): every rank's row equals
    the oracle's count of the whole genome (3 records incl. lowercase, N runs, a short record)."""
    seq = osynth.synth_bases(3_000_017, osynth.genome_seed(5)).tobytes()
    recs = [("a", seq[:1_000_000].lower()), ("b", b"ACGTN" * 3), ("c", seq[1_000_000:2_000_000] + b"NN" + seq[2_000_000:])]
    fa = tmp_path / "g.fa"
    osynth.write_fasta(fa, recs)
    here = os.path.dirname(os.path.abspath(__file__))
    r = _torchrun([os.path.join(here, "split_probe.py"), str(tmp_path), "12", str(fa), backend], nproc=nproc)
    assert r.returncode == 0, _failure(r)
    buf, _ = kmatrix.pack_genomes([str(fa)], 12)
    want = oracle_lib.count_dense(bytes(buf), 12)
    for q in range(nproc):
        got = np.load(tmp_path / f"row{q}.npy").view(np.uint32)
        assert np.array_equal(got, want)


def test_count_host_size_limits(ctx):
    """kmh_count_host rejects an organism of 2^32 - 1 bytes or more at any k before reading a
    byte (DESIGN.md 1 "Limits"; generate.py's docstring).  2^31 windows and more are counted
    (test_count_host_past_2_31_windows)."""
    import ctypes
    buf = np.zeros(64, np.uint8)      # the sizes below are claimed, never read
    out = ctypes.c_void_p()
    lib = _native.lib()
    for n, k in ((2**32 - 1, 21), (2**32 - 1, 12), (2**32, 4), (2**33, 40)):
        rc = lib.kmh_count_host(ctx._h, ctypes.c_void_p(buf.ctypes.data), n, k, 0, ctypes.byref(out))
        assert rc == _native.KMH_ERR_UNSUPPORTED, (n, k, rc)
        assert not out.value


def test_count_result_views_outlive_other_views(ctx):
    """ctx.count returns numpy views of the C result (kmh_kmers_data, no copy): one view stays
    valid after the others are dropped, the garbage collector runs and host memory is reused."""
    import gc
    seq = osynth.synth_bases(2_000_000, osynth.genome_seed(3)).tobytes()
    codes, counts, first = ctx.count(seq, 12)
    n = codes.size
    del codes, first
    gc.collect()
    junk = [np.ones(1 << 20, np.uint64) for _ in range(32)]
    assert counts.size == n and int(counts.sum(dtype=np.uint64)) == len(seq) - 12 + 1
    del junk


def test_context_shared_by_two_streams(ctx, dev, oracle_lib):
    """One context (the process-wide _native.context) used by two threads, each counting its
    own genomes on its own stream, dense k = 12 and sparse k = 21 interleaved: the _dev calls
    return before their kernels finish and share the context's cached workspace, so the C ABI
    orders a call behind the previous call's work on another stream (kmh_api.cpp on_stream).
    Every result matches the oracle."""
    import threading
    sets = [[osynth.synth_bases(3_000_000 + 4096 * i + 37 * t, osynth.genome_seed(40 + 4 * t + i))
             for i in range(3)] for t in range(2)]
    results, errors = [{}, {}], []

    def work(t):
        try:
            st = torch.cuda.Stream(device=dev)
            buf, offs = _layout(sets[t])
            with torch.cuda.stream(st):
                d_seq = torch.from_numpy(buf.copy()).to(dev, non_blocking=False)
                out_off = _native.sparse_out_offsets(offs, 21)
                for rep in range(3):
                    out = torch.full((3, 1 << 24), -7, dtype=torch.int32, device=dev)
                    ctx.count_dense_dev(d_seq.data_ptr(), offs, 12, out.data_ptr(), st.cuda_stream)
                    d_codes = torch.empty(int(out_off[-1]), dtype=torch.int64, device=dev)
                    d_counts = torch.empty(int(out_off[-1]), dtype=torch.int32, device=dev)
                    d_nk = torch.empty(3, dtype=torch.int64, device=dev)
                    ctx.count_sparse_dev(d_seq.data_ptr(), offs, 21, 1, d_codes.data_ptr(), d_counts.data_ptr(),
                                         d_nk.data_ptr(), st.cuda_stream)
                    results[t][rep] = (out, d_codes, d_counts, d_nk)
            st.synchronize()
        except Exception as e:   # noqa: BLE001 -- reported by the main thread
            errors.append(e)

    threads = [threading.Thread(target=work, args=(t,)) for t in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    assert not errors, errors
    torch.cuda.synchronize()
    for t in range(2):
        buf, offs = _layout(sets[t])
        out_off = _native.sparse_out_offsets(offs, 21)
        for rep in range(3):
            out, d_codes, d_counts, d_nk = results[t][rep]
            rows = out.cpu().numpy().view(np.uint32)
            codes = d_codes.cpu().numpy().view(np.uint64)
            counts = d_counts.cpu().numpy().view(np.uint32)
            nk = d_nk.cpu().numpy()
            for g, seq in enumerate(sets[t]):
                assert np.array_equal(rows[g], oracle_lib.count_dense(seq, 12)), (t, rep, g)
                a, n = int(out_off[g]), int(nk[g])
                o = np.argsort(codes[a:a + n], kind="stable")
                wc, wn, _ = oracle_lib.count_sparse(seq, 21, canonical=True)
                assert np.array_equal(codes[a:a + n][o], wc), (t, rep, g)
                assert np.array_equal(counts[a:a + n][o], wn), (t, rep, g)


def test_bench_pipelined_u8_assembly_rccl():
    """bench.py's pipelined u8 all-gather path (the N > 1 default) through RCCL, one rank."""
    r = _torchrun(["bench.py", "--assemble", "u8", "--genomes", "3", "--genome-len", "3000000",
                   "--steps", "3", "--warmup", "1", "--cpu-sample", "0"])
    assert r.returncode == 0, _failure(r)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["rows_checked"] is True and d["config"]["assembly"] == "u8"


def test_bench_pipelined_u4_assembly_rccl():
    """bench.py's pipelined u4 all-gather path (the N > 1 default) through RCCL, one rank."""
    r = _torchrun(["bench.py", "--assemble", "u4", "--genomes", "3", "--genome-len", "3000000",
                   "--steps", "3", "--warmup", "1", "--cpu-sample", "0"])
    assert r.returncode == 0, _failure(r)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["rows_checked"] is True and d["config"]["assembly"] == "u4"
    assert d["allgather"]["allgather_ms"] > 0 and d["allgather"]["received_bytes_per_rank"] == 0


@pytest.mark.parametrize("wire", ["u4", "u4-dense", "u8"])
def test_bench_pipelined_assembly_two_ranks(wire):
    """Two ranks on the one GPU (gloo for the collectives, --single-device): every rank widens
    the other rank's slot, so the assembled matrices pass the row-sum check only if decoding,
    escapes and the double-buffered pipeline are right (6 Mbp at k = 10 averages ~5.7 per bin:
    ~0.1 % of the cells reach 15 and travel in the u4 escape list)."""
    r = _torchrun(["bench.py", "--gpus", "2", "--backend", "gloo", "--single-device", "--assemble", wire,
                   "--genomes", "4", "--genome-len", "6000000", "--k", "10", "--steps", "3", "--warmup", "1",
                   "--cpu-sample", "0"], nproc=2)
    assert r.returncode == 0, _failure(r)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["rows_checked"] is True and d["n_gpus"] == 2 and d["config"]["assembly"] == wire
    ag = d["allgather"]                 # the assembly's all-gather reported on its own
    assert ag["allgather_ms"] > 0 and ag["received_bytes_per_rank"] == ag["slot_bytes"] > 0
    for key in ("received_GBs_per_gpu", "frac_of_7_links", "frac_of_peer_links"):
        assert ag[key] > 0, key


def test_rows_decode_u4_range(ctx, dev):
    """kmh_rows_decode_u4_range_dev (the AssembledMatrix row accessor): any row range of a u4
    block widens to exactly those rows, escapes included (values 15 .. 2^32 - 1)."""
    rng = np.random.default_rng(11)
    B, cols = 5, 2048
    rows = rng.poisson(6, size=(B, cols)).astype(np.uint32)
    rows[1, 7] = 15
    rows[3, 100] = 2**32 - 1
    rows[4, cols - 1] = 70_000
    d = torch.from_numpy(rows.view(np.int32)).to(dev)
    cap, P = kmatrix.slot_layout_u4(B, cols)
    slot = torch.zeros(P, dtype=torch.uint8, device=dev)
    nib = B * cols // 2
    ctx.rows_encode_u4(d.data_ptr(), B, cols, slot.data_ptr(), slot[nib + 16:].data_ptr(), cap, slot[nib:].data_ptr())
    for r0, n in [(0, 5), (1, 2), (4, 1), (3, 2), (2, 0)]:
        out = torch.full((max(n, 1), cols), -1, dtype=torch.int32, device=dev)
        ctx.rows_decode_u4_range(slot.data_ptr(), B, cols, slot[nib + 16:].data_ptr(), cap, slot[nib:].data_ptr(),
                                 r0, n, out.data_ptr())
        torch.cuda.synchronize()
        if n:
            assert np.array_equal(out.cpu().numpy().view(np.uint32), rows[r0:r0 + n])
    with pytest.raises(ValueError):
        ctx.rows_decode_u4_range(slot.data_ptr(), B, cols, slot[nib + 16:].data_ptr(), cap, slot[nib:].data_ptr(),
                                 4, 2, out.data_ptr())


@pytest.mark.parametrize("caps,wire", [({}, "u4"), ({"KMH_ESC_CAP_U4": "0"}, "u8")])
def test_assembled_matrix_compact_two_ranks(tmp_path, caps, wire):
    """count_matrix's compact form (AssembledMatrix: the gathered u4 slots, rows widened on
    access) on two ranks sharing the GPU: every row range equals the ranks' own rows; a forced
    u4 overflow wraps the u8 result instead."""
    env = dict(os.environ, **caps)
    here = os.path.dirname(os.path.abspath(__file__))
    r = _torchrun([os.path.join(here, "assembly_probe.py"), str(tmp_path), "5", "2000000", "10", "gloo",
                   "--single-device", "--compact"], nproc=2, timeout=300, env=env)
    assert r.returncode == 0, _failure(r)
    res = json.load(open(tmp_path / "result.json"))
    assert res == {"wire": wire, "assembly_checked": True, "world": 2}


def test_bench_simulated_rank():
    """bench.py --simulate-ranks: one process doing one rank's share of config 4 (compact u4
    assembly, the all-gather's writes modelled by device copies), labelled as a projection."""
    r = _torchrun(["bench.py", "--simulate-ranks", "4", "--genomes", "8", "--genome-len", "3000000",
                   "--steps", "3", "--warmup", "1", "--cpu-sample", "0"])
    assert r.returncode == 0, _failure(r)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["rows_checked"] is True and d["simulated_ranks"] == 4
    assert d["config"]["workload"].startswith("projection")


def test_bench_config5_object_two_ranks():
    """at N > 1 the dense line carries a config5 object -- every rank counts its
    genomes (k = 21 canonical) and the matrix leg's all-to-all runs in the compact wire -- and the
    global check (values summing to every window of every genome, column ranges in rank order)
    passes.  Two ranks sharing cuda:0 over gloo, at rehearsal sizes (labelled so)."""
    r = _torchrun(["bench.py", "--gpus", "2", "--backend", "gloo", "--single-device", "--genomes", "4",
                   "--genome-len", "3000000", "--k", "10", "--steps", "2", "--warmup", "1", "--cpu-sample", "0",
                   "--config5-genomes-per-rank", "2", "--config5-genome-len", "3000000", "--matrix-wire", "compact"],
                  nproc=2, timeout=600)
    assert r.returncode == 0, _failure(r)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    c5 = d["config5"]
    assert c5["rows_checked"] is True and c5["n_gpus"] == 2 and c5["config"]["workload"].startswith("rehearsal")
    mx = c5["matrix"]
    assert mx["shard_checked"] is True and mx["global"]["values"] == mx["global_windows"] == 4 * (3_000_000 - 20)
    ex = mx["exchange"]   # (3 Mbp genomes: gaps of ~7e5 codes, so nearly every gap is an escape; the
    # byte count of the compact wire on a full config-5 genome: test_wire_round_trip_config5_genome)
    assert ex["wire"] == "compact" and ex["sent_bytes"] > 0 and ex["received_bytes"] > 0, ex


def test_bench_sparse_simulated_rank():
    """bench.py --workload sparse --simulate-ranks N, one rank of config 5's matrix
    at N GPUs on one GPU: the other ranks' slices of its range really counted, packed and unpacked,
    the union at R = N x genomes rows, the shard checked (every entry of the range arrived, columns
    ascending and used); the line is labelled a projection and names the assumed link rate.  (30 Mbp
    genomes: gaps of ~8e4 codes in this range, so ~40 % of them are escapes.)"""
    r = _torchrun(["bench.py", "--workload", "sparse", "--simulate-ranks", "4", "--genomes", "2",
                   "--genome-len", "30000000", "--steps", "1"], timeout=600)
    assert r.returncode == 0, _failure(r)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["simulated_ranks"] == 4 and d["config"]["workload"].startswith("projection")
    assert d["shard"]["checked"] is True and d["shard"]["rows"] == 8
    ex = d["exchange"]
    assert ex["wire"] == "compact" and 0 < ex["received_bytes"] < ex["raw_received_bytes"]
    assert d["projected_ms_per_step"] > d["ms_per_step"] > 0


@pytest.mark.parametrize("k", [6, 10])
def test_from_count_matrix_gpu_equals_file_path(tmp_path, k):
    """Row f4 end to end: the GPU count matrix (kmerml.kmers.matrix.count_matrix, and its
    compact AssembledMatrix form under a one-rank group is covered by the assembly tests) fed
    through KmerFeatureBuilder.from_count_matrix gives the same count matrix as the reference's
    file route -- the drop-in KmerExtractor's k{k}.txt files -> KmerFeatureExtractor CSVs ->
    build_from_statistics_files (features.py:28-117, statistics.py:95-147)."""
    import contextlib as _cl
    import io as _io
    from kmerml.kmers.statistics import KmerFeatureExtractor
    from kmerml.ml.features import KmerFeatureBuilder
    kroot, fdir = tmp_path / "kmers", tmp_path / "features"
    files, orgs = [], []
    for i in range(3):
        org = f"GCF_00000{i}_s{i}"
        seq = osynth.synth_bases(40_000 + 9_000 * i, osynth.genome_seed(20 + i)).tobytes()
        if i == 1:
            seq = b"ACGTTGCA" * 500 + seq[:20_000].lower() + b"NNNN" + seq[20_000:]
        fa = tmp_path / f"{org}.fa"
        osynth.write_fasta(fa, [(org, seq), ("short", b"ACG")])
        files.append(str(fa))
        orgs.append(org)
        with _cl.redirect_stdout(_io.StringIO()):
            KmerExtractor(output_dir=str(kroot), compress=False).extract_kmers_from_fasta(str(fa), [k], organism_id=org)
    with _cl.redirect_stdout(_io.StringIO()):
        kf = find_files(str(kroot), patterns=["k*.txt"], recursive=True)
        KmerFeatureExtractor(input_paths=kf, output_dir=str(fdir)).extract_features()
        want = KmerFeatureBuilder(str(fdir)).build_from_statistics_files()
    m = kmatrix.count_matrix(files, k)
    got = KmerFeatureBuilder().from_count_matrix(m, k, list(want.index))
    assert list(want.index) == ["_".join(o.split("_")[:2]) for o in orgs]   # features.py:79-83
    assert got.to_csv() == want.to_csv()


def test_feature_table_on_gpu():
    """statistics.feature_table computed on the GPU (float64 divisions, products and the
    set-ordered entropy sums in torch on cuda) equals the host's label_features bit for bit."""
    from kmerml.kmers import statistics as st
    from kmerml.ml.features import KmerFeatureBuilder
    assert torch.cuda.is_available()
    st._TABLES.pop(9, None)
    t = st.feature_table(9)
    f = st.label_features(list(KmerFeatureBuilder.compat_labels(9)))
    for name, want in f.items():
        want = np.asarray(want)
        got = t[name]
        if want.dtype.kind == 'f':
            assert np.array_equal(got.view(np.int64), want.view(np.int64)), name
        else:
            assert np.array_equal(got, want), name


@pytest.mark.parametrize("k", [1, 4, 12, 15, 19])
def test_feature_columns_hip_kernel(k):
    """kmh_feature_columns_dev (csrc/kmh_features.hip: one thread per code, the reference's
    float64 operations rounded once each, the entropy in this interpreter's set() order) equals
    label_features on the same compat labels bit for bit: every code for k <= 4, random codes
    (with A...A, T...T and leading-A codes) at larger k.  Reference anchor: statistics.py:188-238."""
    from kmerml.kmers import statistics as st
    rng = np.random.default_rng(70 + k)
    if k <= 4:
        codes = np.arange(4 ** k, dtype=np.int64)
    else:
        codes = rng.integers(0, 4 ** k, 20_000, dtype=np.int64)
        codes[:4] = [0, 4 ** k - 1, 1, 4 ** (k - 3) + 6]
    got = st._code_features_hip(k, codes)
    labels = []
    for c in codes.tolist():
        s = "".join("ACGT"[(c >> (2 * (k - 1 - i))) & 3] for i in range(k)).lstrip("A") or "A"
        labels.append(s)
    want = st.label_features(labels)
    for name, w in want.items():
        w = np.asarray(w)
        g = got[name]
        if w.dtype.kind == "f":
            assert np.array_equal(g.view(np.int64), w.view(np.int64)), (k, name)
        else:
            assert np.array_equal(g, w), (k, name)


def _synth_row(oracle_lib, g, L=100_000_000, k=12, repeat=None):
    seq = oracle_lib.synth(L, osynth.genome_seed(g))
    if repeat:
        seq[:len(repeat)] = np.frombuffer(repeat, np.uint8)
    return oracle_lib.count_dense(seq, k)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("wire", ["u4", "u4-dense", "u8"])
def test_config4_per_rank_workload_eight_ranks(tmp_path, oracle_lib, wire):
    """Config 4 at its real per-rank size, eight ranks sharing the one MI355X (gloo for the
    collectives): 64 synthetic 100 Mbp genomes at k = 12, 8 per rank, every step's matrix
    assembled through the pipelined u4 (or u8) all-gather with ~176 K escapes per rank.  Every
    rank's assembled [64, 4^12] matrix must carry every rank's own count rows (row signatures
    after encode -> all-gather -> decode), and genomes 0 and 63 must equal the oracle's count
    (reference anchor: the organisms x k-mers matrix of features.py:85-117)."""
    r = _torchrun(["bench.py", "--gpus", "8", "--backend", "gloo", "--single-device", "--assemble", wire,
                   "--steps", "2", "--warmup", "1", "--cpu-sample", "0", "--check-dir", str(tmp_path)],
                  nproc=8, timeout=800, gib_per_rank=24)
    assert r.returncode == 0, _failure(r)
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert d["rows_checked"] is True and d["assembly_checked"] is True
    assert d["n_gpus"] == 8 and d["single_device"] is True and d["config"]["assembly"] == wire
    assert d["config"]["workload"].startswith("rehearsal")
    assert np.array_equal(np.load(tmp_path / "row_first.npy"), _synth_row(oracle_lib, 0))
    assert np.array_equal(np.load(tmp_path / "row_last.npy"), _synth_row(oracle_lib, 63))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("caps,wire", [({"KMH_ESC_CAP_U4": "1000"}, "u8"),
                                       ({"KMH_ESC_CAP_U4": "1000", "KMH_ESC_CAP_U8": "0"}, "u32"),
                                       ({}, "u4")])
def test_config4_assembly_fallbacks_full_size(tmp_path, oracle_lib, caps, wire):
    """The library's assembly (kmerml.kmers.matrix.gather_rows_u4) on config 4's per-rank
    workload, eight ranks on the one GPU: with the u4 escape capacity lowered below the ~176 K
    escapes of a rank's 8 x 4^12 block the all-reduced overflow sends every rank to u8, and with
    the u8 capacity at 0 on to the plain u32 all-gather -- each time the assembled matrix is still
    exact (own-row signatures on every rank, genomes 0 and 63 vs the oracle).  Genome 0 starts
    with a 1 Mbp period-8 repeat (counts up to ~125 000: escapes of u4 and u8 alike)."""
    env = dict(os.environ, **caps)
    here = os.path.dirname(os.path.abspath(__file__))
    r = _torchrun([os.path.join(here, "assembly_probe.py"), str(tmp_path), "64", "100000000", "12", "gloo",
                   "--single-device"], nproc=8, timeout=800, env=env, gib_per_rank=24)
    assert r.returncode == 0, _failure(r)
    res = json.load(open(tmp_path / "result.json"))
    assert res == {"wire": wire, "assembly_checked": True, "world": 8}
    rep = b"ACGTTGCA" * 125_000
    first = np.load(tmp_path / "row_first.npy")
    assert first.max() > 100_000
    assert np.array_equal(first, _synth_row(oracle_lib, 0, repeat=rep))
    assert np.array_equal(np.load(tmp_path / "row_last.npy"), _synth_row(oracle_lib, 63))


def test_sparse_dev_config5_full_genome(ctx, dev, oracle_lib):
    """One full config-5 genome: 250 Mbp synthetic genome 0, k = 21 canonical, every distinct
    k-mer and count against the C oracle (≈ 250 M sort pairs on the host, ≈ 9 GB)."""
    seq = oracle_lib.synth(250_000_000, osynth.genome_seed(0))
    got = _sparse_dev(ctx, dev, [seq], 21, 1)[0]
    wc, wn, _ = oracle_lib.count_sparse(seq, 21, canonical=True)
    assert got[0].size == wc.size
    assert np.array_equal(got[0], wc) and np.array_equal(got[1], wn)


def test_sparse_dev_config5_batched_plan(ctx, dev, oracle_lib):
    """The bench's per-GPU config-5 plan (bench.py --workload sparse): 16 synthetic 250 Mbp
    genomes generated on the device and counted at k = 21 canonical in ONE batch (the default
    16 GiB entry budget: one multi-genome item plan, output offsets of 16 genomes).  Every
    genome's distinct k-mers must sum to its windows; genomes 0 and 15 (first and last
    output ranges) are compared k-mer by k-mer with the C oracle.  Reference anchor: the dict
    of /root/reference/kmerml/kmers/generate.py:36,58."""
    L, G, k = 250_000_000, 16, 21
    s = torch.cuda.current_stream().cuda_stream
    d = torch.empty(G * L, dtype=torch.uint8, device=dev)
    ctx.synth_dev(d.data_ptr(), L, L, G, osynth.SEED_BASE, s)
    offs = np.arange(G + 1, dtype=np.uint64) * np.uint64(L)
    out_off = _native.sparse_out_offsets(offs, k)
    cap = int(out_off[-1])
    d_codes = torch.empty(cap, dtype=torch.int64, device=dev)
    d_counts = torch.empty(cap, dtype=torch.int32, device=dev)
    d_nk = torch.full((G,), -1, dtype=torch.int64, device=dev)
    ctx.count_sparse_dev(d.data_ptr(), offs, k, 1, d_codes.data_ptr(), d_counts.data_ptr(), d_nk.data_ptr(), s)
    torch.cuda.synchronize()
    del d
    nk = d_nk.cpu().numpy()
    for g in range(G):
        a, n = int(out_off[g]), int(nk[g])
        assert 0 < n <= int(out_off[g + 1]) - a, g
        assert int(d_counts[a:a + n].to(torch.int64).sum()) == L - k + 1, g
    for g in (0, G - 1):
        a, n = int(out_off[g]), int(nk[g])
        codes, order = torch.sort(d_codes[a:a + n])      # codes < 2^42: int64 order = u64 order
        counts = d_counts[a:a + n][order]
        got_c = codes.cpu().numpy().view(np.uint64)
        got_n = counts.cpu().numpy().view(np.uint32)
        del codes, order, counts
        wc, wn, _ = oracle_lib.count_sparse(oracle_lib.synth(L, osynth.genome_seed(g)), k, canonical=True)
        assert got_c.size == wc.size, g
        assert np.array_equal(got_c, wc) and np.array_equal(got_n, wn), g
        del wc, wn, got_c, got_n


@pytest.mark.parametrize("k,canonical", [(21, True), (9, False), (25, True), (32, False)])
def test_sparse_rows_from_fasta(tmp_path, oracle_lib, k, canonical):
    """kmerml.kmers.matrix.sparse_rows: FASTA files -> per-genome sorted sparse counts (the
    batched hash-table path for 13 <= k <= 32, per-genome GPU counts otherwise)."""
    files, seqs = [], []
    for i in range(3):
        p = tmp_path / f"g{i}.fa"
        seq = osynth.synth_bases(150_000 + 7_000 * i, osynth.genome_seed(10 + i)).tobytes()
        osynth.write_fasta(p, [(f"SYN_{i}", seq), (f"short_{i}", b"ACGT")])   # short record dropped
        files.append(str(p))
        seqs.append(seq)
    lo, rows = kmatrix.sparse_rows(files, k, canonical=canonical)
    assert lo == 0 and len(rows) == 3
    for (codes, counts), seq in zip(rows, seqs):
        wc, wn, _ = oracle_lib.count_sparse(np.frombuffer(seq, np.uint8), k, canonical=canonical)
        assert np.array_equal(codes, wc) and np.array_equal(counts, wn)


def test_dropin_workspace_trim_and_staging(ctx, oracle_lib, monkeypatch):
    """The drop-in's device-memory policy: one 250 Mbp organism
    counted at k = 21 and k = 12 through the drop-in's counting core (generate._count_all: one
    kmh_stage_host, one kmh_count_staged per k, then kmh_ctx_trim).  With a high mark the context
    keeps its workspace (tens of GB after k = 21); with the default-style mark it is released
    after the organism, so the serial loop of generate.py:116-126 does not hold it between
    genomes.  Counts are checked by their sums (every window of an all-ACGT genome)."""
    from kmerml.kmers import generate as kgen
    L = 250_000_000
    packed = oracle_lib.synth(L, osynth.genome_seed(3))
    kept = np.ones(1, bool)
    c = _native.context(0)
    c.release()
    monkeypatch.setenv("KMERML_WORKSPACE_MB", str(1 << 20))      # 1 TiB: nothing is released
    res = kgen._count_all(packed, kept, [21, 12])
    held = c.workspace_bytes()
    assert held > (4 << 30), held
    for k in (21, 12):
        codes, counts, first = res[k]
        assert int(counts.sum(dtype=np.uint64)) == L - k + 1
        assert first[0] == 0 and np.all(np.diff(first.astype(np.int64)) > 0)
    monkeypatch.setenv("KMERML_WORKSPACE_MB", "2048")
    res2 = kgen._count_all(packed, kept, [21])
    assert c.workspace_bytes() <= (2048 << 20)
    assert np.array_equal(res2[21][0], res[21][0]) and np.array_equal(res2[21][1], res[21][1])
    # the staging is gone with the workspace: counting it again must fail loudly, not read freed memory
    with pytest.raises(ValueError):
        c.count_staged(21)


@pytest.mark.parametrize("backend,nproc,k,canonical,wire,G", [
    ("nccl", 1, 21, True, "auto", 3), ("gloo", 2, 21, True, "auto", 3), ("gloo", 2, 21, True, "raw", 3),
    ("gloo", 3, 32, False, "auto", 2), ("gloo", 2, 32, False, "compact", 3), ("gloo", 4, 13, True, "compact", 5)])
def test_sparse_matrix_sharded_on_gpu(tmp_path, oracle_lib, backend, nproc, k, canonical, wire, G):
    """The column-sharded matrix on the GPU path:
    each rank's genomes counted in code order on the GPU (kmh_count_sparse_sorted_dev), the code
    space cut by the rows' device cuts, one all-to-all of the slices in the compact wire format
    (kmh_wire_encode/decode_dev) or raw, and kmh_shard_union_u32_dev (RCCL with one rank; gloo with
    2-4 ranks sharing cuda:0).  The shards side by side must equal the organisms x k-mers matrix of
    the oracle's counts (features.py:85-117's layout: sorted union of k-mers, missing = 0), and every
    rank's global check (shard_check: values summing to every window, ranks' column ranges in order)
    must pass.  Cases: repeated k-mers and a poly-A run (counts > 1 in escapes); k = 32 forward with a
    poly-T run (the code 2^64 - 1, the last top-16-bit bucket) at world 3 > G = 2, so that a rank
    holds no genome; k = 32 forced through the compact wire (every gap escaped); k = 13 at world 4."""
    files, rows, windows = [], [], 0
    for i in range(G):
        p = tmp_path / f"g{i}.fa"
        seq = osynth.synth_bases(120_000 + 9_000 * i, osynth.genome_seed(60 + i)).tobytes()
        if i == 2:
            seq = seq + seq[:30_000]   # k-mers counted twice
        if i == 1:
            seq = seq + b"A" * 5_000 + b"T" * 3_000   # counts of thousands; top-bucket codes
        osynth.write_fasta(p, [(f"SYN_{i}", seq)])
        files.append(str(p))
        windows += len(seq) - k + 1
        c, n, _ = oracle_lib.count_sparse(np.frombuffer(seq, np.uint8), k, canonical=canonical)
        rows.append((c, n))
    here = os.path.dirname(os.path.abspath(__file__))
    extra = (["--single-device"] if nproc > 1 else []) + ([] if canonical else ["--forward"])
    extra += ["--wire", wire, "--windows", str(windows)]
    r = _torchrun([os.path.join(here, "sparse_matrix_probe.py"), str(tmp_path), str(k), backend] + extra + files,
                  nproc=nproc, timeout=300)
    assert r.returncode == 0, _failure(r)
    cols = np.load(tmp_path / "columns.npy")
    vals = np.load(tmp_path / "values.npy")
    want_cols = np.unique(np.concatenate([c for c, _ in rows]))
    assert np.array_equal(cols, want_cols)
    want = np.zeros((G, want_cols.size), np.int64)
    for g, (c, n) in enumerate(rows):
        want[g, np.searchsorted(want_cols, c)] = n
    assert np.array_equal(vals, want) and vals.max() >= 2
    checks = [json.load(open(tmp_path / f"check_{q}.json")) for q in range(nproc)]
    assert all(c["ok"] for c in checks), checks
    assert all(c["index_dtype"] == "torch.int32" for c in checks), checks
    if nproc > 1:
        ex = [c["exchange"] for c in checks]
        assert len({e["wire"] for e in ex}) == 1, ex
        # (auto: the smaller format -- raw for these small genomes, whose gaps are mostly escapes)
        assert ex[0]["wire"] == wire if wire != "auto" else sum(e["sent_bytes"] for e in ex) <= sum(
            e["raw_sent_bytes"] for e in ex), ex
        assert sum(e["sent_bytes"] for e in ex) == sum(e["received_bytes"] for e in ex), ex
    if k == 32 and not canonical:
        assert want_cols[-1] == np.uint64(2**64 - 1)


def test_sparse_skewed_bucket_fallback_grouped(ctx, oracle_lib, monkeypatch):
    """a skewed organism whose largest bucket fails many passes must not run
    one gather + sort per failed pass.  A 1.5 Mbp A-rich stretch (90 % A) puts most of its windows
    in bucket 0 (first five bases AAAAA) -- ~600 passes at the drop-in's k = 22 pass target -- and
    KMH_SP_LIMIT = 64 fails every count item, so every pass goes to the exact fallback.  Failed
    passes are recounted per (genome, bucket): at most one group per bucket, far fewer than the
    passes, and the first-occurrence result equals the oracle's counts and first positions."""
    rng = np.random.default_rng(23)
    rich = np.where(rng.random(1_500_000) < 0.9, ord("A"), np.frombuffer(b"CGT", np.uint8)[rng.integers(0, 3, 1_500_000)])
    seq = np.concatenate([osynth.synth_bases(2_000_000, osynth.genome_seed(81)), rich.astype(np.uint8)])
    monkeypatch.setenv("KMH_SP_LIMIT", "64")
    before = ctx.stats()
    codes, counts, first = ctx.count(seq, 22)
    after = ctx.stats()
    passes = after["fallback_passes"] - before["fallback_passes"]
    groups = after["fallback_groups"] - before["fallback_groups"]
    assert 0 < groups <= 1024 and passes >= 400 + groups, (passes, groups)
    wc, wn, wf = oracle_lib.count_sparse(seq, 22, canonical=False)
    o = np.argsort(codes, kind="stable")
    assert np.array_equal(codes[o], wc) and np.array_equal(counts[o], wn) and np.array_equal(first[o], wf)
    assert np.all(np.diff(first.astype(np.int64)) > 0)


# ---------------------------------------------------------------- sorted rows and the column shard (config 5's matrix)
def _sparse_sorted(ctx, dev, genomes, k, canonical):
    """kmh_count_sparse_sorted_dev on host genomes -> per genome (codes, counts), after checking the
    row contract: rows back to back from entry 0 (row g starts after rows 0 .. g - 1), d_nrows[g] =
    d_ndistinct[g] entries (no padding since round 5: a distinct-count pass places every item),
    codes strictly ascending, every count nonzero, nothing written past the rows."""
    buf, offs = _layout(genomes)
    d_seq = torch.from_numpy(buf.copy()).to(dev)
    out_off = _native.sparse_out_offsets(offs, k)
    cap = max(int(out_off[-1]), 1)
    d_codes = torch.full((cap,), -1, dtype=torch.int64, device=dev)
    d_counts = torch.full((cap,), -7, dtype=torch.int32, device=dev)
    d_nr = torch.full((len(genomes),), -1, dtype=torch.int64, device=dev)
    d_nd = torch.full((len(genomes),), -1, dtype=torch.int64, device=dev)
    ctx.count_sparse_sorted_dev(d_seq.data_ptr(), offs, k, canonical, d_codes.data_ptr(), d_counts.data_ptr(),
                                d_nr.data_ptr(), d_nd.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    nr, nd = d_nr.cpu().numpy(), d_nd.cpu().numpy()
    codes = d_codes.cpu().numpy().view(np.uint64)
    counts = d_counts.cpu().numpy().view(np.uint32)
    res = []
    a = 0
    assert np.all(counts[int(nr.sum()):] == np.uint32(0xFFFFFFF9))   # (the -7 fill)
    for g in range(len(genomes)):
        n = int(nr[g])
        assert 0 <= n == int(nd[g]) <= int(out_off[g + 1]) - int(out_off[g]), g
        c, m = codes[a:a + n], counts[a:a + n]
        a += n
        assert np.all(c[1:] > c[:-1]), g                   # distinct k-mers strictly ascending
        assert np.all(m != 0), g
        res.append((c, m))
    return res


@pytest.mark.parametrize("k,canonical", [(13, 0), (17, 1), (21, 0), (21, 1), (22, 1), (27, 0), (32, 1)])
def test_sparse_sorted_dev_vs_oracle(ctx, dev, oracle_lib, k, canonical):
    """kmh_count_sparse_sorted_dev (the rows of the config-5 matrix): every genome's distinct
    k-mers and counts in code order, equal to the C oracle's sorted output, on ragged genomes
    (lowercase, N, '-', newlines, an empty genome, genomes shorter than k)."""
    rng = np.random.default_rng(900 + k * 2 + canonical)
    genomes = _ragged_genomes(rng, [400_000, 32768 + 21, 1_000_003, 17])
    got = _sparse_sorted(ctx, dev, genomes, k, canonical)
    for g, seq in enumerate(genomes):
        wc, wn, _ = oracle_lib.count_sparse(seq, k, canonical=bool(canonical))
        assert np.array_equal(got[g][0], wc), g
        assert np.array_equal(got[g][1], wn), g


@pytest.mark.parametrize("k", [21, 27])
def test_sparse_sorted_dev_fallback_and_repeats(ctx, dev, oracle_lib, monkeypatch, k):
    """The sorted rows when passes fail: tables capped so that most passes go to the sort
    fallback (counted in the distinct-count pass, then its runs placed in their passes' ranges in
    order), repeats whose big bins fail an item in sorted mode, one genome per batch (rows back to
    back across batches), and low-complexity genomes."""
    rng = np.random.default_rng(77 + k)
    seg = osynth.synth_bases(2000, osynth.genome_seed(71))
    parts = []
    for i in range(30):
        parts.append(osynth.synth_bases(int(rng.integers(500, 20_000)), osynth.genome_seed(2000 + i)))
        parts.append(seg)
    genomes = _ragged_genomes(rng, [600_000, 70_001]) + [
        np.concatenate(parts), np.full(100_000, ord("A"), np.uint8),
        np.frombuffer(b"ACGTTTGACCA" * 20_000, np.uint8).copy()]
    want = [oracle_lib.count_sparse(s, k, canonical=True)[:2] for s in genomes]
    for env in ({}, {"KMH_SP_TARGET": "37", "KMH_SP_LIMIT": "12288"}, {"KMH_SP_TARGET": "100000", "KMH_SP_LIMIT": "40"},
                {"KMH_SP_BUDGET_MB": "1", "KMH_SP_LIMIT": "50"}):
        for key in ("KMH_SP_TARGET", "KMH_SP_LIMIT", "KMH_SP_BUDGET_MB"):
            monkeypatch.delenv(key, raising=False)
        for key, v in env.items():
            monkeypatch.setenv(key, v)
        got = _sparse_sorted(ctx, dev, genomes, k, 1)
        for g in range(len(genomes)):
            assert np.array_equal(got[g][0], want[g][0]), (env, g)
            assert np.array_equal(got[g][1], want[g][1]), (env, g)


def _shard_union(ctx, dev, rows, lo, hi_incl):
    """kmh_shard_union_dev over host rows (sorted uint64 arrays) -> (columns, indices per row)."""
    roff = np.zeros(len(rows) + 1, np.uint64)
    roff[1:] = np.cumsum([r.size for r in rows])
    allc = np.concatenate(rows) if rows else np.zeros(0, np.uint64)
    d = torch.from_numpy(np.ascontiguousarray(allc).view(np.int64).copy()).to(dev)
    cols = torch.full((max(allc.size, 1),), -1, dtype=torch.int64, device=dev)
    idx = torch.full((max(allc.size, 1),), -1, dtype=torch.int64, device=dev)
    n = ctx.shard_union_dev(d.data_ptr(), roff, lo, hi_incl, cols.data_ptr(), idx.data_ptr(),
                            torch.cuda.current_stream().cuda_stream)
    c = cols[:n].cpu().numpy().view(np.uint64)
    ix = idx.cpu().numpy()
    return c, [ix[int(roff[r]):int(roff[r + 1])] for r in range(len(rows))]


@pytest.mark.parametrize("case", ["distinct", "shared", "identical", "mixed", "narrow", "wide", "many_rows", "dense_cell",
                                  "max_rows", "slot_rows64", "rows200", "cell_top"])
def test_shard_union_vs_numpy(ctx, dev, case):
    """kmh_shard_union_dev (the column union and CSR indices of a shard) against numpy's
    union1d / searchsorted: rows of distinct codes (the LDS path), rows sharing half their codes,
    100 identical rows (every bin over its limit: the radix-sort fallback for every unit; rows
    found by binary search, R > 64), a mixture with empty rows, a narrow code range (units of one
    code), the whole 64-bit code space (coarse cells of 2^48 codes: u64 offsets in the union),
    600 rows (R > 512: row starts read without prefetch), one dense cluster of codes inside a
    sparse range (a coarse cell cut into many units) and the API's 4096 rows (row offsets past the
    first 1024 read from memory; ~74 KiB of dynamic LDS beside the static tables).  slot_rows64
    (VERDICT r05 item 4): R = 64, the largest row count whose gathered entries find their rows
    through the 64-entry slot table, with one dense window cut into ~120 units whose row pieces
    range from ~20 entries (inside one slot) to ~500 (spanning 7-8 slots, starting at every offset
    of a slot) -- the shape of the only case (dense_cell) that failed the first slot-table build;
    rows200: 200 rows sharing a pool of codes (the slot table beyond 64 rows, up to its 256).
    cell_top: a 2^48-code range (coarse cells of 2^32 codes, u32 offsets) whose sparse cells are
    single units holding their last code, offset 2^32 - 1 -- the one offset the sizes pass's hash
    set cannot store as offset + 1 (counted apart), shared by two rows."""
    rng = np.random.default_rng({"distinct": 1, "shared": 2, "identical": 3, "mixed": 4, "narrow": 5, "wide": 6,
                                 "many_rows": 7, "dense_cell": 8, "max_rows": 9, "slot_rows64": 10, "rows200": 11,
                                 "cell_top": 12}[case])
    lo, hi = 1 << 40, (1 << 41) - 1
    if case == "distinct":
        rows = [np.unique(rng.integers(lo, hi, 200_000, dtype=np.uint64)) for _ in range(7)]
    elif case == "shared":
        base = rng.integers(lo, hi, 300_000, dtype=np.uint64)
        rows = [np.unique(np.concatenate([base[:150_000], rng.integers(lo, hi, 150_000, dtype=np.uint64)]))
                for _ in range(5)]
    elif case == "identical":
        one = np.unique(rng.integers(lo, hi, 50_000, dtype=np.uint64))
        rows = [one.copy() for _ in range(100)]
    elif case == "mixed":
        one = np.unique(rng.integers(lo, hi, 30_000, dtype=np.uint64))
        rows = [np.zeros(0, np.uint64), one, np.unique(rng.integers(lo, hi, 90_000, dtype=np.uint64))] + \
               [one.copy() for _ in range(40)] + [np.zeros(0, np.uint64)]
    elif case == "narrow":
        lo, hi = 5_000_000, 5_003_999
        rows = [np.unique(rng.integers(lo, hi + 1, 3_000, dtype=np.uint64)) for _ in range(9)]
    elif case == "wide":
        lo, hi = 0, (1 << 64) - 1
        rows = [np.unique(rng.integers(0, 1 << 63, 150_000, dtype=np.uint64) * np.uint64(2) + np.uint64(r % 2))
                for r in range(6)]
        rows[0] = np.unique(np.concatenate([rows[0], np.array([0, hi], np.uint64)]))   # both ends of the range
    elif case == "many_rows":
        pool = rng.integers(lo, hi, 200_000, dtype=np.uint64)
        rows = [np.unique(rng.choice(pool, 500)) for _ in range(600)]
    elif case == "max_rows":
        pool = rng.integers(lo, hi, 100_000, dtype=np.uint64)
        rows = [np.unique(rng.choice(pool, 40)) for _ in range(4096)]
        rows[4000] = np.zeros(0, np.uint64)
    elif case == "rows200":   # R = 200: the slot table's rows past 64 (config 5's N = 8 shard has 128)
        pool = rng.integers(lo, hi, 3_000_000, dtype=np.uint64)
        rows = [np.unique(rng.choice(pool, 1_000 + 37 * r)) for r in range(200)]
    elif case == "cell_top":
        lo, hi = 0, (1 << 48) - 1
        tops = np.array([(c << 32) - 1 for c in range(1, 40)], np.uint64)   # each cell's last code
        rows = [np.unique(np.concatenate([tops[r::2], rng.integers(lo, hi, 3_000, dtype=np.uint64)])) for r in range(2)]
        rows.append(np.unique(np.concatenate([tops, rng.integers(lo, hi, 2_000, dtype=np.uint64)])))
    elif case == "slot_rows64":
        win = lo + (1 << 39) + np.arange(1 << 22, dtype=np.uint64)
        sizes = [40_000 if r % 10 == 0 else 2_000 + 500 * (r % 9) for r in range(64)]
        rows = [np.unique(np.concatenate([rng.choice(win, n, replace=False), rng.integers(lo, hi, 300, dtype=np.uint64)]))
                for n in sizes]
    else:   # dense_cell: 400 K codes in a 1 M-code window of a 2^40 range, plus a sparse background
        dense = lo + (1 << 39) + rng.integers(0, 1 << 20, 400_000, dtype=np.uint64)
        rows = [np.unique(np.concatenate([dense[r::3], rng.integers(lo, hi, 5_000, dtype=np.uint64)])) for r in range(3)]
    cols, idx = _shard_union(ctx, dev, rows, lo, hi)
    want = np.unique(np.concatenate(rows))
    assert np.array_equal(cols, want)
    for r, row in enumerate(rows):
        assert np.array_equal(idx[r], np.searchsorted(want, row)), r


def test_sparse_matrix_two_config5_genomes(tmp_path, ctx, dev, oracle_lib):
    """the device-resident matrix of two full config-5 genomes (250 Mbp
    synthetic genomes 0 and 1, k = 21 canonical): sparse_matrix's shard (sorted rows on the GPU,
    kmh_shard_union_dev) against the C oracle's counts -- columns strictly ascending and every one
    used, and for each genome columns[indices] = its k-mers and values = their counts."""
    seqs = [oracle_lib.synth(250_000_000, osynth.genome_seed(g)) for g in range(2)]
    files = []
    for g, seq in enumerate(seqs):
        p = tmp_path / f"SYN_{g:04d}.fa"
        osynth.write_fasta(p, [(f"SYN_{g:04d}", seq.tobytes())], width=1 << 30)
        files.append(str(p))
    m = kmatrix.sparse_matrix(files, 21, canonical=True, device=0)
    assert m.on_device and m.G == 2 and m.lo_code == 0 and m.hi_code == 1 << 42
    cols = m.columns
    assert bool(torch.all(cols[1:] > cols[:-1]).item())
    assert m.indices.dtype == torch.int32   # u32 indices (fewer than 2^32 - 1 entries)
    assert m.all_columns_used()
    for g, seq in enumerate(seqs):
        wc, wn, _ = oracle_lib.count_sparse(seq, 21, canonical=True)
        a, b = int(m.indptr[g]), int(m.indptr[g + 1])
        assert b - a == wc.size
        got_c = cols[m.column_indices(a, b)].cpu().numpy().view(np.uint64)
        assert np.array_equal(got_c, wc)
        assert np.array_equal(m.values[a:b].cpu().numpy().view(np.uint32), wn)
        del wc, wn


# ---------------------------------------------------------------- the config-5 exchange wire (kmh_wire.hip)
def _wire_encode_np(codes, counts):
    """Restatement of the compact wire format of one slice (include/kmerhip.h, kmh_wire.hip header):
    per 1024 entries a 2320-byte record [u64 first code][u32 first escape word][u32 escape words |
    wide << 31][u16 low 16 bits of every gap][bitmap: gap >> 16 != 0][bitmap: count != 1], then the
    slice's escape words in entry order (gap >> 16 in one word, two in a wide chunk -- one with a
    gap of 2^48 or more -- then a count that is not 1), zero-padded to 16 bytes."""
    n = codes.size
    recs, words = [], []
    for c0 in range(0, n, 1024):
        c = codes[c0:c0 + 1024].astype(np.uint64)
        m = counts[c0:c0 + 1024].astype(np.uint32)
        gap = np.zeros(1024, np.uint64)
        gap[1:c.size] = c[1:] - c[:-1]
        cn = np.ones(1024, np.uint32)
        cn[:c.size] = m
        hi = gap >> np.uint64(16)
        hf, cf = hi != 0, cn != 1
        wide = bool(np.any(hi >> np.uint64(32)))
        w0 = len(words)
        for i in np.nonzero(hf | cf)[0]:
            if hf[i]:
                words.append(int(hi[i]) & 0xFFFFFFFF)
                if wide:
                    words.append(int(hi[i]) >> 32)
            if cf[i]:
                words.append(int(cn[i]))
        head = np.array([c[0]], np.uint64).tobytes() + np.array(
            [w0, (len(words) - w0) | (int(wide) << 31)], np.uint32).tobytes()
        recs.append(head + (gap & np.uint64(0xFFFF)).astype(np.uint16).tobytes()
                    + np.packbits(hf, bitorder="little").tobytes() + np.packbits(cf, bitorder="little").tobytes())
    words += [0] * (-len(words) % 4)
    return b"".join(recs) + np.array(words, np.uint32).tobytes()


def _wire_round_trip(ctx, dev, codes, counts, cuts):
    """Slices of (codes, counts) between consecutive cuts: sized, packed, unpacked in reverse slice
    order into a fresh buffer; returns (packed bytes, unpacked codes, unpacked counts, slice bytes)."""
    d_c = torch.from_numpy(codes.view(np.int64).copy()).to(dev)
    d_n = torch.from_numpy(counts.view(np.int32).copy()).to(dev)
    st = np.array(cuts[:-1], np.uint64)
    sn = np.diff(np.array(cuts, np.uint64))
    s = torch.cuda.current_stream().cuda_stream
    sb = ctx.wire_size_dev(d_c.data_ptr(), d_n.data_ptr(), st, sn, s)
    tot = int(sb.sum())
    out = torch.full((max(tot, 16),), 0xA5, dtype=torch.uint8, device=dev)
    ctx.wire_encode_dev(d_c.data_ptr(), d_n.data_ptr(), st, sn, out.data_ptr(), tot, s)
    packed = out[:tot].cpu().numpy().tobytes()
    # decode the slices in reverse order from a buffer that holds them reversed
    boff = np.concatenate([[0], np.cumsum(sb)]).astype(np.int64)
    rev = b"".join(packed[boff[i]:boff[i + 1]] for i in reversed(range(sn.size)))
    d_in = torch.from_numpy(np.frombuffer(rev, np.uint8).copy()).to(dev) if rev else torch.zeros(16, dtype=torch.uint8,
                                                                                                  device=dev)
    rc = torch.full((max(codes.size, 1),), -1, dtype=torch.int64, device=dev)
    rn = torch.full((max(codes.size, 1),), -1, dtype=torch.int32, device=dev)
    ctx.wire_decode_dev(d_in.data_ptr(), len(rev), sn[::-1].copy(), sb[::-1].copy(), st[::-1].copy(), rc.data_ptr(),
                        rn.data_ptr(), s)
    torch.cuda.synchronize()
    return (packed, rc[:codes.size].cpu().numpy().view(np.uint64), rn[:codes.size].cpu().numpy().view(np.uint32), sb)


@pytest.mark.parametrize("case", ["k21_ragged", "repeats", "k32_wide", "tiny"])
def test_wire_round_trip_small(ctx, dev, oracle_lib, case):
    """The compact wire on small slices: the packed bytes equal the numpy
    restatement of the format byte for byte, and decoding (slices in another order, other
    destinations) gives the exact codes and counts back.  Cases: k = 21 canonical rows of ragged
    genomes; a repeat-rich genome with poly-A (counts up to ~10^5, every count escaped); k = 32
    forward codes (gaps of ~2^46: every gap escaped, wide chunks where one reaches 2^48) with a poly-T run (code
    2^64 - 1); slices of 0, 1, 1023, 1024 and 1025 entries."""
    rng = np.random.default_rng({"k21_ragged": 1, "repeats": 2, "k32_wide": 3, "tiny": 4}[case])
    if case == "k21_ragged":
        seq, k, canon = _ragged_genomes(rng, [300_000])[0], 21, True
    elif case == "repeats":
        unit = osynth.synth_bases(3000, osynth.genome_seed(5))
        seq, k, canon = np.concatenate([np.tile(unit, 30), np.full(100_000, ord("A"), np.uint8)]), 21, True
    elif case == "k32_wide":
        seq = np.concatenate([osynth.synth_bases(200_000, osynth.genome_seed(6)), np.full(500, ord("T"), np.uint8)])
        k, canon = 32, False
    else:
        seq, k, canon = osynth.synth_bases(3_300, osynth.genome_seed(7)), 21, True
    codes, counts, _ = oracle_lib.count_sparse(seq, k, canonical=canon)
    n = codes.size
    cuts = sorted({0, n, n // 3, n // 3, 2 * n // 3 + 5 if 2 * n // 3 + 5 < n else n})
    if case == "tiny":
        cuts = [0, 0, 1, 1024, 2048, 3072, 3073, n]
    packed, rc, rn, sb = _wire_round_trip(ctx, dev, codes, counts, cuts)
    want = b"".join(_wire_encode_np(codes[a:b], counts[a:b]) for a, b in zip(cuts[:-1], cuts[1:]))
    assert packed == want
    assert np.array_equal(rc, codes) and np.array_equal(rn, counts)
    if case == "k32_wide":
        assert codes[-1] == np.uint64(2**64 - 1) and sb.sum() > 6 * n   # every gap escaped


def test_wire_round_trip_config5_genome(ctx, dev, oracle_lib):
    """The compact wire on a full config-5 genome's sorted row (250 Mbp synthetic genome 0, k = 21
    canonical, ~2.5e8 entries from kmh_count_sparse_sorted_dev) cut into the 8 slices an N = 8 run
    sends: exact round trip against the uncompressed row, and the packed size (the VERDICT r05
    target: ~2-2.5 B per entry against 12)."""
    seq = oracle_lib.synth(250_000_000, osynth.genome_seed(0))
    buf, offs = _layout([seq])
    d_seq = torch.from_numpy(buf).to(dev)
    cap = int(_native.sparse_out_offsets(offs, 21)[-1])
    d_c = torch.empty(cap, dtype=torch.int64, device=dev)
    d_n = torch.empty(cap, dtype=torch.int32, device=dev)
    nr = torch.empty(1, dtype=torch.int64, device=dev)
    nd = torch.empty(1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ctx.count_sparse_sorted_dev(d_seq.data_ptr(), offs, 21, 1, d_c.data_ptr(), d_n.data_ptr(), nr.data_ptr(),
                                nd.data_ptr(), s)
    n = int(nr.item())
    del d_seq
    roff = np.array([0, n], np.uint64)
    hist = kmatrix._row_histogram(d_c, roff, 21).cpu().numpy()
    assert int(hist.sum()) == n
    bounds = kmatrix._splitters_from_hist(hist, 21, 8)
    send_len, starts = kmatrix.shard_plan(d_c, roff, bounds, 0)
    assert int(send_len.sum()) == n and np.all(send_len > n // 10)
    st, sn = starts[0].astype(np.uint64), send_len[0].astype(np.uint64)
    sb = ctx.wire_size_dev(d_c.data_ptr(), d_n.data_ptr(), st, sn, s)
    tot = int(sb.sum())
    out = torch.empty(tot, dtype=torch.uint8, device=dev)
    ctx.wire_encode_dev(d_c.data_ptr(), d_n.data_ptr(), st, sn, out.data_ptr(), tot, s)
    rc = torch.empty(n, dtype=torch.int64, device=dev)
    rn = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.wire_decode_dev(out.data_ptr(), tot, sn, sb, st, rc.data_ptr(), rn.data_ptr(), s)
    assert torch.equal(rc, d_c[:n]) and torch.equal(rn, d_n[:n])
    per = tot / n
    print(f"config-5 genome 0: {n} entries, {tot} bytes packed = {per:.3f} B per entry")
    assert per < 2.5, per
