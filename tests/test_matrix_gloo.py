"""CPU: the multi-GPU assembly path (shard genomes by rank, all-gather the rows) with the
gloo backend and world_size 2, counting with the oracle in place of the HIP kernel."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kmerml.kmers import matrix as kmatrix


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_counter(files, k):
    from oracle import corac
    from oracle import fasta as ofasta
    rows = []
    for f in files:
        recs = [s for _, _, s in ofasta.parse_fasta(f) if len(s) >= k]
        packed = "".join(s + "\n" for s in recs).encode()
        rows.append(corac.count_dense(packed, k).view(np.int32))
    return torch.from_numpy(np.stack(rows)) if rows else torch.zeros((0, 1 << (2 * k)), dtype=torch.int32)


def _worker(rank, world, port, files, k, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "kmer-ml_amd"), os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = kmatrix.count_matrix(files, k, count_fn=_oracle_counter)
        np.save(os.path.join(outdir, f"rank{rank}.npy"), m.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_genomes", [5, 1])
def test_count_matrix_gloo_world2(tmp_path, oracle_lib, n_genomes):
    from oracle import synth as osynth
    files = []
    for i in range(n_genomes):
        p = tmp_path / f"g{i}.fa"
        osynth.write_fasta(p, [(f"SYN_{i}", osynth.synth_bases(3000 + 17 * i, osynth.genome_seed(i)).tobytes())])
        files.append(str(p))
    mp.spawn(_worker, args=(2, _free_port(), files, 6, str(tmp_path)), nprocs=2, join=True)
    want = _oracle_counter(files, 6).numpy()
    for r in range(2):
        got = np.load(tmp_path / f"rank{r}.npy")
        assert got.shape == want.shape
        assert np.array_equal(got, want)


def test_shard_bounds_cover_in_order():
    for G in range(0, 20):
        for W in (1, 2, 3, 8):
            spans = [kmatrix.shard_bounds(G, W, r) for r in range(W)]
            assert spans[0][0] == 0 and spans[-1][1] == G
            assert all(spans[i][1] == spans[i + 1][0] for i in range(W - 1))
            assert all(hi - lo <= kmatrix.block_rows(G, W) for lo, hi in spans)


def _oracle_slice_counter(sl, k):
    from oracle import corac
    return torch.from_numpy(corac.count_dense(bytes(sl), k).view(np.int32).copy())


def _split_worker(rank, world, port, path, k, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "kmer-ml_amd"), os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        row = kmatrix.count_genome_split(path, k, count_fn=_oracle_slice_counter)
        np.save(os.path.join(outdir, f"split{rank}.npy"), row.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,n", [(2, 6, 5000), (3, 12, 4099), (3, 4, 20)])
def test_count_genome_split_gloo(tmp_path, oracle_lib, world, k, n):
    """One genome split across ranks with a (k - 1)-byte halo + all-reduce(SUM): every rank's
    row equals the whole genome counted at once (records, lowercase, N runs, a record shorter
    than k, a genome too short for some ranks to own a window)."""
    from oracle import corac
    from oracle import fasta as ofasta
    from oracle import synth as osynth
    seq = osynth.synth_bases(n, osynth.genome_seed(7)).tobytes()
    mid = len(seq) // 2
    recs = [("r1", seq[:mid].lower() + b"NNNN" + seq[mid:mid + 10]), ("r2", b"ACG"), ("r3", seq[mid:])]
    path = tmp_path / "g.fa"
    osynth.write_fasta(path, recs)
    mp.spawn(_split_worker, args=(world, _free_port(), str(path), k, str(tmp_path)), nprocs=world, join=True)
    kept = [s for _, _, s in ofasta.parse_fasta(str(path)) if len(s) >= k]
    want = corac.count_dense("".join(s + "\n" for s in kept).encode(), k)
    for r in range(world):
        got = np.load(tmp_path / f"split{r}.npy").view(np.uint32)
        assert np.array_equal(got, want)


def test_split_bounds_count_every_window_once():
    for n in range(0, 300, 7):
        for W in (1, 2, 3, 8):
            for k in (1, 5, 12):
                seen = np.zeros(max(n - k + 1, 0), np.int64)
                for r in range(W):
                    a, b, e = kmatrix.split_bounds(n, W, r, k)
                    assert a % 16 == 0 and a <= b <= n and e <= n
                    for s in range(a, b):
                        if s + k <= e:
                            seen[s] += 1
                        else:
                            assert s + k > n
                assert np.all(seen == 1)


def _sparse_rows_oracle(files, k):
    """Forward-strand sparse rows of each FASTA file from the C oracle (sorted by code)."""
    from oracle import corac
    from oracle import fasta as ofasta
    rows = []
    for f in files:
        recs = [s for _, _, s in ofasta.parse_fasta(f) if len(s) >= k]
        packed = "".join(s.upper() + "\n" for s in recs).encode()
        c, n, _ = corac.count_sparse(np.frombuffer(packed, np.uint8), k, canonical=False)
        rows.append((c, n))
    return rows


def _sparse_worker(rank, world, port, files, orgs, k, outdir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "kmer-ml_amd"), os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = kmatrix.sparse_matrix(files, k, canonical=False, rows_fn=lambda fs: _sparse_rows_oracle(fs, k))
        shards = [None] * world
        dist.all_gather_object(shards, m)
        assert [s.rank for s in shards] == list(range(world))
        assert all(shards[q].hi_code == shards[q + 1].lo_code for q in range(world - 1))
        if rank == 0:
            df = kmatrix.ShardedSparseMatrix.to_frame(shards, orgs)
            df.to_csv(os.path.join(outdir, f"sharded_k{k}.csv"))
            with open(os.path.join(outdir, f"nnz_k{k}.txt"), "w") as f:
                f.write(" ".join(str(s.nnz) for s in shards))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,k,G", [(2, 13, 3), (2, 21, 3), (3, 21, 5), (4, 32, 5), (3, 32, 2)])
def test_sparse_matrix_column_sharded_gloo(tmp_path, oracle_lib, world, k, G):
    """Config 5's matrix: each of `world` ranks counts its block of genomes, the code
    space is cut into `world` ranges of ~equal entries and one all-to-all-v (gloo here, RCCL on the
    GPUs) gives each rank every organism's counts in its range.  The shards, put side by side,
    equal the reference's matrix built from the per-organism files: k{k}.txt (the restated
    generate.py writer) -> KmerFeatureExtractor CSVs -> KmerFeatureBuilder.build_from_statistics_
    files (features.py:28-117: sorted union of labels, missing = 0; k = 13 has the integer-parsed,
    A-stripped labels, k = 21 the exact k-mer text).  k = 32 with a poly-T run puts the code
    2^64 - 1 in the top histogram bucket, and world 3 > G = 2 leaves a rank without genomes."""
    import contextlib
    import io
    from oracle import kmers as okmers
    from oracle import synth as osynth
    from kmerml.kmers.statistics import KmerFeatureExtractor
    from kmerml.ml.features import KmerFeatureBuilder
    from kmerml.utils.path_utils import find_files
    kroot, fdir = tmp_path / "kmers", tmp_path / "features"
    files, orgs = [], []
    for i in range(G):
        org = f"GCF_00000{i}"
        seq = osynth.synth_bases(2500 + 700 * i, osynth.genome_seed(30 + i)).tobytes().decode()
        if i == 1:   # shared stretch (counts > 1 across and within organisms), lowercase, N run
            seq = seq[:600] + seq[:600].lower() + "NNNNN" + seq[600:]
        if i == 2:
            seq = seq + "ACGTTGCA" * 40
        if i == 1 and k == 32:   # TTT...T: the code 2^64 - 1, in the histogram's last bucket
            seq = seq + "T" * 50
        fa = tmp_path / f"{org}.fa"
        osynth.write_fasta(fa, [(org, seq.encode()), ("short", b"ACGTA")])
        files.append(str(fa))
        orgs.append(org)
        table = okmers.count_records([(org, seq), ("short", "ACGTA")], [k])[k]
        (kroot / org).mkdir(parents=True)
        (kroot / org / f"k{k}.txt").write_text(okmers.kmer_text(table))
    with contextlib.redirect_stdout(io.StringIO()):
        kf = find_files(str(kroot), patterns=["k*.txt"], recursive=True)
        KmerFeatureExtractor(input_paths=kf, output_dir=str(fdir)).extract_features()
        want = KmerFeatureBuilder(str(fdir)).build_from_statistics_files()
    mp.spawn(_sparse_worker, args=(world, _free_port(), files, orgs, k, str(tmp_path)), nprocs=world, join=True)
    got = (tmp_path / f"sharded_k{k}.csv").read_text()
    assert list(want.index) == orgs
    assert got == want.to_csv()
    nnz = [int(x) for x in (tmp_path / f"nnz_k{k}.txt").read_text().split()]
    assert len(nnz) == world
    assert min(nnz) > 0.5 * sum(nnz) / world   # the code ranges balance the entries


def test_sparse_matrix_many_rows_takes_host_path(tmp_path, monkeypatch, oracle_lib):
    """kmh_shard_union_dev holds at most SHARD_MAX_ROWS organism rows, so a
    matrix with more organisms than that is routed to the host assembly (sparse_rows + the sorted
    union on the host), not to the device shard that would fail at its last step.  The limit is
    lowered to 2 here, with 3 genomes and the GPU counter replaced by the C oracle's rows."""
    from oracle import synth as osynth
    files = []
    for i in range(3):
        fa = tmp_path / f"g{i}.fa"
        osynth.write_fasta(fa, [(f"g{i}", osynth.synth_bases(3000, osynth.genome_seed(90 + i)).tobytes())])
        files.append(str(fa))
    monkeypatch.setattr(kmatrix, "SHARD_MAX_ROWS", 2)

    def no_device(*a, **k):
        raise AssertionError("the device shard was chosen for more rows than it holds")
    monkeypatch.setattr(kmatrix, "_sparse_matrix_dev", no_device)
    monkeypatch.setattr(kmatrix, "sparse_rows", lambda fs, k, canonical=True, device=None, group=None:
                        (0, _sparse_rows_oracle(fs, k)))
    m = kmatrix.sparse_matrix(files, 21, canonical=False)
    rows = _sparse_rows_oracle(files, 21)
    want = np.unique(np.concatenate([c for c, _ in rows]))
    assert m.G == 3 and np.array_equal(m.columns, want)
    for g, (c, n) in enumerate(rows):
        a, b = int(m.indptr[g]), int(m.indptr[g + 1])
        assert np.array_equal(m.columns[m.indices[a:b]], c) and np.array_equal(m.values[a:b], n)
