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
