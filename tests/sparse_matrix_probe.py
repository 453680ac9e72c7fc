"""Helper for tests/test_gpu_parity.py (not a test module): kmerml.kmers.matrix.sparse_matrix
under torch.distributed.run -- each rank counts its genomes on the GPU (the batched hash-table
path), the code space is cut into ranges and one all-to-all-v (RCCL, or gloo with every rank on
cuda:0) assembles each rank's column shard.  Rank 0 writes every shard's dense block in rank
order, and every rank's global check (kmerml.kmers.matrix.shard_check) and exchange record go to
check_<rank>.json.  Usage: sparse_matrix_probe.py OUTDIR K BACKEND [--single-device] [--forward]
[--wire auto|compact|raw] [--windows N] FASTA...  (--windows: the total windows of the genomes, for
the global sum check)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "kmer-ml_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kmerml.kmers import matrix as kmatrix  # noqa: E402


def main():
    outdir, k, backend = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    args = sys.argv[4:]
    single = "--single-device" in args
    forward = "--forward" in args
    wire, windows, files, i = "auto", None, [], 0
    while i < len(args):
        if args[i] == "--wire":
            wire, i = args[i + 1], i + 2
        elif args[i] == "--windows":
            windows, i = int(args[i + 1]), i + 2
        else:
            if args[i] not in ("--single-device", "--forward"):
                files.append(args[i])
            i += 1
    local = 0 if single else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    try:
        lo, codes, counts, roff = kmatrix.sorted_rows_dev(files, k, canonical=not forward, device=local)
        m = kmatrix.shard_from_rows(codes, counts, roff, len(files), k, wire=wire)
        del codes, counts
        ok, summ = kmatrix.shard_check(m, windows if windows is not None else -1)
        with open(os.path.join(outdir, f"check_{dist.get_rank()}.json"), "w") as f:
            json.dump({"ok": ok, "summary": summ, "exchange": kmatrix.LAST_EXCHANGE, "lo_code": m.lo_code,
                       "hi_code": m.hi_code, "index_dtype": str(m.indices.dtype)}, f)
        shards = [None] * dist.get_world_size()
        dist.all_gather_object(shards, m)
        if dist.get_rank() == 0:
            np.save(os.path.join(outdir, "columns.npy"), np.concatenate([s.columns for s in shards]))
            np.save(os.path.join(outdir, "values.npy"), np.concatenate([s.dense() for s in shards], axis=1))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    from kmerml.utils.devmem import run_guarded
    run_guarded(main)
