"""Helper for tests/test_gpu_parity.py (not a test module): count ONE genome split across the
ranks of a torch.distributed.run launch (kmerml.kmers.matrix.count_genome_split: slice + halo on
the GPU, all-reduce of the rows) and save each rank's row.
Usage: split_probe.py OUTDIR K FASTA BACKEND   (BACKEND "nccl" = RCCL; "gloo" puts every rank on
cuda:0 so that two ranks can share the test box's one GPU)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "kmer-ml_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kmerml.kmers.matrix import count_genome_split  # noqa: E402


def main():
    outdir, k, fasta, backend = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    rank = int(os.environ.get("RANK", "0"))
    dev = 0 if backend == "gloo" else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo")
    try:
        row = count_genome_split(fasta, k, device=dev)
        torch.cuda.synchronize()
        np.save(os.path.join(outdir, f"row{rank}.npy"), row.cpu().numpy())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    from kmerml.utils.devmem import run_guarded
    run_guarded(main)
