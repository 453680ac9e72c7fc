"""Helper for tests/test_gpu_parity.py (not a test module): run kmerml.kmers.matrix.count_matrix
under a torch.distributed process group ("nccl" = RCCL) launched by torch.distributed.run, and
save this rank's matrix.  Usage: rccl_probe.py OUT.npy K FASTA..."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "kmer-ml_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from kmerml.kmers.matrix import count_matrix  # noqa: E402


def main():
    out, k, files = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    try:
        m = count_matrix(files, k)
        torch.cuda.synchronize()
        np.save(out, m.cpu().numpy())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    from kmerml.utils.devmem import run_guarded
    run_guarded(main)
