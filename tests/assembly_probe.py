"""Helper for tests/test_gpu_parity.py (not a test module): config 4's per-rank assembly through
the library path kmerml.kmers.matrix.gather_rows_u4 (u4 -> u8 -> u32 fallbacks) under
torch.distributed.run.  Every rank generates its block of G synthetic genomes of L bases on the
device (the bench's genomes), counts them at k, assembles the matrix, and checks it against every
rank's own rows (bench.check_assembly); rank 0 writes result.json (wire format used, check
result) and the assembled rows of genomes 0 and G - 1.  The first REPEAT_BYTES of genome 0
are overwritten with a period-8 repeat (REPEAT), so its block has counts far above 255 (u8 and
u4 escapes with large values).
--compact keeps the matrix in the AssembledMatrix form (u4 slots, rows widened on access).
Usage: assembly_probe.py OUT_DIR G L K BACKEND [--single-device] [--compact]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "kmer-ml_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import SEED_BASE, check_assembly  # noqa: E402
from kmerml import _native  # noqa: E402
from kmerml.kmers import matrix as kmatrix  # noqa: E402


REPEAT = b"ACGTTGCA"
REPEAT_BYTES = 1_000_000


def main():
    out, G, L, k, backend = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    single = "--single-device" in sys.argv
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_index = 0 if single else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    try:
        world, rank = dist.get_world_size(), dist.get_rank()
        lo, hi = kmatrix.shard_bounds(G, world, rank)
        B = kmatrix.block_rows(G, world)
        bins = 1 << (2 * k)
        ctx = _native.context(dev_index)
        s = torch.cuda.current_stream(dev).cuda_stream
        stride = (L + 15) // 16 * 16
        d_seq = torch.full((max(hi - lo, 1) * stride,), ord("N"), dtype=torch.uint8, device=dev)
        padded = torch.zeros((B, bins), dtype=torch.int32, device=dev)
        if hi > lo:
            ctx.synth_dev(d_seq.data_ptr(), L, stride, hi - lo, SEED_BASE + lo, s)
            if lo == 0:
                rep = np.frombuffer(REPEAT * (REPEAT_BYTES // len(REPEAT)), dtype=np.uint8)
                d_seq[:rep.size].copy_(torch.from_numpy(rep.copy()))
            offsets = np.arange(hi - lo + 1, dtype=np.uint64) * np.uint64(stride)
            ctx.count_dense_dev(d_seq.data_ptr(), offsets, k, padded.data_ptr(), s)
        del d_seq
        if "--compact" in sys.argv:
            am = kmatrix.gather_rows_u4(padded, None, compact=True, G=G)
            assert am.shape == (G, bins)
            full = torch.zeros((world * B, bins), dtype=torch.int32, device=dev)
            for q in range(world):
                qlo, qhi = kmatrix.shard_bounds(G, world, q)
                full[q * B:q * B + (qhi - qlo)] = am.rows(qlo, qhi)
            # single rows and a range across a slot boundary agree with the block widening
            assert torch.equal(am.row(G - 1), full[(world - 1) * B + (G - 1 - kmatrix.shard_bounds(G, world, world - 1)[0])])
            if G >= 2:
                mid = kmatrix.shard_bounds(G, world, 0)[1]
                a0, a1 = max(0, mid - 1), min(G, mid + 1)
                assert torch.equal(am.rows(a0, a1), torch.cat([am.row(g)[None] for g in range(a0, a1)]))
        else:
            full = kmatrix.gather_rows_u4(padded, None)
        torch.cuda.synchronize()
        ok = check_assembly(full, padded[:hi - lo], B, G, world, rank, k, out)
        okt = torch.tensor([int(ok)], dtype=torch.int32)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        if rank == 0:
            with open(os.path.join(out, "result.json"), "w") as f:
                json.dump({"wire": kmatrix.LAST_WIRE, "assembly_checked": bool(okt.item()), "world": world}, f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    from kmerml.utils.devmem import run_guarded
    run_guarded(main)
