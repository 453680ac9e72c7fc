"""PCIe-inclusive rates of the host-buffer boundary: genome bytes in host memory,
counts back in host memory, k = 12, synthetic 100 Mbp genomes.

    python profiles/pcie_r01.py [--genomes 16]

1. pageable: kmh_count_dense_host (one genome per call: H2D, count, D2H of the 4^12 row);
2. pinned: G genomes in pinned host memory -> one H2D, kmh_count_dense_dev on the batch, one D2H
   of the [G, 4^12] rows into pinned memory.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "kmer-ml_amd"), os.path.dirname(HERE)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from kmerml import _native  # noqa: E402

SEED_BASE = 0x6B6D65724D4C0000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genomes", type=int, default=16)
    a = ap.parse_args()
    L, k, G = 100_000_000, 12, a.genomes
    dev = torch.device("cuda", 0)
    ctx = _native.context(0)
    s = torch.cuda.current_stream().cuda_stream
    d_seq = torch.empty(G * L, dtype=torch.uint8, device=dev)
    ctx.synth_dev(d_seq.data_ptr(), L, L, G, SEED_BASE, s)
    h_seq = torch.empty(G * L, dtype=torch.uint8, pin_memory=True)
    h_seq.copy_(d_seq)
    torch.cuda.synchronize()
    one = h_seq[:L].numpy().copy()            # pageable copy of genome 0

    # 1. pageable, one genome per call
    ctx.count_dense(one, k)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        row = ctx.count_dense(one, k)
        ts.append(time.perf_counter() - t0)
    assert int(row.sum()) == L - k + 1
    t = float(np.median(ts))
    print(json.dumps({"path": "pageable kmh_count_dense_host", "genomes": 1, "s_per_genome": t,
                      "bases_per_s": L / t}), flush=True)

    # 2. pinned batch
    out = torch.empty((G, 1 << (2 * k)), dtype=torch.int32, device=dev)
    h_out = torch.empty((G, 1 << (2 * k)), dtype=torch.int32, pin_memory=True)
    offs = np.arange(G + 1, dtype=np.uint64) * np.uint64(L)

    def run():
        d_seq.copy_(h_seq, non_blocking=True)
        ctx.count_dense_dev(d_seq.data_ptr(), offs, k, out.data_ptr(), s)
        h_out.copy_(out, non_blocking=True)
        torch.cuda.synchronize()

    run()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        run()
        ts.append(time.perf_counter() - t0)
    assert bool((h_out.sum(1, dtype=torch.int64) == L - k + 1).all())
    t = float(np.median(ts))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ctx.count_dense_dev(d_seq.data_ptr(), offs, k, out.data_ptr(), s)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"path": "pinned batch: H2D + kmh_count_dense_dev + D2H", "genomes": G,
                      "s_per_batch": t, "bases_per_s": G * L / t, "h2d_bytes": G * L,
                      "d2h_bytes": G * (4 << (2 * k)), "count_only_ms": e0.elapsed_time(e1)}), flush=True)


if __name__ == "__main__":
    main()
