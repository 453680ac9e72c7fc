"""Phase clocks of k_sp_count (experiment build, KMH_SP_PROF=1) for the unordered count and the
count in code order (ORD) of the same 16 synthetic 250 Mbp genomes at k = 21 canonical.
usage: KMH_LIB_PATH=build_ab/exp/libkmerhip.so KMH_SP_PROF=1 python3 profiles/r05/prof_ord.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "kmer-ml_amd"))
from kmerml import _native  # noqa: E402

G, L, k = 16, 250_000_000, 21
dev = torch.device("cuda", 0)
ctx = _native.context(0)
s = torch.cuda.current_stream(dev).cuda_stream
stride = (L + 15) // 16 * 16
d_seq = torch.empty(G * stride, dtype=torch.uint8, device=dev)
ctx.synth_dev(d_seq.data_ptr(), L, stride, G, 1000, s)
offsets = np.arange(G + 1, dtype=np.uint64) * np.uint64(stride)
cap = int(_native.sparse_out_offsets(offsets, k)[-1])
codes = torch.empty(cap, dtype=torch.int64, device=dev)
counts = torch.empty(cap, dtype=torch.int32, device=dev)
nk = torch.zeros(G, dtype=torch.int64, device=dev)
nd = torch.zeros(G, dtype=torch.int64, device=dev)
for name in ("unordered", "ordered", "unordered", "ordered"):
    torch.cuda.synchronize()
    print(f"--- {name}", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    if name == "unordered":
        ctx.count_sparse_dev(d_seq.data_ptr(), offsets, k, 1, codes.data_ptr(), counts.data_ptr(), nk.data_ptr(), s)
    else:
        ctx.count_sparse_sorted_dev(d_seq.data_ptr(), offsets, k, 1, codes.data_ptr(), counts.data_ptr(), nk.data_ptr(),
                                    nd.data_ptr(), s)
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) * 1e3:.1f} ms", file=sys.stderr, flush=True)
