"""Times kmh_shard_union_dev alone on 16 synthetic sorted rows of 250 M random k = 21 codes (the
config-5 matrix's shard at W = 1), for A/B builds of the library (KMH_LIB_PATH).
usage: KMH_LIB_PATH=build_ab/<v>/libkmerhip.so python3 profiles/r05/time_union.py <label>"""
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
gen = torch.Generator(device=dev)
gen.manual_seed(5)
rows = []
for g in range(G):
    r = torch.randint(0, 4 ** k, (L,), dtype=torch.int64, device=dev, generator=gen)
    rows.append(torch.unique(r, sorted=True))
    del r
roff = np.zeros(G + 1, np.uint64)
roff[1:] = np.cumsum([r.numel() for r in rows])
codes = torch.cat(rows)
del rows
n = codes.numel()
cols = torch.empty(n, dtype=torch.int64, device=dev)
idx = torch.empty(n, dtype=torch.int64, device=dev)
torch.cuda.synchronize()
out = []
for rep in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nc = ctx.shard_union_dev(codes.data_ptr(), roff, 0, 4 ** k - 1, cols.data_ptr(), idx.data_ptr(), s)
    torch.cuda.synchronize()
    out.append((time.perf_counter() - t0) * 1e3)
chk = int(idx[:: 9973].sum().item()) if True else 0
print(f"{sys.argv[1] if len(sys.argv) > 1 else '?'}: entries {n} columns {nc} ms {' '.join(f'{x:.1f}' for x in out)} "
      f"idxsum {chk} colsum {int(cols[:nc:9973].sum().item())}", flush=True)
