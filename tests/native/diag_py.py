"""Staged diagnostic of the Python -> ctypes -> HIP path (prints after every stage)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "kmer-ml_amd"), REPO]
T0 = time.time()


def say(msg):
    print(f"[{time.time() - T0:7.2f}s] {msg}", flush=True)


mode = sys.argv[1] if len(sys.argv) > 1 else "torch-first"
if mode == "torch-first":
    import torch
    say(f"torch {torch.__version__} hip {torch.version.hip} avail={torch.cuda.is_available()}")
    x = torch.zeros(1024, device="cuda")
    torch.cuda.synchronize()
    say("torch tensor ok")
import numpy as np
from kmerml import _native
_native.lib()
say("lib loaded")
ctx = _native.Context(0)
say("ctx ok")
rng = np.random.default_rng(0)
seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 100_000)]
for k in (4, 8, 12):
    c = ctx.count_dense(seq, k)
    say(f"count_dense host k={k} sum={int(c.sum())} expect={100_000 - k + 1}")
codes, counts, first = ctx.count(seq, 21)
say(f"count k=21 distinct={codes.size}")
if mode == "torch-first":
    import torch
    d = torch.empty(2 * 1_000_000, dtype=torch.uint8, device="cuda")
    ctx.synth_dev(d.data_ptr(), 1_000_000, 1_000_000, 2, 0x6B6D65724D4C0000, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    say("synth_dev ok")
    out = torch.zeros((2, 1 << 24), dtype=torch.int32, device="cuda")
    ctx.count_dense_dev(d.data_ptr(), np.array([0, 1_000_000, 2_000_000], np.uint64), 12, out.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    say(f"count_dense_dev k=12 sums={out.sum(1, dtype=torch.int64).tolist()}")
say("diag done")
