"""One simulated config-4 rank (8 x 100 Mbp, k = 12, fused count + u4 slot): consecutive steps on
one context and stream vs alternating between two contexts on two streams (step i+1's partition
may start while step i's count runs), with and without the all-gather's writes modelled as 7
device copies of the slot.  usage: python3 profiles/r05/overlap_steps.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "kmer-ml_amd"))
from kmerml import _native  # noqa: E402
from kmerml.kmers.matrix import slot_layout_u4  # noqa: E402

G, L, k, SPAN = 8, 100_000_000, 12, 8
bins = 1 << (2 * k)
dev = torch.device("cuda", 0)
ctxs = [_native.context(0), _native.context(0)]
streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
side = torch.cuda.Stream(dev)
stride = (L + 15) // 16 * 16
d_seq = torch.empty(G * stride, dtype=torch.uint8, device=dev)
ctxs[0].synth_dev(d_seq.data_ptr(), L, stride, G, 1000, streams[0].cuda_stream)
offsets = np.arange(G + 1, dtype=np.uint64) * np.uint64(stride)
cap, P = slot_layout_u4(G, bins)
payload = G * bins // 2
locs = [torch.zeros((G, bins), dtype=torch.int32, device=dev) for _ in range(2)]
recv = [torch.zeros(SPAN * P, dtype=torch.uint8, device=dev) for _ in range(2)]
torch.cuda.synchronize()


def run(nctx, copies, steps=20, warmup=3):
    inflight = [None, None]

    def step(i):
        b = i % 2
        c = ctxs[i % nctx]
        st = streams[i % nctx]
        if inflight[b] is not None:
            st.wait_event(inflight[b])
            inflight[b] = None
        sb = recv[b][:P]
        c.count_dense_u4_dev(d_seq.data_ptr(), offsets, k, locs[i % nctx].data_ptr(), sb.data_ptr(),
                             sb[payload + 16:].data_ptr(), cap, sb[payload:].data_ptr(), st.cuda_stream, rows=False)
        side.wait_stream(st)
        with torch.cuda.stream(side):
            if copies:
                for q in range(1, SPAN):
                    recv[b][q * P:(q + 1) * P].copy_(sb)
            ev = torch.cuda.Event()
            ev.record(side)
        inflight[b] = ev

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        step(i)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    # every slot of the last step's buffer holds a full count (the u4 nibbles sum is not cheap to
    # check; the escape count must be within its cap)
    esc = int(recv[(warmup + steps - 1) % 2][payload:payload + 4].view(torch.int32).item())
    return ms, esc


for rep in range(2):
    for nctx in (1, 2):
        for copies in (False, True):
            ms, esc = run(nctx, copies)
            print(f"contexts {nctx} copies {int(copies)}: {ms:.4f} ms/step (escapes {esc})", flush=True)
