"""u4 / u8 + escape row encode / decode throughput (the multi-GPU assembly kernels):
8 count rows of synthetic 100 Mbp genomes at k = 12 (a rank's block at N = 8), round trip
checked, HIP events on the launch stream; KMH_U4_OLD=1 selects the per-thread-contiguous
kernels for the A/B.

    python profiles/u4_r01.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "kmer-ml_amd"), os.path.dirname(HERE)]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from kmerml import _native  # noqa: E402
from kmerml.kmers.matrix import slot_layout, slot_layout_u4  # noqa: E402

SEED_BASE = 0x6B6D65724D4C0000


def main():
    L, k, B = 100_000_000, 12, 8
    cols = 1 << (2 * k)
    dev = torch.device("cuda", 0)
    ctx = _native.context(0)
    s = torch.cuda.current_stream().cuda_stream
    d_seq = torch.empty(B * L, dtype=torch.uint8, device=dev)
    ctx.synth_dev(d_seq.data_ptr(), L, L, B, SEED_BASE, s)
    rows = torch.empty((B, cols), dtype=torch.int32, device=dev)
    ctx.count_dense_dev(d_seq.data_ptr(), np.arange(B + 1, dtype=np.uint64) * np.uint64(L), k, rows.data_ptr(), s)
    del d_seq
    cap, P = slot_layout_u4(B, cols)
    nib = B * cols // 2
    slot = torch.zeros(P, dtype=torch.uint8, device=dev)
    back = torch.empty_like(rows)
    cells = B * cols
    for variant in ("new", "old"):
        if variant == "old":
            os.environ["KMH_U4_OLD"] = "1"
        else:
            os.environ.pop("KMH_U4_OLD", None)
        te, td = [], []
        for it in range(8):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            ctx.rows_encode_u4(rows.data_ptr(), B, cols, slot.data_ptr(), slot[nib + 16:].data_ptr(), cap,
                               slot[nib:].data_ptr(), s)
            e1.record()
            ctx.rows_decode_u4(slot.data_ptr(), B, cols, slot[nib + 16:].data_ptr(), cap, slot[nib:].data_ptr(),
                               back.data_ptr(), s)
            e2.record()
            torch.cuda.synchronize()
            if it >= 2:
                te.append(e0.elapsed_time(e1))
                td.append(e1.elapsed_time(e2))
        ok = bool(torch.equal(rows, back))
        nesc = int(slot[nib:nib + 4].view(torch.int32).item())
        me, md = float(np.median(te)), float(np.median(td))
        print(json.dumps({"variant": variant, "rows": B, "cols": cols, "escapes": nesc, "cap": cap,
                          "round_trip_exact": ok, "encode_ms": me, "decode_ms": md,
                          "encode_GBs": cells * 4.5 / me / 1e6, "decode_GBs": cells * 4.5 / md / 1e6}), flush=True)
        back.zero_()
        # u8 + escapes (the fallback wire format)
        cap8, P8 = slot_layout(B, cols)
        slot8 = torch.zeros(P8, dtype=torch.uint8, device=dev)
        te, td = [], []
        for it in range(8):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            ctx.rows_encode_u8(rows.data_ptr(), B, cols, slot8.data_ptr(), slot8[cells + 16:].data_ptr(), cap8,
                               slot8[cells:].data_ptr(), s)
            e1.record()
            ctx.rows_decode_u8(slot8.data_ptr(), B, cols, slot8[cells + 16:].data_ptr(), cap8, slot8[cells:].data_ptr(),
                               1, B, back.data_ptr(), s)
            e2.record()
            torch.cuda.synchronize()
            if it >= 2:
                te.append(e0.elapsed_time(e1))
                td.append(e1.elapsed_time(e2))
        me, md = float(np.median(te)), float(np.median(td))
        print(json.dumps({"variant": variant, "wire": "u8", "round_trip_exact": bool(torch.equal(rows, back)),
                          "encode_ms": me, "decode_ms": md, "encode_GBs": cells * 5 / me / 1e6,
                          "decode_GBs": cells * 5 / md / 1e6}), flush=True)
        back.zero_()
        del slot8


if __name__ == "__main__":
    main()
