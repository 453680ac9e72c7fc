"""End-to-end timing of the drop-in KmerExtractor on
FASTA files: parse -> count on the GPU -> first-occurrence order -> text -> file.

    python profiles/e2e_r01.py [--mbp 100] [--out gpurun_out/e2e]

Cases: the 12.16 Mbp, 17-record yeast stand-in at k = 4 (BASELINE config 1) and k = 12, and a
synthetic single-record genome (default 100 Mbp) at k = 12, uncompressed and gzip.  Each case
is timed as a whole and per stage (parse, count, format, write).  The reference path's own
count loop is timed by bench.py's cpu_baseline; here only this implementation runs.
"""
import argparse
import io
import json
import os
import sys
import time
import contextlib

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "kmer-ml_amd"), REPO]

import numpy as np  # noqa: E402

from kmerml import _native  # noqa: E402
from kmerml.kmers.generate import KmerExtractor  # noqa: E402
from oracle import synth as osynth  # noqa: E402  (input generator only)


def stages(fasta, k):
    t = {}
    t0 = time.perf_counter()
    f = _native.FastaFile(fasta)
    packed, kept = f.pack(k)
    t["parse_s"] = time.perf_counter() - t0
    ctx = _native.context(0)
    t0 = time.perf_counter()
    codes, counts, _ = ctx.count(packed, k)
    t["count_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    text = _native.format_lines_array(k, codes, np.multiply(counts, np.uint64(1), dtype=np.uint64))
    t["format_s"] = time.perf_counter() - t0
    f.close()
    t["bases"] = int(packed.size)
    t["distinct"] = int(codes.size)
    t["text_MB"] = round(len(text) / 1e6, 1)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mbp", type=int, default=100)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "e2e"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    yeast = os.path.join(a.out, "yeast_standin.fa")
    osynth.write_fasta(yeast, osynth.yeast_standin_records())
    big = os.path.join(a.out, f"syn_{a.mbp}mbp.fa")
    osynth.write_fasta(big, [("SYN_0000", osynth.synth_bases(a.mbp * 1_000_000, osynth.genome_seed(0)).tobytes())])
    _native.context(0)  # initialise the device before timing
    results = []
    for fasta, k in ((yeast, 4), (yeast, 12), (big, 12)):
        for compress in (False, True):
            ext = KmerExtractor(output_dir=os.path.join(a.out, "kmers"), compress=compress)
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                ext.extract_kmers_from_fasta(fasta, [k], organism_id=f"e2e_{os.path.basename(fasta)}_{k}")
            dt = time.perf_counter() - t0
            r = {"fasta": os.path.basename(fasta), "k": k, "compress": compress, "total_s": round(dt, 3)}
            r.update({kk: (round(v, 4) if isinstance(v, float) else v) for kk, v in stages(fasta, k).items()})
            r["bases_per_s"] = r["bases"] / dt
            results.append(r)
            print(json.dumps(r), flush=True)
    for p in (yeast, big):
        os.remove(p)


if __name__ == "__main__":
    main()
