#!/bin/bash
# Round 6: ring bench without the hand-off protocol (data movement floor), modes and shapes.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06f}
mkdir -p $OUT
for args in "8 64 3 3 4x1" "8 64 2 3 4x1" "8 64 3 3 8x2" "8 64 2 3 8x2" "8 64 3 3 12x2"; do
  timeout -k 10 120 kmer-ml_amd/kmerml/_lib/ring_bench $args >> $OUT/ring_bench.log 2>&1 || { echo "ring_bench $args rc=$?" >> $OUT/ring_bench.log; break; }
done
cat $OUT/ring_bench.log
