#!/bin/bash
# Ablations of k_sp_count (experiments; counts are wrong when KMH_SP_ABL != 0):
# 1 = no hash inserts, 2 = no output stores, 4 = no segment reads, 8 = no output-cursor atomic.
export TMPDIR=/tmp
OUT=gpurun_out/spabl
mkdir -p $OUT
for a in 0 1 2 8 10 4; do
  KMH_SP_ABL=$a timeout -k 10 300 python3 -u bench.py --workload sparse --genomes 2 --steps 2 --warmup 1 --cpu-sample 0 > $OUT/abl$a.log 2>&1 || [ $a != 0 ] || exit 10
done
echo done > $OUT/done
