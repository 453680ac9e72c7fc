#!/bin/bash
# Batch-size sweep: genomes per partition/count launch via KMH_SUF_BUDGET_MB (config 3),
# with per-kernel events (the bench default) and without (--no-kernel-events).
export TMPDIR=/tmp
OUT=gpurun_out/batch
mkdir -p $OUT
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
for mb in 2048 4096 16384; do
  KMH_SUF_BUDGET_MB=$mb timeout -k 10 200 python3 -u $B > $OUT/b$mb.log 2>&1 || exit 10
  KMH_SUF_BUDGET_MB=$mb timeout -k 10 200 python3 -u $B --no-kernel-events > $OUT/b${mb}_noev.log 2>&1 || exit 11
done
echo done > $OUT/done
