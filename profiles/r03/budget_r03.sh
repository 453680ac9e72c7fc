#!/bin/bash
# Exchange budget sweep of the config-3 bench with round 3's kernels (KMH_SUF_BUDGET_MB: genomes
# per partition / count launch pair).  Usage (GPU box): bash profiles/r03/budget_r03.sh <tag>
export TMPDIR=/tmp
tag=${1:-budget}
OUT=gpurun_out/$tag
mkdir -p $OUT
for mb in 4096 8192 12288 16384 8192 12288 16384 4096; do
  KMH_SUF_BUDGET_MB=$mb timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-config5 >> $OUT/b$mb.log 2>&1 || exit 11
done
echo done > $OUT/done
