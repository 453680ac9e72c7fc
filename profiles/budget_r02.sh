#!/bin/bash
# Exchange budget sweep of the config-3 bench with the three-workgroup partition
# (KMH_SUF_BUDGET_MB: genomes per launch pair).  Usage (GPU box): bash profiles/budget_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-budget}
OUT=gpurun_out/$tag
mkdir -p $OUT
for mb in 1024 2048 4096 8192 16384 1024 2048 8192; do
  KMH_SUF_BUDGET_MB=$mb timeout -k 10 200 python3 -u bench.py --cpu-sample 0 --no-config5 >> $OUT/b$mb.log 2>&1 || exit 11
done
echo done > $OUT/done
