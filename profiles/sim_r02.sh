#!/bin/bash
# One rank of config 4 at N = 2 / 4 / 8 projected on one GPU (bench.py --simulate-ranks), each
# run twice.  Usage (GPU box): bash profiles/sim_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-sim}
OUT=gpurun_out/$tag
mkdir -p $OUT
for n in 2 4 8 8 4 2; do
  timeout -k 10 200 python3 -u bench.py --simulate-ranks $n --steps 20 --warmup 3 --cpu-sample 0 >> $OUT/sim$n.log 2>&1 || exit 11
done
echo done > $OUT/done
