#!/bin/bash
# Step-gap experiment: config-3 step time with and without per-kernel HIP events in the timed
# region, and with 2 / 4 genomes per partition batch (KMH_SUF_BUDGET_MB).
export TMPDIR=/tmp
OUT=gpurun_out/gap
mkdir -p $OUT
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 200 python3 -u $B > $OUT/base.log 2>&1 || exit 10
timeout -k 10 200 python3 -u $B --no-kernel-events > $OUT/noev.log 2>&1 || exit 11
KMH_SUF_BUDGET_MB=512 timeout -k 10 200 python3 -u $B > $OUT/b512.log 2>&1 || exit 12
KMH_SUF_BUDGET_MB=1024 timeout -k 10 200 python3 -u $B > $OUT/b1024.log 2>&1 || exit 13
echo done > $OUT/done
