#!/bin/bash
# 16384-window partition tiles (KMH_SUBT=1, three partition workgroups per CU) with the count
# kernel's pipelined variant (KMH_GSU=4) and a larger batch budget; default for reference.
export TMPDIR=/tmp
OUT=gpurun_out/s1
mkdir -p $OUT
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 200 python3 -u $B > $OUT/base.log 2>&1 || exit 11
KMH_SUBT=1 timeout -k 10 200 python3 -u $B > $OUT/s1.log 2>&1 || exit 12
KMH_SUBT=1 KMH_GSU=4 timeout -k 10 200 python3 -u $B > $OUT/s1_gsu4.log 2>&1 || exit 13
KMH_SUBT=1 KMH_GSU=6 timeout -k 10 200 python3 -u $B > $OUT/s1_gsu6.log 2>&1 || exit 14
KMH_SUBT=1 KMH_SUF_BUDGET_MB=8192 timeout -k 10 200 python3 -u $B > $OUT/s1_b8g.log 2>&1 || exit 15
echo done > $OUT/done
