#!/bin/bash
# A/B of the partition variants at the current defaults (config 3, kernel times per launch):
# default (32768-window tiles), KMH_SUBT=1 (16384-window tiles), KMH_FC=2 (fixed-capacity rows
# on 16384-window tiles).
export TMPDIR=/tmp
OUT=gpurun_out/fcab
mkdir -p $OUT
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 200 python3 -u $B > $OUT/base.log 2>&1 || exit 11
KMH_SUBT=1 timeout -k 10 200 python3 -u $B > $OUT/subt1.log 2>&1 || exit 12
KMH_FC=2 timeout -k 10 200 python3 -u $B > $OUT/fc2.log 2>&1 || exit 13
echo done > $OUT/done
