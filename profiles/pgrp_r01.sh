#!/bin/bash
# Grouped (pipelined) scatter in k_partition: dense parity tests with it, then config-3 bench
# A/B: default, KMH_PGRP=8/16/32 (32768-window tiles) and KMH_SUBT=1 KMH_PGRP=16.
export TMPDIR=/tmp
OUT=gpurun_out/pgrp
mkdir -p $OUT
KMH_PGRP=16 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "dense or config3 or smoke" > $OUT/tests.log 2>&1 || exit 10
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 200 python3 -u $B > $OUT/base.log 2>&1 || exit 11
KMH_PGRP=8 timeout -k 10 200 python3 -u $B > $OUT/g8.log 2>&1 || exit 12
KMH_PGRP=16 timeout -k 10 200 python3 -u $B > $OUT/g16.log 2>&1 || exit 13
KMH_PGRP=32 timeout -k 10 200 python3 -u $B > $OUT/g32.log 2>&1 || exit 14
KMH_SUBT=1 KMH_PGRP=16 timeout -k 10 200 python3 -u $B > $OUT/s1g16.log 2>&1 || exit 15
echo done > $OUT/done
