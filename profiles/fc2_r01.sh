#!/bin/bash
# Fixed-capacity partition on 16384-window tiles (KMH_FC=2, 2 workgroups per CU): dense parity
# tests with it, then config-3 bench with it and with the default.
export TMPDIR=/tmp
OUT=gpurun_out/fc2
mkdir -p $OUT
KMH_FC=2 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "dense or config3" > $OUT/tests.log 2>&1 || exit 10
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
KMH_FC=2 timeout -k 10 200 python3 -u $B > $OUT/bench_fc2.log 2>&1 || exit 11
timeout -k 10 200 python3 -u $B > $OUT/bench_base.log 2>&1 || exit 12
echo done > $OUT/done
