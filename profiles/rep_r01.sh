#!/bin/bash
# Persistent replica-counter partition (k_partition_rep): dense parity tests, then the
# config-3 bench with it (default) and with the classic partition (KMH_PART=0).
export TMPDIR=/tmp
OUT=gpurun_out/rep
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "dense or config3" > $OUT/tests.log 2>&1 || exit 10
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 200 python3 -u $B > $OUT/bench_rep.log 2>&1 || exit 11
KMH_PART=0 timeout -k 10 200 python3 -u $B > $OUT/bench_classic.log 2>&1 || exit 12
timeout -k 10 200 python3 -u $B --no-kernel-events > $OUT/bench_rep_noev.log 2>&1 || exit 13
echo done > $OUT/done
