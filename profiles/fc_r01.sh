#!/bin/bash
# Fixed-capacity partition (KMH_FC=1): dense parity tests with it, then bench with and without.
export TMPDIR=/tmp
OUT=gpurun_out/fc
mkdir -p $OUT
KMH_FC=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "dense or config or dropin or count_matrix or first" > $OUT/tests.log 2>&1 || exit 10
KMH_FC=1 timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $OUT/bench_fc.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $OUT/bench_base.log 2>&1 || exit 12
echo done > $OUT/done
