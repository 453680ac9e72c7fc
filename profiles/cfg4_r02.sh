#!/bin/bash
# Config 4's real per-rank workload on one MI355X (8 ranks sharing cuda:0, gloo), the
# assembly tests at full size, then the default bench line (with the new CPU baselines).
export TMPDIR=/tmp
tag=${1:-cfg4}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "config4 or assembly or bench_pipelined" > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
echo done > $OUT/done
