#!/bin/bash
# Sparse path change: sparse parity tests, then the config-5 bench line.
export TMPDIR=/tmp
tag=${1:-spt}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sparse" > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 600 python3 -u bench.py --workload sparse --steps 5 --warmup 2 --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 12
echo done > $OUT/done
