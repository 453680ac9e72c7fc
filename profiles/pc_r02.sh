#!/bin/bash
# Persistent count kernel: dense parity tests, the default bench line, the one-rank-of-8 projection.
export TMPDIR=/tmp
tag=${1:-pc}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "dense or u4 or config3 or low_complex or wraps or smoke or dropin" > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 > $OUT/sim8.log 2>&1 || exit 13
echo done > $OUT/done
