#!/bin/bash
# Fused count + u4 with the wrap check after the widening: dense / u4 / assembly / config-4
# GPU tests, the default bench line and the one-rank-of-8 projection.
export TMPDIR=/tmp
tag=${1:-u4post}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "dense or u4 or config3 or low_complex or wraps or smoke or dropin or assembly or config4" > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 --no-config5 > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 > $OUT/sim8.log 2>&1 || exit 13
echo done > $OUT/done
