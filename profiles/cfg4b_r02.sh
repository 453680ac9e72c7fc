#!/bin/bash
# Compact u4 assembly: the assembly / rank-simulation GPU tests, then the one-rank-of-N projection
# (--simulate-ranks 2 / 4 / 8 at config 4's size) beside the default config-3 line.
export TMPDIR=/tmp
tag=${1:-cfg4b}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "config4 or assembl or bench_ or decode_u4" > $OUT/gpu_tests.log 2>&1 || exit 10
for n in 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --simulate-ranks $n --cpu-sample 0 > $OUT/sim$n.log 2>&1 || exit 12
  timeout -k 10 300 python3 -u bench.py --simulate-ranks $n --cpu-sample 0 --assemble u4-dense > $OUT/sim${n}_dense.log 2>&1 || true
done
echo done > $OUT/done
