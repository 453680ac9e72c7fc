#!/bin/bash
# Fused count + u4 encode (kmh_count_dense_u4_dev): parity tests, then the one-rank-of-8 projection
# fused vs --separate-encode.
export TMPDIR=/tmp
tag=${1:-fused}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "u4 or dense or assembl or bench_ or config4" > $OUT/gpu_tests.log 2>&1 || exit 10
for n in 8 4; do
  timeout -k 10 300 python3 -u bench.py --simulate-ranks $n --cpu-sample 0 > $OUT/sim$n.log 2>&1 || exit 12
  timeout -k 10 300 python3 -u bench.py --simulate-ranks $n --cpu-sample 0 --separate-encode > $OUT/sim${n}_sep.log 2>&1 || exit 13
done
echo done > $OUT/done
