#!/bin/bash
# enc4 on the dot-product unit + interior tiles without tail masks: dense and sparse parity,
# then the config-3 bench (no config 5) twice.
export TMPDIR=/tmp
tag=${1:-dot}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "dense or sparse_dev or synth or config3 or u4_fused or low_complex or wraps" > $OUT/gpu_tests.log 2>&1 || exit 10
for i in 1 2; do timeout -k 10 300 python3 -u bench.py --cpu-sample 0 --no-config5 > $OUT/bench$i.log 2>&1 || exit 12; done
echo done > $OUT/done
