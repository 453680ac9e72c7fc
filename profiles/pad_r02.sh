#!/bin/bash
# Dense exchange without chunk padding: dense parity tests, the default bench line (config 3).
export TMPDIR=/tmp
tag=${1:-pad}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  -k "dense or u4 or config3 or low_complex or wraps or smoke or dropin or assembly or config4" > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 --no-config5 > $OUT/bench.log 2>&1 || exit 12
echo done > $OUT/done
