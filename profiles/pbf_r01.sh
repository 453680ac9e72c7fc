#!/bin/bash
# k_partition with branch-free histogram/scatter atomics: dense GPU parity tests, then the
# default bench (config 3) twice.
export TMPDIR=/tmp
OUT=gpurun_out/pbf
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "not sparse" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $OUT/bench1.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $OUT/bench2.log 2>&1 || exit 12
echo done > $OUT/done
