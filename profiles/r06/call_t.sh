#!/bin/bash
# The shard union parity cases.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06t}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "shard_union" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; exit $rc
