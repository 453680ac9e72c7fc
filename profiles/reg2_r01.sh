#!/bin/bash
# Regression after batching + u4 assembly: every GPU test, smoke(), the default bench line.
export TMPDIR=/tmp
OUT=gpurun_out/reg2
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
echo done > $OUT/done
