#!/bin/bash
# Regression pass after the sparse / assembly / feature work: every GPU test, smoke(),
# the default bench line (config 3) and its kernel-trace stats.
export TMPDIR=/tmp
OUT=gpurun_out/reg
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 13
echo done > $OUT/done
