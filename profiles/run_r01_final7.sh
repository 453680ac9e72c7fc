#!/bin/bash
# Round-1 final (7), after the wave-coalesced assembly kernels and the kernel-event filter: every GPU
# test, smoke(), the default bench line (config 3) and rocprofv3 kernel stats of it.
export TMPDIR=/tmp
OUT=gpurun_out/final7
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -x --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 14
echo done > $OUT/done
