#!/bin/bash
# Round 4 regression: every GPU test, the default bench line (config 3 + config 5 + e2e), then
# the count kernel's output what-ifs on the new kernels.
out=gpurun_out/${1:-r04f}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1
rc=$?
tail -c 600 $out/bench.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_sparse.sh ${1:-r04f}/ab 1 exp0 outexp1 outexp2
