#!/bin/bash
# Round 5: shard union with rank-ordered bins and counted row lookup: shard / matrix GPU tests,
# phase clocks of the ordered vs unordered count (experiment build), the matrix kernel trace.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05l}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "shard or matrix" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
KMH_LIB_PATH=$PWD/build_ab/exp/libkmerhip.so KMH_SP_PROF=1 timeout -k 10 200 python3 -u profiles/r05/prof_ord.py > $out/prof_ord.log 2>&1 || exit 12
grep -v "^$" $out/prof_ord.log | tail -24
bash profiles/r05/call_g.sh ${1:-r05l}/g
