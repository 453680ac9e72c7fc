#!/bin/bash
# Round 5: sorted rows (bins of 2-4 keys sorted by a network, parallel item offsets): the sorted /
# shard / matrix GPU tests, then the kernel trace of the config-5 bench with its matrix leg.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05j}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sorted or shard or matrix" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r05/call_g.sh ${1:-r05j}/g
