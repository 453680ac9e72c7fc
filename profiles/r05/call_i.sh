#!/bin/bash
# Round 5: shard union with its gather loads in flight together: the shard / matrix GPU tests, then
# the kernel trace of the config-5 bench with its matrix leg.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05k}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "shard or matrix" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r05/call_g.sh ${1:-r05k}/g
