#!/bin/bash
# Round 5: shard union test cases for the paths the config-5 bench does not take (u64 code offsets
# over the whole 64-bit range, 600 rows, one dense cell cut into many units).
export TMPDIR=/tmp
out=gpurun_out/${1:-r05v}
mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "shard_union" > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
exit $rc
