#!/bin/bash
# Round 5, after the split-item target change (kmh_hash.hip): the sparse / sorted / shard / matrix
# / drop-in GPU tests, then final_b.sh (bench line, kernel stats, FETCH / WRITE passes for this
# build, one simulated N = 8 rank, the sparse bench with the matrix leg).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05fd}
mkdir -p $OUT
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_parity.py tests/test_integration_binding.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sorted or shard or matrix or sparse or dropin or binding or count_host" > $OUT/gpu_tests.log 2>&1
rc=$?
tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r05/final_b.sh ${1:-r05fd}
