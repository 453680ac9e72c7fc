#!/bin/bash
# One-pass shard union (look-back column bases): the shard / matrix GPU tests (one-pass and, with
# KMH_SHARD_TWO_PASS=1, the two passes), then config 5's matrix leg at N = 1 and one simulated
# N = 8 rank.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06lb}
mkdir -p $OUT
K="shard or sparse_matrix or wire or config5 or simulated"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit 10
KMH_SHARD_TWO_PASS=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "shard_union" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests2.log 2>&1
rc=$?; tail -2 $OUT/tests2.log; [ $rc -eq 0 ] || exit 11
timeout -k 10 400 python3 -u bench.py --workload sparse --steps 3 --cpu-sample 0 > $OUT/sparse.log 2>&1 || exit 12
grep -o '"matrix": {[^}]*}' $OUT/sparse.log | head -1
timeout -k 10 400 python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim8_sparse.log 2>&1 || exit 13
grep -o '"phases_ms": {[^}]*}' $OUT/sim8_sparse.log | head -1
echo done > $OUT/done
