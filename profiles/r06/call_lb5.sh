#!/bin/bash
# Deferred-store one-pass union: shard tests, then look-back stats on config 5's matrix leg (N = 1).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06lb6}
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "shard_union or sparse_matrix_sharded or two_config5" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 10
KMH_SHARD_LB_STATS=1 timeout -k 10 400 python3 -u bench.py --workload sparse --steps 2 --cpu-sample 0 > $OUT/one.log 2>&1 || exit 12
grep "shard lb" $OUT/one.log | tail -2
grep -o '"shard_phases_rank0": {[^}]*}' $OUT/one.log | head -1
echo done > $OUT/done
