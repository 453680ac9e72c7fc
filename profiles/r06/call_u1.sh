#!/bin/bash
# Shard union A/B: the shard tests, kernel stats of config 5's matrix leg (N = 1), one simulated N = 8 rank.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06u1}
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "shard_union or sparse_matrix_sharded or two_config5" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/one -o t -- python3 -u bench.py --workload sparse --steps 2 --cpu-sample 0 > $OUT/one.log 2>&1 || exit 12
grep -o '"matrix": {[^}]*}' $OUT/one.log | head -1
timeout -k 10 400 python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim8_sparse.log 2>&1 || exit 13
grep -o '"phases_ms": {[^}]*}' $OUT/sim8_sparse.log | head -1
echo done > $OUT/done
