#!/bin/bash
# One-pass shard union A/B: the shard union tests, config 5's matrix leg at N = 1, one simulated N = 8 rank.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06lb2}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "shard_union" --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; [ $rc -eq 0 ] || exit 10
timeout -k 10 400 python3 -u bench.py --workload sparse --steps 3 --cpu-sample 0 > $OUT/sparse.log 2>&1 || exit 12
grep -o '"shard_phases_rank0": {[^}]*}' $OUT/sparse.log | head -1
timeout -k 10 400 python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim8_sparse.log 2>&1 || exit 13
grep -o '"phases_ms": {[^}]*}' $OUT/sim8_sparse.log | head -1
echo done > $OUT/done
