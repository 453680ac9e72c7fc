#!/bin/bash
# Look-back cost per unit (KMH_SHARD_LB_STATS=1): config 5's matrix leg at N = 1.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06lb5}
mkdir -p $OUT
KMH_SHARD_LB_STATS=1 timeout -k 10 400 python3 -u bench.py --workload sparse --steps 2 --cpu-sample 0 > $OUT/one.log 2>&1 || exit 12
grep "shard lb" $OUT/one.log | tail -3
grep -o '"shard_phases_rank0": {[^}]*}' $OUT/one.log | head -1
echo done > $OUT/done
