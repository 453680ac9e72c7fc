#!/bin/bash
# One-pass vs two-pass shard union on the same box: kernel stats of config 5's matrix leg (N = 1).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06lb3}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/one -o t -- python3 -u bench.py --workload sparse --steps 2 --cpu-sample 0 > $OUT/one.log 2>&1 || exit 12
grep -o '"shard_phases_rank0": {[^}]*}' $OUT/one.log | head -1
KMH_SHARD_TWO_PASS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/two -o t -- python3 -u bench.py --workload sparse --steps 2 --cpu-sample 0 > $OUT/two.log 2>&1 || exit 13
grep -o '"shard_phases_rank0": {[^}]*}' $OUT/two.log | head -1
echo done > $OUT/done
