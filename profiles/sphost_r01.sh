#!/bin/bash
# Host phases of the sparse path (KMH_SP_PROF=1), config 5 bench shape.
export TMPDIR=/tmp
OUT=gpurun_out/sphost
mkdir -p $OUT
KMH_SP_PROF=2 timeout -k 10 300 python3 -u bench.py --workload sparse --steps 3 --warmup 1 --cpu-sample 0 > $OUT/prof.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 11
echo done > $OUT/done
