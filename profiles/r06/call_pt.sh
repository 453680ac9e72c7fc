#!/bin/bash
# KMH_EXPERIMENTS build: per-phase clocks of the union's write pass (config 5 matrix leg, N = 1).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06pt}
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py --workload sparse --steps 2 --cpu-sample 0 > $OUT/one.log 2>&1 || exit 12
grep "union write phases" $OUT/one.log | tail -2
timeout -k 10 400 python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 1 > $OUT/sim.log 2>&1 || exit 13
grep "union write phases" $OUT/sim.log | tail -1
echo done > $OUT/done
