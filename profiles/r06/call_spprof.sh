#!/bin/bash
# KMH_EXPERIMENTS build: k_sp_count (ordered pass) and k_sp_split phase clocks on config 5's matrix leg.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06spp}
mkdir -p $OUT
KMH_SP_PROF=1 timeout -k 10 400 python3 -u bench.py --workload sparse --steps 1 --cpu-sample 0 > $OUT/one.log 2>&1 || exit 12
grep -E "k_sp_count per wave|k_sp_split|union" $OUT/one.log | tail -8
echo done > $OUT/done
