#!/bin/bash
# k_sp_count load factor sweep (keys per 16384-slot table, KMH_SP_TARGET) after the device
# item plan and the balanced count kernel: config 5 bench per target.
export TMPDIR=/tmp
OUT=gpurun_out/sptarget2
mkdir -p $OUT
for t in 5120 6144 8192 10240; do
  KMH_SP_TARGET=$t timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/t$t.log 2>&1 || exit 10
done
echo done > $OUT/done
