#!/bin/bash
# k_sp_count load factor: keys per 16384-slot table (KMH_SP_TARGET, default 8192), config 5.
export TMPDIR=/tmp
OUT=gpurun_out/sptarget
mkdir -p $OUT
for t in 8192 6144 4096 3072; do
  KMH_SP_TARGET=$t timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/t$t.log 2>&1 || exit 10
done
echo done > $OUT/done
