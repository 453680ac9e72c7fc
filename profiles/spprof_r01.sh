#!/bin/bash
# In-kernel phase counters of k_sp_count (KMH_SP_PROF=1) and the table-size sweep,
# 2 genomes, config-5 shape.
export TMPDIR=/tmp
OUT=gpurun_out/spprof
mkdir -p $OUT
for tb in 14 13 12; do
  KMH_SP_TABLE_BITS=$tb KMH_SP_PROF=1 timeout -k 10 300 python3 -u bench.py --workload sparse --genomes 2 --steps 1 --warmup 0 --cpu-sample 0 > $OUT/prof_tb$tb.log 2>&1 || exit 10
  KMH_SP_TABLE_BITS=$tb timeout -k 10 300 python3 -u bench.py --workload sparse --genomes 2 --steps 2 --warmup 1 --cpu-sample 0 > $OUT/bench_tb$tb.log 2>&1 || exit 11
done
echo done > $OUT/done
