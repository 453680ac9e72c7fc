#!/bin/bash
# k_sp_count ablations (counts wrong when KMH_SP_ABL != 0): 1 = no hash inserts, 2 = no output
# stores, 4 = no segment reads; KMH_SP_PROF=1 per-phase cycles; table 2^13 (2 WG/CU).
export TMPDIR=/tmp
OUT=gpurun_out/spabl2
mkdir -p $OUT
B="bench.py --workload sparse --genomes 4 --steps 2 --warmup 1 --cpu-sample 0"
for a in 0 1 2 4 3; do
  KMH_SP_ABL=$a timeout -k 10 200 python3 -u $B > $OUT/abl$a.log 2>&1 || [ $a != 0 ] || exit 10
done
KMH_SP_PROF=1 timeout -k 10 200 python3 -u $B > $OUT/prof.log 2>&1 || exit 11
KMH_SP_TABLE_BITS=13 timeout -k 10 200 python3 -u $B > $OUT/tb13.log 2>&1 || exit 12
echo done > $OUT/done
