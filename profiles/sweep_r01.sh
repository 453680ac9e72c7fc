#!/bin/bash
# Count-kernel lane-group sweep + SQ/TA counters on the current kernels (config 3 / 8 genomes).
export TMPDIR=/tmp
OUT=gpurun_out/sweep
mkdir -p $OUT
for v in 0 84 48 28 12 162; do
  KMH_GSU=$v timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > $OUT/gsu_$v.log 2>&1
  echo "gsu=$v $(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}' $OUT/gsu_$v.log)" >> $OUT/summary.txt
done
B="bench.py --steps 2 --warmup 1 --cpu-sample 0 --genomes 8"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 $B > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/summary.txt
done
echo done >> $OUT/summary.txt
