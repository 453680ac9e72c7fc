#!/bin/bash
# k_sp_count: bench at NS=1 (regression check), then SQ counter passes (each --pmc set in its
# own run) at NS=1 and NS=2 on 2 genomes.
export TMPDIR=/tmp
OUT=gpurun_out/spsq2
mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/ns1.log 2>&1 || exit 10
B="bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 --genomes 2"
i=0
for ns in 1 2; do
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM"; do
  i=$((i+1))
  KMH_SP_STREAMS=$ns timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/status; exit 11; }
done
done
echo ok >> $OUT/status
