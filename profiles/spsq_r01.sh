#!/bin/bash
# SQ counter passes (each --pmc set in its own run) for the sparse k=21 kernels, 2 genomes.
export TMPDIR=/tmp
OUT=gpurun_out/spsq
mkdir -p $OUT
B="bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 --genomes 2"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/status; exit 1; }
done
echo ok >> $OUT/status
