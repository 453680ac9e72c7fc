#!/bin/bash
# SQ / TCC counter passes (one --pmc set per run) of the config-5 kernels, 4 genomes.
# Usage: bash profiles/spsq_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-spsq}
OUT=gpurun_out/$tag
mkdir -p $OUT
B="bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 --genomes 4"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 11; }
done
python3 profiles/sq_summary.py $OUT > $OUT/summary.txt
