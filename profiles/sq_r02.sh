#!/bin/bash
# SQ / TCC counter passes (one --pmc set per run) of the dense k = 12 kernels, 8 genomes.
# Usage: bash profiles/sq_r02.sh <tag> [libpath]   (libpath: KMH_LIB_PATH for an A/B build)
export TMPDIR=/tmp
tag=${1:-sq}
OUT=gpurun_out/$tag
mkdir -p $OUT
[ -n "$2" ] && export KMH_LIB_PATH=$2
B="bench.py --steps 1 --warmup 1 --cpu-sample 0 --genomes 8"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/p$i -o p$i -- python3 $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 11; }
done
python3 profiles/sq_summary.py $OUT
