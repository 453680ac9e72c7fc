#!/bin/bash
# Counter passes (one --pmc set per run, each under its own time limit) of the config-5 kernels
# on 4 genomes of 250 Mbp (bench.py --workload sparse --genomes 4), then a per-kernel summary.
# usage: bash profiles/r03/pmc_sparse.sh <tag> [extra bench args]
export TMPDIR=/tmp
tag=${1:-pmcsp}; shift
out=gpurun_out/$tag
mkdir -p $out
B="bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 --genomes 4 $*"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $out/p$i -o p$i -- python3 $B > $out/p$i.log 2>&1 || { echo "pass $i failed"; exit 11; }
done
python3 profiles/sq_summary.py $out > $out/summary.txt
grep -A20 "k_sp_" $out/summary.txt | head -80
