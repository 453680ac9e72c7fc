#!/bin/bash
# Round-1 profiling recipe (run on the GPU box from the repo root via gpurun).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01
mkdir -p $OUT
B="bench.py --steps 5 --warmup 2 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $B > $OUT/trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o write -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/write.log 2>&1 || exit 13
# footprint experiment: same 6.4 Gbases, smaller genomes -> smaller suffix buffers per batch
for cfg in "256 25000000 64" "256 25000000 256" "1024 6250000 16" "64 100000000 256"; do
  set -- $cfg
  KMH_SUF_BUDGET_MB=$3 timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 --genomes $1 --genome-len $2 > $OUT/fp_$1_$3.log 2>&1 || exit 14
done
echo done > $OUT/done
