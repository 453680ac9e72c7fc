#!/bin/bash
# Kernel-trace stats and PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes) of the default
# config-3 bench after the batching change (18 genomes per partition/count launch).
export TMPDIR=/tmp
OUT=gpurun_out/prof2
mkdir -p $OUT
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $B > $OUT/trace.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/fetch.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o write -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/write.log 2>&1 || exit 15
echo done > $OUT/done
