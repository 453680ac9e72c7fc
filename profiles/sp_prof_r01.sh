#!/bin/bash
# Config 3 bench line (with the threaded C baseline), then config 5 (sparse) kernel-trace
# stats and separate FETCH_SIZE / WRITE_SIZE passes.
export TMPDIR=/tmp
OUT=gpurun_out/spp
mkdir -p $OUT
S="bench.py --workload sparse --cpu-sample 0"
timeout -k 10 300 python3 -u bench.py > $OUT/bench3.log 2>&1 || exit 9
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $S --steps 3 --warmup 1 > $OUT/trace.log 2>&1 || exit 10
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o fetch -- python3 $S --steps 1 --warmup 0 > $OUT/fetch.log 2>&1 || exit 11
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o write -- python3 $S --steps 1 --warmup 0 > $OUT/write.log 2>&1 || exit 12
echo done > $OUT/done
