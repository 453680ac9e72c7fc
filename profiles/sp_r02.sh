#!/bin/bash
# Config 5 (sparse k = 21 canonical, 16 x 250 Mbp per GPU): bench line + kernel stats.
export TMPDIR=/tmp
tag=${1:-sp}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 600 python3 -u bench.py --workload sparse --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --workload sparse --steps 3 --warmup 1 --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 13
echo done > $OUT/done
