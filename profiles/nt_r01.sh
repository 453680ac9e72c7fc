#!/bin/bash
# Non-temporal streaming stores: config-3 bench line and a kernel trace for inter-kernel gaps.
export TMPDIR=/tmp
OUT=gpurun_out/nt
mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o trace -- python3 bench.py --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 11
echo done > $OUT/done
