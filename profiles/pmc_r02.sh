#!/bin/bash
# HBM traffic of the default bench command (config 3 and its config-5 leg), one rocprofv3 pass
# per counter, for profiles/pmc_traffic.json (merged on the CPU side by pmc_summary.py; bench.py
# prints `traffic` only while the loaded library has the build id stamped there).
# Usage (GPU box): bash profiles/pmc_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-pmc}
OUT=gpurun_out/$tag
mkdir -p $OUT
B="bench.py --steps 2 --warmup 1 --cpu-sample 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/f -o f -- python3 $B > $OUT/f.log 2>&1 || exit 11
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/w -o w -- python3 $B > $OUT/w.log 2>&1 || exit 12
echo done > $OUT/done
