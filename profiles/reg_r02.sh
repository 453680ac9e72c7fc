#!/bin/bash
# Round-2 regression of the committed HEAD: every GPU test, smoke(), the default bench line,
# rocprofv3 kernel stats of the same bench, and the fabric / Infinity-Cache microbenchmarks.
# Usage (GPU box): bash profiles/reg_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-reg}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 13
if [ -n "$MICRO" ]; then
  timeout -k 10 120 kmer-ml_amd/kmerml/_lib/fabric_bench > $OUT/fabric.txt 2>&1 || exit 14
  timeout -k 10 120 kmer-ml_amd/kmerml/_lib/mall_pass_bench > $OUT/mall_pass.txt 2>&1 || exit 15
fi
echo done > $OUT/done
