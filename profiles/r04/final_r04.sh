#!/bin/bash
# Round-4 regression of the committed HEAD on one MI355X: every GPU test, smoke(), the default
# bench line, rocprofv3 kernel stats of the same bench, then the FETCH_SIZE / WRITE_SIZE passes
# that profiles/pmc_traffic.json is rebuilt from (profiles/pmc_summary.py, CPU side).
# Usage (GPU box): bash profiles/r04/final_r04.sh <tag> [skip-tests]
export TMPDIR=/tmp
tag=${1:-final}
OUT=gpurun_out/$tag
mkdir -p $OUT
if [ -z "$2" ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
  tail -2 $OUT/gpu_tests.log
fi
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-e2e > $OUT/trace.log 2>&1 || exit 13
B="bench.py --steps 2 --warmup 1 --cpu-sample 0 --no-e2e"   # (the e2e cases launch the same kernels on small genomes)
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/f -o f -- python3 $B > $OUT/f.log 2>&1 || exit 14
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/w -o w -- python3 $B > $OUT/w.log 2>&1 || exit 15
echo done > $OUT/done
