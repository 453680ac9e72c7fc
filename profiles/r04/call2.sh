#!/bin/bash
# Round 4: contiguous pass regions + neighbour emission in the config-5 count kernel.
# Sparse / drop-in GPU tests, then the config-5 bench line.
tag=${1:-r04b}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
  -k "sparse or dropin or long or count_host or first_order or cli or synthetic or past_2_31 or workspace" > $out/tests.log 2>&1
rc=$?
tail -5 $out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload sparse --steps 5 --warmup 2 --cpu-sample 0 > $out/bench5.log 2>&1
rc2=$?
tail -c 1500 $out/bench5.log
exit $rc2
