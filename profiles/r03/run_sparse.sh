#!/bin/bash
# Round 3: the sparse / drop-in GPU tests, then the config-5 bench line, on one MI355X.
tag=${1:-r03b}
sel=${2:-"sparse or dropin or long or count_host or first_order or cli or synthetic or past_2_31"}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -k "$sel" > $out/tests.log 2>&1
rc=$?
tail -5 $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --workload sparse --steps 5 --warmup 2 --cpu-sample 0 > $out/bench5.log 2>&1
rc2=$?
tail -c 1500 $out/bench5.log
exit $(( rc > rc2 ? rc : rc2 ))
