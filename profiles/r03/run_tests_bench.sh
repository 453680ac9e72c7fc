#!/bin/bash
# Round 3: full -m gpu suite, then the default bench line (config 3 + config 5), on one MI355X.
# usage (from the repo root, via gpurun): bash profiles/r03/run_tests_bench.sh <tag>
tag=${1:-r03a}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $out/tests.log 2>&1
rc=$?
tail -3 $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = failed tests (still bench); others = stop
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1
rc2=$?
tail -c 600 $out/bench.log
exit $(( rc > rc2 ? rc : rc2 ))
