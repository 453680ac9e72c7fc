#!/bin/bash
# Round 5: every GPU test, the smoke run and the default bench line on the current build.
out=gpurun_out/${1:-r05b}
mkdir -p $out
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $out/build_id.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py > $out/bench.log 2>&1
rc=$?
tail -c 600 $out/bench.log
exit $rc
