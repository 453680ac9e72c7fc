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
timeout -k 10 400 python3 -u bench.py > $out/bench.log 2>&1 || exit $?
tail -c 300 $out/bench.log
# one rank of config 4 at N = 8 (the all-gather modelled by device copies, and without them)
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 > $out/sim8_torch.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 --sim-copy none > $out/sim8_none.log 2>&1
rc=$?
tail -c 300 $out/sim8_none.log
exit $rc
