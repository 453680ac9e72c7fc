#!/bin/bash
# Round 6 final, part A, on the committed HEAD: every GPU test, smoke(), the default bench line.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06fa}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?
tail -2 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit 10
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit 12
tail -c 300 $OUT/bench.log
