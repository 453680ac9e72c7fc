#!/bin/bash
# Round 5: build_ab/pipe (ordered count: 8-key network for bins of 5..8 keys; union count pass
# without sorting, u32 code offsets): sorted / shard / matrix GPU tests, phase clocks of the
# ordered count (experiment build of the same sources), matrix kernel trace.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05q}
mkdir -p $out
export KMH_LIB_PATH=$PWD/build_ab/pipe/libkmerhip.so
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id(), _native.lib()._name)" > $out/build_id.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sorted or shard or matrix" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
KMH_LIB_PATH=$PWD/build_ab/exp/libkmerhip.so KMH_SP_PROF=1 timeout -k 10 200 python3 -u profiles/r05/prof_ord.py > $out/prof_ord.log 2>&1 || exit 12
grep "k_sp_count\|ms$" $out/prof_ord.log | tail -4
bash profiles/r05/call_g.sh ${1:-r05q}/g
