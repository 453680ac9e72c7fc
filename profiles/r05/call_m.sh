#!/bin/bash
# Round 5: the software-pipelined shard union (build_ab/pipe): sorted / shard / matrix GPU tests on
# that library, then the matrix kernel trace with it.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05o}
mkdir -p $out
export KMH_LIB_PATH=$PWD/build_ab/pipe/libkmerhip.so
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id(), _native.lib()._name)" > $out/build_id.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sorted or shard or matrix" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r05/call_g.sh ${1:-r05o}/g
