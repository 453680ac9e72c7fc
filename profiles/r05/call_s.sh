#!/bin/bash
# Round 5: the shard union in one pass (column bases by decoupled look-back, no sizes pass): the
# shard union cases first (short limit), then the sorted / shard / matrix / sparse GPU tests, then
# the kernel trace of the config-5 bench with its matrix leg.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05x}
mkdir -p $out
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $out/build_id.txt
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 60 --timeout-method thread -p no:cacheprovider \
  -k "shard_union" > $out/gpu_shard.log 2>&1
rc=$?
tail -3 $out/gpu_shard.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_integration_binding.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sorted or shard or matrix or sparse or binding" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r05/call_g.sh ${1:-r05x}/g
