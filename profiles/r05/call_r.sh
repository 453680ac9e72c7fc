#!/bin/bash
# Round 5: ordered count in two passes (distinct counts first, then compact rows back to back: no
# padding, no compaction kernel): sorted / shard / matrix / sparse GPU tests, then the matrix
# kernel trace.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05u}
mkdir -p $out
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $out/build_id.txt
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_integration_binding.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sorted or shard or matrix or sparse or binding" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r05/call_g.sh ${1:-r05u}/g
