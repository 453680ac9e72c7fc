#!/bin/bash
# Count output by plain stores (default since r04n): sparse parity tests, then the final profiling
# of this build (smoke, bench, kernel trace, FETCH/WRITE passes; profiles/r04/final_r04.sh).
out=gpurun_out/${1:-r04fin3}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "sparse or hash or dropin or kmers" --timeout 300 --timeout-method thread > $out/gpu_tests_sparse.log 2>&1
rc=$?
tail -3 $out/gpu_tests_sparse.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/final_r04.sh ${1:-r04fin3} skip
