#!/bin/bash
# Count-kernel LDS swizzle: sparse parity tests on the default (swizzled) build, then config-5
# A/B against the unswizzled (swz0) and histogram-only (swz1) builds.
out=gpurun_out/${1:-r04h}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "sparse or hash or dropin or kmers" --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_sparse.sh ${1:-r04h}/ab 3 swz0 swz1
