#!/bin/bash
# Config-5 kernel changes of b286c47: sparse parity tests on the default build, then a config-5
# A/B against one switch reverted each: count bins by multiply (binmul), split reservations after
# the item's own histogram (late), split stores one read at a time (stb0), no LDS swizzle (swz0).
out=gpurun_out/${1:-r04j}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "sparse or hash or dropin or kmers" --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_sparse.sh ${1:-r04j}/ab 2 binmul late stb0 swz0 || exit 12
