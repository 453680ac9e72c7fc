#!/bin/bash
# Round 4: the split's 16-byte region stores (build_ab/v4) on the sparse tests, then an A/B of
# config 5: default, v4, and experiment builds with phase clocks (exp0) and without the split's
# returning-atomic wait (splitexp2).
out=gpurun_out/r04c
mkdir -p $out
KMH_LIB_PATH=$PWD/build_ab/v4/libkmerhip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "sparse_dev or sparse_host or past_2_31 or sparse_rows" > $out/tests_v4.log 2>&1
rc=$?
tail -3 $out/tests_v4.log
[ $rc -eq 0 ] || exit $rc
export KMH_SP_PROF=1
bash profiles/r04/ab_sparse.sh r04c/ab 2 v4 exp0 splitexp2
