#!/bin/bash
# Round 4: count slow path (parallel reads, registers), split atomics before the scan.
out=gpurun_out/${1:-r04e}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "sparse_dev or sparse_host or past_2_31 or sparse_rows or dropin_edge or workspace or sparse_matrix or skewed" > $out/tests.log 2>&1
rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || exit $rc
export KMH_SP_PROF=1
bash profiles/r04/ab_sparse.sh ${1:-r04e}/ab 2 exp0
grep -h "per wave" $out/ab/exp0.log | tail -2
