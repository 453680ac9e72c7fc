#!/bin/bash
# Round 4, first GPU call: the host-side changes (staged counting, workspace trim) on their
# GPU tests, then the config-5 what-if A/B (which kernel's bytes bound the step).
out=gpurun_out/r04a
mkdir -p $out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "workspace or dropin or count_host or cli or first_order or synthetic_hashes or sparse_host" > $out/tests.log 2>&1
rc=$?
tail -4 $out/tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_sparse.sh r04a/ab 2 exp0 outexp1 outexp2 splitexp partexp
