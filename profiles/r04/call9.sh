#!/bin/bash
# Split: region reservations one item early (default) vs after the item's own histogram (late):
# sparse parity tests on the default build, config-5 A/B; then call8's measurements (integer
# multiply rates, sim8 with and without copies, 8/32-genome launches).
out=gpurun_out/${1:-r04j}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "sparse or hash or dropin or kmers" --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?
tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash profiles/r04/ab_sparse.sh ${1:-r04j}/ab 2 binmul late stb0 || exit 12
bash profiles/r04/call8.sh ${1:-r04j}/m
