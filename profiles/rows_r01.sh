#!/bin/bash
# sparse_rows at k = 9 / 21 / 25 / 32 (batched hash tables for 13..21, per-genome GPU sort otherwise).
export TMPDIR=/tmp
OUT=gpurun_out/rows
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse_rows or long_kmers or edge_cases" > $OUT/tests.log 2>&1 || exit 10
echo done > $OUT/done
