#!/bin/bash
# k_sp_count at 2^13 slots with 8 waves/SIMD (two workgroups per CU) vs 2^14: parity + bench.
export TMPDIR=/tmp
OUT=gpurun_out/sp4
mkdir -p $OUT
KMH_SP_TABLE_BITS=13 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse_dev" > $OUT/tests.log 2>&1 || exit 10
for tb in 13 14; do
  KMH_SP_TABLE_BITS=$tb timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/tb$tb.log 2>&1 || exit 11
done
echo done > $OUT/done
