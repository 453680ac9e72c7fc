#!/bin/bash
# k_sp_count with table-scan emission (no claimed-slot list): sparse parity tests, then the
# config-5 bench at table sizes 2^14 (default), 2^13 and 2^12 (KMH_SP_TABLE_BITS).
export TMPDIR=/tmp
OUT=gpurun_out/sp3
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse" > $OUT/tests.log 2>&1 || exit 10
for tb in 14 13 12; do
  KMH_SP_TABLE_BITS=$tb timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/tb$tb.log 2>&1 || exit 11
done
echo done > $OUT/done
