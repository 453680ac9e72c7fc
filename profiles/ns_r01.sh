#!/bin/bash
# k_sp_count with NS independent probe streams per lane (KMH_SP_STREAMS 1/2/4): sparse parity
# tests at the default (2), then config 5 bench for each NS.
export TMPDIR=/tmp
OUT=gpurun_out/ns
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse" > $OUT/tests.log 2>&1 || exit 10
for ns in 1 2 4; do
  KMH_SP_STREAMS=$ns timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/ns$ns.log 2>&1 || exit 11
done
KMH_SP_STREAMS=4 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse_dev" > $OUT/tests4.log 2>&1 || exit 12
echo done > $OUT/done
