#!/bin/bash
# k_sp_count A/B: match add issued by every lane (VAR 0) or only by matching lanes (VAR 1).
export TMPDIR=/tmp
OUT=gpurun_out/spvar
mkdir -p $OUT
KMH_SP_VAR=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse_dev" > $OUT/tests1.log 2>&1 || exit 10
for v in 0 1 0 1; do
  KMH_SP_VAR=$v timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 >> $OUT/var$v.log 2>&1 || exit 11
done
echo done > $OUT/done
