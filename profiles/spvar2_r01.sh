#!/bin/bash
# k_sp_count match-add variants (KMH_SP_VAR): 0 = unconditional add of 0/1 on the probed slot
# (default), 1 = non-matching lanes add to their own dummy slot, 2 = wave-uniform skip when no
# lane matched, 3 = both.  Device sparse parity tests with 3, then the config-5 bench A/B.
export TMPDIR=/tmp
OUT=gpurun_out/spvar2
mkdir -p $OUT
KMH_SP_VAR=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse_dev" > $OUT/tests3.log 2>&1 || exit 10
S="bench.py --workload sparse --steps 5 --warmup 2 --cpu-sample 0"
timeout -k 10 200 python3 -u $S > $OUT/v0.log 2>&1 || exit 11
KMH_SP_VAR=1 timeout -k 10 200 python3 -u $S > $OUT/v1.log 2>&1 || exit 12
KMH_SP_VAR=2 timeout -k 10 200 python3 -u $S > $OUT/v2.log 2>&1 || exit 13
KMH_SP_VAR=3 timeout -k 10 200 python3 -u $S > $OUT/v3.log 2>&1 || exit 14
echo done > $OUT/done
