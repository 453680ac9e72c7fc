#!/bin/bash
# k_sp_count with branch-free k_sp_split atomics (dummy passes, scratch tail):
# sparse parity tests, config-5 bench, per-phase cycles.
export TMPDIR=/tmp
OUT=gpurun_out/spsbf
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 11
echo done > $OUT/done
