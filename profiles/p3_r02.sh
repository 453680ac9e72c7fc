#!/bin/bash
# k_partition at three workgroups per CU (u16 rank counters, starts aliased into the stage,
# codes derived twice from six encoded registers): dense parity tests, then the config-3 bench
# and its kernel stats.  Usage (GPU box): bash profiles/p3_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-p3}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "dense or u4_fused or u16_wraps or count_host or count_matrix_single or first_order" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 200 python3 -u bench.py --cpu-sample 0 --no-config5 > $OUT/bench.log 2>&1 || exit 11
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-config5 > $OUT/trace.log 2>&1 || exit 12
echo done > $OUT/done
