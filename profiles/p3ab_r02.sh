#!/bin/bash
# A/B of k_partition variants on one box (config-3 bench, kernel events): the default library
# (three workgroups per CU) against build_ab/head (the two-workgroup kernel of the last commit),
# after the dense parity tests of the default library.  Usage: bash profiles/p3ab_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-p3ab}
OUT=gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  -k "dense or u4_fused or u16_wraps or count_host or count_matrix_single or first_order" > $OUT/tests.log 2>&1 || exit 10
for v in default head default head; do
  if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
  timeout -k 10 200 python3 -u bench.py --cpu-sample 0 --no-config5 >> $OUT/bench_$v.log 2>&1 || exit 11
done
echo done > $OUT/done
