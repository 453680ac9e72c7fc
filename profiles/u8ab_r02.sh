#!/bin/bash
# EXPERIMENT (library not in the tree's sources): the config-3 count with u8 LDS tables in
# 512-thread workgroups (two per CU; no exact recount: uniform genomes never pass 255 per bin
# at k = 12, and the bench's row sums check that) against the default u16 / 1024-thread count.
# Usage (GPU box): bash profiles/u8ab_r02.sh <tag>   (needs build_ab/u8/libkmerhip.so)
export TMPDIR=/tmp
tag=${1:-u8ab}
OUT=gpurun_out/$tag
mkdir -p $OUT
for v in default u8 default u8; do
  if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
  timeout -k 10 200 python3 -u bench.py --cpu-sample 0 --no-config5 >> $OUT/bench_$v.log 2>&1 || exit 11
done
echo done > $OUT/done
