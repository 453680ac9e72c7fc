#!/bin/bash
# A/B of the dense count kernel's loads in flight per lane with plain-add counting (experiment
# builds with -DKMH_COUNT_U=4/8 vs the default 6), config 3, twice each.
export TMPDIR=/tmp
tag=${1:-abu2}
OUT=gpurun_out/$tag
mkdir -p $OUT
for v in q u4 u8 q u4 u8; do
  KMH_LIB_PATH=kmer-ml_amd/kmerml/_lib/libkmh_${v}_exp.so timeout -k 10 300 python3 -u bench.py --cpu-sample 0 --no-config5 --steps 10 --warmup 3 >> $OUT/b_$v.log 2>&1 || exit 10
done
echo done > $OUT/done
