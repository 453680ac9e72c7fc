#!/bin/bash
# A/B: config-3 count kernel with LDS adds whose returned values are unused (ds_add_u32 instead of
# ds_add_rtn_u32; wrong past 65535 per bin, never reached by the bench genomes) vs the default.
export TMPDIR=/tmp
tag=${1:-noret}
OUT=gpurun_out/$tag
mkdir -p $OUT
for v in q noret q noret; do
  KMH_LIB_PATH=kmer-ml_amd/kmerml/_lib/libkmh_${v}_exp.so timeout -k 10 300 python3 -u bench.py --cpu-sample 0 --no-config5 --steps 10 --warmup 3 >> $OUT/b_$v.log 2>&1 || exit 10
done
echo done > $OUT/done
