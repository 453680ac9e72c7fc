#!/bin/bash
# k_sp_count emission stores: non-temporal (KMH_SP_NTS=1, default) vs plain (0): bench each
# twice, then a WRITE_SIZE pass with plain stores.
export TMPDIR=/tmp
OUT=gpurun_out/spnts
mkdir -p $OUT
S="bench.py --workload sparse --cpu-sample 0"
for v in 0 1 0 1; do
  KMH_SP_NTS=$v timeout -k 10 300 python3 -u $S >> $OUT/nts$v.log 2>&1 || exit 11
done
KMH_SP_NTS=0 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/swrite -o swrite -- python3 $S --steps 1 --warmup 1 > $OUT/swrite.log 2>&1 || exit 12
echo done > $OUT/done
