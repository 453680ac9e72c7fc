#!/bin/bash
# Config 3 with small batches (the exchange of one or two genomes stays in the Infinity Cache)
# and one count workgroup per bucket (no split rows): experiment build, KMH_COUNT_S=1.
export TMPDIR=/tmp
tag=${1:-mall}
OUT=gpurun_out/$tag
mkdir -p $OUT
LIB=kmer-ml_amd/kmerml/_lib/libkmh_q_exp.so
for mb in 230 460 920 8192; do
  KMH_LIB_PATH=$LIB KMH_SUF_BUDGET_MB=$mb KMH_COUNT_S=1 timeout -k 10 300 python3 -u bench.py --cpu-sample 0 --no-config5 --steps 10 --warmup 3 > $OUT/b$mb.log 2>&1 || exit 10
done
echo done > $OUT/done
