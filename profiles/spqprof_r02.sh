#!/bin/bash
# k_sp_count phase counters (KMH_SP_PROF=1, experiment builds): per-lane queue vs the
# committed 8-key calls, 2 config-5 genomes; then both at 16 genomes without counters.
export TMPDIR=/tmp
tag=${1:-spqprof}
OUT=gpurun_out/$tag
mkdir -p $OUT
for v in old q; do
  KMH_LIB_PATH=kmer-ml_amd/kmerml/_lib/libkmh_${v}_exp.so KMH_SP_PROF=1 timeout -k 10 300 python3 -u bench.py --workload sparse --genomes 2 --steps 1 --warmup 0 --cpu-sample 0 > $OUT/prof_$v.log 2>&1 || exit 10
done
for v in old q; do
  KMH_LIB_PATH=kmer-ml_amd/kmerml/_lib/libkmh_${v}_exp.so timeout -k 10 300 python3 -u bench.py --workload sparse --steps 3 --warmup 1 --cpu-sample 0 > $OUT/bench_$v.log 2>&1 || exit 11
done
echo done > $OUT/done
