#!/bin/bash
# k_sp_count with a wave-level key queue: phase clocks (experiment build, 2 genomes),
# sparse parity tests, the config-5 bench line and rocprofv3 kernel stats of the same bench.
# Usage (GPU box): bash profiles/spq_r02.sh <tag> [noprof]
export TMPDIR=/tmp
tag=${1:-spq}
OUT=gpurun_out/$tag
mkdir -p $OUT
if [ -z "$2" ]; then
KMH_LIB_PATH=kmer-ml_amd/kmerml/_lib/libkmh_q_exp.so KMH_SP_PROF=1 timeout -k 10 300 python3 -u bench.py --workload sparse --genomes 2 --steps 1 --warmup 0 --cpu-sample 0 > $OUT/prof_q.log 2>&1 || exit 9
fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sparse" > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 600 python3 -u bench.py --workload sparse --steps 5 --warmup 2 --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --workload sparse --steps 3 --warmup 1 --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 13
echo done > $OUT/done
