#!/bin/bash
# Phase clocks of the config-5 kernels (experiment build, KMH_SP_PROF=1: per wave, k_sp_split's
# and k_sp_count's phases) on the default bench workload.  usage: bash profiles/r03/sprof_r03.sh <tag> [variant]
tag=${1:-sprof}
out=gpurun_out/$tag
mkdir -p $out
KMH_LIB_PATH=$PWD/build_ab/${2:-exp}/libkmerhip.so KMH_SP_PROF=1 timeout -k 10 200 python3 -u bench.py --workload sparse \
  --steps 2 --warmup 1 --cpu-sample 0 > $out/bench.log 2> $out/prof.txt || exit 11
grep "k_sp_" $out/prof.txt | tail -2
