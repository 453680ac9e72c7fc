#!/bin/bash
# Phase clocks of the config-3 count kernel (experiment build, KMH_DENSE_PROF=1): per wave, the
# table clear, the walk over the exchange, the reduction, the widening + row stores, the check.
tag=${1:-dprof}
out=gpurun_out/$tag
mkdir -p $out
KMH_LIB_PATH=$PWD/build_ab/${2:-exp}/libkmerhip.so KMH_DENSE_PROF=1 timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 \
  --cpu-sample 0 --no-config5 --no-kernel-events > $out/bench.log 2> $out/prof.txt || exit 11
tail -4 $out/prof.txt
