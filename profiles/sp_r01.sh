#!/bin/bash
# Config 5 (sparse k = 21 canonical) bring-up: device sparse parity tests, then a short bench.
export TMPDIR=/tmp
OUT=gpurun_out/sp
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "sparse_dev" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --workload sparse --genomes 2 --steps 2 --warmup 1 --cpu-sample 0 > $OUT/bench_g2.log 2>&1 || exit 11
timeout -k 10 600 python3 -u bench.py --workload sparse --steps 3 --warmup 1 > $OUT/bench_g16.log 2>&1 || exit 12
echo done > $OUT/done
