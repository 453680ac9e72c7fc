#!/bin/bash
# k_sp_count with next-item prefetch (bounds + first chunk) before the emission:
# sparse parity tests, config-5 bench, per-phase cycles.
export TMPDIR=/tmp
OUT=gpurun_out/sppre
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 11
KMH_SP_PROF=1 timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 --steps 2 --warmup 1 --genomes 4 > $OUT/prof.log 2>&1 || exit 12
echo done > $OUT/done
