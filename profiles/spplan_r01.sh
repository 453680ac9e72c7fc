#!/bin/bash
# Device-planned sparse work items (no host item building / uploads; one batch of 16 genomes):
# sparse parity tests, config-5 bench twice (step-time variance), host-phase timing.
export TMPDIR=/tmp
OUT=gpurun_out/spplan
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/bench1.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/bench2.log 2>&1 || exit 12
KMH_SP_PROF=2 timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 --steps 3 > $OUT/hprof.log 2>&1 || exit 13
echo done > $OUT/done
