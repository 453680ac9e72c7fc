#!/bin/bash
# k_sp_count with the low-VALU insert loop: sparse parity tests, config-5 bench, one SQ pass.
export TMPDIR=/tmp
OUT=gpurun_out/spv3
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "sparse" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 > $OUT/bench.log 2>&1 || exit 11
B="bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 --genomes 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $OUT/p1 -o p1 -- python3 $B > $OUT/p1.log 2>&1 || exit 12
echo done > $OUT/done
