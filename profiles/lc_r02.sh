#!/bin/bash
export TMPDIR=/tmp
# Low-complexity dense / sparse parity tests (one bucket per tile, both counter halves).
# Usage (GPU box): bash profiles/lc_r02.sh
mkdir -p gpurun_out/lc
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider -k "low_complexity or partition_many or long_runs" > gpurun_out/lc/tests.log 2>&1
