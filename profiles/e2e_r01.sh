#!/bin/bash
# Drop-in path: parity tests touching the host count / ordering / writer, then end-to-end
# timing (parse, count, format, write; gzip on/off).
export TMPDIR=/tmp
mkdir -p gpurun_out/e2e
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "dropin or first or sparse or cli or count_matrix" > gpurun_out/e2e/tests.log 2>&1 || exit 9
timeout -k 10 600 python3 -u profiles/e2e_r01.py --mbp 100 > gpurun_out/e2e/e2e.log 2>&1 || exit 10
rm -rf gpurun_out/e2e/kmers
echo done > gpurun_out/e2e/done
