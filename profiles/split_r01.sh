#!/bin/bash
# One genome split across ranks (count_genome_split): RCCL with one rank, gloo with 2/3 ranks on cuda:0.
export TMPDIR=/tmp
OUT=gpurun_out/split
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "genome_split" > $OUT/tests.log 2>&1 || exit 10
echo done > $OUT/done
