#!/bin/bash
# Multi-rank assembly check on one GPU: the u8 + escape all-gather and the plain u32
# all-gather through bench.py with gloo and every rank on cuda:0 (logic only, not a number).
export TMPDIR=/tmp
OUT=gpurun_out/mg
mkdir -p $OUT
R="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "rows_u8" > $OUT/tests.log 2>&1 || exit 10
timeout -k 10 300 $R bench.py --gpus 2 --steps 3 --warmup 1 --genomes 5 --genome-len 3000000 --backend gloo --single-device --assemble u8 > $OUT/u8_w2.log 2>&1 || exit 11
timeout -k 10 300 $R bench.py --gpus 2 --steps 3 --warmup 1 --genomes 5 --genome-len 3000000 --backend gloo --single-device --assemble u32 > $OUT/u32_w2.log 2>&1 || exit 12
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 3 --steps 4 --warmup 2 --genomes 8 --genome-len 2000001 --k 10 --backend gloo --single-device > $OUT/u8_w3.log 2>&1 || exit 13
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --cpu-sample 0 > $OUT/bench1.log 2>&1 || exit 14
echo done > $OUT/done
