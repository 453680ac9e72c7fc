#!/bin/bash
# Four ranks on the one GPU (gloo, every rank on cuda:0): the default u4 + escape assembly at
# k = 12 through bench.py, even (8 genomes) and uneven (10 genomes) shards -- logic only.
export TMPDIR=/tmp
OUT=gpurun_out/mg4
mkdir -p $OUT
R="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1"
timeout -k 10 400 $R --master-port 29541 bench.py --gpus 4 --steps 3 --warmup 1 --genomes 8 --genome-len 10000000 --backend gloo --single-device > $OUT/u4_w4_g8.log 2>&1 || exit 11
timeout -k 10 400 $R --master-port 29542 bench.py --gpus 4 --steps 3 --warmup 1 --genomes 10 --genome-len 10000000 --backend gloo --single-device > $OUT/u4_w4_g10.log 2>&1 || exit 12
echo done > $OUT/done
