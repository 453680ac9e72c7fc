#!/bin/bash
# Kernel-event scope A/B: HIP event pairs around every instrumented launch (--kernel-events all)
# vs only the kernels the roofline names (default); config 3 at N = 1, and two ranks on the one
# GPU (gloo, u4 assembly: encode + decode launches in the step).
export TMPDIR=/tmp
OUT=gpurun_out/kev
mkdir -p $OUT
B="bench.py --steps 10 --warmup 3 --cpu-sample 0"
timeout -k 10 200 python3 -u $B --kernel-events all > $OUT/n1_all.log 2>&1 || exit 11
timeout -k 10 200 python3 -u $B > $OUT/n1_roof.log 2>&1 || exit 12
T="-m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --single-device --genomes 8 --steps 5 --warmup 2 --cpu-sample 0"
timeout -k 10 300 python3 -u $T --kernel-events all > $OUT/n2_all.log 2>&1 || exit 13
timeout -k 10 300 python3 -u $T > $OUT/n2_roof.log 2>&1 || exit 14
echo done > $OUT/done
