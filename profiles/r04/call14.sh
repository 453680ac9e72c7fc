#!/bin/bash
# Split items in tile order (order: neighbouring buckets of one tile range adjacent, sharing their
# segments' boundary lines in one XCD's L2) vs bucket order (default); config-5 A/B, 3 rounds,
# then a FETCH_SIZE pass of config 5 on the order variant.
export TMPDIR=/tmp
out=gpurun_out/${1:-r04o}
bash profiles/r04/ab_sparse.sh ${1:-r04o}/ab 3 order || exit 12
export KMH_LIB_PATH=$PWD/build_ab/order/libkmerhip.so
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/f -o f -- python3 bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 > $out/f.log 2>&1 || exit 13
