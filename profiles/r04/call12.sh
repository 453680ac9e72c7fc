#!/bin/bash
# Config-5 stores: non-temporal (default) vs plain stores in the count (cntplain), in the split
# (splplain) and both (bothplain), 3 rounds; then a WRITE_SIZE pass of config 5 on bothplain
# (default's is in profiles/pmc_traffic.json): do partial lines of non-temporal stores reach HBM?
export TMPDIR=/tmp
out=gpurun_out/${1:-r04n}
bash profiles/r04/ab_sparse.sh ${1:-r04n}/ab 3 cntplain splplain bothplain || exit 12
export KMH_LIB_PATH=$PWD/build_ab/bothplain/libkmerhip.so
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/w -o w -- python3 bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 > $out/w.log 2>&1 || exit 13
