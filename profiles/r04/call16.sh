#!/bin/bash
# Phase clocks of k_sp_split and k_sp_count on the final round-4 kernels (experiment build,
# KMH_SP_PROF=1): where the split's and count's wave time goes now.
out=gpurun_out/${1:-r04p}
export KMH_SP_PROF=1
bash profiles/r04/ab_sparse.sh ${1:-r04p}/ab 1 exp0
grep -h "per wave" $out/ab/exp0.log | tail -4
