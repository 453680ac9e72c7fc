#!/bin/bash
# A/B + ablation sweep of the k=12 partition/count kernels (bench.py, config 3).
OUT=gpurun_out/ablate
mkdir -p $OUT
run() { name=$1; shift; env "$@" timeout -k 10 150 python3 bench.py --steps 5 --warmup 2 --cpu-sample 0 > $OUT/$name.log 2>&1; echo "$name rc=$?" >> $OUT/summary.txt; }
run base
run tpb1024 KMH_TPB=1024
run p1_nohist KMH_ABLATE_P=1
run p2_noscatter KMH_ABLATE_P=2
run p4_nowrite KMH_ABLATE_P=4
run c1_noatomic KMH_ABLATE_C=1
run c2_noload KMH_ABLATE_C=2
run budget512 KMH_SUF_BUDGET_MB=512
for f in $OUT/*.log; do echo "$f $(grep -o '"kernels": {[^}]*}[^}]*}[^}]*}' $f)" >> $OUT/summary.txt; done
