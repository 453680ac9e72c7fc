#!/bin/bash
# Experiment: is the config-3 exchange served from the Infinity Cache when a batch is one genome
# (214 MB of suffixes) and the partition stores it with plain instead of non-temporal stores?
# build_ab/exp (the default kernels, experiment knobs on: nt stores) vs build_ab/plain, each at the
# default 8 GiB budget and at one genome per batch (KMH_SUF_BUDGET_MB=230), one count workgroup
# per bucket (KMH_COUNT_S=1: no split rows added with atomics).  usage: bash profiles/r03/mall_r03.sh <tag>
tag=${1:-mall}
out=gpurun_out/$tag
mkdir -p $out
for v in exp plain; do
  for b in 8192 230; do
    export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so
    KMH_COUNT_S=1 KMH_SUF_BUDGET_MB=$b timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-config5 \
      > $out/${v}_$b.log 2>&1 || exit 11
  done
done
python3 - "$out" <<'P'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.log")):
    r = [json.loads(l) for l in open(f) if l.startswith("{")][-1]
    print(os.path.basename(f), round(r["ms_per_step"], 3), {k: (v["launches"], round(v["mean_ms"], 3)) for k, v in r["kernels"].items()})
P
