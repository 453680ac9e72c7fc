#!/bin/bash
# A/B of config 5 (bench.py --workload sparse) between the default library and variants built
# by profiles/r03/build_ab.sh.  usage: bash profiles/r03/ab_sparse.sh <tag> <variant>...
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for round in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
    timeout -k 10 200 python3 -u bench.py --workload sparse --steps 5 --warmup 2 --cpu-sample 0 >> $out/$v.log 2>&1 || exit 11
  done
done
python3 - "$out" default "$@" <<'P'
import json, sys, glob
out = sys.argv[1]
for v in sys.argv[2:]:
    rows = [json.loads(l) for l in open(f"{out}/{v}.log") if l.startswith("{")]
    print(v, [round(r["ms_per_step"], 2) for r in rows],
          {k: [round(r["kernels"][k]["mean_ms"], 2) for r in rows] for k in rows[0]["kernels"]})
P
