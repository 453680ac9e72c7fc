#!/bin/bash
# A/B of config 3 (bench.py, no config-5 leg) between the default library and variants built by
# profiles/r03/build_ab.sh (experiment variants may count wrong on purpose: the JSON line is
# printed before the row check).  usage: bash profiles/r03/ab_dense.sh <tag> <variant>...
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for round in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-config5 >> $out/$v.log 2>&1
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
python3 - "$out" default "$@" <<'P'
import json, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    rows = [json.loads(l) for l in open(f"{out}/{v}.log") if l.startswith("{")]
    print(v, [round(r["ms_per_step"], 3) for r in rows],
          {k: [round(r["kernels"][k]["mean_ms"], 3) for r in rows] for k in rows[0]["kernels"]})
P
