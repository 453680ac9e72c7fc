#!/bin/bash
# A/B of config 5 (bench.py --workload sparse) between the default library and variants built
# by profiles/r04/build_ab.sh.  What-if variants count wrong by design (their rows check fails
# and the fallback is off: KMH_SP_NO_FALLBACK); only their kernel times are read.
# usage: bash profiles/r04/ab_sparse.sh <tag> <rounds> <variant>...
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for round in $(seq $rounds); do
  for v in default "$@"; do
    if [ $v = default ]; then unset KMH_LIB_PATH KMH_SP_NO_FALLBACK
    else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so KMH_SP_NO_FALLBACK=1; fi
    timeout -k 10 240 python3 -u bench.py --workload sparse --steps 5 --warmup 2 --cpu-sample 0 >> $out/$v.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && ! grep -q '^{' $out/$v.log; then echo "variant $v failed rc=$rc"; tail -20 $out/$v.log; exit 11; fi
    if [ $rc -ge 124 ]; then echo "variant $v rc=$rc"; exit 12; fi
  done
done
python3 - "$out" default "$@" <<'P'
import json, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    rows = [json.loads(l) for l in open(f"{out}/{v}.log") if l.startswith("{")]
    print(v, [round(r["ms_per_step"], 2) for r in rows],
          {k: [round(r["kernels"][k]["mean_ms"], 2) for r in rows] for k in rows[0]["kernels"]},
          "checked", [r["rows_checked"] for r in rows])
P
