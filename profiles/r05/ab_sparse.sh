#!/bin/bash
# A/B of config 5 (bench.py --workload sparse, count only) between the default library and
# variants built by profiles/r05/build_ab.sh (build_ab/<name>/libkmerhip.so), <rounds> rounds
# on one box; each variant's sparse GPU tests first (they must pass before it is timed).
# usage: bash profiles/r05/ab_sparse.sh <tag> <rounds> <variant>...
tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for v in "$@"; do
  KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider -k "sparse_dev and not config5_full" > $out/tests_$v.log 2>&1 || { tail -5 $out/tests_$v.log; exit 10; }
  tail -1 $out/tests_$v.log
done
for round in $(seq $rounds); do
  for v in default "$@"; do
    if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
    timeout -k 10 240 python3 -u bench.py --workload sparse --no-matrix --steps 5 --warmup 2 --cpu-sample 0 >> $out/$v.log 2>&1 || { tail -5 $out/$v.log; exit 11; }
  done
done
unset KMH_LIB_PATH
python3 - "$out" default "$@" <<'P'
import json, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    rows = [json.loads(l) for l in open(f"{out}/{v}.log") if l.startswith("{")]
    print(v, [round(r["ms_per_step"], 2) for r in rows],
          {k: [round(r["kernels"][k]["mean_ms"], 2) for r in rows] for k in rows[0]["kernels"]},
          "checked", [r["rows_checked"] for r in rows])
P
