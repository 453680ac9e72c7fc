#!/bin/bash
# Round 5: k_sp_split counting the next item's pass histogram before this item's stores
# (build_ab/split2): sparse / drop-in GPU tests on that library, then an A/B of the config-5 step
# against the tree's library (two rounds of 5 steps).
export TMPDIR=/tmp
out=gpurun_out/${1:-r05s}
mkdir -p $out
KMH_LIB_PATH=$PWD/build_ab/split2/libkmerhip.so timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sparse or sorted or shard or dropin or count_host" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
for round in 1 2; do
  for v in default split2; do
    if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
    timeout -k 10 240 python3 -u bench.py --workload sparse --no-matrix --steps 5 --warmup 2 --cpu-sample 0 >> $out/ab_$v.log 2>&1 || exit 11
  done
done
unset KMH_LIB_PATH
python3 - "$out" <<'P'
import json, sys
out = sys.argv[1]
for v in ("default", "split2"):
    rows = [json.loads(l) for l in open(f"{out}/ab_{v}.log") if l.startswith("{")]
    print(v, [round(r["ms_per_step"], 2) for r in rows],
          {k: [round(r["kernels"][k]["mean_ms"], 2) for r in rows] for k in rows[0]["kernels"]})
P
