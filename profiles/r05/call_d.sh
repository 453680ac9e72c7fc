#!/bin/bash
# Round 5: replicated partition counters + device padding compaction: sparse / sorted / shard GPU
# tests on the tree's library, the sparse bench with the matrix leg, then an A/B of the count
# against the previous build (build_ab/base: single partition counters).
out=gpurun_out/${1:-r05d}
mkdir -p $out
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $out/build_id.txt
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sparse or sorted or shard or dropin or count_host" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 --steps 3 --warmup 1 > $out/sparse.log 2>&1 || exit $?
tail -c 400 $out/sparse.log
for round in 1 2; do
  for v in default base; do
    if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
    timeout -k 10 240 python3 -u bench.py --workload sparse --no-matrix --steps 5 --warmup 2 --cpu-sample 0 >> $out/ab_$v.log 2>&1 || exit 11
  done
done
unset KMH_LIB_PATH
python3 - "$out" <<'P'
import json, sys
out = sys.argv[1]
for v in ("default", "base"):
    rows = [json.loads(l) for l in open(f"{out}/ab_{v}.log") if l.startswith("{")]
    print(v, [round(r["ms_per_step"], 2) for r in rows],
          {k: [round(r["kernels"][k]["mean_ms"], 2) for r in rows] for k in rows[0]["kernels"]})
P
