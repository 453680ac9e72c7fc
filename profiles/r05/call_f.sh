#!/bin/bash
# Round 5: split items ordered by tile range (k_sp_gplan): sparse GPU tests, an A/B of the
# config-5 step against build_ab/base (items in (genome, bucket) order), FETCH_SIZE / WRITE_SIZE
# of both on 4 genomes, then the sparse bench with the matrix leg.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05f}
mkdir -p $out
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $out/build_id.txt
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sparse or sorted or shard or dropin or count_host" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
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
B="bench.py --workload sparse --no-matrix --steps 1 --warmup 1 --cpu-sample 0 --genomes 4"
for v in default base; do
  if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
  mkdir -p $out/pmc_$v
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $out/pmc_$v/f -o f -- python3 $B > $out/pmc_$v/f.log 2>&1 || exit 12
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $out/pmc_$v/w -o w -- python3 $B > $out/pmc_$v/w.log 2>&1 || exit 13
  python3 profiles/sq_summary.py $out/pmc_$v > $out/pmc_$v/summary.txt
  grep -A3 "^k_sp_split\|^k_sp_count\|^k_sp_partition" $out/pmc_$v/summary.txt
done
unset KMH_LIB_PATH
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 --steps 3 --warmup 1 > $out/sparse.log 2>&1 || exit 14
tail -c 1200 $out/sparse.log
