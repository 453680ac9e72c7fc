#!/bin/bash
# Round 5: the sorted rows' phases (alloc / count / compaction) in the sparse bench's matrix leg,
# an A/B of the partition's counters (tree: one counter per bucket; build_ab/rep16: bank-replicated
# counters), and the LDS counter pass of both on 4 genomes.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05e}
mkdir -p $out
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $out/build_id.txt
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 --steps 3 --warmup 1 > $out/sparse.log 2>&1 || exit $?
tail -c 900 $out/sparse.log
for round in 1 2; do
  for v in default rep16; do
    if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
    timeout -k 10 240 python3 -u bench.py --workload sparse --no-matrix --steps 5 --warmup 2 --cpu-sample 0 >> $out/ab_$v.log 2>&1 || exit 11
  done
done
unset KMH_LIB_PATH
python3 - "$out" <<'P'
import json, sys
out = sys.argv[1]
for v in ("default", "rep16"):
    rows = [json.loads(l) for l in open(f"{out}/ab_{v}.log") if l.startswith("{")]
    print(v, [round(r["ms_per_step"], 2) for r in rows],
          {k: [round(r["kernels"][k]["mean_ms"], 2) for r in rows] for k in rows[0]["kernels"]})
P
B="bench.py --workload sparse --no-matrix --steps 1 --warmup 1 --cpu-sample 0 --genomes 4"
for v in default rep16; do
  if [ $v = default ]; then unset KMH_LIB_PATH; else export KMH_LIB_PATH=$PWD/build_ab/$v/libkmerhip.so; fi
  mkdir -p $out/sq_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $out/sq_$v/p2 -o p2 -- python3 $B > $out/sq_$v/p2.log 2>&1 || exit 12
  python3 profiles/sq_summary.py $out/sq_$v > $out/sq_$v/summary.txt
  grep -A9 "^k_sp_partition" $out/sq_$v/summary.txt
done
