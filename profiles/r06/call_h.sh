#!/bin/bash
# Round 6: union per-row delta tables (A/B against r06d/r06e), wire sizing cache one-shot.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06h}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "shard_union or sharded_on_gpu or two_config5_genomes or wire_round_trip" > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit 10
for w in sparse sim; do
  if [ $w = sparse ]; then args="--workload sparse --steps 3 --cpu-sample 0"; else args="--workload sparse --simulate-ranks 8 --steps 2"; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$w -o trace -- python3 -u bench.py $args > $OUT/$w.log 2>&1 || exit 12
  f=$(find $OUT/trace_$w -name "*kernel_stats.csv" | head -1)
  cp "$f" $OUT/kernel_stats_$w.csv
  python3 - $OUT/kernel_stats_$w.csv <<'P'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "shard" in r["Name"] or "wire" in r["Name"]]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e6:9.3f} ms')
P
done
grep -o '"phases_ms[^}]*}' $OUT/sim.log
grep -o '"matrix": {"matrix_ms[^,]*,[^,]*,[^,]*' $OUT/sparse.log
