#!/bin/bash
# Round 6: config 5 at N = 1 (count + matrix leg) under a kernel trace; ring bench with per-XCD flags.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06e}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
for shape in 4x1 8x2; do
  timeout -k 10 120 kmer-ml_amd/kmerml/_lib/ring_bench 8 64 1 3 $shape >> $OUT/ring_bench.log 2>&1 || { echo "ring_bench $shape rc=$?" >> $OUT/ring_bench.log; break; }
done
cat $OUT/ring_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 -u bench.py --workload sparse --steps 3 --cpu-sample 0 > $OUT/sparse.log 2>&1 || exit 12
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e6:9.3f} ms tot {float(r["TotalDurationNs"])/1e6:9.2f}')
P
grep -o '"matrix": {"matrix_ms[^,]*,[^,]*,[^,]*' $OUT/sparse.log
grep -o '"shard_phases_rank0[^}]*}' $OUT/sparse.log
