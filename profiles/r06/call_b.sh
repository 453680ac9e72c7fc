#!/bin/bash
# Round 6: kernel trace of one simulated N = 8 rank of the config-5 matrix (R = 128 union).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06b}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim8.log 2>&1 || exit 12
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e6:9.3f} ms tot {float(r["TotalDurationNs"])/1e6:9.2f}')
P
tail -c 1500 $OUT/sim8.log
