#!/bin/bash
# Round 5: kernel trace of the config-5 bench with its matrix leg (sorted rows, compaction, shard
# union): per-kernel times of the device-resident matrix path.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05g2}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 bench.py --workload sparse --steps 1 --warmup 1 --cpu-sample 0 > $out/trace.log 2>&1 || exit 12
tail -c 600 $out/trace.log
f=$(ls $out/trace/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] || f=$(find $out/trace -name "*kernel_stats.csv" | head -1)
cp "$f" $out/kernel_stats.csv
python3 - $out/kernel_stats.csv <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e6:10.2f} ms  avg {float(r["AverageNs"])/1e3:10.1f} us')
P
