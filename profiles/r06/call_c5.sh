#!/bin/bash
# Config 5 count A/B: kernel stats of the default bench (config 3 + config 5 count, no matrix / e2e).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06c5}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t -o t -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-matrix > $OUT/bench.log 2>&1 || exit 12
python3 - "$OUT" <<'PY'
import csv, json, sys
out = sys.argv[1]
for r in csv.DictReader(open(out + "/t/t_kernel_stats.csv")):
    if any(k in r["Name"] for k in ("k_sp_", "k_partition", "k_bucket")):
        print(f'{r["Name"][:60]:60s} {r["Calls"]:>4s} {float(r["AverageNs"])/1e3:9.1f}us')
l = [x for x in open(out + "/bench.log") if x.startswith("{")][-1]
d = json.loads(l)
print("config3", d["ms_per_step"], "config5", d.get("config5", {}).get("ms_per_step"))
PY
echo done > $OUT/done
