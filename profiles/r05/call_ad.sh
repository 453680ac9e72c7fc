#!/bin/bash
# Round 5: SQ / TCC counters of the shard union's two passes (profiles/r05/time_union.py, 16 x
# 250 M sorted random k = 21 codes), one --pmc set per run.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05al}
mkdir -p $out
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $out/p$i -o p$i -- python3 profiles/r05/time_union.py pmc$i > $out/p$i.log 2>&1 || { echo "pass $i failed"; exit 11; }
done
python3 - $out <<'P'
import csv, glob, sys
from collections import defaultdict
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "shard_union" not in n:
            continue
        key = "union<" + n.split("k_shard_union<")[1].split(">")[0] + ">"
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(sys.argv[1] + "/summary.txt", "w") as o:
    for k in sorted(vals):
        print(k, file=o)
        for c in sorted(vals[k]):
            v = vals[k][c]
            print(f"   {c:24s} n={len(v):3d} mean={sum(v) / len(v):.4g}", file=o)
print(open(sys.argv[1] + "/summary.txt").read())
P
