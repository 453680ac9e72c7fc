"""HBM traffic of config 5's matrix leg per kernel, from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python profiles/matrix_traffic.py PMC_DIR OUT_JSON

PMC_DIR holds mf/mw (the matrix leg at N = 1: bench.py --workload sparse) and sf/sw (one
simulated N = 8 rank: --simulate-ranks 8) counter collections, as profiles/r06/final_b.sh writes
them.  read = 2 x FETCH_SIZE (gfx950 reports half the bytes of 16-B-per-lane loads,
MI355X_MICROARCH.md HBM section), written = WRITE_SIZE; KB x 1024, in GB.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = re.sub(r"^void ", "", name.split("(")[0]).replace("kmh::", "")
        vals[name].append(float(row["Counter_Value"]) * 1024.0 / 1e9)
    return vals


def main():
    d, out = sys.argv[1:3]
    res = {}
    for tag, f, w in (("N1_matrix", "mf", "mw"), ("N8_rank_sim", "sf", "sw")):
        fp = os.path.join(d, f"{f}_counter_collection.csv")
        wp = os.path.join(d, f"{w}_counter_collection.csv")
        if not (os.path.exists(fp) and os.path.exists(wp)):
            continue
        fe, wr = per_kernel(fp, "FETCH_SIZE"), per_kernel(wp, "WRITE_SIZE")
        for k in sorted(set(fe) | set(wr)):
            if not re.search(r"k_shard|k_wire|k_rows_cuts|k_sp_", k):
                continue
            rd = [2.0 * x for x in fe.get(k, [])]
            wt = wr.get(k, [])
            res[f"{tag}:{k}"] = {"dispatches": max(len(rd), len(wt)),
                                 "read_GB_per_launch_max": round(max(rd, default=0.0), 2),
                                 "written_GB_per_launch_max": round(max(wt, default=0.0), 2),
                                 "read_GB_total": round(sum(rd), 2), "written_GB_total": round(sum(wt), 2)}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(f"{len(res)} kernels -> {out}")


if __name__ == "__main__":
    main()
