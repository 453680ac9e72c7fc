"""Per-kernel mean of every counter in the rocprofv3 counter_collection CSVs under a directory.

    python profiles/sq_summary.py gpurun_out/<tag>
"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)", "")
    return re.sub(r"<.*", "", name.split("(")[0]).split("::")[-1].split()[-1]


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(path)):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(vals):
        print(k)
        for c in sorted(vals[k]):
            v = vals[k][c]
            print(f"   {c:24s} n={len(v):3d} mean={sum(v) / len(v):.4g}")


if __name__ == "__main__":
    main()
