"""Merge rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

    python profiles/pmc_summary.py FETCH_CSV WRITE_CSV KEY_SUFFIX [NOTE] [KERNELS]

KERNELS (comma-separated short names) keeps only those kernels' entries.

For each kernel: mean FETCH_SIZE and WRITE_SIZE (KB) per dispatch and
hbm_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 (FETCH_SIZE doubled: gfx950
reports half the bytes of 16-B-per-lane loads, MI355X_MICROARCH.md HBM section).  Entries are
stored under "<kernel><KEY_SUFFIX>", e.g. "k_partition:k12:L100000000:G64", which bench.py
reads, and stamped with the build id of the library that was profiled (kmh_build_id): bench.py
prints the figure only while the loaded library has the same build id.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "pmc_traffic.json")
sys.path.insert(0, os.path.join(HERE, "..", "kmer-ml_amd"))


def per_kernel(path, counter):
    vals = defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        name = row["Kernel_Name"].replace("(anonymous namespace)", "")
        short = re.sub(r"<.*", "", name.split("(")[0]).split("::")[-1].split()[-1]
        vals[short].append(float(row["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in vals.items()}


def main():
    from kmerml import _native

    fetch_csv, write_csv, suffix = sys.argv[1:4]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    keep = set(sys.argv[5].split(",")) if len(sys.argv) > 5 and sys.argv[5] else None
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    d = json.load(open(OUT)) if os.path.exists(OUT) else {}
    bid = _native.build_id()
    for k in sorted(set(f) & set(w)):
        if keep is not None and k not in keep:
            continue
        fk, n = f[k]
        wk, _ = w[k]
        entry = {"FETCH_SIZE_KB": round(fk, 1), "WRITE_SIZE_KB": round(wk, 1), "dispatches": n,
                 "hbm_bytes_per_launch": int(round((2 * fk + wk) * 1024)), "build_id": bid,
                 "source": os.path.relpath(fetch_csv, os.path.join(HERE, ".."))}
        if note:
            entry["note"] = note
        d[k + suffix] = entry
        print(k + suffix, entry)
    json.dump(d, open(OUT, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
