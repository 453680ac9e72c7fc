#!/bin/bash
# Round 5: the union sizes pass on a 4-slot table per bin (u32 offsets), adds issued before the
# stores: the shard union cases, then the union alone (tree vs the two-pass base) under a kernel
# trace.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05ab}
mkdir -p $out
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 60 --timeout-method thread -p no:cacheprovider \
  -k "shard_union" > $out/gpu_shard.log 2>&1
rc=$?
tail -2 $out/gpu_shard.log
[ $rc -eq 0 ] || exit $rc
for v in tree base; do
  if [ $v = tree ]; then lib=kmer-ml_amd/kmerml/_lib/libkmerhip.so; else lib=build_ab/$v/libkmerhip.so; fi
  KMH_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$v -o trace -- python3 -u profiles/r05/time_union.py $v >> $out/time_union.log 2>&1 || exit $?
  f=$(find $out/trace_$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $out/kernel_stats_$v.csv
  python3 - $out/kernel_stats_$v.csv <<'P'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "shard" in r["Name"]]
for r in rows:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):4d} avg {float(r["AverageNs"])/1e6:8.2f} ms')
P
done
grep ": entries" $out/time_union.log
