#!/bin/bash
# Round 5: union A/B (tree vs build_ab/base = the committed union), here the sizes pass counted bin by bin:
# the shard union cases, then the union alone (tree vs base, twice) under a kernel trace.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05am}
mkdir -p $out
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 60 --timeout-method thread -p no:cacheprovider \
  -k "shard_union" > $out/gpu_shard.log 2>&1
rc=$?
tail -2 $out/gpu_shard.log
[ $rc -eq 0 ] || exit $rc
for v in tree ${AB:-base}; do
  if [ $v = tree ]; then lib=kmer-ml_amd/kmerml/_lib/libkmerhip.so; else lib=build_ab/$v/libkmerhip.so; fi
  KMH_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace_$v -o trace -- python3 -u profiles/r05/time_union.py $v >> $out/time_union.log 2>&1 || exit $?
  f=$(find $out/trace_$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $out/kernel_stats_$v.csv
  python3 - $out/kernel_stats_$v.csv <<'P'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "shard_union" in r["Name"]]
for r in rows:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):4d} avg {float(r["AverageNs"])/1e6:8.2f} ms')
P
done
KMH_LIB_PATH=kmer-ml_amd/kmerml/_lib/libkmerhip.so timeout -k 10 240 python3 -u profiles/r05/time_union.py tree2 >> $out/time_union.log 2>&1 || exit $?
grep ": entries" $out/time_union.log
