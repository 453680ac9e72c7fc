#!/bin/bash
# Round 6: transposed ustarts; union tests; simulated N = 8 rank under a kernel trace; ring shapes.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06d}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "shard_union or sharded_on_gpu or two_config5_genomes" > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit 10
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim8.log 2>&1 || exit 12
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/kernel_stats.csv
python3 - $OUT/kernel_stats.csv <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):5d} avg {float(r["AverageNs"])/1e6:9.3f} ms tot {float(r["TotalDurationNs"])/1e6:9.2f}')
P
grep -o '"phases_ms[^}]*}' $OUT/sim8.log
for shape in 4x2 8x1 8x2 12x2; do
  timeout -k 10 120 kmer-ml_amd/kmerml/_lib/ring_bench 8 64 1 3 $shape >> $OUT/ring_bench.log 2>&1 || { echo "ring_bench $shape rc=$?" >> $OUT/ring_bench.log; break; }
done
cat $OUT/ring_bench.log
