#!/bin/bash
# Round 6: wire kernels with coalesced loads / stores (count strided, pack and unpack LDS-staged).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06i}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sharded_on_gpu or wire_round_trip or config5_object or sparse_simulated" > $OUT/tests.log 2>&1
rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit 10
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_sim -o trace -- python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim.log 2>&1 || exit 12
python3 - $OUT/trace_sim/trace_kernel_trace.csv <<'P'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for name in ['k_wire_count', 'k_wire_pack', 'k_wire_unpack', 'k_shard_union<true', 'k_shard_union<false']:
    d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if name in r['Kernel_Name']]
    print(name, [round(x, 2) for x in d][-3:])
P
grep -o '"phases_ms[^}]*}' $OUT/sim.log
grep -o '"ms_per_step": [0-9.]*' $OUT/sim.log
