#!/bin/bash
# Round 6 final, part B: rocprofv3 kernel stats of the bench (config 3 + config 5 count), the
# FETCH_SIZE / WRITE_SIZE passes profiles/pmc_traffic.json is rebuilt from (profiles/pmc_summary.py,
# CPU side), the same for config 5's matrix leg (union, wire) at N = 1 and for one simulated N = 8
# rank of it, kernel stats of both, and one simulated N = 8 rank of config 4.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06fb}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-matrix > $OUT/trace.log 2>&1 || exit 13
B="bench.py --steps 2 --warmup 1 --min-warmup-ms 0 --cpu-sample 0 --no-e2e --no-matrix"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/f -o f -- python3 $B > $OUT/f.log 2>&1 || exit 14
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/w -o w -- python3 $B > $OUT/w.log 2>&1 || exit 15
M="bench.py --workload sparse --steps 1 --warmup 0 --cpu-sample 0"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/mf -o f -- python3 $M > $OUT/mf.log 2>&1 || exit 16
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/mw -o w -- python3 $M > $OUT/mw.log 2>&1 || exit 17
S="bench.py --workload sparse --simulate-ranks 8 --steps 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/sf -o f -- python3 $S > $OUT/sf.log 2>&1 || exit 18
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/sw -o w -- python3 $S > $OUT/sw.log 2>&1 || exit 19
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_sparse -o trace -- python3 -u bench.py --workload sparse --steps 3 --cpu-sample 0 > $OUT/sparse.log 2>&1 || exit 20
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_sim -o trace -- python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim8_sparse.log 2>&1 || exit 21
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --steps 20 --warmup 5 --cpu-sample 0 --no-e2e --no-config5 > $OUT/sim8.log 2>&1 || exit 22
tail -c 300 $OUT/sim8.log
echo done > $OUT/done
