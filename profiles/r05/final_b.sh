#!/bin/bash
# Round-5 regression, part B, on the committed HEAD: the default bench line, rocprofv3 kernel
# stats of the same bench, the FETCH_SIZE / WRITE_SIZE passes that profiles/pmc_traffic.json is
# rebuilt from (profiles/pmc_summary.py, CPU side), one simulated N = 8 rank, and the config-5
# bench with its matrix leg.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05fb}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 400 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
tail -c 300 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --no-e2e --no-matrix > $OUT/trace.log 2>&1 || exit 13
B="bench.py --steps 2 --warmup 1 --min-warmup-ms 0 --cpu-sample 0 --no-e2e --no-matrix"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/f -o f -- python3 $B > $OUT/f.log 2>&1 || exit 14
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/w -o w -- python3 $B > $OUT/w.log 2>&1 || exit 15
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --steps 20 --warmup 5 --cpu-sample 0 --no-e2e --no-config5 > $OUT/sim8.log 2>&1 || exit 16
tail -c 400 $OUT/sim8.log
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 --steps 3 --warmup 1 > $OUT/sparse.log 2>&1 || exit 17
tail -c 600 $OUT/sparse.log
echo done > $OUT/done
