#!/bin/bash
# Round-1 final (4): every GPU test, smoke(), the default bench line (config 3) and the config-5
# bench, rocprofv3 kernel-trace stats of both, and separate FETCH_SIZE / WRITE_SIZE passes of
# the config-5 bench (16 genomes per launch since the device item plan).
export TMPDIR=/tmp
OUT=gpurun_out/final4
mkdir -p $OUT
S="bench.py --workload sparse"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -x --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 300 python3 -u bench.py > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 python3 -u $S --cpu-sample 0 > $OUT/bench_sparse.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/strace -o strace -- python3 $S --cpu-sample 0 > $OUT/strace.log 2>&1 || exit 15
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/sfetch -o sfetch -- python3 $S --steps 1 --warmup 1 --cpu-sample 0 > $OUT/sfetch.log 2>&1 || exit 16
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/swrite -o swrite -- python3 $S --steps 1 --warmup 1 --cpu-sample 0 > $OUT/swrite.log 2>&1 || exit 17
echo done > $OUT/done
