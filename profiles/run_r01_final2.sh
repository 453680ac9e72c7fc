#!/bin/bash
# Round-1 final (2): every GPU test, smoke(), the default bench line (config 3), rocprofv3
# kernel-trace stats of the same command, and separate FETCH_SIZE / WRITE_SIZE passes.
export TMPDIR=/tmp
OUT=gpurun_out/final2
mkdir -p $OUT
B="bench.py --steps 10 --warmup 3"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 300 python3 -u $B > $OUT/bench.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $B --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/fetch.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o write -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > $OUT/write.log 2>&1 || exit 15
echo done > $OUT/done
