#!/bin/bash
# Final round-4 regression of the committed build (profiles/r04/final_r04.sh: every GPU test,
# smoke, bench, kernel trace, FETCH/WRITE passes), then a kernel trace of one simulated rank of
# N = 8 (its small kernels and gaps beside partition and count).
export TMPDIR=/tmp
bash profiles/r04/final_r04.sh ${1:-r04fin4} || exit $?
out=gpurun_out/${1:-r04fin4}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/sim8 -o sim8 -- python3 bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 > $out/sim8.log 2>&1 || exit 16
