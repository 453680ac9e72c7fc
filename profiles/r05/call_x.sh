#!/bin/bash
# Round 5: one simulated N = 8 rank with consecutive steps overlapped on two contexts / streams.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05ad}
mkdir -p $out
timeout -k 10 300 python3 -u profiles/r05/overlap_steps.py > $out/overlap.log 2>&1
rc=$?
cat $out/overlap.log | tail -12
exit $rc
