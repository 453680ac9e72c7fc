#!/bin/bash
# Every GPU test on the committed round-4 build (10451cd31594da40).
out=gpurun_out/${1:-r04fin6}
mkdir -p $out
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
exit $rc
