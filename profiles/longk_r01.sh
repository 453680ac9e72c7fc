#!/bin/bash
# Long k-mers (33 <= k <= 1024) on the GPU: the full GPU suite (golden k = 33 / 40 drop-in
# cases now byte-identical; long-k parity vs the Python oracle) and smoke().
export TMPDIR=/tmp
OUT=gpurun_out/longk
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -x --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || exit 10
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 11
echo done > $OUT/done
