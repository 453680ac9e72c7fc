#!/bin/bash
# Round 5: bench.py with a minimum warm-up time: the bench GPU tests, one simulated N = 8 rank at
# the default warm-up (3 steps + up to 60 ms), and the default config-3 line.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05ag}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "bench" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 > $out/sim8_torch.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 > $out/sim8_torch2.log 2>&1 || exit $?
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 --sim-copy none > $out/sim8_none.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --no-e2e --no-config5 > $out/bench.log 2>&1 || exit $?
for f in sim8_torch sim8_torch2 sim8_none bench; do python3 - $out/$f.log $f <<'P'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], round(d["ms_per_step"], 4), d["warmup"], d.get("warmup_steps_run"), {k: v["mean_ms"] for k, v in (d.get("kernels") or {}).items()})
P
done
