#!/bin/bash
# Round 5: the warm-up effect on config 3 (N = 1) and on the simulated N = 8 rank.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05af}
mkdir -p $out
run() { timeout -k 10 300 python3 -u bench.py --cpu-sample 0 --no-config5 --no-e2e "$@" > $out/b_$tag.log 2>&1 || exit $?; python3 - $out/b_$tag.log $tag <<'P'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], round(d["ms_per_step"], 4), {k: v["mean_ms"] for k, v in (d.get("kernels") or {}).items()})
P
}
tag=c3_w3 run --steps 20 --warmup 3
tag=c3_w30 run --steps 20 --warmup 30
tag=c3_w3b run --steps 20 --warmup 3
tag=sim8_w30 run --simulate-ranks 8 --steps 20 --warmup 30
tag=sim8_w100 run --simulate-ranks 8 --steps 50 --warmup 100
