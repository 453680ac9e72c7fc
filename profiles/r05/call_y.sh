#!/bin/bash
# Round 5: what the simulated N = 8 rank's line pays for: kernel event pairs and a short warm-up.
export TMPDIR=/tmp
out=gpurun_out/${1:-r05ae}
mkdir -p $out
run() { timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 "$@" > $out/sim8_$tag.log 2>&1 || exit $?; python3 - $out/sim8_$tag.log $tag <<'P'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], round(d["ms_per_step"], 4), d.get("kernels"))
P
}
tag=default run
tag=noev run --no-kernel-events
tag=warm30 run --warmup 30
tag=warm30_noev run --warmup 30 --no-kernel-events
tag=default2 run
