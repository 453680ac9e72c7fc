#!/bin/bash
# Round 5: config 5 over the count items' key target (KMH_SP_TARGET, default 7680).
export TMPDIR=/tmp
out=gpurun_out/${1:-r05ay}
mkdir -p $out
run() { timeout -k 10 300 python3 -u bench.py --workload sparse --no-matrix --steps 5 --warmup 2 --cpu-sample 0 > $out/sp_$tag.log 2>&1 || exit $?; python3 - $out/sp_$tag.log $tag <<'P'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], round(d["ms_per_step"], 3), {k: v["mean_ms"] for k, v in (d.get("kernels") or {}).items()})
P
}
tag=default run
for v in 7424 7552 7808 7680; do tag=pass$v; export KMH_SP_TARGET=$v; run; unset KMH_SP_TARGET; done
tag=default2 run
