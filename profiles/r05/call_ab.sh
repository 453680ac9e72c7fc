#!/bin/bash
# Round 5: config 5 (--workload sparse, no matrix leg) over the split items' entry target
# (KMH_SP_SPLIT, default 12288) and the count items' key target (KMH_SP_TARGET, default 7680).
export TMPDIR=/tmp
out=gpurun_out/${1:-r05ah}
mkdir -p $out
run() { timeout -k 10 300 python3 -u bench.py --workload sparse --no-matrix --steps 5 --warmup 2 --cpu-sample 0 > $out/sp_$tag.log 2>&1 || exit $?; python3 - $out/sp_$tag.log $tag <<'P'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(sys.argv[2], round(d["ms_per_step"], 3), {k: v["mean_ms"] for k, v in (d.get("kernels") or {}).items()}, d.get("fallback_passes"))
P
}
tag=${SWEEP_TAGS:-default} run
for v in ${SWEEP_SPLIT:-}; do tag=split$v; export KMH_SP_SPLIT=$v; run; unset KMH_SP_SPLIT; done
