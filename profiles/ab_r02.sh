#!/bin/bash
# A/B of the dense k = 12 path on one MI355X: bench at several exchange budgets.
# Usage (GPU box): bash profiles/ab_r02.sh <tag>
set -o pipefail
tag=${1:-ab}
mkdir -p gpurun_out/$tag
for b in ${BUDGETS:-1024 4096}; do
  KMH_SUF_BUDGET_MB=$b timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 \
    > gpurun_out/$tag/bench_b$b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$tag/bench_b$b.log').read().strip().splitlines()[-1]); print('budget $b', round(d['ms_per_step'],3), 'ms', {k:v['mean_ms'] for k,v in d['kernels'].items()}, d['rows_checked'])"
done
