#!/bin/bash
# A/B of dense k = 12 scheduling: KMH_DENSE_STREAMS (1 | 2) x KMH_SUF_BUDGET_MB.
set -o pipefail
tag=${1:-ab}
mkdir -p gpurun_out/$tag
for st in ${STREAMS:-1 2}; do
for b in ${BUDGETS:-4096}; do
  KMH_DENSE_STREAMS=$st KMH_SUF_BUDGET_MB=$b timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 \
    > gpurun_out/$tag/bench_s${st}_b$b.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$tag/bench_s${st}_b$b.log').read().strip().splitlines()[-1]); print('streams $st budget $b', round(d['ms_per_step'],3), 'ms', {k:(v['mean_ms'],v['launches']) for k,v in d['kernels'].items()}, d['rows_checked'])"
done
done
