#!/bin/bash
# A/B of the count kernel's loads in flight per lane (KMH_COUNT_U builds in build_ab/) on config 3.
set -o pipefail
tag=${1:-abu}
mkdir -p gpurun_out/$tag
for lib in kmer-ml_amd/kmerml/_lib/libkmerhip.so build_ab/libkmerhip_u4.so build_ab/libkmerhip_u5.so build_ab/libkmerhip_u7.so; do
  n=$(basename $lib .so)
  KMH_LIB_PATH=$PWD/$lib timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --cpu-sample 0 > gpurun_out/$tag/$n.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/$tag/$n.log').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],3), {k:v['mean_ms'] for k,v in d['kernels'].items()}, d['rows_checked'])"
done
