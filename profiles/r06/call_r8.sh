#!/bin/bash
# Round 6: the N = 8 code path rehearsed with 8 ranks sharing cuda:0 over gloo (small sizes):
# config 4's u4 all-gather and the config5 object's count + compact all-to-all + global check.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06r8}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 8 --backend gloo --single-device --genomes 16 --genome-len 3000000 --k 12 --steps 2 --warmup 1 \
  --cpu-sample 0 --config5-genomes-per-rank 2 --config5-genome-len 30000000 > $OUT/rehearsal8.log 2>&1 || exit 10
grep '^{' $OUT/rehearsal8.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config5']; m=c['matrix']; print(d['rows_checked'], d['allgather']['wire'], c['n_gpus'], c['rows_checked'], m['shard_checked'], m['global'], m['global_windows'], m['exchange']['wire'], m['exchange']['bytes_per_entry'])"
