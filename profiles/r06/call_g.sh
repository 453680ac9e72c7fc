#!/bin/bash
# Round 6: rehearsal of the N > 1 dense line's config5 object at full genome length: 2 ranks sharing
# cuda:0 (gloo), 4 genomes of 250 Mbp per rank (config 5 has 16; 2 x 16 would not fit one GPU).
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06g}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --backend gloo --single-device --genomes 4 --genome-len 20000000 --k 12 --steps 3 --warmup 1 --cpu-sample 0 \
  --config5-genomes-per-rank 4 --config5-genome-len 250000000 > $OUT/rehearsal2.log 2>&1 || exit 10
grep '^{' $OUT/rehearsal2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config5']; m=c['matrix']; print(c['ms_per_step'], m['matrix_ms'], m['shard_checked'], m['global'], m['exchange']['wire'], m['exchange']['bytes_per_entry'], m['exchange']['sent_bytes'], m['shard_phases_rank0'])"
