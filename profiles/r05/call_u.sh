#!/bin/bash
# Round 5: the one-pass union with a 512-unit look-back window: the shard union cases, then the
# union alone on 16 x 250 M codes (tree vs the two-pass base).
export TMPDIR=/tmp
out=gpurun_out/${1:-r05z}
mkdir -p $out
timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 60 --timeout-method thread -p no:cacheprovider \
  -k "shard_union" > $out/gpu_shard.log 2>&1
rc=$?
tail -2 $out/gpu_shard.log
[ $rc -eq 0 ] || exit $rc
for v in tree base tree; do
  if [ $v = tree ]; then lib=kmer-ml_amd/kmerml/_lib/libkmerhip.so; else lib=build_ab/$v/libkmerhip.so; fi
  KMH_LIB_PATH=$lib timeout -k 10 240 python3 -u profiles/r05/time_union.py $v >> $out/time_union.log 2>&1 || exit $?
done
grep ": entries" $out/time_union.log
