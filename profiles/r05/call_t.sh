#!/bin/bash
# Round 5: the shard union alone (16 x 250 M sorted random k = 21 codes) for the two-pass union
# (base), the one-pass look-back union (tree), and two what-ifs of the one-pass union: no look-back
# wait (nolb) and no look-back with static unit assignment instead of tickets (nolbst).
export TMPDIR=/tmp
out=gpurun_out/${1:-r05y}
mkdir -p $out
for v in base tree nolb nolbst; do
  if [ $v = tree ]; then lib=kmer-ml_amd/kmerml/_lib/libkmerhip.so; else lib=build_ab/$v/libkmerhip.so; fi
  KMH_LIB_PATH=$lib timeout -k 10 240 python3 -u profiles/r05/time_union.py $v >> $out/time_union.log 2>&1 || exit $?
done
cat $out/time_union.log | grep ": entries"
