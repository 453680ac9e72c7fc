#!/bin/bash
# Round 6, first GPU call: the new exchange (rows' cuts, compact wire, u32 shard indices) and the
# config-5 measurement paths, then config 5 at N = 1 and one simulated N = 8 rank of its matrix.
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06a}
mkdir -p $OUT
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $OUT/build_id.txt
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "wire_round_trip or sharded_on_gpu or config5_object or sparse_simulated or shard_union or two_config5_genomes" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit 10
timeout -k 10 300 python3 -u bench.py --workload sparse --steps 3 --cpu-sample 0 > $OUT/sparse.log 2>&1 || exit 11
tail -c 3000 $OUT/sparse.log
timeout -k 10 400 python3 -u bench.py --workload sparse --simulate-ranks 8 --steps 2 > $OUT/sim8.log 2>&1 || exit 12
tail -c 3000 $OUT/sim8.log
