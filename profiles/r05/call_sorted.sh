#!/bin/bash
# Round 5: sorted sparse rows, the shard union, the device sparse matrix (GPU tests), then one
# simulated N = 8 rank (layout cache, counters cleared by the partition).
out=gpurun_out/${1:-r05c}
mkdir -p $out
python3 -c "import sys; sys.path.insert(0, 'kmer-ml_amd'); from kmerml import _native; print(_native.build_id())" > $out/build_id.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sorted or shard_union or sparse_matrix or count_dense_u4_fused or context_shared or config4 or dense_partition" > $out/gpu_tests.log 2>&1
rc=$?
tail -2 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 > $out/sim8_torch.log 2>&1 || exit $?
tail -c 300 $out/sim8_torch.log
# config 5 with the device-resident matrix leg (16 x 250 Mbp, one rank)
timeout -k 10 300 python3 -u bench.py --workload sparse --cpu-sample 0 --steps 3 --warmup 1 > $out/sparse.log 2>&1
rc=$?
tail -c 600 $out/sparse.log
exit $rc
