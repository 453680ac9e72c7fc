export TMPDIR=/tmp
OUT=gpurun_out/spqp2; mkdir -p $OUT
KMH_LIB_PATH=kmer-ml_amd/kmerml/_lib/libkmh_q_exp.so KMH_SP_PROF=1 timeout -k 10 300 python3 -u bench.py --workload sparse --genomes 2 --steps 1 --warmup 0 --cpu-sample 0 > $OUT/prof_q.log 2>&1
