#!/bin/bash
# Integer multiply issue rates (bin_of / pass_of), and where one simulated rank of N = 8 loses
# time: sim8 with and without the modelled all-gather copies, plain 8- and 32-genome launches,
# and a kernel trace of sim8 (the copies' kernels beside the count's).
export TMPDIR=/tmp
out=gpurun_out/${1:-r04i}
mkdir -p $out
timeout -k 10 60 ./build_ab/bin/mulrate > $out/mulrate.log 2>&1 || { cat $out/mulrate.log; exit 11; }
cat $out/mulrate.log
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 > $out/sim8_torch.log 2>&1 || exit 12
# (without the copies the gathered slots are never written, so its row-sum check fails by design:
# only a run that printed no JSON line is an error)
timeout -k 10 300 python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 --sim-copy none > $out/sim8_none.log 2>&1
rc=$?; [ $rc -ge 124 ] && exit 12; grep -q '^{' $out/sim8_none.log || exit 12
timeout -k 10 300 python3 -u bench.py --genomes 8 --cpu-sample 0 --steps 20 --no-config5 --no-e2e > $out/g8_plain.log 2>&1 || exit 13
timeout -k 10 300 python3 -u bench.py --genomes 32 --cpu-sample 0 --steps 20 --no-config5 --no-e2e > $out/g32_plain.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o sim8 -- python3 -u bench.py --simulate-ranks 8 --cpu-sample 0 --steps 20 > $out/sim8_prof.log 2>&1 || exit 15
python3 - $out <<'P'
import json, sys
out = sys.argv[1]
for n in ("sim8_torch", "sim8_none", "g8_plain", "g32_plain"):
    r = [json.loads(l) for l in open(f"{out}/{n}.log") if l.startswith("{")][-1]
    print(n, round(r["ms_per_step"], 4), {k: round(v["mean_ms"], 4) for k, v in r["kernels"].items()})
P
