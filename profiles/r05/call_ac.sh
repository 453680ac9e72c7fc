#!/bin/bash
# Round 5: config 5 over larger split-item targets (KMH_SP_SPLIT), two rounds.
export SWEEP_SPLIT="14336 16384 18432 20480 12288 16384 20480"
bash profiles/r05/call_ab.sh ${1:-r05ai}
