#!/bin/bash
# Count bins: bit-field (default) vs multiply (binmul); split descriptors by vector loads (vdesc); 3 rounds; then call8's measurements
# (integer multiply rates; sim8 with and without the modelled all-gather copies; 8/32-genome
# launches; kernel trace of sim8).
bash profiles/r04/ab_sparse.sh ${1:-r04l}/ab 3 binmul vdesc || exit 12
bash profiles/r04/call8.sh ${1:-r04l}/m
