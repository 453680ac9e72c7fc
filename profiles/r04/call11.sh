#!/bin/bash
# Split descriptor two items ahead: scalar load (default) vs one vector load spread over lanes
# 0-7 of one VGPR, read by readlane (vdesc); config-5 A/B, 3 rounds.
bash profiles/r04/ab_sparse.sh ${1:-r04m}/ab 3 vdesc || exit 12
