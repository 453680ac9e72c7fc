#!/bin/bash
# End-of-round regression on the committed HEAD: every GPU test, smoke(), the default bench line,
# rocprofv3 kernel stats of the same bench, then the FETCH_SIZE / WRITE_SIZE passes that
# profiles/pmc_traffic.json is built from (profiles/pmc_summary.py, CPU side).
# Usage (GPU box): bash profiles/final_r02.sh <tag>
export TMPDIR=/tmp
tag=${1:-final}
bash profiles/reg_r02.sh $tag || exit $?
bash profiles/pmc_r02.sh ${tag}_pmc || exit $?
