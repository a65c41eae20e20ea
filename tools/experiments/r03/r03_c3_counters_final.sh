#!/bin/bash
# Round 3 final build: the C3 counter passes (TA/TD/TCP and VALU sets) of the headline kernel,
# binary16 field, serial whole-frame launches (tools/pmc_passes.sh), and their summary.
set -o pipefail
TAG=${1:-r03_c3_counters_final}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
cat tools/pmc_sets_ta.txt tools/pmc_sets_valu.txt > $O/sets.txt
PASS_TIMEOUT=90 bash tools/pmc_passes.sh $TAG/half $O/sets.txt --frames 10 || exit $?
python tools/gather_report.py $O/half > $O/half_summary.json 2> $O/half_summary.err
echo done > $O/rc.txt
