#!/bin/bash
# Round 3: the TA/TD/TCP and SQ/VALU counter sets on the round-3 C3 headline kernel (binary16
# field, deferred shading; serial whole-frame launches), and the same for the exact f32 field
# (exact_gradient = 1), as round 2 did for its C3 kernel.  One rocprofv3 --pmc run per group.
set -o pipefail
TAG=${1:-r03_c3_counters}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
cat tools/pmc_sets_ta.txt tools/pmc_sets_valu.txt > $O/sets.txt
PASS_TIMEOUT=90 bash tools/pmc_passes.sh $TAG/half $O/sets.txt --frames 10 || exit $?
PASS_TIMEOUT=90 bash tools/pmc_passes.sh $TAG/exact $O/sets.txt --frames 10 --exact-gradient 1 || exit $?
python tools/gather_report.py $O/half > $O/half_summary.json 2> $O/half_summary.err
python tools/gather_report.py $O/exact > $O/exact_summary.json 2> $O/exact_summary.err
echo done > $O/rc.txt
