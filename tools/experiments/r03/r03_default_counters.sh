#!/bin/bash
# Round 3: TA/TD/TCP and SQ counter sets on the reference's default camera (r = 3; C3 volume,
# 1080p), shaded (15x15x8 z-pair copy, stencil gradient) and unshaded (plain copy): serial
# whole-frame launches, one rocprofv3 --pmc run per group.
set -o pipefail
TAG=${1:-r03_default_counters}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
cat tools/pmc_sets_ta.txt tools/pmc_sets_valu.txt > $O/sets.txt
PASS_TIMEOUT=90 bash tools/pmc_passes.sh $TAG/shaded $O/sets.txt --frames 10 --cam default || exit $?
PASS_TIMEOUT=90 bash tools/pmc_passes.sh $TAG/unshaded $O/sets.txt --frames 10 --cam default --shading 0 --ert 0 || exit $?
for a in shaded unshaded; do
  python tools/gather_report.py $O/$a > $O/${a}_summary.json 2> $O/${a}_summary.err
done
echo done > $O/rc.txt
