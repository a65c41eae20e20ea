#!/bin/bash
# Round 3: the GPU suite (up to 10 failures reported), then, only if it passed, the round
# measurement (tools/measure_round.sh <tag>).  Each GPU step under its own time limit.
set -o pipefail
TAG=${1:-r03_suite_measure}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
VR_PARITY_LOG=$O/parity_fullsize.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q \
    --maxfail=10 --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
echo "suite rc=$rc" > $O/rc_suite.txt
[ $rc -eq 0 ] || exit $rc
bash tools/measure_round.sh $TAG/measure
