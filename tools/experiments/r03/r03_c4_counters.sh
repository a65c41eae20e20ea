#!/bin/bash
# Round 3: GPU suite, the default bench line, then the C4 (1024^3 u8 @ 2048^2) counter passes
# (TA/TD/TCP and SQ/VALU sets, as for C3 in round 2) on serial whole-frame launches.
# Every GPU step under its own time limit, chained with && (the first failure ends it).
set -o pipefail
TAG=${1:-r03_first}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
C4="--n 1024 --dtype uint8 --size 2048x2048 --shading 0 --ert 0 --frames 10" &&
cat tools/pmc_sets_ta.txt tools/pmc_sets_valu.txt > $O/sets.txt &&
PASS_TIMEOUT=90 bash tools/pmc_passes.sh $TAG/c4_counters $O/sets.txt $C4
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
