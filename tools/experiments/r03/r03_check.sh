#!/bin/bash
# Round 3 check on the GPU box: the GPU suite, then bench lines (default; frames in flight 3;
# the multi-device-context path forced at N = 1).  Each GPU step under its own time limit,
# chained with && (the first failure ends it).
set -o pipefail
TAG=${1:-r03_check}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
VR_PARITY_LOG=$O/parity_fullsize.jsonl timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_f4.json 2> $O/bench_f4.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --frames-in-flight 3 > $O/bench_f3.json 2> $O/bench_f3.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variants --multi-device-context > $O/bench_group.json 2> $O/bench_group.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
