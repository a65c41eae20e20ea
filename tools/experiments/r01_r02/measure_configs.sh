#!/bin/bash
# Every BASELINE config through bench.py on one GPU (C3 is the default bench line; the rest
# are reported in DESIGN.md §8).  C4/C5 skip the CPU baseline (the oracle would need minutes
# per frame).  Each run has its own time limit; chained with &&.
# Usage: bash tools/experiments/r01_r02/measure_configs.sh <tag>
set -o pipefail
TAG=${1:-configs}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --config c1 --steps 30 --warmup 5 > $O/c1.json 2> $O/c1.err &&
timeout -k 10 300 python bench.py --config c2 --steps 30 --warmup 5 > $O/c2.json 2> $O/c2.err &&
timeout -k 10 400 python bench.py --config c4 --steps 30 --warmup 5 --no-cpu-baseline --no-variants > $O/c4.json 2> $O/c4.err &&
timeout -k 10 600 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-variants > $O/c5.json 2> $O/c5.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
