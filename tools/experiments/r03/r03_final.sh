#!/bin/bash
# Round 3 final: the GPU suite and the round measurement (r03_suite_measure.sh), then bench
# lines of the other BASELINE configurations (C2, C4, C5; no variants, no CPU baseline).
set -o pipefail
TAG=${1:-r03_final}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
bash tools/experiments/r03/r03_suite_measure.sh $TAG || exit $?
for cfg in c2 c4 c5; do
  st=100; [ $cfg = c5 ] && st=30
  timeout -k 10 300 python bench.py --config $cfg --no-variants --no-cpu-baseline --steps $st --warmup 30 \
      > $O/b_$cfg.json 2> $O/b_$cfg.err || exit $?
done
echo done > $O/rc_final.txt
