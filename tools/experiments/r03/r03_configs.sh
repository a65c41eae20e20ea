#!/bin/bash
# Round 3: bench lines of the other BASELINE configurations (C2, C4, C5; 3 frames in flight,
# as the headline) and their PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs of
# bench.py itself), so their roofline fields are measured on this build too.  Each GPU step
# under its own time limit; chained (the first failure ends it).
set -o pipefail
TAG=${1:-r03_configs}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for cfg in c2 c4 c5; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${cfg}_$ctr -o run \
        --output-format csv -- python3 bench.py --config $cfg --no-variants --no-cpu-baseline \
        --steps 10 --warmup 3 > $O/pmc_${cfg}_$ctr.log 2>&1 || exit $?
  done
done
python tools/traffic_json.py $O $O/pmc_traffic_configs.json > /dev/null || exit $?
for cfg in c2 c4 c5; do
  steps=100; warm=50
  [ $cfg = c5 ] && steps=40 && warm=20
  timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline --steps $steps --warmup $warm \
      > $O/bench_$cfg.json 2> $O/bench_$cfg.err || exit $?
done
echo done > $O/rc.txt
