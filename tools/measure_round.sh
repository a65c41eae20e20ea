#!/bin/bash
# Round measurement on the GPU box: smoke, bench (with CPU baseline), its rocprofv3 kernel-trace
# summary, and PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs of bench.py
# itself) for the headline C3, its default-camera and reference-semantics variants, then
# profiles/pmc_traffic.json from them (bench.py's roofline reads it).  Each GPU step has its
# own time limit; chained with && (the first failure ends the script).
# Usage: bash tools/measure_round.sh <tag> [configs for PMC, default "c3 c3_default c3_ref"]
set -o pipefail
TAG=${1:-measure}
CFGS=${2:-"c3 c3_default c3_ref"}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
# the headline's own launches (no variants): rocprof's average march duration is the one
# roofline.kernel_ms reports (bench_noV.json is the same command without the profiler)
timeout -k 10 600 python bench.py --no-cpu-baseline --no-variants > $O/bench_noV.json 2> $O/bench_noV.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-variants > $O/trace.log 2>&1 &&
for cfg in $CFGS; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${cfg}_$ctr -o run \
        --output-format csv -- python3 bench.py --config $cfg --no-variants --no-cpu-baseline \
        --steps 10 --warmup 3 > $O/pmc_${cfg}_$ctr.log 2>&1 || exit $?
  done
done &&
python tools/traffic_json.py $O $O/pmc_traffic.json > /dev/null &&
cp $O/pmc_traffic.json profiles/pmc_traffic.json &&
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
