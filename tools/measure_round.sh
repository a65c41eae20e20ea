#!/bin/bash
# Round measurement on the GPU box: bench (with CPU baseline), its rocprofv3 kernel-trace
# summary, and PMC HBM-traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs) for C3 and the
# reference-semantics variant.  Each GPU step has its own time limit; chained with &&.
# Usage: bash tools/measure_round.sh <tag>
set -o pipefail
TAG=${1:-measure}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err &&
# the headline's own launches (no variants): rocprof's average march duration is the one
# roofline.kernel_ms reports (bench_noV.json is the same command without the profiler)
timeout -k 10 600 python bench.py --no-cpu-baseline --no-variants > $O/bench_noV.json 2> $O/bench_noV.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-variants > $O/trace.log 2>&1 &&
for cfg in c3 c3_ref; do
  if [ $cfg = c3 ]; then A="--shading 1 --ert 1e-5"; else A="--shading 0 --ert 0"; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${cfg}_$ctr -o run \
        --output-format csv -- python3 tools/prof_run.py $A --frames 10 > $O/pmc_${cfg}_$ctr.log 2>&1 || exit $?
  done
done
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
