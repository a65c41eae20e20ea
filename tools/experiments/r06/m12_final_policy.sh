#!/bin/bash
# Round 6, after the layout-policy change (kernels unchanged: profiles/pmc_traffic.json's
# machine-code key still matches, so no PMC passes): smoke, the headline alone, its rocprofv3
# kernel-trace summary, and the driver's bench command with variants and the CPU baseline.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r06_policy}
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --no-cpu-baseline --no-variants > $O/bench_noV.json 2> $O/bench_noV.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --no-variants > $O/trace.log 2>&1 &&
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
