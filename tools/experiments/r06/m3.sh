#!/bin/bash
# round 6: host-cost breakdown, the ABI-9 eviction/downgrade tests, the orbit under the budgets
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/m3; mkdir -p $O
timeout -k 10 180 tools/bin/host_cost 3000 > $O/host_cost.json 2> $O/host_cost.err
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread --durations=0 \
  tests/test_gpu_round6.py tests/test_gpu_round4.py tests/test_gpu_round5.py > $O/pytest_r6.log 2>&1
for B in default unlimited; do
  timeout -k 10 200 python -u tools/orbit.py --budget $B > $O/orbit_$B.json 2> $O/orbit_$B.err
done
