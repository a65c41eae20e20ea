#!/bin/bash
# round 6: new frame schedule (fewer cross-stream edges) + fences: host cost, dist/group/member
# GPU tests, ABI-9 tests, the orbit
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/m6; mkdir -p $O
timeout -k 10 180 tools/bin/host_cost 3000 > $O/host_cost.json 2> $O/host_cost.err
timeout -k 10 560 python -u -m pytest -v --timeout 120 --timeout-method thread --durations=20 \
  tests/test_gpu_dist.py tests/test_gpu_members.py tests/test_gpu_group.py tests/test_gpu_round6.py \
  tests/test_gpu_round4.py tests/test_gpu_round5.py tests/test_gpu_bench.py > $O/pytest.log 2>&1 || true
for B in default unlimited; do
  timeout -k 10 200 python -u tools/orbit.py --budget $B > $O/orbit_$B.json 2> $O/orbit_$B.err
done
