#!/bin/bash
# Round 6: lane groups for serial frames of sparse oblique-copy views -- the affected GPU tests,
# the orbit and grid sweeps with every variant (the policy's own choice now includes the lane
# groups), and the orbit variant.
set -o pipefail
O=gpurun_out/m13
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_round6.py tests/test_gpu_random.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/orbit_policy.py --stride 4 > $O/orbit_policy.jsonl 2> $O/err1.log &&
timeout -k 10 300 python -u tools/orbit_policy.py --path grid > $O/grid_shaded.jsonl 2> $O/err2.log &&
timeout -k 10 300 python -u tools/orbit.py > $O/orbit_budget5x.json 2> $O/err3.log &&
timeout -k 10 300 python -u tools/far_views.py > $O/far_views.jsonl 2> $O/err4.log
