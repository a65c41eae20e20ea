#!/bin/bash
# Round 6, launch policy by ray axis and row alignment: the affected GPU tests, the orbit and
# grid sweeps (every variant forced beside the policy's own choice), the orbit variant under the
# default budget, and the host cost with the multi-device member rows.
set -o pipefail
O=gpurun_out/m11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_round6.py tests/test_gpu_members.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -u tools/orbit_policy.py --stride 4 > $O/orbit_policy.jsonl 2> $O/err1.log &&
timeout -k 10 300 python -u tools/orbit_policy.py --stride 4 --shading 0 > $O/orbit_policy_unshaded.jsonl 2> $O/err2.log &&
timeout -k 10 300 python -u tools/orbit_policy.py --path grid > $O/grid_shaded.jsonl 2> $O/err3.log &&
timeout -k 10 300 python -u tools/orbit_policy.py --path grid --shading 0 > $O/grid_unshaded.jsonl 2> $O/err4.log &&
timeout -k 10 300 python -u tools/orbit.py > $O/orbit_budget5x.json 2> $O/err5.log &&
timeout -k 10 300 tools/bin/host_cost 3000 > $O/host_cost.json 2> $O/err6.log
