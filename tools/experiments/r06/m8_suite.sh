#!/bin/bash
# round 6: the whole GPU suite (as the driver runs it) and smoke
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/m8; mkdir -p $O
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > $O/pytest_gpu.log 2>&1
echo "rc=$?" >> $O/pytest_gpu.log
