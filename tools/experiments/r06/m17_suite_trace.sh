#!/bin/bash
# Round 6: the whole GPU suite and smoke on the current sources, then a kernel-trace summary of
# the bench with its variants (build kernels included).
set -o pipefail
O=gpurun_out/m17
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
    -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $O/trace.log 2>&1
