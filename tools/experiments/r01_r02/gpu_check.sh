#!/bin/bash
# GPU check of one build: parity tests, bench (C3 + reference-semantics variant), view sweeps.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
# Usage (on the box, via gpurun): bash tools/experiments/r01_r02/gpu_check.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-check}
shift || true
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python tools/view_sweep.py > $O/views_f32.txt 2>&1 &&
timeout -k 10 300 python tools/view_sweep.py --shading 1 --ert 1e-5 > $O/views_f32_shaded.txt 2>&1 &&
timeout -k 10 300 python tools/view_sweep.py --dtype uint8 --n 256 --size 1024x1024 > $O/views_u8.txt 2>&1 &&
timeout -k 10 300 python tools/view_sweep.py --shading 1 --ert 1e-5 --skip-empty 1 > $O/views_f32_shaded_skip.txt 2>&1 &&
timeout -k 10 300 python tools/view_sweep.py --skip-empty 1 > $O/views_f32_skip.txt 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
