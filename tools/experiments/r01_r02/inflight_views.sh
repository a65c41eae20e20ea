#!/bin/bash
# Frames-in-flight throughput over views, shaded (C3) and unshaded, N = 1 and the N = 8 share;
# every GPU step under its own time limit, chained with &&.
# Usage (on the box, via gpurun): bash tools/experiments/r01_r02/inflight_views.sh <tag> [extra sweep args]
set -o pipefail
TAG=${1:-inflight}
shift || true
O=gpurun_out/$TAG
mkdir -p $O
: > $O/views.jsonl
for v in fill fill_oblique side_x top_z diag default; do
  timeout -k 10 120 python tools/inflight_sweep.py --view $v --ranks 1,8 --frames 100 --streams 1,2,3,4 "$@" >> $O/views.jsonl 2>>$O/err.log &&
  timeout -k 10 120 python tools/inflight_sweep.py --view $v --ranks 1,8 --frames 100 --streams 1,2,3,4 --shading 0 --ert 0 "$@" >> $O/views.jsonl 2>>$O/err.log || exit $?
done
