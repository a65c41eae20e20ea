#!/bin/bash
# Round 6: wave footprint (16x4 default, 8x8, 4x16) on the sparse views, C3 volume and params,
# serial and 3 frames in flight.
set -o pipefail
O=gpurun_out/m19
mkdir -p $O
for ws in 0 1 3; do
  for fl in 1 3; do
    timeout -k 10 200 python tools/view_sweep.py --shading 1 --ert 1e-5 --views fill,default,far_oblique,far_side,diag \
        --wave-shape $ws --inflight $fl --reps 20 > $O/ws${ws}_fl${fl}.txt 2>&1 || exit $?
  done
done
