#!/bin/bash
# Round 6: the C4 launch knobs re-swept on the current kernels (1024^3 u8 @ 2048^2, unshaded,
# 3 frames in flight, fill view): wave footprint (16x4 default, 8x8, 4x16) x tile order (4 default,
# 1 raster, 2 XCD bands, 3 XCD super-tiles).
set -o pipefail
O=gpurun_out/m15
mkdir -p $O
for ws in 0 1 3; do
  for to in 0 1 2 3; do
    timeout -k 10 200 python tools/view_sweep.py --n 1024 --dtype uint8 --size 2048x2048 --views fill,diag,default \
        --wave-shape $ws --tile-order $to --inflight 3 --reps 30 > $O/ws${ws}_to${to}.txt 2>&1 || exit $?
  done
done
