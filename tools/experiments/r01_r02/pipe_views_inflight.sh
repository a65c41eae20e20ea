#!/bin/bash
# Unshaded full frames, 3 frames in flight: pipelined vs single-stage march per view (C3 volume).
O=gpurun_out/${TAG:-r02_pipeviews}; mkdir -p $O
SH=${SH:-"--shading 0 --ert 0"}
for v in fill fill_oblique side_x top_z diag default; do for pp in 0 1; do
  r=$(VR_PIPELINE=$pp timeout -k 10 120 python tools/inflight_sweep.py --view $v $SH --ranks 1 --streams 3 --frames 150 2>>$O/err.txt | grep '"view"') || exit 1
  echo "pipe=$pp $r" | tee -a $O/out.txt
done; done
