#!/bin/bash
# Default-camera (r = 3) shaded C3 with 3 frames in flight: launch knobs on the stencil-gradient path.
O=gpurun_out/${TAG:-r02_defknobs}; mkdir -p $O
for r in 1 2; do for arm in base pipe field; do
  unset VR_PIPELINE VR_FIELD_MAX_SPAN
  [ $arm = pipe ] && export VR_PIPELINE=1
  [ $arm = field ] && export VR_FIELD_MAX_SPAN=1e30
  x=$(timeout -k 10 120 python tools/inflight_sweep.py --view default --shading 1 --ert 1e-5 --ranks 1 --streams 3 --frames 150 2>>$O/err.txt | grep '"view"') || exit 1
  echo "r=$r $arm $x" | tee -a $O/out.txt
done; done
