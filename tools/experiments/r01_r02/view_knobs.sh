#!/bin/bash
# Shaded C3 views with 3 frames in flight: launch knobs (base / pipelined / stencil+pipelined / stencil).
O=gpurun_out/${TAG:-r02_viewknobs}; mkdir -p $O
for r in 1 2; do for v in ${VIEWS:-diag side_x}; do for arm in base pipe nfpipe nf; do
  unset VR_PIPELINE VR_NO_GRAD_FIELD
  case $arm in pipe) export VR_PIPELINE=1;; nfpipe) export VR_PIPELINE=1 VR_NO_GRAD_FIELD=1;; nf) export VR_NO_GRAD_FIELD=1;; esac
  x=$(timeout -k 10 120 python tools/inflight_sweep.py --view $v --shading 1 --ert 1e-5 --ranks 1 --streams 3 --frames 150 2>>$O/err.txt | grep '"view"') || exit 1
  echo "r=$r $arm $x" | tee -a $O/out.txt
done; done; done
