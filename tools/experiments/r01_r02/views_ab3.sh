#!/bin/bash
# Shaded C3 views, 3 frames in flight, several libraries alternating (fresh process per arm), two rounds.
O=gpurun_out/${TAG:-r02_viewsab3}; mkdir -p $O
for r in 1 2; do for v in ${VIEWS:-side_x diag default}; do for L in "$@"; do
  x=$(VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 120 python tools/inflight_sweep.py --view $v --shading ${SH:-1} --ert 1e-5 --ranks 1 --streams 3 --frames 150 2>>$O/err.txt | grep '"view"') || exit 1
  echo "r=$r $L $x" | tee -a $O/out.txt
done; done; done
