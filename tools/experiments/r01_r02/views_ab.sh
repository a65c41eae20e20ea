#!/bin/bash
# Shaded C3 views, 3 frames in flight, two libraries alternating (fresh process per arm), two rounds.
A=$1; B=$2; O=gpurun_out/${3:-r02_viewsab}; mkdir -p $O
for r in 1 2; do for v in ${VIEWS:-fill side_x diag default}; do for L in $A $B; do
  x=$(VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 120 python tools/inflight_sweep.py --view $v --shading 1 --ert 1e-5 --ranks 1 --streams 3 --frames 150 2>>$O/err.txt | grep '"view"') || exit 1
  echo "r=$r $L $x" | tee -a $O/out.txt
done; done; done
