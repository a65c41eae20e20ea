#!/bin/bash
# Shaded C3 views, 3 frames in flight: difference field (default) vs stencil gradient (VR_NO_GRAD_FIELD)
# vs plain one-voxel f32 elements (lib_plain), alternating, two rounds (fresh process per arm).
O=gpurun_out/${TAG:-r02_gradviews}; mkdir -p $O
for r in 1 2; do for v in fill side_x diag default; do for arm in base nofield plain; do
  unset VR_NO_GRAD_FIELD VR_AMD_LIB
  [ $arm = nofield ] && export VR_NO_GRAD_FIELD=1
  [ $arm = plain ] && export VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_plain/libvr_amd.so
  x=$(timeout -k 10 120 python tools/inflight_sweep.py --view $v --shading 1 --ert 1e-5 --ranks 1 --streams 3 --frames 150 2>>$O/err.txt | grep '"view"') || exit 1
  echo "r=$r $arm $x" | tee -a $O/out.txt
done; done; done
