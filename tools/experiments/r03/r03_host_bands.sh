#!/bin/bash
# Round 3: host-output frames (vr_render -> pageable host memory, the drop-in record() path)
# with 4 (lib), 8 (lib_b8) and 16 (lib_b16) row bands per frame; C3 shaded and unshaded;
# three alternating rounds.
set -o pipefail
TAG=${1:-r03_host_bands}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
for r in 1 2 3; do
  for L in lib lib_b8 lib_b16; do
    for sh in 1 0; do
      VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 200 python tools/host_output.py --shading $sh \
          >> $O/host_s$sh.jsonl 2>> $O/host.err || exit $?
    done
  done
done
echo done > $O/rc.txt
