#!/bin/bash
# Round 3: host-output frames into a page-locked buffer against a pageable one, with 2, 4
# (lib) and 8 row bands; C3 shaded; two alternating rounds.
set -o pipefail
TAG=${1:-r03_host_pinned}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
for r in 1 2; do
  for L in lib lib_b2 lib_b8; do
    for pin in 0 1; do
      VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 200 python tools/host_output.py --pinned $pin \
          >> $O/host.jsonl 2>> $O/host.err || exit $?
    done
  done
done
echo done > $O/rc.txt
