#!/bin/bash
# Round 3: which brick geometry the f32 alt copy should use: lib (7x7x8) against
# lib_a1578 (15x7x8), lib_a7158 (7x15x8), lib_a7716 (7x7x16), lib_a15158 (15x15x8), on the views
# the copy serves (default camera, diagonal), alt forced on, 4 frames in flight, two rounds.
set -o pipefail
TAG=${1:-r03_altgeom_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 240 \
      python tools/view_sweep.py --reps 60 --views default,diag,fill_oblique "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(11), sys.argv[2].ljust(6), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for R in 1 2; do
  for L in lib lib_a1578 lib_a7158 lib_a7716 lib_a15158; do
    run $L s --shading 1 --ert 1e-5 --inflight 4 --knob alt_geometry=1 || exit $?
    run $L u --shading 0 --inflight 4 --knob alt_geometry=1 || exit $?
  done
done
echo done > $O/rc.txt
