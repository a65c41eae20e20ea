#!/bin/bash
# Round 3: f32 layout A/B per view: lib (z-pair 8^3 bricks), lib_plain (-DVR_F32_PLAIN=1: one
# voxel per element, 4 x 8-B loads per sample, half the bytes), lib_778 (-DVR_BRICK_CELLS=7,7,8).
# tools/view_sweep.py per library, shaded (policy) and unshaded, 4 frames in flight and serial,
# two alternating rounds.  Usage (GPU box): bash tools/experiments/r03/r03_layout_ab.sh <tag>
set -o pipefail
TAG=${1:-r03_layout_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 240 \
      python tools/view_sweep.py --reps 30 "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(9), sys.argv[2].ljust(12), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for R in 1 2; do
  for L in lib lib_plain lib_778; do
    run $L c3s_f4 --shading 1 --ert 1e-5 --inflight 4 --reps 60 || exit $?
    run $L c3u_f4 --shading 0 --inflight 4 --reps 60 || exit $?
    run $L c3s --shading 1 --ert 1e-5 || exit $?
  done
done
echo done > $O/rc.txt
