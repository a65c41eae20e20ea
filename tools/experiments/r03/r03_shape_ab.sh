#!/bin/bash
# Round 3: wavefront pixel footprint (vr_params.wave_shape: 0 auto = 16x4, 1 = 8x8, 3 = 4x16)
# and tile order (0 auto = 4 adaptive, 3 static super-tiles) on the round-3 C3 shaded kernel,
# 3 frames in flight, two rounds.
set -o pipefail
TAG=${1:-r03_shape_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 --shading 1 --ert 1e-5 \
      --views fill,fill_oblique,top_z,side_x,diag,default "$@" > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(8), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  run ws0 || exit $?
  run ws1 --wave-shape 1 || exit $?
  run ws3 --wave-shape 3 || exit $?
  run to3 --tile-order 3 || exit $?
done
echo done > $O/rc.txt
