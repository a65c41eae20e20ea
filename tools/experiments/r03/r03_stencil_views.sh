#!/bin/bash
# Round 3: the stencil copy (29^3 cells; knob alt_geometry=4) on the oblique views against the
# oblique copy (alt_geometry=1, their policy), shaded; and unshaded on the default camera
# against the plain copy (alt_geometry=3, its policy).  3 frames in flight, two rounds.
set -o pipefail
TAG=${1:-r03_stencil_views}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag views args...
  T=$1; V=$2; shift 2
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
      --views $V "$@" > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(12), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  run s_oblique diag,diag2,fill_oblique --shading 1 --ert 1e-5 --knob alt_geometry=1 || exit $?
  run s_stencil diag,diag2,fill_oblique --shading 1 --ert 1e-5 --knob alt_geometry=4 || exit $?
  run u_plain default --knob alt_geometry=3 || exit $?
  run u_stencil default --knob alt_geometry=4 || exit $?
done
echo done > $O/rc.txt
