#!/bin/bash
# Round 3: the plain f32 copy (F32P, 15^3 bricks, knob alt_geometry=3) on the dense-row views,
# unshaded (reference semantics) and shaded (stencil gradient), against the policy (8^3
# z-pairs; shaded: binary16 field), 3 frames in flight, two rounds.
set -o pipefail
TAG=${1:-r03_plain_dense}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
      --views fill,fill_oblique,top_z,side_x "$@" > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(10), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  run u_policy || exit $?
  run u_plain --knob alt_geometry=3 || exit $?
  run s_policy --shading 1 --ert 1e-5 || exit $?
  run s_plain --shading 1 --ert 1e-5 --knob alt_geometry=3 --knob grad_field=0 || exit $?
done
echo done > $O/rc.txt
