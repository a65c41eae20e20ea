#!/bin/bash
# Round 3: launch policy on the alternative-geometry views: pipelined vs single-stage (knob) for
# the default camera and the diagonal, shaded and unshaded, 4 frames in flight and serial.
set -o pipefail
TAG=${1:-r03_policy_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --views default,diag,side_x "$@" > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(14), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for R in 1 2; do
  for pp in 0 1; do
    run s_f4_pipe$pp --shading 1 --ert 1e-5 --inflight 4 --knob pipeline=$pp || exit $?
    run u_f4_pipe$pp --shading 0 --inflight 4 --knob pipeline=$pp || exit $?
    run s_f1_pipe$pp --shading 1 --ert 1e-5 --knob pipeline=$pp || exit $?
    run u_f1_pipe$pp --shading 0 --knob pipeline=$pp || exit $?
  done
  for f in 2 3 6; do
    run s_f$f --shading 1 --ert 1e-5 --inflight $f || exit $?
  done
done
echo done > $O/rc.txt
