#!/bin/bash
# Round 3: the stencil copy's shaded sparse view (default camera), pipelined kernel (policy;
# 106 VGPRs, 4 waves) against the single-stage kernel (knob pipeline=0; 78 VGPRs, 6 waves).
# 3 frames in flight, two rounds.
set -o pipefail
TAG=${1:-r03_stencil_pipe}
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
  run s_pipe default --shading 1 --ert 1e-5 --knob alt_geometry=4 --knob pipeline=1 || exit $?
  run s_single default --shading 1 --ert 1e-5 --knob alt_geometry=4 --knob pipeline=0 || exit $?
  run u_pipe default --knob alt_geometry=3 --knob pipeline=1 || exit $?
  run u_single default --knob alt_geometry=3 --knob pipeline=0 || exit $?
done
echo done > $O/rc.txt
