#!/bin/bash
# Round 3: lane groups (march_pair_kernel, 2 or 4 lanes per ray) on the reference's default
# camera and the diagonal with 3 frames in flight (the launch policy uses them only for serial
# frames), shaded and unshaded, two rounds.
set -o pipefail
TAG=${1:-r03_pair_sparse}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 --views default,diag "$@" \
      > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(10), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
S="--shading 1 --ert 1e-5"
for r in 1 2; do
  run s_policy $S || exit $?
  run s_pair2 $S --knob pair=1 --knob pair_lanes=2 || exit $?
  run s_pair4 $S --knob pair=1 --knob pair_lanes=4 || exit $?
  run u_policy || exit $?
  run u_pair2 --knob pair=1 --knob pair_lanes=2 || exit $?
done
echo done > $O/rc.txt
