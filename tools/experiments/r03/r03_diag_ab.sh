#!/bin/bash
# Round 3: work placement for oblique views (diagonal, and a second oblique camera): tile
# order 3 (static super-tiles) and/or 8x8 wavefronts against the defaults (adaptive order,
# 16x4), shaded and unshaded, 3 frames in flight, two rounds.
set -o pipefail
TAG=${1:-r03_diag_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 --views diag,diag2 "$@" \
      > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(10), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
S="--shading 1 --ert 1e-5"
for r in 1 2; do
  run s_def $S || exit $?
  run s_to3 $S --tile-order 3 || exit $?
  run s_ws1 $S --wave-shape 1 || exit $?
  run s_both $S --tile-order 3 --wave-shape 1 || exit $?
  run u_def || exit $?
  run u_to3 --tile-order 3 || exit $?
  run u_ws1 --wave-shape 1 || exit $?
  run u_both --tile-order 3 --wave-shape 1 || exit $?
done
echo done > $O/rc.txt
