#!/bin/bash
# Round 3: work placement on the stencil copy's view (shaded default camera, 3 frames in
# flight): wavefront shape (0 auto = 16x4, 1 = 8x8, 3 = 4x16) and tile order (0 auto = adaptive
# (4), 1..3 the static orders).  Two rounds.
set -o pipefail
TAG=${1:-r03_stencil_place}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 --views default \
      --shading 1 --ert 1e-5 "$@" > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(12), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  run auto || exit $?
  run wave8x8 --wave-shape 1 || exit $?
  run wave4x16 --wave-shape 3 || exit $?
  run order1 --tile-order 1 || exit $?
  run order2 --tile-order 2 || exit $?
  run order3 --tile-order 3 || exit $?
done
echo done > $O/rc.txt
