#!/bin/bash
# Round 3: with the binary16 field, does reading the field pay on the views that form the
# gradient from the stencil today (side, diagonal, default camera)?  C3 shaded, 3 frames in
# flight: launch policy (auto) vs the field forced on every view (knob grad_field=1) vs the
# exact f32 field forced (grad_field=1 + exact gradient is not a knob: f32 via lib only).
set -o pipefail
TAG=${1:-r03_field_views}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 --shading 1 --ert 1e-5 "$@" \
      > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(10), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  run auto || exit $?
  run field --knob grad_field=1 || exit $?
  run field_p0 --knob grad_field=1 --knob pipeline=0 || exit $?
done
echo done > $O/rc.txt
