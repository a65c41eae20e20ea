#!/bin/bash
# Round 3: the f32 GeomAlt copy (oblique/sparse views): GPU suite, per-view sweeps of the
# policy build (lib) against the copy forced off (knob) and on, 4 frames in flight, and the
# bench line.  Chained with && per step.
set -o pipefail
TAG=${1:-r03_alt}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || exit $?
run() {  # tag args...
  T=$1; shift
  timeout -k 10 240 python tools/view_sweep.py --reps 60 "$@" > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(16), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for R in 1 2; do
  run s_policy --shading 1 --ert 1e-5 --inflight 4 || exit $?
  run s_alt0 --shading 1 --ert 1e-5 --inflight 4 --knob alt_geometry=0 || exit $?
  run u_policy --shading 0 --inflight 4 || exit $?
  run u_alt0 --shading 0 --inflight 4 --knob alt_geometry=0 || exit $?
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
echo done > $O/rc.txt
