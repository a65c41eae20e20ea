#!/bin/bash
# Round 3: 8-bit z-pairs in 3x8x8-cell bricks (ZPair8, knob u8_layout=2: one 16-B load per
# sample, 3.4x the voxels) against the default layouts (plain 7x8x8 bricks: two 16-B loads,
# 1.45x; yz-quads for <= 2^25 voxels).  GPU suite first (ZPair8 renders the same bytes), then
# unshaded C4 / C5 / C2 views, 3 frames in flight.
set -o pipefail
TAG=${1:-r03_zpair8_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
VR_PARITY_LOG=$O/parity_fullsize.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q \
    --maxfail=10 --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
run() {  # tag args...
  T=$1; shift
  timeout -k 10 300 python tools/view_sweep.py --inflight 3 "$@" > $O/vs_$T.txt 2> $O/vs_$T.err || return $?
  python - "$T" "$O/vs_$T.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(12), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
C4="--dtype uint8 --n 1024 --size 2048x2048 --reps 60 --views fill,fill_oblique,side_x,top_z,diag,default"
for r in 1 2; do
  run c4_default $C4 || exit $?
  run c4_zpair $C4 --knob u8_layout=2 || exit $?
done
C2="--dtype uint8 --n 256 --size 1024x1024 --reps 60 --views fill,diag,default"
run c2_default $C2 || exit $?
run c2_zpair $C2 --knob u8_layout=2 || exit $?
run c2_plain $C2 --knob u8_layout=0 || exit $?
C5="--dtype uint8 --n 2048 --size 4096x4096 --reps 20 --views fill,diag"
run c5_default $C5 || exit $?
run c5_zpair $C5 --knob u8_layout=2 || exit $?
echo done > $O/rc.txt
