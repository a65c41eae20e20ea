#!/bin/bash
# Round 3: the stencil copy (F32S, knob alt_geometry=4: plain f32 in 13^3-cell bricks with a
# 1-below / 2-above apron, gradient taps at constant in-brick offsets) against the z-pair
# 15x15x8 copy (alt_geometry=2, today's shaded sparse choice), the oblique copy (1) and the plain
# copy (3), on the default camera and the diagonal; shaded and unshaded; 3 frames in flight.
# lib: x differences from one 16-B load per row at shade time; lib_sw (-DVR_STENCIL_WIDE=1):
# the density loads themselves are 16 B from x - 1.  Parity first (the alt-geometry test on
# both builds), then the A/B, then the whole GPU suite on lib.
set -o pipefail
TAG=${1:-r03_stencil_copy}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
for L in lib lib_sw; do
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
      -k alt_geometry --timeout 150 --timeout-method thread > $O/parity_$L.log 2>&1 || exit $?
done
run() {  # lib tag views args...
  L=$1; T=$2; V=$3; shift 3
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
      --views $V "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(9), sys.argv[2].ljust(10), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  echo "round $r" >> $O/ab.txt
  run lib s_wide default,diag --shading 1 --ert 1e-5 --knob alt_geometry=2 || exit $?
  run lib s_obl diag --shading 1 --ert 1e-5 --knob alt_geometry=1 || exit $?
  for L in lib lib_sw; do
    run $L s_stencil default,diag --shading 1 --ert 1e-5 --knob alt_geometry=4 || exit $?
    run $L u_stencil default --knob alt_geometry=4 || exit $?
  done
  run lib u_plain default --knob alt_geometry=3 || exit $?
done
VR_PARITY_LOG=$O/parity_fullsize.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q \
    --maxfail=10 --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
echo "rc=$?" > $O/rc.txt
