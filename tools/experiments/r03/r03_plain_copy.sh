#!/bin/bash
# Round 3: a plain one-voxel f32 copy (F32P, knob alt_geometry=3) for sparse views against the
# z-pair 15x15x8 copy (alt_geometry=2, today's choice) and the policy, on the views that would
# read it: the reference's default camera (r = 3) and a sparser r = 4 view; shaded and unshaded;
# 3 frames in flight.  Geometries: lib (15x15x15 cells), lib_p157 (15x15x7), lib_p31 (31x15x7).
# The GPU suite first (the F32P copy renders byte-identical frames).
set -o pipefail
TAG=${1:-r03_plain_copy}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
VR_PARITY_LOG=$O/parity_fullsize.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -q \
    --maxfail=10 --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit $?
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
      --views default,diag "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(9), sys.argv[2].ljust(10), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  for L in lib lib_p157 lib_p31; do
    run $L s_wide --shading 1 --ert 1e-5 --knob alt_geometry=2 || exit $?
    run $L s_plain --shading 1 --ert 1e-5 --knob alt_geometry=3 || exit $?
    run $L u_wide --knob alt_geometry=2 || exit $?
    run $L u_plain --knob alt_geometry=3 || exit $?
  done
done
echo done > $O/rc.txt
