#!/bin/bash
# Round 3, stencil copy step 4: brick geometry of the stencil copy (lib 29x13x13 cells, lib_g2
# 29x13x29, lib_g4 29x29x29, lib_g5 29x13x61, lib_g6 13x13x29), shaded default camera, 3 in flight.
# Parity of each build first (the alt-geometry test), then two alternating rounds.
set -o pipefail
TAG=${1:-r03_stencil4}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
ALL="lib_g2 lib_g4 lib_g5 lib_g6 lib"
for L in $ALL; do
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
  for L in $ALL; do
    run $L s_stencil default --shading 1 --ert 1e-5 --knob alt_geometry=4 || exit $?
  done
done
echo done > $O/rc.txt
