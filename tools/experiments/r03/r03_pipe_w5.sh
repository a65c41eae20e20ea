#!/bin/bash
# Round 3: the pipelined stencil kernels (shaded sparse and oblique views) with a 5-wave floor
# on the final build (lib_pw5, -DVR_PIPE_MIN_WAVES=5: 102 -> 96 VGPRs, 4-10 spilled) against 4
# waves (lib).  Shaded default camera and diagonal views, 3 frames in flight, two rounds.
set -o pipefail
TAG=${1:-r03_pipe_w5}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
VR_AMD_LIB=$LIBS/lib_pw5/libvr_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
    -k alt_geometry --timeout 150 --timeout-method thread > $O/parity_lib_pw5.log 2>&1 || exit $?
for r in 1 2; do
  for L in lib lib_pw5; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
        --views default,diag,diag2 --shading 1 --ert 1e-5 > $O/vs_$L.txt 2> $O/vs_$L.err || exit $?
    python - "$L" "$O/vs_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(9), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
  done
done
echo done > $O/rc.txt
