#!/bin/bash
# Round 3: a 5-wave floor on the pipelined stencil-gradient kernels (lib_pw5:
# -DVR_PIPE_MIN_WAVES=5, 96 VGPRs + 44 B spilled, against 126 VGPRs at 4 waves): shaded views
# that use the stencil (default camera, diagonal, a second oblique view), 3 in flight, 2 rounds.
set -o pipefail
TAG=${1:-r03_stencil_waves}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
for r in 1 2; do
  for L in lib lib_pw5; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
        --shading 1 --ert 1e-5 --views default,diag,diag2 > $O/vs_$L.txt 2> $O/vs_$L.err || exit $?
    python - "$L" "$O/vs_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(8), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
  done
done
echo done > $O/rc.txt
