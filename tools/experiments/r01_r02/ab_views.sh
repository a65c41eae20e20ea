#!/bin/bash
# Per-view A/B of experiment builds: tools/view_sweep.py (non-shaded, and shaded + ERT) per
# library.  Usage (GPU box): bash tools/experiments/r01_r02/ab_views.sh <tag> lib lib_a ...
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for L in "$@"; do
  if [ -n "${AB_CFGS:-}" ]; then CFGS=("$AB_CFGS"); else CFGS=("--shading 0" "--shading 1 --ert 1e-5"); fi
  for cfg in "${CFGS[@]}"; do
    VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so \
      timeout -k 10 200 python tools/view_sweep.py $cfg --reps 30 > $O/run.txt 2> $O/run.err || exit $?
    python - "$L" "$cfg" "$O/run.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(9), sys.argv[2].ljust(22), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
  done
done
