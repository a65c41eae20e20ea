#!/bin/bash
# NOTE (round 3): the VR_* launch-policy variables only act on an experiment build
# (make -C volumetric-renderer_amd EXTRA=-DVR_EXPERIMENTS LIBDIR=lib_exp BUILDDIR=build_exp, then
# VR_AMD_LIB=.../lib_exp/libvr_amd.so); the product library reads no environment (vr_debug.h).
# Per-view A/B of one build under environment settings (e.g. VR_PIPELINE=0 / 1).
# Usage (GPU box): bash tools/experiments/r01_r02/ab_env.sh <tag> "<cfg args>" "ENV=a" "ENV=b" ...
set -o pipefail
TAG=$1; CFG=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for E in "$@"; do
  env $E timeout -k 10 200 python tools/view_sweep.py $CFG --reps 30 > $O/run.txt 2> $O/run.err || exit $?
  python - "$E" "$CFG" "$O/run.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(14), sys.argv[2].ljust(40), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
done
