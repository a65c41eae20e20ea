#!/bin/bash
# NOTE (round 3): the VR_* launch-policy variables only act on an experiment build
# (make -C volumetric-renderer_amd EXTRA=-DVR_EXPERIMENTS LIBDIR=lib_exp BUILDDIR=build_exp, then
# VR_AMD_LIB=.../lib_exp/libvr_amd.so); the product library reads no environment (vr_debug.h).
# Per-view kernel-choice sweep (serial frames, tools/view_sweep.py) over the launch-policy
# overrides: pipelined / lane-pair (2, 4 lanes per ray) kernels and wavefront shapes.
# Usage (GPU box): bash tools/experiments/r01_r02/knob_sweep.sh <tag> "<view_sweep args>"
TAG=$1; ARGS=$2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for arm in "base:" "pipe1:VR_PIPELINE=1" "pipe0:VR_PIPELINE=0" "pair2:VR_PAIR=1 VR_PAIR_LANES=2" "pair4:VR_PAIR=1 VR_PAIR_LANES=4" "ws8x8:VS=--wave-shape=1" "ws4x16:VS=--wave-shape=3"; do
  name=${arm%%:*}; envs=${arm#*:}
  VS=""
  case "$envs" in VS=*) VS=${envs#VS=}; envs="";; esac
  env $envs timeout -k 10 200 python tools/view_sweep.py $ARGS $VS --reps 30 > $O/run.txt 2> $O/run.err || { echo "rc=$? $name" >> $O/knobs.txt; exit 1; }
  python - "$name" "$O/run.txt" <<'PY' | tee -a $O/knobs.txt
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(7), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
done
