#!/bin/bash
# NOTE (round 3): the VR_* launch-policy variables only act on an experiment build
# (make -C volumetric-renderer_amd EXTRA=-DVR_EXPERIMENTS LIBDIR=lib_exp BUILDDIR=build_exp, then
# VR_AMD_LIB=.../lib_exp/libvr_amd.so); the product library reads no environment (vr_debug.h).
# A/B of the LDS-staged march against the bricked gather kernels on the GPU box: parity suites
# under VR_LDS=1 first (every frame checked against the oracle), then per-view kernel times of
# each arm (f32 shaded + ERT, f32 reference semantics, u8 1024^3 @ 2048^2).  Each GPU step has
# its own time limit; chained (the first failure ends the script).
# Usage: bash tools/experiments/r01_r02/ab_lds.sh <tag> "<name>:<env settings>" ...
#   e.g. "gather:VR_LDS=0" "lds:VR_LDS=1" "lds3wg:VR_LDS=1 VR_AMD_LIB=$PWD/volumetric-renderer_amd/lib_b23/libvr_amd.so"
set -o pipefail
TAG=${1:-ab_lds}
shift
O=gpurun_out/$TAG
mkdir -p $O
T="timeout -k 10"
env VR_LDS=1 $T 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py tests/test_gpu_inputs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests_lds.log 2>&1 || { echo "rc=$?" > $O/rc.txt; exit 1; }
for arm in "$@"; do
  name=${arm%%:*}; envs=${arm#*:}
  for v in "--shading 1 --ert 1e-5" "--shading 0" "--dtype uint8 --n 1024 --size 2048x2048"; do
    f=$O/views_${name}_$(echo $v | tr -d ' -').txt
    env $envs $T 200 python tools/view_sweep.py $v --reps 10 > $f 2>&1 || { echo "rc=$? $name $v" > $O/rc.txt; exit 1; }
    python - "$name" "$v" "$f" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(10), sys.argv[2].ljust(42), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
  done
done
echo "rc=0" > $O/rc.txt
