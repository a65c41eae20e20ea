#!/bin/bash
# Alternating A/B of library builds on the whole bench line (C3 headline + its default-camera,
# reference-semantics and skip-empty variants, 4 frames in flight) and serial per-view kernel
# times (unshaded, shaded + ERT), after the parity suites under the first candidate build.
# Usage (GPU box): bash tools/experiments/r01_r02/ab_full.sh <tag> <rounds> lib lib_b ...
set -o pipefail
TAG=$1; R=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
T="timeout -k 10"
for L in "$@"; do
  [ "$L" = lib ] && continue
  VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so $T 300 python -u -m pytest \
    tests/test_gpu_parity.py tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > $O/tests_$L.log 2>&1 || exit 1
done
for r in $(seq 1 $R); do
  for L in "$@"; do
    VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so $T 300 python bench.py \
      --no-cpu-baseline --steps 50 > $O/b.json 2> $O/b.err || exit 1
    python - "$r" "$L" "$O/b.json" <<'PY' | tee -a $O/ab_bench.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
v = d["variants"]
print(sys.argv[1], sys.argv[2].ljust(8), "C3", d["value"], d["ms_per_step"],
      "default", v["default_camera"]["ms_per_step"],
      "ref", v["reference_semantics_no_shading_no_ert"]["ms_per_step"],
      "skip", v["c3_skip_empty"]["ms_per_step"])
PY
  done
done
for r in $(seq 1 $R); do
  bash tools/experiments/r01_r02/ab_views.sh $TAG "$@" || exit 1
done
