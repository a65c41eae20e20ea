#!/bin/bash
# Alternating A/B of library builds on the headline bench line (C3, 3 frames in flight, no
# variants) and the shaded view sweep.  Usage (GPU box): bash tools/experiments/r01_r02/ab_bench.sh <tag> <rounds> lib_a lib_b ...
TAG=$1; R=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $R); do
  for L in "$@"; do
    VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-variants --no-cpu-baseline --steps 100 > $O/b.json 2> $O/b.err || exit 1
    python -c "import json; d=json.load(open('$O/b.json')); print('$r', '$L'.ljust(12), 'C3', d['value'], d['ms_per_step'])" | tee -a $O/ab_bench.txt
  done
done
AB_CFGS="--shading 1 --ert 1e-5" bash tools/experiments/r01_r02/ab_views.sh $TAG "$@" "$@"
