#!/bin/bash
# A/B of experiment builds (make LIBDIR=lib_<name> BUILDDIR=build_<name> EXTRA=...): kernel
# time of C3 (shaded + ERT) and the reference-semantics frame per build, alternating builds
# over R rounds.  Usage (GPU box): bash tools/experiments/r01_r02/ab_libs.sh <tag> <rounds> lib lib_a lib_b ...
set -o pipefail
TAG=$1; R=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $R); do
  for L in "$@"; do
    for cfg in "--shading 1 --ert 1e-5" "--shading 0 --ert 0"; do
      VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so \
        timeout -k 10 120 python tools/prof_run.py $cfg --frames 20 > $O/run.json 2> $O/run.err || exit $?
      python -c "import json,sys; d=json.load(open('$O/run.json')); print('$L', '$cfg', round(d['kernel_ms'],4), round(d['gsamples_s'],1))" | tee -a $O/ab.txt
    done
  done
done
