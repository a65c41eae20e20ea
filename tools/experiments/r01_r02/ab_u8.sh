#!/bin/bash
# NOTE (round 3): the VR_* launch-policy variables only act on an experiment build
# (make -C volumetric-renderer_amd EXTRA=-DVR_EXPERIMENTS LIBDIR=lib_exp BUILDDIR=build_exp, then
# VR_AMD_LIB=.../lib_exp/libvr_amd.so); the product library reads no environment (vr_debug.h).
# 8-bit layout A/B (plain 7x8x8-cell bricks vs yz-quads): GPU tests on the default build, view
# sweeps of C4 and C2 per library, the pipelined override on C4, C4/C5 bench lines and PMC
# HBM bytes of a C4 frame.  Usage (GPU box): bash tools/experiments/r01_r02/ab_u8.sh <tag> <lib_a> <lib_b>
set -o pipefail
TAG=$1; A=$2; B=$3
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $O/tests.log 2>&1 || exit $?
C4="--dtype uint8 --n 1024 --size 2048x2048 --shading 0"
C2="--dtype uint8 --n 256 --size 1024x1024 --shading 0"
AB_CFGS="$C4" bash tools/experiments/r01_r02/ab_views.sh $TAG $A $B $A $B || exit $?
AB_CFGS="$C2" bash tools/experiments/r01_r02/ab_views.sh $TAG $A $B || exit $?
VR_PIPELINE=1 AB_CFGS="$C4" bash tools/experiments/r01_r02/ab_views.sh $TAG/pipe1 $A $B || exit $?
VR_PIPELINE=0 AB_CFGS="$C4" bash tools/experiments/r01_r02/ab_views.sh $TAG/pipe0 $A $B || exit $?
for L in $A $B; do
  for cfg in c4 c5; do
    VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --config $cfg --no-variants --no-cpu-baseline --steps 20 > $O/bench_${cfg}_$L.json 2> $O/bench_${cfg}_$L.err || exit $?
  done
  for ctr in FETCH_SIZE WRITE_SIZE; do
    VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_c4_${L}_$ctr -o run --output-format csv -- python3 tools/prof_run.py --n 1024 --dtype uint8 --size 2048x2048 --shading 0 --ert 0 --frames 10 > $O/pmc_c4_${L}_$ctr.log 2>&1 || exit $?
  done
done
