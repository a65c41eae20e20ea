#!/bin/bash
# PMC passes (tools/pmc_sets_view.txt: TLB, L1/L2, HBM, TA/TD) of one march configuration on
# several cameras, to compare views.  Usage: bash tools/experiments/r01_r02/view_pmc.sh <tag> "<cams>" [prof_run args]
TAG=$1; CAMS=$2; shift 2
for c in $CAMS; do
  PASS_TIMEOUT=60 bash tools/pmc_passes.sh $TAG/$c tools/pmc_sets_view.txt --cam $c "$@" || exit $?
done
