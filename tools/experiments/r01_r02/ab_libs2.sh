#!/bin/bash
# A/B of builds (make LIBDIR=lib_<name> BUILDDIR=build_<name> EXTRA=...) or environment settings,
# alternating arms over R rounds: kernel ms of C3 (shaded + ERT), C3 reference semantics, the C3
# default camera and C4 (u8 1024^3 @ 2048^2) per arm, via tools/prof_run.py (20 frames).
# Usage (GPU box): bash tools/experiments/r01_r02/ab_libs2.sh <tag> <rounds> "<name>:<env>" ...
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $R); do
  for arm in "$@"; do
    name=${arm%%:*}; envs=${arm#*:}
    for cfg in "--shading 1 --ert 1e-5" "--shading 0 --ert 0" "--shading 1 --ert 1e-5 --cam default" "--shading 1 --ert 1e-5 --cam diag" "--shading 0 --ert 0 --n 1024 --dtype uint8 --size 2048x2048"; do
      env $envs timeout -k 10 120 python tools/prof_run.py $cfg --frames 20 > $O/run.json 2> $O/run.err || { echo "rc=$? $name $cfg" >> $O/ab.txt; exit 1; }
      python -c "import json,sys; d=json.load(open('$O/run.json')); print('$r', '$name'.ljust(8), '$cfg'.ljust(60), round(d['kernel_ms'],4), round(d['gsamples_s'],1))" | tee -a $O/ab.txt
    done
  done
done
