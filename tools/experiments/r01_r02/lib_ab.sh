#!/bin/bash
# Library A/B: headline bench at the driver's K=20/W=5 and at K=200, alternating libraries.
A=$1; B=$2; O=gpurun_out/${3:-r02_ab}; mkdir -p $O
for r in 1 2; do for L in $A $B; do for kw in "20 5" "200 10"; do set -- $kw
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-variants --no-cpu-baseline --steps $1 --warmup $2 > $O/b.json 2> $O/b.err || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); print('$r', '$L'.ljust(8), 'K=$1 W=$2', d['value'], d['ms_per_step'])" | tee -a $O/out.txt
done; done; done
