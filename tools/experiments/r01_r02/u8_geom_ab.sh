#!/bin/bash
# Plain 8-bit brick geometry A/B (7x8x8 = 8-B rows vs 3x8x8 = 4-B rows): GPU tests on the
# second library, C4/C5 bench lines alternating, C4 views.  GPU box.
A=$1; B=$2; O=gpurun_out/r02_u8geom; mkdir -p $O
VR_AMD_LIB=$PWD/volumetric-renderer_amd/$B/libvr_amd.so timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests_$B.log 2>&1 || exit 1
for r in 1 2; do for L in $A $B; do for c in c4 c5; do
  VR_AMD_LIB=$PWD/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --config $c --no-variants --no-cpu-baseline --steps 30 > $O/b.json 2> $O/b.err || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); print('$r', '$L'.ljust(8), '$c', d['value'], d['ms_per_step'], d['config']['volume_resident_bytes'])" | tee -a $O/out.txt
done; done; done
AB_CFGS="--dtype uint8 --n 1024 --size 2048x2048 --shading 0" bash tools/experiments/r01_r02/ab_views.sh r02_u8geom $A $B
