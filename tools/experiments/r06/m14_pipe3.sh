#!/bin/bash
# Round 6 A/B (rejected; the variant is tools/experiments/r06/pipe3_u8.patch): three samples in flight for the unshaded plain 8-bit march (VR_PIPE3_U8=1,
# volumetric-renderer_amd/ab_pipe3) against the product library, C4 and C5 alternating, after a
# whole-frame C4 parity check of the variant.
set -o pipefail
O=gpurun_out/m14
mkdir -p $O
AB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/ab_pipe3/libvr_amd.so
VR_AMD_LIB=$AB timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread \
    tests/test_gpu_fullsize.py -k "c4" > $O/pytest_c4_pipe3.log 2>&1 || exit $?
for cfg in c4 c5; do
  for rep in 1 2; do
    timeout -k 10 300 python bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 5 \
        > $O/${cfg}_lib_$rep.json 2> $O/${cfg}_lib_$rep.err || exit $?
    VR_AMD_LIB=$AB timeout -k 10 300 python bench.py --config $cfg --no-variants --no-cpu-baseline \
        --steps 40 --warmup 5 > $O/${cfg}_pipe3_$rep.json 2> $O/${cfg}_pipe3_$rep.err || exit $?
  done
done
