#!/bin/bash
# Round 3: 8-bit plain bricks sampled with 4 byte-aligned dword loads (lib_u8d, -DVR_U8_DWORD=1:
# 4 B per lane per row) against 2 x 16-B loads from the 4-aligned address (lib).  Parity of the
# variant first (the GPU tests that render 8-bit volumes, and the full-size C4/C5 rows), then
# C4, C5 and C2 bench lines, alternating, 3 frames in flight.
set -o pipefail
TAG=${1:-r03_u8_dword}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
VR_AMD_LIB=$LIBS/lib_u8d/libvr_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_random.py -m gpu -q -x \
    --timeout 150 --timeout-method thread > $O/parity_lib_u8d.log 2>&1 || exit $?
for r in 1 2; do
  for cfg in c4 c5 c2; do
    for L in lib lib_u8d; do
      st=60; [ $cfg = c5 ] && st=20
      VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
          python bench.py --config $cfg --no-variants --no-cpu-baseline --steps $st --warmup 20 \
          > $O/b_${cfg}_${L}_$r.json 2> $O/b_${cfg}_${L}_$r.err || exit $?
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" \
          $O/b_${cfg}_${L}_$r.json $cfg $L | tee -a $O/bench.txt
    done
  done
done
echo done > $O/rc.txt
