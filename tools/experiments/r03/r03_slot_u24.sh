#!/bin/bash
# Round 3: the brick slot with 24-bit multiplies (lib, VR_SLOT_U24=1: v_mad_u32_u24, full rate)
# against 32-bit ones (lib_no24: the compiler's quarter-rate v_mad_u64_u32).  The GPU suite on
# lib first, then C3 and C4 bench lines (K = 100 / 60, no variants), three alternating rounds.
set -o pipefail
TAG=${1:-r03_slot_u24}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || exit $?
for r in 1 2 3; do
  for L in lib lib_no24; do
    for cfg in c3 c4; do
      st=100; [ $cfg = c4 ] && st=60
      VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
          python bench.py --config $cfg --no-variants --no-cpu-baseline --steps $st --warmup 50 \
          > $O/b_${cfg}_${L}_$r.json 2> $O/b_${cfg}_${L}_$r.err || exit $?
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" \
          $O/b_${cfg}_${L}_$r.json $L $cfg | tee -a $O/bench.txt
    done
  done
done
echo done > $O/rc.txt
