#!/bin/bash
# Round 3: compiler flags on top of the final build (-O3 -fno-slp-vectorize): lib_o2 (-O2),
# lib_nv (-fno-vectorize), lib_nu (-fno-unroll-loops; the explicit #pragma unroll loops stay).
# Parity of each variant (parity + full-size tests), then C3 and C4 bench lines, two rounds.
set -o pipefail
TAG=${1:-r03_flags}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
for L in lib_o2 lib_nv lib_nu; do
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -q -x \
      --timeout 150 --timeout-method thread > $O/parity_$L.log 2>&1 || exit $?
done
for r in 1 2; do
  for L in lib lib_o2 lib_nv lib_nu; do
    for cfg in c3 c4; do
      st=100; [ $cfg = c4 ] && st=60
      VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
          python bench.py --config $cfg --no-variants --no-cpu-baseline --steps $st --warmup 50 \
          > $O/b_${cfg}_${L}_$r.json 2> $O/b_${cfg}_${L}_$r.err || exit $?
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2].ljust(8), sys.argv[3].ljust(4), d['value'], d['ms_per_step'])" \
          $O/b_${cfg}_${L}_$r.json $L $cfg | tee -a $O/bench.txt
    done
  done
done
echo done > $O/rc.txt
