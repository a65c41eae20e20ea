#!/bin/bash
# Round 3: packed-FP32 pairs measured slower when written by hand (pack_sample/, tri_pairs/), so
# without the compiler's own pairs: lib_noslp (-fno-slp-vectorize) and lib_noslp2 (+ the
# explicit lerp2 pairs as two scalar lerps, -DVR_LERP2_SCALAR=1) against lib.  Parity of both
# variants first, then C3, reference-semantics C3 and C4 bench lines, two alternating rounds.
set -o pipefail
TAG=${1:-r03_noslp}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
for L in lib_noslp lib_noslp2; do
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_random.py -m gpu -q -x \
      --timeout 150 --timeout-method thread > $O/parity_$L.log 2>&1 || exit $?
done
for r in 1 2; do
  for L in lib lib_noslp lib_noslp2; do
    for cfg in c3 c3_ref c4; do
      st=100; [ $cfg = c4 ] && st=60
      VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
          python bench.py --config $cfg --no-variants --no-cpu-baseline --steps $st --warmup 50 \
          > $O/b_${cfg}_${L}_$r.json 2> $O/b_${cfg}_${L}_$r.err || exit $?
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2].ljust(11), sys.argv[3].ljust(7), d['value'], d['ms_per_step'])" \
          $O/b_${cfg}_${L}_$r.json $L $cfg | tee -a $O/bench.txt
    done
  done
done
echo done > $O/rc.txt
