#!/bin/bash
# Round 3: the binary16 field's x lerps as v_fma_mix_f32 (lib_mix, -DVR_FIELD_MIX=1: halves read
# in place, 12 fewer VALU per shaded sample) against convert-then-lerp (lib).  Parity of the
# variant first (half-field, full-size and random-sweep GPU tests), then C3 bench lines
# (K = 100, W = 50, no variants), three alternating rounds.
set -o pipefail
TAG=${1:-r03_field_mix}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
VR_AMD_LIB=$LIBS/lib_mix/libvr_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_random.py -m gpu -q -x \
    --timeout 150 --timeout-method thread > $O/parity_lib_mix.log 2>&1 || exit $?
for r in 1 2 3; do
  for L in lib lib_mix; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config c3 --no-variants --no-cpu-baseline --steps 100 --warmup 50 \
        > $O/b_${L}_$r.json 2> $O/b_${L}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" \
        $O/b_${L}_$r.json $L | tee -a $O/bench.txt
  done
done
echo done > $O/rc.txt
