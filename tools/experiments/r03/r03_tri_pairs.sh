#!/bin/bash
# Round 3: the f32 z-pair trilinear filter alone as packed-FP32 pairs (lib_tri, -DVR_TRI_PAIRS=1)
# against scalar (lib). Parity of the
# variant first (half-field, full-size and random-sweep GPU tests), then C3 bench lines
# (K = 100, W = 50, no variants), three alternating rounds.
set -o pipefail
TAG=${1:-r03_tri_pairs}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
VR_AMD_LIB=$LIBS/lib_tri/libvr_amd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_random.py -m gpu -q -x \
    --timeout 150 --timeout-method thread > $O/parity_lib_tri.log 2>&1 || exit $?
for r in 1 2 3; do
  for L in lib lib_tri; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config c3 --no-variants --no-cpu-baseline --steps 100 --warmup 50 \
        > $O/b_${L}_$r.json 2> $O/b_${L}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" \
        $O/b_${L}_$r.json $L | tee -a $O/bench.txt
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config c3_ref --no-variants --no-cpu-baseline --steps 100 --warmup 50 \
        > $O/bref_${L}_$r.json 2> $O/bref_${L}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ref', d['value'], d['ms_per_step'])" \
        $O/bref_${L}_$r.json $L | tee -a $O/bench.txt
  done
done
echo done > $O/rc.txt
