#!/bin/bash
# Round 3: the binary16 field loads as device-scope (sc1) loads that skip the L1 (lib_byp,
# inline asm + manual waits) against cached loads (lib): parity tests of the field path on
# lib_byp first, then C3 shaded views (3 in flight) and C3 bench lines, alternating rounds.
set -o pipefail
TAG=${1:-r03_field_bypass}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
VR_AMD_LIB=$LIBS/lib_byp/libvr_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    -k "half_field or sparse_views or kernel_variants or f32_gradient_field" -q --timeout 150 \
    --timeout-method thread > $O/parity_byp.log 2>&1 || exit $?
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
      --views fill,fill_oblique,top_z,side_x "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(8), sys.argv[2].ljust(4), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  for L in lib lib_byp; do
    run $L s --shading 1 --ert 1e-5 || exit $?
  done
done
for r in 1 2 3; do
  for L in lib lib_byp; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config c3 --no-variants --no-cpu-baseline --steps 40 --warmup 10 \
        > $O/b_${L}_$r.json 2> $O/b_${L}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
        $O/b_${L}_$r.json $L | tee -a $O/bench.txt
  done
done
echo done > $O/rc.txt
