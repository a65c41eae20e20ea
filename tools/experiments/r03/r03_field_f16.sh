#!/bin/bash
# Round 3 experiment: the difference field as f16 yz-quads, 3 x 16-B loads
# per shaded sample instead of 6 (lib_f16: -DVR_FIELD_F16=1, 5 waves; lib_f16w6: 6 waves),
# against the exact f32 field (lib/).  Not exact, so: the whole-frame C1/C3 parity tests on
# lib_f16 log their errors (VR_PARITY_LOG) without stopping at a failure, then per-view C3
# shaded kernel times and C3 bench lines per library.
set -o pipefail
TAG=${1:-r03_field_f16}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
VR_AMD_LIB=$LIBS/lib_f16/libvr_amd.so VR_PARITY_LOG=$O/parity_f16.jsonl timeout -k 10 300 \
    python -u -m pytest tests/test_gpu_fullsize.py -k "c1 or c3" -q --timeout 200 \
    --timeout-method thread > $O/parity_f16.log 2>&1
rc=$?
echo "parity rc=$rc" > $O/rc_parity.txt
[ $rc -le 1 ] || exit $rc   # 1 = assertion failures (expected to be possible); worse = stop
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 \
      python tools/view_sweep.py --reps 30 "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(9), sys.argv[2].ljust(8), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for L in lib lib_f16 lib_f16w6 lib lib_f16 lib_f16w6; do
  run $L c3s --shading 1 --ert 1e-5 || exit $?
  run $L c3s_f3 --shading 1 --ert 1e-5 --inflight 3 --reps 60 || exit $?
done
for L in lib lib_f16 lib_f16w6 lib lib_f16 lib_f16w6; do
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
      python bench.py --config c3 --no-variants --no-cpu-baseline --steps 40 --warmup 10 \
      >> $O/bench_c3_$L.json 2>> $O/bench_c3_$L.err || exit $?
done
echo done > $O/rc.txt
