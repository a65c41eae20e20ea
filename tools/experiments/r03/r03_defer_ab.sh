#!/bin/bash
# Round 3: deferred shading in the pipelined difference-field kernel (lib/: VR_DEFER_SHADE=1,
# 5 waves) against the committed kernel (lib_old/: VR_DEFER_SHADE=0, 6 waves) and an occupancy
# control (lib_o5/: VR_DEFER_SHADE=0, 5 waves).  GPU suite on lib/ (whole-frame parity), then
# per-view kernel times of C3 shaded (serial and 3 in flight), then C3 bench lines per library.
set -o pipefail
TAG=${1:-r03_defer_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || exit $?
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 240 \
      python tools/view_sweep.py --reps 30 "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(8), sys.argv[2].ljust(14), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for L in lib_old lib lib_o5 lib_old lib lib_o5; do
  run $L c3s --shading 1 --ert 1e-5 || exit $?
  run $L c3s_f3 --shading 1 --ert 1e-5 --inflight 3 --reps 60 || exit $?
done
for L in lib_old lib lib_old lib; do
  VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 \
      python bench.py --config c3 --no-variants --no-cpu-baseline --steps 40 --warmup 10 \
      >> $O/bench_c3_$L.json 2>> $O/bench_c3_$L.err || exit $?
done
echo done > $O/rc.txt
