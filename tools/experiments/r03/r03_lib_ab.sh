#!/bin/bash
# Round 3: generic A/B of library builds (volumetric-renderer_amd/<lib>/libvr_amd.so): C3
# views shaded and unshaded (3 frames in flight), then C3 bench lines, alternating rounds.
# usage: r03_lib_ab.sh TAG lib libA [libB ...]
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
      --views fill,fill_oblique,top_z,side_x,diag,default "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(10), sys.argv[2].ljust(4), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  for L in "$@"; do
    run $L s --shading 1 --ert 1e-5 || exit $?
    run $L u || exit $?
  done
done
for r in 1 2 3; do
  for L in "$@"; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config c3 --no-variants --no-cpu-baseline --steps 40 --warmup 10 \
        > $O/b_${L}_$r.json 2> $O/b_${L}_$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
        $O/b_${L}_$r.json $L | tee -a $O/bench.txt
  done
done
echo done > $O/rc.txt
