#!/bin/bash
# Round 3: the binary16-field headline kernel -- deferred shading at 5 waves (lib, 86 VGPRs)
# against no deferral at 6 waves (lib_nd, 76 VGPRs) and deferred at 6 waves (lib_d6, 80 VGPRs
# + 20 B spilled).  C3 shaded views that read the field, 3 frames in flight, then C3 bench
# lines; two alternating rounds.
set -o pipefail
TAG=${1:-r03_occupancy_ab}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
LIBS=$GRAFT_REPO_ROOT/volumetric-renderer_amd
run() {  # lib tag args...
  L=$1; T=$2; shift 2
  VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 240 python tools/view_sweep.py --reps 60 --inflight 3 \
      --views fill,fill_oblique,top_z,side_x "$@" > $O/vs_${T}_$L.txt 2> $O/vs_${T}_$L.err || return $?
  python - "$L" "$T" "$O/vs_${T}_$L.txt" <<'PY' | tee -a $O/ab.txt
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(sys.argv[1].ljust(7), sys.argv[2].ljust(6), " ".join(f"{k}={v['kernel_ms']:.4f}" for k, v in d["views"].items()))
PY
}
for r in 1 2; do
  for L in lib lib_nd lib_d6; do
    run $L s --shading 1 --ert 1e-5 || exit $?
  done
done
for r in 1 2; do
  for L in lib lib_nd lib_d6; do
    VR_AMD_LIB=$LIBS/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config c3 --no-variants --no-cpu-baseline --steps 40 --warmup 10 \
        >> $O/bench_c3_$L.json 2>> $O/bench_c3_$L.err || exit $?
  done
done
echo done > $O/rc.txt
