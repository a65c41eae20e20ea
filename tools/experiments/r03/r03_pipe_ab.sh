#!/bin/bash
# Round 3: the pipelined march as a wave-uniform loop (VR_PIPE_UNIFORM=1, lib/) against the
# round-2 loop (lib_old/, -DVR_PIPE_UNIFORM=0): GPU suite on lib/, per-view kernel times
# (serial frames and 4 in flight) for C3 unshaded (policy and pipelined forced), C3 shaded,
# C4 u8, C2 u8, then C3/C4/C5 bench lines per library.  Chained with && per step.
set -o pipefail
TAG=${1:-r03_pipe_ab}
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
for L in lib_old lib lib_old lib; do
  run $L c3u --shading 0 || exit $?
  run $L c3u_pipe --shading 0 --knob pipeline=1 || exit $?
  run $L c3s --shading 1 --ert 1e-5 || exit $?
  run $L c4 --dtype uint8 --n 1024 --size 2048x2048 --shading 0 || exit $?
  run $L c2 --dtype uint8 --n 256 --size 1024x1024 --shading 0 || exit $?
  run $L c3u_f4 --shading 0 --inflight 4 --reps 60 || exit $?
  run $L c3u_pipe_f4 --shading 0 --knob pipeline=1 --inflight 4 --reps 60 || exit $?
  run $L c3s_f4 --shading 1 --ert 1e-5 --inflight 4 --reps 60 || exit $?
  run $L c4_f4 --dtype uint8 --n 1024 --size 2048x2048 --shading 0 --inflight 4 --reps 60 || exit $?
done
for L in lib_old lib; do
  for cfg in c3 c4 c5; do
    VR_AMD_LIB=$GRAFT_REPO_ROOT/volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 \
        python bench.py --config $cfg --no-variants --no-cpu-baseline --steps 40 --warmup 10 \
        > $O/bench_${cfg}_$L.json 2> $O/bench_${cfg}_$L.err || exit $?
  done
done
echo done > $O/rc.txt
