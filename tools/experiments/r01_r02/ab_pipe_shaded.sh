# shaded full frame: pipelined (default) vs one-lane (VR_PIPELINE=0) under the stable tile order
set -o pipefail
O=gpurun_out/ab_pipes; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python tools/view_sweep.py --shading 1 --ert 1e-5 > $O/views_def_$r.txt 2>&1 &&
  VR_PIPELINE=0 timeout -k 10 200 python tools/view_sweep.py --shading 1 --ert 1e-5 > $O/views_nopipe_$r.txt 2>&1 || exit $?
done
