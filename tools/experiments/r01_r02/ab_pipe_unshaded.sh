# full-frame unshaded: pipelined (VR_PIPELINE=1) vs one-lane (default) under the stable tile order
set -o pipefail
O=gpurun_out/ab_pipeu; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python tools/view_sweep.py > $O/views_def_$r.txt 2>&1 &&
  VR_PIPELINE=1 timeout -k 10 200 python tools/view_sweep.py > $O/views_pipe_$r.txt 2>&1 || exit $?
done
for r in 1 2; do
  timeout -k 10 200 python tools/view_sweep.py --n 256 --dtype uint8 --size 1024x1024 > $O/u8_def_$r.txt 2>&1 &&
  VR_PIPELINE=0 timeout -k 10 200 python tools/view_sweep.py --n 256 --dtype uint8 --size 1024x1024 > $O/u8_nopipe_$r.txt 2>&1 || exit $?
done
