#!/bin/bash
# round 6, first measurement: host cost breakdown of a multi-GPU frame; u8 layouts at C4/C5
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/m1; mkdir -p $O
timeout -k 10 180 tools/bin/host_cost 3000 > $O/host_cost.json 2> $O/host_cost.err
for L in 0 1; do
  timeout -k 10 240 python -u tools/view_sweep.py --n 1024 --dtype uint8 --size 2048x2048 \
    --knob u8_layout=$L --inflight 3 --reps 40 --views fill,fill_oblique,diag,default > $O/c4_layout$L.txt 2>&1
done
for L in 0 1; do
  timeout -k 10 300 python -u tools/view_sweep.py --n 2048 --dtype uint8 --size 4096x4096 \
    --knob u8_layout=$L --inflight 3 --reps 12 --views fill > $O/c5_layout$L.txt 2>&1
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=0 \
  tests/test_gpu_fullsize.py tests/test_gpu_bench.py -k "c4 or c5 or rehearses or device_count" > $O/pytest_new.log 2>&1
