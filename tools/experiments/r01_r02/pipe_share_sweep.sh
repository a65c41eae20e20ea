#!/bin/bash
# Pipelined vs single-stage march for unshaded rank shares (N = 1..8) with 3 frames in flight:
# C3 volume (f32 512^3 @ 1080p) and C2-size u8 (256^3 @ 1024^2).  GPU box; tools/inflight_sweep.py.
O=gpurun_out/r02_pipe_share; mkdir -p $O
for pp in 0 1; do
  for args in "--n 512 --dtype float32 --size 1920x1080" "--n 256 --dtype uint8 --size 1024x1024"; do
    echo "== VR_PIPELINE=$pp $args" >> $O/out.txt
    VR_PIPELINE=$pp timeout -k 10 200 python tools/inflight_sweep.py --shading 0 --ert 0 --streams 3 --ranks 1,2,4,8 --frames 150 $args 2>>$O/err.txt | grep -v '^{"args' >> $O/out.txt || exit 1
  done
done
