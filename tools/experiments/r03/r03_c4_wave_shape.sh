set -e
mkdir -p gpurun_out/c4ws
for r in 1 2; do
 for ws in 2 1 3; do
  timeout -k 10 120 python tools/view_sweep.py --n 1024 --dtype uint8 --size 2048x2048 --inflight 3 --reps 40 --wave-shape $ws --views fill,diag,default,side_x > gpurun_out/c4ws/r${r}_ws${ws}.log 2>&1
 done
done
