#!/bin/bash
# Round 6, final sources: the driver's multi-GPU launch path rehearsed on one GPU (gloo ranks
# through launch_ranks) and three members of one context on device 0 (copy exchange).
set -o pipefail
O=gpurun_out/m18
mkdir -p $O
timeout -k 10 400 python bench.py --gpus 2 --rehearse-launch --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_rehearse_launch2.json 2> $O/bench_rehearse_launch2.err &&
timeout -k 10 300 python bench.py --members-on-one-gpu 3 --steps 20 --warmup 5 --no-cpu-baseline --no-variants > $O/bench_members3.json 2> $O/bench_members3.err
