#!/bin/bash
# round 6: the fence-event scope A/B (C3 headline, alternating libraries), bench lines of
# C2/C4/C5, the driver-launch rehearsal and the member rehearsal
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06_final; mkdir -p $O
for r in 1 2; do
  for L in lib ab_sysfence; do
    VR_AMD_LIB=volumetric-renderer_amd/$L/libvr_amd.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-variants --steps 100 --warmup 5 > $O/ab_fence_${L}_$r.json 2> $O/ab_fence_${L}_$r.err || exit $?
  done
done
for c in c2 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 40 --warmup 5 > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
timeout -k 10 400 python bench.py --gpus 2 --rehearse-launch --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_rehearse_launch2.json 2> $O/bench_rehearse_launch2.err || exit $?
timeout -k 10 300 python bench.py --members-on-one-gpu 3 --steps 20 --warmup 5 --no-cpu-baseline --no-variants > $O/bench_members3.json 2> $O/bench_members3.err
