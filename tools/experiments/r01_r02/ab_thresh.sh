# unshaded launches of 12-24 K wavefronts (C2 full frame, N=2 rank share): pipelined (policy) vs one-lane
set -o pipefail
O=gpurun_out/ab_thresh; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-variants > $O/c2_def_$r.json 2> $O/c2_def_$r.err &&
  VR_PIPELINE=0 timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-variants > $O/c2_one_$r.json 2> $O/c2_one_$r.err &&
  timeout -k 10 200 python tools/inflight_sweep.py --ranks 1,2,4 --frames 200 --streams 1,3 --shading 0 --ert 0 > $O/share_def_$r.json 2> $O/share_def_$r.err &&
  VR_PIPELINE=0 timeout -k 10 200 python tools/inflight_sweep.py --ranks 1,2,4 --frames 200 --streams 1,3 --shading 0 --ert 0 > $O/share_one_$r.json 2> $O/share_one_$r.err || exit $?
done
