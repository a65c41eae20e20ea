#!/bin/bash
# Round 3: frames in flight for the bench (the box's 4 hardware queues): F = 3, 4, 6, two
# alternating rounds of bench.py (variants on, no CPU baseline).
set -o pipefail
TAG=${1:-r03_fif}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for R in 1 2; do
  for F in 3 4 6; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --frames-in-flight $F \
        > $O/bench_f${F}_r$R.json 2> $O/bench_f${F}_r$R.err || exit $?
    python - $O/bench_f${F}_r$R.json $F <<'PY' | tee -a $O/summary.txt
import json, sys
d = json.load(open(sys.argv[1]))
v = d["variants"]
print(f"F={sys.argv[2]} headline {d['value']:.1f} ({d['ms_per_step']:.4f} ms)  default {v['default_camera']['value']:.1f}  "
      f"ref {v['reference_semantics_no_shading_no_ert']['value']:.1f}  skip {v['c3_skip_empty']['fps']:.0f} fps")
PY
  done
done
echo done > $O/rc.txt
