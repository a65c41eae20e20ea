#!/bin/bash
# C3 bench line (headline + default-camera / reference-semantics / skip-empty variants) per
# hardware-queue count and frames in flight, alternating.  Each run has its own time limit;
# the first failure ends the script.  Usage (GPU box): bash tools/experiments/r01_r02/queues_fif.sh <tag> <rounds>
set -o pipefail
TAG=${1:-queues_fif}; R=${2:-2}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $R); do
  for q in 8 16; do
    for f in 4 6; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 \
        --frames-in-flight $f > $O/b.json 2> $O/b.err || exit 1
      python - "$r" "q=$q" "fif=$f" "$O/b.json" <<'PY' | tee -a $O/qf.txt
import json, sys
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
v = d["variants"]
print(sys.argv[1], sys.argv[2], sys.argv[3], "C3", d["value"], d["ms_per_step"],
      "default", v["default_camera"]["ms_per_step"],
      "ref", v["reference_semantics_no_shading_no_ert"]["ms_per_step"],
      "skip", v["c3_skip_empty"]["ms_per_step"])
PY
    done
  done
done
