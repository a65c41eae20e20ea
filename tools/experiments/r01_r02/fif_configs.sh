#!/bin/bash
# Frames in flight per 8-bit configuration (C2/C4/C5), alternating settings, past the
# cold-device ramp (50 / 20 warm-up frames).  Each run has its own time limit; the first
# failure ends the script.  Usage (GPU box): bash tools/experiments/r01_r02/fif_configs.sh <tag> <rounds> "<fifs>"
set -o pipefail
TAG=${1:-fif_configs}; R=${2:-2}; FIFS=${3:-"3 4 6"}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $R); do
  for cfg in c2 c4 c5; do
    if [ $cfg = c5 ]; then S="--steps 40 --warmup 20"; else S="--steps 100 --warmup 50"; fi
    for f in $FIFS; do
      timeout -k 10 300 python bench.py --config $cfg $S --no-cpu-baseline --no-variants \
        --frames-in-flight $f > $O/b.json 2> $O/b.err || exit 1
      python - "$r" "$cfg" "$f" "$O/b.json" <<'PY' | tee -a $O/fif.txt
import json, sys
d = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
print(sys.argv[1], sys.argv[2], "fif=" + sys.argv[3], d["value"], d["ms_per_step"], "frac", d["roofline"]["frac"])
PY
    done
  done
done
